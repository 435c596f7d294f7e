"""Site-mean collectives with explicit payload precision and FP32 accumulation.

The reference's remote averages the sites' gradients it received as files, 16-bit ones as IEEE
half when ``precision_bits`` is 16 (``/root/reference/compspec.json:161-176``).  Here every site
holds the mean after a two-phase DIRECT exchange (``csrc/kernels/payload.hip``):

    pack (fp32 -> payload, zero-padded to world * chunk)
    all_to_all        rank r receives chunk r from every site
    rowsum            fp32 sum of the world chunks, * 1/world, one rounding to the payload type
    all_gather        of the mean chunks
    unpack (payload -> fp32)

Traffic per rank is the reduce-scatter + all-gather volume of a ring all-reduce, but every chunk
goes straight to its owner: on the MI355X node's fully-connected xGMI mesh (7 links per GPU) an
all-to-all drives all links at once instead of walking a ring one link per hop, and there is no
16-bit accumulation anywhere (an all-reduce on a 16-bit buffer rounds its partial sums at every
hop; SURVEY.md §2.4 asks for a direct 7-peer path for these <=4 MB payloads).

``payload`` names the wire type: ``"fp16"`` (the reference's half, default for
``precision_bits=16``), ``"bf16"`` (wider range, 3 fewer mantissa bits) or ``"fp32"``.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.distributed as dist

from ..ops import _lib

Tensor = torch.Tensor

PAYLOAD_TYPES = {"bf16": (0, torch.bfloat16), "fp16": (1, torch.float16), "fp32": (2, torch.float32)}

_lib.register("dn_payload_pack", [_lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_long,
                                  _lib.c_float, _lib.c_int, _lib.c_int, _lib.c_void_p])
_lib.register("dn_payload_unpack", [_lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_float,
                                    _lib.c_int, _lib.c_void_p])
_lib.register("dn_payload_rowsum", [_lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_long, _lib.c_float,
                                    _lib.c_int, _lib.c_void_p])

HDR = 8    # header elements per sub-block: [e, 0 x 7], the sub-block holds payload(x * 2^e)
SB = 2048  # data elements per sub-block (payload.hip): fp16 scales are per sub-block


def payload_name(cfg: Optional[dict]) -> str:
    """The wire type a config asks for: ``payload_dtype`` if set, else fp16 at
    ``precision_bits=16`` and fp32 otherwise."""
    cfg = cfg or {}
    name = cfg.get("payload_dtype")
    if name is None:
        name = "fp16" if str(cfg.get("precision_bits", "32")) == "16" else "fp32"
    name = str(name).lower()
    if name not in PAYLOAD_TYPES:
        raise ValueError(f"payload_dtype {name!r}: expected one of {sorted(PAYLOAD_TYPES)}")
    return name


def _code(dtype) -> int:
    return next(c for c, t in PAYLOAD_TYPES.values() if t == dtype)


def _scale_exp(amax: float) -> int:
    """max|x| * 2^e < 2^15 (payload.hip scale_exp)."""
    if not (amax > 0.0) or amax == float("inf"):
        return 0
    e = 15 - math.frexp(amax)[1]
    return max(-100, min(100, e))


def payload_numel(elems: int) -> int:
    """Payload elements holding ``elems`` data elements: whole sub-blocks of [HDR | SB]."""
    return -(-int(elems) // SB) * (HDR + SB)


def blocks_numel(world: int, chunk: int) -> int:
    """``world`` rank-blocks of ``chunk`` data elements (a multiple of SB) each."""
    return world * payload_numel(chunk)


def chunk_for(n: int, world: int) -> int:
    """Per-rank data elements of a ``world``-way exchange of ``n``: whole sub-blocks."""
    return max(SB, -(-int(n) // (SB * world)) * SB)


def to_payload(src: Tensor, dst: Tensor, world: int, chunk: int, scale: float = 1.0,
               scaled: Optional[bool] = None):
    """fp32 ``src`` -> ``dst``: ``world`` rank-blocks of ``chunk`` elements (a multiple of SB) as
    sub-blocks of [header | SB] in the payload dtype, zero past ``src``.  fp16 sub-blocks are
    scaled by 2^e from their own max |x| (``scaled``, default: fp16), computed inside the pack
    launch (payload.hip)."""
    n = src.numel()
    fp16 = dst.dtype == torch.float16
    scaled = fp16 if scaled is None else bool(scaled and fp16)
    if chunk % SB or world * chunk < n or dst.numel() < blocks_numel(world, chunk):
        raise ValueError(f"to_payload: {n} elements into {world} x {chunk} (sub-blocks of {SB}) "
                         f"in {dst.numel()}")
    if dst.is_cuda:
        _lib.call("dn_payload_pack", src.data_ptr(), dst.data_ptr(), n, world, chunk, scale,
                  int(scaled), _code(dst.dtype), _lib.stream())
        return
    nsb = world * chunk // SB
    body = torch.zeros(nsb * SB, dtype=torch.float32)
    body[:n] = src.reshape(-1).float()
    b = body.view(nsb, SB)
    if scaled:
        e = torch.tensor([_scale_exp(float(a)) for a in b.abs().max(1).values], dtype=torch.float32)
    else:
        e = torch.zeros(nsb)
    v = dst[:nsb * (HDR + SB)].view(nsb, HDR + SB)
    v[:, :HDR] = 0
    v[:, 0] = e.to(dst.dtype)
    v[:, HDR:] = (b * (scale * torch.pow(2.0, e))[:, None]).to(dst.dtype)


def from_payload(src: Tensor, dst: Tensor, world: Optional[int] = None,
                 chunk: Optional[int] = None, scale: float = 1.0):
    """The first ``dst.numel()`` data elements of a payload (sub-blocks back to back: one
    rank-block or several whole ones) -> fp32 ``dst``, each sub-block unscaled by its 2^-e."""
    n = dst.numel()
    if dst.is_cuda:
        _lib.call("dn_payload_unpack", src.data_ptr(), dst.data_ptr(), n, scale, _code(src.dtype),
                  _lib.stream())
        return
    nsb = -(-n // SB)
    v = src[:nsb * (HDR + SB)].view(nsb, HDR + SB)
    un = torch.pow(2.0, -v[:, :1].float())
    body = (v[:, HDR:].float() * un).reshape(-1)[:n]
    dst.reshape(-1).copy_(body * scale if scale != 1.0 else body)


def rowsum(src: Tensor, dst: Tensor, world: int, chunk: int, scale: float):
    """``dst`` (one rank-block) = payload(scale * sum_w unscaled fp32(src[w])) per sub-block --
    fp32 accumulation in rank order, rescaled by the sub-block's smallest exponent."""
    if dst.is_cuda:
        _lib.call("dn_payload_rowsum", src.data_ptr(), dst.data_ptr(), world, chunk, scale,
                  _code(dst.dtype), _lib.stream())
        return
    nsb = chunk // SB
    v = src[:blocks_numel(world, chunk)].view(world, nsb, HDR + SB)
    es = v[:, :, 0].float()
    acc = torch.zeros(nsb, SB, dtype=torch.float32)
    for w in range(world):
        acc += v[w, :, HDR:].float() * torch.pow(2.0, -es[w])[:, None]
    e = es.min(0).values
    out = dst[:nsb * (HDR + SB)].view(nsb, HDR + SB)
    out[:, :HDR] = 0
    out[:, 0] = e.to(dst.dtype)
    out[:, HDR:] = (acc * (scale * torch.pow(2.0, e))[:, None]).to(dst.dtype)


class DirectMean:
    """Mean over sites of one fp32 range of ``n`` elements with a ``payload`` wire type.  The
    buffers are allocated once (they live across steps, which keeps the exchange free of
    allocator traffic and lets it run on a side stream)."""

    def __init__(self, group, n: int, payload: str, device):
        self.group = group
        self.n = int(n)
        self.code, self.dtype = PAYLOAD_TYPES[payload]
        W = group.world
        self.chunk = chunk_for(self.n, W)   # per-rank slice: whole sub-blocks
        self.send = torch.zeros(blocks_numel(W, self.chunk), dtype=self.dtype, device=device)
        self.recv = torch.zeros_like(self.send)
        self.mine = torch.zeros(payload_numel(self.chunk), dtype=self.dtype, device=device)

    def _a2a(self):
        g = self.group
        if g.backend == "gloo" and self.send.is_cuda:  # one-GPU multi-site rehearsal
            r = torch.empty(self.recv.numel(), dtype=self.dtype)
            dist.all_to_all_single(r, self.send.cpu(), group=g.pg)
            self.recv.copy_(r)
        else:
            dist.all_to_all_single(self.recv, self.send, group=g.pg)

    def run_(self, x: Tensor, scale: float = 1.0):
        """``x`` (fp32, ``n`` elements, contiguous) <- scale * mean over sites, on the current
        stream (RCCL orders its collectives after it)."""
        W, c = self.group.world, self.chunk
        to_payload(x.reshape(-1), self.send, W, c)
        self._a2a()
        rowsum(self.recv, self.mine, W, c, 1.0 / W)
        self.group.all_gather_into(self.send, self.mine)
        from_payload(self.send, x.reshape(-1), W, c, scale)
        return self.n * self.send.element_size()  # this site's payload


class _EventWork:
    """``Work``-like handle of an exchange running on a side stream."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class _DoneWork:
    def wait(self):
        pass


def launch_on(stream, fn):
    """Run ``fn`` on ``stream`` after everything already queued on the current stream; returns a
    handle whose ``wait()`` orders the current stream after it (no host synchronisation)."""
    if stream is None:
        fn()
        return _DoneWork()
    cur = torch.cuda.current_stream()
    stream.wait_stream(cur)
    with torch.cuda.stream(stream):
        fn()
        ev = torch.cuda.Event()
        ev.record(stream)
    return _EventWork(ev)
