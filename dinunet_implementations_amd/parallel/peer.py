"""Peer exchange over IPC-mapped HBM: the engines' site-means and factor all-gathers without RCCL
(``csrc/kernels/peer.hip``).

The reference's sites reach the mean through a remote aggregator, one file round trip per step
(``/root/reference/local.py:49``, ``/root/reference/remote.py:37``).  On an MI355X node every
GPU has its own xGMI link to each of its 7 peers, and these payloads are small (<= 4.25 MB): the
exchange here is one-sided writes straight into the peers' HBM, synchronised by flag words,
issued as ordinary kernels on the step's stream -- so it is captured in the step's HIP graph like
any other launch, with any process-group backend (the group only carries the one-time handle
exchange):

* every site allocates one uncached arena and exports it (``hipIpcGetMemHandle``); every peer
  maps it (``hipIpcOpenMemHandle``) -- ``PeerArena``, one per site group, carved into regions in
  the same order on every site;
* ``PeerMean``: push (my chunk d -> site d's inbox), reduce (my chunk: fp32 sum in site order,
  * 1/W, written into every site's gather slot), unpack -- three launches, each waiting only for
  an earlier phase of its peers, never for a peer launch to be co-resident with it;
* ``PeerGather``: the factor all-gather of rank-dAD (credit-based slot reuse).

Wire types as ``collective``: fp32, bf16, or the reference's fp16 with a power-of-two scale per
2,048-element sub-block; the sums are always fp32.  A wait that times out (a dead peer; default
20 s, ``DINUNET_PEER_TIMEOUT_MS``) sets the arena's sticky error word, which
``runtime.health.check`` reports instead of the step silently using stale data.
"""
from __future__ import annotations

import ctypes
import os
import weakref
from typing import Dict, List, Optional

import torch

from ..ops import _lib
from .collective import PAYLOAD_TYPES, SB, payload_numel

MAXW = 16
ALIGN = 256
ARENA_BYTES = 64 << 20

_lib.register("dn_peer_alloc", [_lib.c_long, _lib.c_void_p])
_lib.register("dn_peer_free", [_lib.c_void_p])
_lib.register("dn_peer_export", [_lib.c_void_p, _lib.c_void_p])
_lib.register("dn_peer_open", [_lib.c_void_p, _lib.c_void_p])
_lib.register("dn_peer_close", [_lib.c_void_p])
_lib.register("dn_peer_fill_u32", [_lib.c_void_p, ctypes.c_uint, _lib.c_long])
_lib.register("dn_peer_launch", [_lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_void_p])
_lib.register("dn_peer_wait", [_lib.c_void_p, _lib.c_int, _lib.c_void_p])
_lib.register("dn_peer_set_timeout_ms", [_lib.c_long])

PUSH, REDUCE, UNPACK, GPUSH, GCOLLECT = range(5)
# error-word codes (peer.hip): phase << 8 | peer
PHASES = {1: "reduce-scatter wait (peer push)", 2: "all-gather wait (owner reduce)",
          3: "gather credit wait (reader)", 4: "gather data wait (peer push)"}


class _PxArgs(ctypes.Structure):
    _fields_ = [("inbox", ctypes.c_void_p * MAXW), ("gath", ctypes.c_void_p * MAXW),
                ("flags", ctypes.c_void_p * MAXW), ("src", ctypes.c_void_p),
                ("dst", ctypes.c_void_p), ("err", ctypes.c_void_p), ("n", ctypes.c_long),
                ("chunk", ctypes.c_long), ("dstride", ctypes.c_long), ("timeout", ctypes.c_long),
                ("W", ctypes.c_int), ("me", ctypes.c_int), ("scaled", ctypes.c_int),
                ("scale", ctypes.c_float), ("scale_red", ctypes.c_float), ("mode", ctypes.c_int)]


# hand-off form (peer.hip PxArgs.mode): bit 0 = release by store drain only, bit 1 = system-scope
# payload loads instead of an acquire invalidate.  Default 3: every byte a peer reads -- payload
# and flag words -- is an uncached store / a system-scope load, so the full system fences' L2
# write-back and invalidate touch nothing the exchange uses; the release is each storing wave's
# vmcnt(0) drain (the completion the memory model's system release waits for after its
# write-back).  Loopback fp16 step (split form) 0.3643 (fences) -> 0.3564 (bit 1) -> 0.3497-0.3502
# ms (both; one unsplit exchange since: 0.3255, profiles/r6_peer_unsplit_ab.jsonl), the multi-process peer and oracle suites pass with it (profiles/r6_peer_mode_ab.jsonl,
# profiles/r6_peer_mode3.jsonl); DINUNET_PEER_MODE=0 restores the fences.
MODE = int(os.environ.get("DINUNET_PEER_MODE", "3"))


def available(group, device) -> bool:
    """Can ``group`` run the peer exchange on ``device``?  Needs the kernel library, a GPU
    tensor device and at most ``MAXW`` sites."""
    dev = torch.device(device)
    return (dev.type == "cuda" and getattr(group, "distributed", False) and group.world <= MAXW
            and _lib.native_available())


class PeerArena:
    """One site's uncached, IPC-exported HBM, mapped by every peer of the group.  Regions are
    carved in request order, which every site follows identically (the engines build their
    exchanges in the same order), so a region's offset is the same in every site's arena."""

    def __init__(self, group, device):
        if group.world > MAXW:
            raise ValueError(f"peer exchange: at most {MAXW} sites ({group.world})")
        self.group = group
        self.device = torch.device(device)
        self.W, self.me = max(1, group.world), group.rank if group.world > 1 else 0
        self._chunks: List[tuple] = []  # (local base, [site bases], bytes)
        self._used = 0
        self._cache: Dict[tuple, object] = {}
        # waits as one-workgroup launches of their own when site processes share this GPU (a
        # waiting data launch there can starve a peer's whole-CU kernels: peer.hip px_wait_kernel);
        # DINUNET_PEER_WAIT=inline|launch forces one form
        forced = os.environ.get("DINUNET_PEER_WAIT", "")
        self.wait_launch = (forced == "launch") if forced in ("inline", "launch") else bool(
            getattr(group, "gpu_shared", False))
        # sticky error word of every wait on this site (normal device memory)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        ms = os.environ.get("DINUNET_PEER_TIMEOUT_MS")
        if ms is not None:
            _lib.call("dn_peer_set_timeout_ms", int(ms))
        _ARENAS.add(self)

    def _new_chunk(self, nbytes: int):
        if torch.cuda.is_current_stream_capturing():
            # the allocation, its zero fill and the handle exchange are host work: an exchange
            # must first run (or be built) outside a capture -- the engines build theirs eagerly
            raise RuntimeError("peer exchange: a new arena region was requested inside a HIP "
                               "graph capture; build the exchange before capturing")
        nbytes = max(ARENA_BYTES, -(-nbytes // ALIGN) * ALIGN)
        with torch.cuda.device(self.device):
            p = ctypes.c_void_p()
            _lib.call("dn_peer_alloc", nbytes, ctypes.byref(p))
            bases = [p.value]
            if self.group.world > 1:
                h = ctypes.create_string_buffer(int(_lib.lib().dn_peer_handle_size()))
                _lib.call("dn_peer_export", p, h)
                handles = self.group.all_gather_object(bytes(h.raw))
                bases = []
                for w, hb in enumerate(handles):
                    if w == self.me:
                        bases.append(p.value)
                        continue
                    q = ctypes.c_void_p()
                    buf = ctypes.create_string_buffer(hb, len(hb))
                    _lib.call("dn_peer_open", buf, ctypes.byref(q))
                    bases.append(q.value)
        self._chunks.append((p.value, bases, nbytes))
        self._used = 0

    def region(self, nbytes: int) -> List[int]:
        """``nbytes`` (ALIGN-rounded) of a fresh region: the base address of that region in
        every site's arena, as mapped in this process (index = site)."""
        nbytes = -(-int(nbytes) // ALIGN) * ALIGN
        if not self._chunks or self._used + nbytes > self._chunks[-1][2]:
            self._new_chunk(nbytes)
        _, bases, _ = self._chunks[-1]
        off = self._used
        self._used += nbytes
        return [b + off for b in bases]

    def get(self, key: tuple, make):
        """The exchange object cached under ``key`` (built by ``make()`` on first use): engines
        rebuilt in the same process (folds, pretrain -> finetune) reuse their regions."""
        ex = self._cache.get(key)
        if ex is None:
            ex = self._cache[key] = make()
        return ex

    def error(self) -> int:
        return int(self.err.item())

    def close(self):
        """Unmap the peers' arenas and free this one (every site must be done with them)."""
        for base, bases, _ in self._chunks:
            for w, b in enumerate(bases):
                if w != self.me:
                    _lib.lib().dn_peer_close(ctypes.c_void_p(b))
            _lib.lib().dn_peer_free(ctypes.c_void_p(base))
        self._chunks.clear()
        self._cache.clear()


_ARENAS: "weakref.WeakSet[PeerArena]" = weakref.WeakSet()


def arena(group, device) -> PeerArena:
    a = getattr(group, "_peer_arena", None)
    if a is None:
        a = PeerArena(group, device)
        group._peer_arena = a
    return a


def arenas() -> List[PeerArena]:
    return list(_ARENAS)


def _elem(wire: str) -> int:
    return 4 if wire == "fp32" else 2


class _Exchange:
    def __init__(self, ar: PeerArena, wire: str):
        self.ar = ar
        self.wire = wire
        self.code, self.dtype = PAYLOAD_TYPES[wire]
        self.scaled = 1 if wire == "fp16" else 0

    def _args(self, inbox, gath, flags, src, dst, n, chunk, dstride=0, scale=1.0, a=None):
        a = _PxArgs() if a is None else a
        for w in range(self.ar.W):
            a.inbox[w], a.gath[w], a.flags[w] = inbox[w], gath[w], flags[w]
        a.src, a.dst, a.err = src, dst, self.ar.err.data_ptr()
        a.n, a.chunk, a.dstride = int(n), int(chunk), int(dstride)
        a.W, a.me, a.scaled, a.scale = self.ar.W, self.ar.me, self.scaled, float(scale)
        a.scale_red = 1.0 / self.ar.W
        a.mode = MODE | (4 if self.ar.wait_launch else 0)
        return a

    def _launch(self, args, phase):
        if self.ar.wait_launch and phase != PUSH:  # the phase's wait, as a launch of its own
            _lib.call("dn_peer_wait", ctypes.byref(args), phase, _lib.stream())
        _lib.call("dn_peer_launch", ctypes.byref(args), phase, self.code, _lib.stream())


class PeerMean(_Exchange):
    """Mean over sites of an fp32 range of ``n`` elements, ``wire`` type on the links, fp32 sums.
    ``start`` (push) and ``finish`` (reduce + unpack) may be split around other work: the push
    never waits, so the peers' data travel while this site computes."""

    def __init__(self, ar: PeerArena, n: int, wire: str):
        super().__init__(ar, wire)
        W = ar.W
        self.n = int(n)
        self.chunk = max(SB, -(-self.n // (SB * W)) * SB)
        self.nsbc = self.chunk // SB
        slot = payload_numel(self.chunk) * _elem(wire)
        self.inbox = ar.region(W * slot)
        self.gath = ar.region(W * slot)
        self.flags = ar.region(2 * W * self.nsbc * 4)
        self.bytes_sent = W * payload_numel(self.chunk) * _elem(wire)

    def start(self, x: torch.Tensor):
        if x.numel() != self.n or x.dtype != torch.float32 or not x.is_contiguous():
            raise ValueError(f"PeerMean.start: {self.n} contiguous fp32 elements expected")
        self._launch(self._args(self.inbox, self.gath, self.flags, x.data_ptr(), 0, self.n,
                                self.chunk), PUSH)

    def finish_args(self, x: torch.Tensor, scale: float = 1.0, into=None):
        if x.numel() != self.n or x.dtype != torch.float32 or not x.is_contiguous():
            raise ValueError(f"PeerMean.finish: {self.n} contiguous fp32 elements expected")
        return self._args(self.inbox, self.gath, self.flags, 0, x.data_ptr(), self.n, self.chunk,
                          scale=scale, a=into)

    def finish(self, x: torch.Tensor, scale: float = 1.0):
        """Reduce my chunk (waits for every site's push) and unpack every owner's mean into
        ``x`` (waits for the owners' reduce)."""
        finish_many([(self, x, scale)])

    def run_(self, x: torch.Tensor, scale: float = 1.0) -> int:
        """``x`` <- scale * mean over sites, on the current stream; returns bytes this site sent."""
        self.start(x)
        self.finish(x, scale)
        return self.bytes_sent


class PeerGather(_Exchange):
    """All-gather of ``m`` fp32 elements per site into ``dst[w * dstride : w * dstride + m]``
    (the rank-dAD factors), ``wire`` type on the links."""

    def __init__(self, ar: PeerArena, m: int, wire: str):
        super().__init__(ar, wire)
        W = ar.W
        self.m = int(m)
        self.chunk = max(SB, -(-self.m // SB) * SB)
        self.nsb = self.chunk // SB
        self.gath = ar.region(W * payload_numel(self.chunk) * _elem(wire))
        self.flags = ar.region(2 * W * self.nsb * 4)
        # credits of the slots this site writes at every peer start free (1): my own arena only
        _lib.call("dn_peer_fill_u32", self.flags[ar.me] + 4 * W * self.nsb, 1, W * self.nsb)
        self.bytes_sent = W * payload_numel(self.chunk) * _elem(wire)

    def run(self, src: torch.Tensor, dst: torch.Tensor, dstride: Optional[int] = None,
            scale: float = 1.0) -> int:
        dstride = self.m if dstride is None else int(dstride)
        if src.numel() < self.m or src.dtype != torch.float32 or not src.is_contiguous():
            raise ValueError(f"PeerGather.run: {self.m} contiguous fp32 source elements expected")
        if dst.dtype != torch.float32 or dst.numel() < (self.ar.W - 1) * dstride + self.m:
            raise ValueError("PeerGather.run: destination too small")
        # (the gather kinds read no inbox: the gather slots stand in for the launcher's checks)
        a = self._args(self.gath, self.gath, self.flags, src.data_ptr(), dst.data_ptr(), self.m,
                       self.chunk, dstride, scale)
        self._launch(a, GPUSH)
        self._launch(a, GCOLLECT)
        return self.bytes_sent


def finish_many(items) -> None:
    """Reduce + unpack of several pushed exchanges ``[(PeerMean, x, scale), ...]`` in the given
    order (every site must pass the same sequence): two launches per exchange.  (One launch for
    reduce + unpack of several exchanges -- the blocks' own reduce tasks first, then unpack tasks
    waiting on the peers' -- timed out intermittently on a shared GPU while the separate
    launches never did: ``profiles/r6_peer_fused_index.jsonl``; not kept.)"""
    for pm, x, scale in items:
        a = pm.finish_args(x, scale)
        pm._launch(a, REDUCE)
        pm._launch(a, UNPACK)


def mean(group, device, n: int, wire: str, tag) -> PeerMean:
    ar = arena(group, device)
    return ar.get(("mean", tag, int(n), wire), lambda: PeerMean(ar, n, wire))


def gather(group, device, m: int, wire: str, tag) -> PeerGather:
    ar = arena(group, device)
    return ar.get(("gather", tag, int(m), wire), lambda: PeerGather(ar, m, wire))


_lib.register("dn_peer_peek", [_lib.c_void_p, _lib.c_void_p, _lib.c_long])


def flag_state(ex) -> dict:
    """Diagnostics: the set flag words of an exchange in THIS site's arena (after a timeout:
    which wait never saw its flag)."""
    import numpy as np
    W = ex.ar.W
    if isinstance(ex, PeerMean):
        n = 2 * W * ex.nsbc
    else:
        n = 2 * W * ex.nsb
    buf = np.zeros(n, dtype=np.uint32)
    _lib.call("dn_peer_peek", ex.flags[ex.ar.me], buf.ctypes.data, 4 * n)
    half = n // 2
    return {"kind": type(ex).__name__, "words": n,
            "set_first_half": [int(i) for i in np.nonzero(buf[:half])[0][:16]],
            "set_second_half": [int(i) for i in np.nonzero(buf[half:])[0][:16]],
            "nsub": ex.nsbc if isinstance(ex, PeerMean) else ex.nsb}


def errors(reset: bool = True) -> List[tuple]:
    """``[(site, code, what)]`` of every arena whose error word is set (then cleared)."""
    out = []
    for ar in arenas():
        if not ar._chunks:  # never exchanged anything (or closed)
            continue
        code = ar.error()
        if code:
            out.append((ar.me, code, f"{PHASES.get(code >> 8, 'wait')} on site {code & 0xff}"))
            if reset:
                ar.err.zero_()
    return out
