"""Fused bidirectional LSTM (forward + backward) on the persistent gfx950 kernels.

Per training step (both directions together):

forward
  1. ``dn_lstm_pack``: fp32 reference-layout params -> bf16 kernel layouts (gate rows permuted to
     ``m = 4u + g``, units zero-padded to HD in {64,128,192,256,384,512}), fused bias ``b_ih + b_hh``.
  2. input projection of both directions as ONE GEMM ``[B*S, I] x [I, ndir*4*HD]`` (bf16 out).
  3. ``dn_lstm_fwd``: persistent recurrence (grid = batch-row chunks x directions), stores
     ``c_t`` and ``h_{t-1}`` per step and, when a backward will follow, the gate
     pre-activations ``x W_ih^T + h_{t-1} W_hh^T + b`` (fp32, one 16-B store per lane and
     step, no extra GEMM).
backward
  4. (nothing to recompute: the forward stored the pre-activations).
  5. ``dn_lstm_bwd``: reverse-time recurrence -> gate grads ``dpre`` (bf16, original time order).
  6. parameter grads ACCUMULATED straight into ``.grad`` (flat buffer) by GEMM epilogues with a
     row map back to the reference ``[i|f|o|g]`` layout: ``dW_ih += dpre^T x``,
     ``dW_hh += dpre^T h_{t-1}``, bias grads ``+= dpre^T 1`` (all in one grouped launch).
  7. ``dx = dpre W_ih`` only when the input needs a gradient.  The weight-gradient GEMMs of (6)
     are deferred (``ops._grad.defer``) and issued with the encoder's as ONE grouped launch when
     the autograd pass ends; the engines are notified then.

Reference math: ``comps/icalstm/models.py:5-66`` (oracle: ``ops.reference.bilstm``).
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _grad
from . import _lib
from . import _streams
from . import capture as _cap
from .gemm import PLAIN_BLAS, mm, mm_grouped, mm_plain

Tensor = torch.Tensor

_lib.register("dn_lstm_pack", [_lib.c_void_p] * 8 + [_lib.c_int] * 3 + [_lib.c_void_p] * 4
              + [_lib.c_int] + [_lib.c_void_p] * 3 + [_lib.c_void_p])
_lib.register("dn_lstm_pack_prologue", [_lib.c_void_p] * 8 + [_lib.c_int] * 3
              + [_lib.c_void_p] * 4 + [_lib.c_int] + [_lib.c_void_p] * 3
              + [_lib.c_void_p, _lib.c_long, _lib.c_void_p, _lib.c_void_p, _lib.c_long,
                 _lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_void_p, _lib.c_void_p])
_lib.register("dn_lstm_pack_gather", [_lib.c_void_p] * 8 + [_lib.c_int] * 3
              + [_lib.c_void_p] * 4 + [_lib.c_int] + [_lib.c_void_p] * 3
              + [_lib.c_void_p, _lib.c_int, _lib.c_long, _lib.c_void_p, _lib.c_void_p, _lib.c_long,
                 _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                 _lib.c_long, _lib.c_void_p, _lib.c_void_p])
_lib.register("dn_lstm_fwd", [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_int,
                              _lib.c_int, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                              _lib.c_void_p, _lib.c_float, _lib.c_void_p, _lib.c_void_p,
                              _lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_void_p])
_lib.register("dn_lstm_bwd", [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                              _lib.c_long, _lib.c_long, _lib.c_float, _lib.c_void_p,
                              _lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_int, _lib.c_int,
                              _lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_void_p])
_lib.register("dn_lstm_rows_per_wg", [_lib.c_int, _lib.c_int])
_lib.register("dn_lstm_pre_bf16_used", [_lib.c_int, _lib.c_int])
# Gate pre-activations stored for the backward in bf16 instead of fp32 (the forward writes and the
# backward reads half the bytes per step; the backward then recomputes its gates from the rounded
# values, an error of the order of the bf16 dpre it already stores).  DINUNET_LSTM_PRE_BF16:
# "0" never, "1" always where the kernels offer it (192-unit resident-weight geometry, temporal
# mean), "auto" (default) from PRE_BF16_MIN_BATCH rows on -- the HBM-bound large batches (B=2048
# step 3.091 -> 2.956 ms, profiles/r4_pre_bf16_b2048.jsonl; B=512 hard-cohort training, 3 seeds x
# 300 steps: final validation AUC 0.8583 vs 0.8612 with the fp32 store, seed spread 0.009,
# profiles/r4_pre_bf16_fidelity_b512.jsonl).  The B=32 headline step keeps the fp32 store.
PRE_BF16 = os.environ.get("DINUNET_LSTM_PRE_BF16", "auto")
PRE_BF16_MIN_BATCH = int(os.environ.get("DINUNET_LSTM_PRE_BF16_MIN_BATCH", "512"))


def pre_dtype(B: int, Hd: int, mode: str) -> torch.dtype:
    """Element type of the stored gate pre-activations for this forward."""
    if PRE_BF16 == "0" or (PRE_BF16 == "auto" and B < PRE_BF16_MIN_BATCH):
        return torch.float32
    used = _lib.lib().dn_lstm_pre_bf16_used(int(Hd), int(mode != "mean"))
    return torch.bfloat16 if used else torch.float32


_ROWMAP_CACHE: Dict[Tuple[int, int, str], Tensor] = {}


def padded_hidden(hd: int) -> int:
    if hd <= 0:
        return 0
    # <= 192: W_hh resident in registers; 256 / 384 / 512: streamed from L2 every step
    for p in (64, 128, 192, 256, 384, 512):
        if hd <= p:
            return p
    return 0


def lstm_supported(batch: int, input_size: int, hidden: int, ndir: int,
                   seq: Optional[int] = None) -> bool:
    """Shapes the persistent kernels take: per-direction hidden <= 512, any batch (the forward's
    buffer descriptors are based per workgroup), and a sequence whose per-workgroup span fits the
    descriptors' 32-bit offsets (<= 16 rows x S x ndir x 4 HD fp32 < 2 GiB: S < 8,192 at
    HD = 512, < 21,845 at HD = 192)."""
    HD = padded_hidden(hidden)
    if not (HD > 0 and ndir in (1, 2) and batch > 0 and input_size > 0):
        return False
    return seq is None or 16 * seq * ndir * 4 * HD * 4 < (1 << 31)


def _row_map(Hd: int, HD: int, device) -> Tensor:
    """kernel gate row m = 4u+g (u < HD) -> reference row g*Hd + u, or -1 for padded units."""
    key = (Hd, HD, str(device))
    rm = _ROWMAP_CACHE.get(key)
    if rm is None:
        m = torch.arange(4 * HD)
        u, g = m // 4, m % 4
        rm = torch.where(u < Hd, g * Hd + u, torch.full_like(m, -1)).to(torch.int32).to(device)
        _ROWMAP_CACHE[key] = rm
    return rm


def _ones(n: int, device) -> Tensor:
    from .gemm import ones_operand
    return ones_operand(n, device)


class _BiLSTMFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, enc: Tensor, mode: str, modules, packed, xp_pre, relu_in: bool,
                *params: Tensor):
        ctx.set_materialize_grads(False)  # unused hT / cT -> None (no zero tensors, no syncs)
        B, S, I = enc.shape
        ndir = len(params) // 4
        Hd = params[2].shape[1]
        HD = padded_hidden(Hd)
        GP = 4 * HD
        BR = int(_lib.lib().dn_lstm_rows_per_wg(B, Hd))  # rows per workgroup the kernels use
        Bp = (B + BR - 1) // BR * BR
        dev = enc.device
        st = _lib.stream()
        if packed is None:
            packed = pack_params(params, I, dev)
        wih_p, bias_p, whh_p, whhT_p, ev = packed
        if ev is not None:  # packed on the side stream while the encoder ran
            torch.cuda.current_stream(dev).wait_event(ev)
        x2d = enc.reshape(B * S, I)
        if x2d.dtype != torch.bfloat16:
            x2d = x2d.to(torch.bfloat16)
        x2d = x2d.contiguous()
        if xp_pre is not None:  # the caller's own input projection (same layout as below)
            if xp_pre.shape != (B * S, ndir * GP) or xp_pre.dtype != torch.bfloat16:
                raise ValueError("precomputed LSTM input projection has the wrong shape/dtype")
            xp = xp_pre
        else:
            # bf16 projection: half the bytes the recurrence streams per step (large batches
            # are HBM-bound there); the sum with the recurrent part stays fp32
            xp = mm_plain(x2d, wih_p, trans_b=True, out_dtype=torch.bfloat16)  # [B*S, ndir*GP]
        c_save = torch.empty(ndir, Bp, S, HD, dtype=torch.float32, device=dev)
        hprev = torch.empty(ndir, Bp, S, HD, dtype=torch.bfloat16, device=dev)
        hT = torch.empty(B, ndir * Hd, dtype=torch.float32, device=dev)
        cT = torch.empty(B, ndir * Hd, dtype=torch.float32, device=dev)
        hmean = hseq = None
        if mode == "mean":
            hmean = torch.empty(B, ndir * Hd, dtype=torch.float32, device=dev)
        else:
            hseq = torch.empty(Bp, S, ndir * HD, dtype=torch.float32, device=dev)
        need_bwd = any(ctx.needs_input_grad)
        # gate pre-activations (x W_ih^T + h W_hh^T + b) for the backward (fp32, or bf16: pre_dtype)
        pre = (torch.empty(B * S, ndir * GP, dtype=pre_dtype(B, Hd, mode), device=dev)
               if need_bwd else None)
        # a persistent pack (PersistentPack) keeps b_ih and b_hh as two images: summed in-kernel
        bsplit = ndir * GP if bias_p.numel() == 2 * ndir * GP else 0
        _lib.call("dn_lstm_fwd", xp.data_ptr(), bias_p.data_ptr(), whh_p.data_ptr(), B, S, Hd,
                  ndir, c_save.data_ptr(), hprev.data_ptr(), _lib.ptr(hseq), _lib.ptr(hmean),
                  1.0 / S, hT.data_ptr(), cT.data_ptr(), _lib.ptr(pre), bsplit,
                  int(pre is not None and pre.dtype == torch.bfloat16), st)
        if mode == "mean":
            out = hmean
        else:
            out = hseq.view(Bp, S, ndir, HD)[:B, :, :, :Hd].reshape(B, S, ndir * Hd)
        ctx.save_for_backward(x2d, wih_p, whh_p, whhT_p, bias_p, pre, c_save, hprev)
        ctx.params = params
        ctx.relu_in = bool(relu_in)
        ctx.meta = (B, S, I, Hd, HD, ndir, mode, enc.dtype)
        ctx.modules = modules
        return out, hT, cT

    @staticmethod
    def backward(ctx, dout: Optional[Tensor], dhT: Optional[Tensor], dcT: Optional[Tensor]):
        dx, dpre_v = _lstm_backward(ctx, ctx.saved_tensors, dout, dhT, dcT,
                                    ctx.needs_input_grad[0])
        # a differentiable precomputed projection (``project``: split capture at the projection
        # output) receives the gate gradients themselves: d xp = dpre
        dxp = dpre_v if ctx.needs_input_grad[4] else None
        return (dx, None, None, None, dxp, None) + (None,) * len(ctx.params)


def _lstm_backward(ctx, saved, dout: Optional[Tensor], dhT: Optional[Tensor],
                   dcT: Optional[Tensor], need_dx: bool):
    """Backward of the fused bi-LSTM (steps 4-7 of the module docstring); ``saved`` = the
    forward's ``(x2d, wih_p, whh_p, whhT_p, bias_p, pre, c_save, hprev)``.  Returns ``(dx,
    dpre)``: the input gradient (``need_dx``, premasked by the input ReLU when ``ctx.relu_in``)
    and the gate gradients ``[B*S, ndir*4HD]`` (bf16)."""
    x2d, wih_p, whh_p, whhT_p, bias_p, pre, c_save, hprev = saved
    params = ctx.params
    B, S, I, Hd, HD, ndir, mode, enc_dtype = ctx.meta
    GP = 4 * HD
    N = B * S
    Bp = c_save.shape[1]
    dev = x2d.device
    st = _lib.stream()
    # (4) the forward kernel stored the gate pre-activations
    # (5) reverse-time recurrence
    if dout is None:
        dout = torch.zeros((B, ndir * Hd) if mode == "mean" else (B, S, ndir * Hd),
                           dtype=torch.float32, device=dev)
    dout = dout.float().contiguous()
    if mode == "mean":
        sb, stt, scale = ndir * Hd, 0, 1.0 / S
    else:
        sb, stt, scale = S * ndir * Hd, ndir * Hd, 1.0
    dhT = None if dhT is None else dhT.float().contiguous()
    dcT = None if dcT is None else dcT.float().contiguous()
    dpre = torch.empty(Bp * S, ndir * GP, dtype=torch.bfloat16, device=dev)
    dpre_v = dpre[:N]
    capturing = _cap.active() is not None and ctx.modules is not None
    # the backward addresses the forward's padded buffers (Bp rows) whatever rows per workgroup
    # it tiles with
    _lib.call("dn_lstm_bwd", pre.data_ptr(), c_save.data_ptr(), whhT_p.data_ptr(),
              dout.data_ptr(), sb, stt, scale, _lib.ptr(dhT), _lib.ptr(dcT), B, S, Hd,
              ndir, dpre.data_ptr(), Bp, int(pre.dtype == torch.bfloat16), st)
    # (6) parameter grads accumulated into .grad (reference layout via row map): queued
    # for the end-of-backward grouped launch together with the encoder's (ops._grad.defer)
    probs = _param_grad_problems(params, dpre_v, x2d, hprev, B, S, Hd, HD, ndir, dev)
    _grad.defer(probs, [p for p in params if p is not None])
    # (7) input grad
    dx = None
    if need_dx:
        if ctx.relu_in and not PLAIN_BLAS:
            # the input is a ReLU output consumed only here: the ReLU backward's mask rides
            # in this GEMM's epilogue (d input where input <= 0 cannot reach anything), and
            # the encoder backward skips its own mask launch for exactly this tensor
            dx = mm(dpre_v, wih_p, out_dtype=torch.bfloat16, mask=x2d)
            from .linear import mark_premasked
            mark_premasked(dx)
            dx = dx.view(B, S, I)
        else:
            dx = mm_plain(dpre_v, wih_p, out_dtype=torch.bfloat16).view(B, S, I)
        if enc_dtype != torch.bfloat16:
            dx = dx.to(enc_dtype)
    if capturing:
        dref = dpre_v.view(N, ndir, HD, 4)[:, :, :Hd, :].transpose(2, 3).reshape(N, ndir, 4 * Hd)
        for d, cell in enumerate(ctx.modules):
            _cap.record(cell.i2h, x2d, dref[:, d])
            _cap.record(cell.h2h, hprev[d].view(Bp * S, HD)[:N, :Hd], dref[:, d])
    return dx, dpre_v


class _ProjFn(torch.autograd.Function):
    """The LSTM input projection of both directions, ``xp = enc W_ih^T`` (bf16, packed gate
    columns), as an autograd node of its own: the split capture of a multi-site step cuts the
    backward HERE (``runtime.step.TrainStep``), so everything after the projection -- the
    recurrences, the head and every LSTM / head weight gradient -- is final before the input
    gradient ``d enc = dpre W_ih`` (ReLU mask in its epilogue) and the encoder's gradients run,
    and the all-reduce of the LSTM + head gradients overlaps those."""

    @staticmethod
    def forward(ctx, enc: Tensor, wih_p: Tensor, relu_in: bool):
        B, S, I = enc.shape
        x2d = enc.reshape(B * S, I)
        if x2d.dtype != torch.bfloat16:
            x2d = x2d.to(torch.bfloat16)
        x2d = x2d.contiguous()
        ctx.save_for_backward(x2d, wih_p)
        ctx.meta = (B, S, I, enc.dtype, bool(relu_in))
        return mm_plain(x2d, wih_p, trans_b=True, out_dtype=torch.bfloat16)

    @staticmethod
    def backward(ctx, dxp: Tensor):
        x2d, wih_p = ctx.saved_tensors
        B, S, I, dt, relu_in = ctx.meta
        dxp = dxp.to(torch.bfloat16).contiguous()
        if relu_in and not PLAIN_BLAS:
            dx = mm(dxp, wih_p, out_dtype=torch.bfloat16, mask=x2d)
            from .linear import mark_premasked
            mark_premasked(dx)
        else:
            dx = mm_plain(dxp, wih_p, out_dtype=torch.bfloat16)
        dx = dx.view(B, S, I)
        return (dx if dt == torch.bfloat16 else dx.to(dt)), None, None


def project(enc: Tensor, packed, relu_input: bool = False) -> Tensor:
    """Differentiable LSTM input projection ``[B, S, I] -> [B*S, ndir*4HD]`` with the packed
    weights of ``pack_params`` (see :class:`_ProjFn`); feed it to :func:`bilstm` as ``xp``."""
    wih_p, _, _, _, ev = packed
    if ev is not None:
        torch.cuda.current_stream(enc.device).wait_event(ev)
    return _ProjFn.apply(enc, wih_p, bool(relu_input))


def pack_params(params: Sequence[Tensor], input_size: int, device, side: bool = False,
                casts: Sequence[Tensor] = (), cast_out: Optional[List[Tensor]] = None):
    """``dn_lstm_pack``: fp32 reference-layout params -> bf16 kernel layouts + fused bias.

    With ``side=True`` the pack runs on the side stream (it depends only on the parameters, so
    it overlaps the encoder GEMM) and the returned event orders the consumer after it.
    ``casts`` (<= 4 fp32 tensors) are rounded to bf16 by the same launch; the copies are
    appended to ``cast_out``.
    """
    pp = _PERSIST
    if pp is not None and not side and pp.matches(params, casts):
        # the fused Adam keeps these images current (optim.hip adam_pack_kernel): no launch
        if cast_out is not None:
            cast_out.extend(pp.casts)
        pp.used = True
        return pp.wih_p, pp.bias_p, pp.whh_p, pp.whhT_p, None
    ndir = len(params) // 4
    Hd = params[2].shape[1]
    HD = padded_hidden(Hd)
    GP = 4 * HD
    I = int(input_size)
    stream = _streams.fork(device) if side else None
    ctx = torch.cuda.stream(stream) if side else _nullctx()
    with ctx:
        wih_p = torch.empty(ndir * GP, I, dtype=torch.bfloat16, device=device)
        bias_p = torch.empty(ndir * GP, dtype=torch.float32, device=device)
        whh_p = torch.empty(ndir, GP, HD, dtype=torch.bfloat16, device=device)
        whhT_p = torch.empty(ndir, HD, GP, dtype=torch.bfloat16, device=device)
        ps = [p.detach().contiguous() for p in params] + [None] * (8 - len(params))
        if len(casts) > 4:
            raise ValueError("pack_params: at most 4 extra casts")
        srcs = [c.detach().contiguous() for c in casts]
        dsts = [torch.empty(c.shape, dtype=torch.bfloat16, device=device) for c in srcs]
        nc = len(srcs)
        P, I_ = ctypes.c_void_p, ctypes.c_int
        args = ([_lib.ptr(p) for p in ps] + [I, Hd, ndir, wih_p.data_ptr(), bias_p.data_ptr(),
                whh_p.data_ptr(), whhT_p.data_ptr(), nc,
                (P * max(nc, 1))(*[c.data_ptr() for c in srcs]),
                (P * max(nc, 1))(*[d.data_ptr() for d in dsts]),
                (I_ * max(nc, 1))(*[c.numel() for c in srcs])])
        rp = _RIDE
        if rp is not None and not rp.consumed and not side and _DEFERRED is None:
            # the step's device-fed prologue (batch gather, labels, gradient zeroing, Adam's
            # counter) rides in this launch: the step's first kernel
            _lib.call("dn_lstm_pack_gather", *args, *rp.tail, _lib.stream())
            rp.consumed = True
        elif _DEFERRED is not None and not side:
            # recorded, launched before each replay (run_deferred_pack); the record keeps every
            # operand alive so the graph pool never hands the packed buffers to another tensor
            _DEFERRED.append((args, (ps, srcs, dsts, wih_p, bias_p, whh_p, whhT_p)))
        else:
            _lib.call("dn_lstm_pack", *args, _lib.stream())
        if cast_out is not None:
            cast_out.extend(dsts)
        ev = None
        if side:
            ev = torch.cuda.Event()
            ev.record(stream)
    if side:
        # the packed tensors are consumed on the main stream: keep their blocks alive there
        main = torch.cuda.current_stream(device)
        for t in (wih_p, bias_p, whh_p, whhT_p):
            t.record_stream(main)
    return wih_p, bias_p, whh_p, whhT_p, ev


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


_DEFERRED: Optional[list] = None
_RIDE = None
_PERSIST = None

# PackKind of csrc/kernels/optim.hip
PK_CAST, PK_WIH, PK_WHH, PK_BIAS = 1, 2, 3, 4


class PersistentPack:
    """Packed LSTM operand images (and bf16 copies of ``casts``, e.g. the encoder weights) that
    live across steps and are rewritten by the fused Adam as it updates each parameter
    (``FusedAdam.step_pack``), so the training step needs no repack launch.  Same layouts as
    :func:`pack_params` except the bias: ``[2][ndir*4HD]`` (the ``b_ih`` image, then ``b_hh``),
    which ``dn_lstm_fwd`` sums as it loads (``bias_split``) -- the same fp32 sum the pack forms.
    Padded units / columns are zero from allocation and never written.  While
    :class:`use_persistent` is active, :func:`pack_params` on the same parameters returns these
    buffers without a launch."""

    def __init__(self, params: Sequence[Tensor], input_size: int, device,
                 casts: Sequence[Tensor] = (), extra: Sequence[Tensor] = ()):
        self.params = list(params)
        if len(self.params) % 4 or any(p is None for p in self.params):
            raise ValueError("PersistentPack: every direction needs W_ih, b_ih, W_hh, b_hh")
        self.ndir = len(self.params) // 4
        self.Hd = self.params[2].shape[1]
        self.HD = padded_hidden(self.Hd)
        self.I = int(input_size)
        GP = 4 * self.HD
        z = dict(device=device)
        self.wih_p = torch.zeros(self.ndir * GP, self.I, dtype=torch.bfloat16, **z)
        self.bias_p = torch.zeros(2 * self.ndir * GP, dtype=torch.float32, **z)
        self.whh_p = torch.zeros(self.ndir, GP, self.HD, dtype=torch.bfloat16, **z)
        self.whhT_p = torch.zeros(self.ndir, self.HD, GP, dtype=torch.bfloat16, **z)
        self.cast_src = list(casts)
        self.casts = [torch.zeros(c.shape, dtype=torch.bfloat16, **z) for c in casts]
        # further bf16 copies kept current by the same Adam launch, looked up by parameter
        # (bf16_of): the classifier weights the replicated head kernel reads (head_rep.hip)
        self.extra_src = list(extra)
        self.extra = [torch.zeros(c.shape, dtype=torch.bfloat16, **z) for c in extra]
        self.used = False

    def bf16_of(self, t: Tensor) -> Optional[Tensor]:
        """The bf16 image of parameter ``t`` this pack keeps current, or None."""
        for src, dst in zip(self.cast_src + self.extra_src, self.casts + self.extra):
            if src is t:
                return dst
        return None

    def matches(self, params, casts) -> bool:
        return (len(params) == len(self.params)
                and all(a is b for a, b in zip(params, self.params))
                and len(casts) == len(self.cast_src)
                and all(a is b for a, b in zip(casts, self.cast_src)))

    def rows(self, flat) -> list:
        """``(flat offset, numel, kind, direction, dst ptr, dst2 ptr)`` per packed parameter of
        the flat buffer ``flat`` (``ops.FlatParams``), sorted by offset."""
        offs = {id(p): o for p, o, _ in flat.segments()}
        GP = 4 * self.HD
        out = []
        for d in range(self.ndir):
            w_ih, b_ih, w_hh, b_hh = self.params[4 * d:4 * d + 4]
            out.append((offs[id(w_ih)], w_ih.numel(), PK_WIH, d, self.wih_p.data_ptr(), 0))
            out.append((offs[id(w_hh)], w_hh.numel(), PK_WHH, d, self.whh_p.data_ptr(),
                        self.whhT_p.data_ptr()))
            out.append((offs[id(b_ih)], b_ih.numel(), PK_BIAS, d, self.bias_p.data_ptr(), 0))
            out.append((offs[id(b_hh)], b_hh.numel(), PK_BIAS, d,
                        self.bias_p.data_ptr() + 4 * self.ndir * GP, 0))
        for src, dst in zip(self.cast_src + self.extra_src, self.casts + self.extra):
            out.append((offs[id(src)], src.numel(), PK_CAST, 0, dst.data_ptr(), 0))
        return sorted(out)


class use_persistent:
    """While active, :func:`pack_params` on ``pp``'s parameters returns ``pp``'s buffers."""

    def __init__(self, pp: Optional[PersistentPack]):
        self.pp = pp

    def __enter__(self):
        global _PERSIST
        self._prev, _PERSIST = _PERSIST, self.pp
        return self.pp

    def __exit__(self, *a):
        global _PERSIST
        _PERSIST = self._prev
        return False


class ride_pack:
    """While active, the next in-stream ``pack_params`` launch also runs the device-fed step
    prologue (``dn_lstm_pack_gather``; ``tail`` = ``ops.DeviceSource.prologue_args``), so the
    batch gather costs no launch of its own.  ``consumed`` tells the caller it happened."""

    def __init__(self, tail):
        self.tail = tail
        self.consumed = False

    def __enter__(self):
        global _RIDE
        self._prev, _RIDE = _RIDE, self
        return self

    def __exit__(self, *a):
        global _RIDE
        _RIDE = self._prev
        return False


class defer_pack:
    """While active (a graph capture in ``runtime.step.TrainStep``), ``pack_params`` allocates
    its outputs but records its launch instead of issuing it: the pack depends only on the
    parameters, so it runs before each replay in the same launch as the step prologue
    (``run_deferred_pack``), and the graph starts at the encoder GEMM.  The packed layouts are
    identical either way."""

    def __init__(self):
        self.records: list = []

    def __enter__(self):
        global _DEFERRED
        self._prev, _DEFERRED = _DEFERRED, self.records
        return self

    def __exit__(self, *a):
        global _DEFERRED
        _DEFERRED = self._prev
        return False


def run_deferred_pack(records: list, prologue=None, bump: Optional[Tensor] = None) -> None:
    """Issue the recorded pack launches; the LAST one also runs the step prologue
    ``(x fp32, xb bf16, y int64, yd int64, grad fp32)`` when given (``dn_lstm_pack_prologue``),
    advancing the int32 counter ``bump`` once when given."""
    if bump is not None and prologue is None:
        raise ValueError("run_deferred_pack: a step-counter bump rides on the prologue only")
    for k, (args, _keep) in enumerate(records):
        if prologue is not None and k == len(records) - 1:
            x, xb, y, yd, g = prologue
            _lib.call("dn_lstm_pack_prologue", *args, x.data_ptr(), x.numel(), xb.data_ptr(),
                      y.data_ptr(), y.numel(), yd.data_ptr(), g.data_ptr(), g.numel(),
                      _lib.ptr(bump), _lib.stream())
        else:
            _lib.call("dn_lstm_pack", *args, _lib.stream())


def _param_grad_problems(params, dpre_v, x2d, hprev, B, S, Hd, HD, ndir, dev):
    """Grouped-GEMM problems accumulating dW_ih, dW_hh, b_ih, b_hh of every direction into
    ``.grad`` (``out += dpre^T @ operand``, gate rows mapped back to the reference layout)."""
    GP = 4 * HD
    N = B * S
    Bp = hprev.shape[1]
    rmap = _row_map(Hd, HD, dev)
    probs = []
    for d in range(ndir):
        w_ih, b_ih, w_hh, b_hh = params[4 * d:4 * d + 4]
        dsl = dpre_v[:, d * GP:(d + 1) * GP]
        probs.append(dict(a=dsl, b=x2d, out=_grad.grad_buffer(w_ih), beta=1.0, row_map=rmap))
        # bias grads = column sums of dpre = dpre^T @ 1, requested with dW_hh (ops.gemm
        # _place_colsums: a virtual ones column in dW_hh's spare tile columns on large-batch
        # launches, else its own problem).  d b_ih == d b_hh (both add to the same
        # pre-activation): ONE column sum, stored twice
        bs = tuple(_grad.grad_buffer(b) for b in (b_ih, b_hh) if b is not None)
        probs.append(dict(a=dsl, b=hprev[d].view(Bp * S, HD)[:N, :Hd],
                          out=_grad.grad_buffer(w_hh), beta=1.0, row_map=rmap,
                          colsum=bs or None))
    return probs


def bilstm(x: Tensor, params: Sequence[Tuple[Tensor, Tensor, Tensor, Tensor]],
           reduce: str = "none", modules=None, packed=None, xp: Optional[Tensor] = None,
           relu_input: bool = False):
    """Fused bi-LSTM: returns ``(hmean [B, ndir*Hd] | hseq [B, S, ndir*Hd], (hT, cT))``.

    ``relu_input``: ``x`` is a ReLU output whose only consumer is this LSTM (the ICA encoder);
    the backward then fuses the ReLU mask into its input-gradient GEMM."""
    if not _lib.native_available():
        raise RuntimeError("fused LSTM requested but the gfx950 kernel library is not built")
    flat: List[Tensor] = []
    for p in params:
        flat.extend(p)
    out, hT, cT = _BiLSTMFn.apply(x, "mean" if reduce == "mean" else "seq", modules, packed, xp,
                                  bool(relu_input), *flat)
    return out, (hT, cT)
