"""Flat-buffer parameters and fused optimizers.

All parameters of the site's model(s) are re-homed into ONE contiguous fp32 buffer (16-byte
aligned per tensor) and their ``.grad`` into a matching flat gradient buffer.  Consequences:

* the dSGD all-reduce is one collective on one buffer (or a few buckets) with zero packing;
* Adam is a single fused HIP launch over the whole model (``csrc/kernels/optim.hip``);
* checkpoints still save per-module ``state_dict``s with the reference key names.

Semantics match ``torch.optim.Adam`` / ``torch.optim.SGD`` (checked against them in tests).
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Optional

import torch
import torch.nn as nn

from . import _lib

_lib.register("dn_adam", [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                          _lib.c_long] + [_lib.c_float] * 8 + [_lib.c_void_p, _lib.c_void_p])
_lib.register("dn_adam_dev", [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                              _lib.c_long, _lib.c_float, _lib.c_double, _lib.c_double,
                              _lib.c_float, _lib.c_float, _lib.c_float, _lib.c_void_p,
                              _lib.c_int, _lib.c_void_p, _lib.c_void_p])
_lib.register("dn_step_gather", [_lib.c_void_p, _lib.c_int, _lib.c_long, _lib.c_void_p,
                                 _lib.c_void_p, _lib.c_long, _lib.c_void_p, _lib.c_int,
                                 _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_long,
                                 _lib.c_void_p, _lib.c_void_p])
_lib.register("dn_step_prologue", [_lib.c_void_p, _lib.c_long, _lib.c_void_p, _lib.c_void_p,
                                   _lib.c_long, _lib.c_void_p, _lib.c_void_p, _lib.c_long,
                                   _lib.c_void_p, _lib.c_void_p])
_lib.register("dn_sgd", [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_long,
                         _lib.c_float, _lib.c_float, _lib.c_float, _lib.c_float, _lib.c_int,
                         _lib.c_void_p])
_lib.register("dn_cast_f32_bf16", [_lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_float,
                                   _lib.c_void_p])
_lib.register("dn_cast_bf16_f32", [_lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_float,
                                   _lib.c_void_p])

_lib.register("dn_adam_pack", [_lib.c_void_p] * 4 + [_lib.c_long, _lib.c_float, _lib.c_double,
                               _lib.c_double, _lib.c_float, _lib.c_float, _lib.c_float,
                               _lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_void_p, _lib.c_int,
                               _lib.c_int, _lib.c_int, _lib.c_int, _lib.c_void_p, _lib.c_int,
                               _lib.c_long, _lib.c_void_p, _lib.c_void_p, _lib.c_long,
                               _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p,
                               _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p])
_lib.register("dn_step_record", [_lib.c_void_p, _lib.c_int, _lib.c_void_p])


def ctypes_addr(obj) -> int:
    import ctypes
    return ctypes.addressof(obj)


ALIGN = 4  # elements (16 bytes)


class FlatParams:
    """Re-home ``params`` into one flat buffer; ``.grad`` of each becomes a view of ``self.grad``."""

    def __init__(self, params: Iterable[nn.Parameter], device=None):
        self.params: List[nn.Parameter] = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("no trainable parameters")
        device = device or self.params[0].device
        self.offsets: List[int] = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self.data = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            self.data[o:o + n].copy_(p.detach().reshape(-1).float())
            p.data = self.data[o:o + n].view_as(p)
            p.grad = self.grad[o:o + n].view_as(p)

    def zero_grad(self):
        self.grad.zero_()

    def rebind_grads(self):
        """Autograd may replace ``.grad`` with a fresh tensor when it was None; keep views."""
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            if p.grad is None or p.grad.data_ptr() != self.grad[o:o + n].data_ptr():
                g = p.grad
                p.grad = self.grad[o:o + n].view_as(p)
                if g is not None:
                    p.grad.copy_(g)

    def segments(self):
        for p, o in zip(self.params, self.offsets):
            yield p, o, p.numel()

    def numel_of(self, ps) -> int:
        return sum(p.numel() for p in ps)


class FusedAdam:
    """``torch.optim.Adam`` on a :class:`FlatParams` buffer in one kernel launch per step."""

    def __init__(self, flat: FlatParams, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0):
        self.flat = flat
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.exp_avg = torch.zeros_like(flat.data)
        self.exp_avg_sq = torch.zeros_like(flat.data)
        self.step_count = 0
        self._tdev: Optional[torch.Tensor] = None  # device step counter (graph-captured steps)
        # device-fed batches (ops.DeviceSource): the update advances the source's cursor
        self.cursor: Optional[torch.Tensor] = None

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    def step(self, grad_scale: float = 1.0):
        self.step_count += 1
        b1, b2 = self.betas
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        d = self.flat.data
        if d.is_cuda:
            _lib.call("dn_adam", d.data_ptr(), self.flat.grad.data_ptr(), self.exp_avg.data_ptr(),
                      self.exp_avg_sq.data_ptr(), d.numel(), self.lr, b1, b2, self.eps,
                      self.weight_decay, bc1, 1.0 / math.sqrt(bc2), grad_scale,
                      _lib.ptr(self.cursor), _lib.stream())
            return
        g = self.flat.grad * grad_scale
        if self.weight_decay:
            g = g + self.weight_decay * d
        self.exp_avg.mul_(b1).add_(g, alpha=1 - b1)
        self.exp_avg_sq.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (self.exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(self.eps)
        d.addcdiv_(self.exp_avg, denom, value=-self.lr / bc1)

    # HIP-graph form --------------------------------------------------------------------------
    def sync_device_step(self):
        """Copy the host step count to the device counter :meth:`step_graphable` reads."""
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            # inside a capture the fill (and a first allocation) would become graph nodes that
            # reset the counter at every replay
            raise RuntimeError("FusedAdam.sync_device_step inside a HIP graph capture")
        if self._tdev is None:
            self._tdev = torch.zeros(1, dtype=torch.int32, device=self.flat.data.device)
        self._tdev.fill_(self.step_count)

    def step_graphable(self, grad_scale: float = 1.0, prebumped: bool = False):
        """One Adam step whose bias corrections come from the device step counter (advanced by
        the same launch), so it can be captured once and replayed every step.  The caller keeps
        ``step_count`` in sync (one increment per replay).  ``prebumped``: the caller advances
        the counter in its step prologue instead (it passes :meth:`device_step` to the
        prologue launch before each replay), so the update is ONE graph node, not Adam + a
        one-thread bump kernel."""
        d = self.flat.data
        if self._tdev is None:
            self.sync_device_step()
        b1, b2 = self.betas
        _lib.call("dn_adam_dev", d.data_ptr(), self.flat.grad.data_ptr(), self.exp_avg.data_ptr(),
                  self.exp_avg_sq.data_ptr(), d.numel(), self.lr, b1, b2, self.eps,
                  self.weight_decay, grad_scale, self._tdev.data_ptr(), int(prebumped),
                  _lib.ptr(self.cursor), _lib.stream())

    # Adam that also emits the next step's operands (optim.hip adam_pack_kernel) ------------------
    def attach_pack(self, pack, src=None, xb: Optional[torch.Tensor] = None,
                    yd: Optional[torch.Tensor] = None, sd: Optional[torch.Tensor] = None,
                    copy_x: bool = True):
        """Keep ``pack`` (``ops.lstm.PersistentPack``) current from every :meth:`step_pack`, and
        gather the next batch of ``src`` (``DeviceSource``) into ``xb`` / ``yd`` there too.
        ``sd`` (int64 [B + 1]): the next batch's dataset rows go there as well; ``copy_x=False``
        then skips the batch copy (the GEMMs read the rows in place: ``ops.gemm.rows_from``)."""
        import ctypes
        rows = pack.rows(self.flat)

        class _Seg(ctypes.Structure):
            _fields_ = [("off", ctypes.c_long), ("n", ctypes.c_int), ("kind", ctypes.c_int),
                        ("d", ctypes.c_int), ("dst", ctypes.c_void_p), ("dst2", ctypes.c_void_p)]
        L = _lib.lib()
        L.dn_pack_seg_size.restype = ctypes.c_long
        if ctypes.sizeof(_Seg) != L.dn_pack_seg_size():
            raise RuntimeError("pack segment layout mismatch with the kernel library")
        tab = (_Seg * max(1, len(rows)))()
        for i, (off, n, kind, d, dst, dst2) in enumerate(rows):
            tab[i] = _Seg(off, n, kind, d, dst, dst2 or None)
        if not copy_x and sd is None:
            raise ValueError("attach_pack: without the batch copy the step needs its row indices")
        self._pack = (pack, tab, len(rows), src, xb, yd, sd, copy_x)

    def step_pack(self, grad_scale: float = 1.0, update: bool = True, gofs: int = 1,
                  record=None):
        """ONE launch: the graph-capturable Adam step (bias corrections from the device counter,
        which the step's first GEMM advanced: ``dn_gemm_arm_bump``), the attached packed images
        rewritten from the updated parameters, the gradient zeroed, and the batch at
        ``cursor + gofs`` gathered.  ``update=False``: images + gather + zeroing only (priming).
        ``record``: a :meth:`StepRecorder.args` struct -- the step's score column and loss go to
        the recorder's rings at the cursor (one more workgroup of the same launch)."""
        pack, tab, cnt, src, xb, yd, sd, copy_x = self._pack
        d = self.flat.data
        if self._tdev is None:
            self.sync_device_step()
        b1, b2 = self.betas
        if src is not None:
            gx = [src.X.data_ptr(), src._mode(xb), src.row,
                  src.Y.data_ptr(), _lib.ptr(src.order), src.nb, src.cursor.data_ptr(), src.B,
                  xb.data_ptr() if copy_x else None, yd.data_ptr(), _lib.ptr(sd)]
        else:
            gx = [None, 0, 0, None, None, 1, None, 0, None, None, None]
        _lib.call("dn_adam_pack", d.data_ptr(), self.flat.grad.data_ptr(), self.exp_avg.data_ptr(),
                  self.exp_avg_sq.data_ptr(), d.numel(), self.lr, b1, b2, self.eps,
                  self.weight_decay, grad_scale, self._tdev.data_ptr(), int(update), 1,
                  ctypes_addr(tab), cnt, pack.I, pack.Hd, pack.HD, *gx, int(gofs),
                  ctypes_addr(record) if (record is not None and update) else None, _lib.stream())

    def device_step(self) -> torch.Tensor:
        """The device step counter (int32[1]) the graph-captured update reads; a step prologue
        given it advances it once per launch."""
        if self._tdev is None:
            self.sync_device_step()  # (raises inside a capture: create it before)
        return self._tdev

    def state_dict(self) -> Dict:
        return {"lr": self.lr, "betas": self.betas, "eps": self.eps,
                "weight_decay": self.weight_decay, "step": self.step_count,
                "exp_avg": self.exp_avg.detach().cpu(), "exp_avg_sq": self.exp_avg_sq.detach().cpu()}

    def load_state_dict(self, sd: Dict):
        self.lr = sd.get("lr", self.lr)
        self.betas = tuple(sd.get("betas", self.betas))
        self.eps = sd.get("eps", self.eps)
        self.weight_decay = sd.get("weight_decay", self.weight_decay)
        self.step_count = int(sd.get("step", 0))
        if "exp_avg" in sd:
            self.exp_avg.copy_(sd["exp_avg"].to(self.exp_avg.device))
            self.exp_avg_sq.copy_(sd["exp_avg_sq"].to(self.exp_avg_sq.device))


def step_prologue(x: torch.Tensor, xb: Optional[torch.Tensor], y: torch.Tensor,
                  yd: torch.Tensor, grad: torch.Tensor, bump: Optional[torch.Tensor] = None):
    """ONE launch before a graph replay: ``xb <- bf16(x)`` (skipped when ``xb`` is None),
    ``yd <- y`` (int64), ``grad <- 0`` and, when given, ``bump += 1`` (the captured Adam's
    device step counter, :meth:`FusedAdam.device_step`)."""
    nx = x.numel() if xb is not None else 0
    if nx % 8 or grad.numel() % 4 or y.dtype != torch.int64 or yd.dtype != torch.int64:
        raise ValueError("step_prologue: x numel % 8, grad numel % 4 and int64 labels required")
    _lib.call("dn_step_prologue", x.data_ptr() if nx else None, nx,
              xb.data_ptr() if nx else None, y.data_ptr(), y.numel(), yd.data_ptr(),
              grad.data_ptr(), grad.numel(), _lib.ptr(bump), _lib.stream())


def cast_f32_to_bf16(src: torch.Tensor, dst: torch.Tensor, scale: float = 1.0):
    if src.is_cuda:
        _lib.call("dn_cast_f32_bf16", src.data_ptr(), dst.data_ptr(), src.numel(), scale,
                  _lib.stream())
    else:
        dst.copy_((src * scale).to(dst.dtype))


def cast_bf16_to_f32(src: torch.Tensor, dst: torch.Tensor, scale: float = 1.0):
    if src.is_cuda:
        _lib.call("dn_cast_bf16_f32", src.data_ptr(), dst.data_ptr(), src.numel(), scale,
                  _lib.stream())
    else:
        dst.copy_(src.float() * scale)


class DeviceSource:
    """Training batches resident in HBM (BASELINE config 5 sizing: a site's whole dataset fits one
    MI355X): ``X [N, *sample]`` (bf16, or fp32), labels ``Y [N]`` int64, an optional per-pass order
    ``[nb * B]`` of row indices, and a device batch cursor.  Step ``c`` trains on rows
    ``order[(c mod nb) * B : ... + B]``; the gather runs in the step's first launch and the cursor
    advances in its Adam launch, so a HIP graph can hold several whole steps
    (``runtime.step.TrainStep.run``)."""

    def __init__(self, X: torch.Tensor, Y: torch.Tensor, batch: int,
                 order: Optional[torch.Tensor] = None):
        if not X.is_cuda or X.dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("DeviceSource: X must be a bf16 / fp32 GPU tensor")
        self.width = None  # the real feature count of a padded fp32 feature matrix
        if X.dtype == torch.float32 and X.dim() == 2 and X.shape[1] % 8:
            # fp32 feature rows (FS: 66 features) padded with zero columns to whole 16-B chunks
            # once; the step's static input keeps the padded width and the model reads the
            # first `width` columns (``view``)
            self.width = int(X.shape[1])
            Xp = torch.zeros(X.shape[0], -(-X.shape[1] // 8) * 8, dtype=X.dtype, device=X.device)
            Xp[:, :self.width] = X
            X = Xp
        self.X = X.contiguous()
        self.Y = Y.to(device=X.device, dtype=torch.int64).contiguous()
        self.B = int(batch)
        self.row = self.X[0].numel()
        if self.row % 8:
            raise ValueError("DeviceSource: sample size must be a multiple of 8 elements")
        self.order = None
        self.set_order(order)
        self.cursor = torch.zeros(1, dtype=torch.int64, device=X.device)

    def set_order(self, order: Optional[torch.Tensor]):
        """A new pass order (e.g. the next epoch's shuffle) in place: captured graphs keep
        reading the same buffer."""
        n = self.X.shape[0] if order is None else order.numel()
        nb = n // self.B
        if nb < 1:
            raise ValueError("DeviceSource: fewer samples than one batch")
        if order is None:
            self.order = None
        else:
            o = order.to(device=self.X.device, dtype=torch.int64).reshape(-1)[:nb * self.B]
            if self.order is not None and self.order.numel() == o.numel():
                self.order.copy_(o)
            else:
                self.order = o.clone()
        self.nb = nb

    @property
    def sample_shape(self):
        return tuple(self.X.shape[1:])

    def batch(self, c: int):
        """Host-side view of batch ``c`` (tests / eager fallbacks): ``(x, y)``."""
        j = (c % self.nb) * self.B
        rows = (self.order[j:j + self.B] if self.order is not None
                else torch.arange(j, j + self.B, device=self.X.device))
        return self.X[rows], self.Y[rows]

    def view(self, xb: torch.Tensor) -> torch.Tensor:
        """What the model reads of a static input ``xb`` this source gathers into (the real
        columns of padded feature rows)."""
        return xb if self.width is None else xb[:, :self.width]

    def _mode(self, xb: torch.Tensor) -> int:
        # dn_step_gather's source / destination mode (prologue.h): 1 bf16 -> bf16, 0 fp32 ->
        # bf16 (rounded), 2 fp32 -> fp32 (exact)
        if self.X.dtype == torch.bfloat16:
            if xb.dtype != torch.bfloat16:
                raise ValueError("DeviceSource: a bf16 dataset gathers into a bf16 static input")
            return 1
        return 2 if xb.dtype == torch.float32 else 0

    def gather(self, xb: torch.Tensor, yd: torch.Tensor, grad: torch.Tensor,
               bump: Optional[torch.Tensor] = None):
        """The standalone device-fed prologue launch (``dn_step_gather``)."""
        _lib.call("dn_step_gather", self.X.data_ptr(), self._mode(xb),
                  self.row, self.Y.data_ptr(), _lib.ptr(self.order), self.nb,
                  self.cursor.data_ptr(), self.B, xb.data_ptr(), yd.data_ptr(), grad.data_ptr(),
                  grad.numel(), _lib.ptr(bump), _lib.stream())

    def labels_of(self, steps: int) -> torch.Tensor:
        """Labels of batches ``0 .. steps-1`` of the current order, flattened (what a
        :class:`StepRecorder`'s score ring pairs with)."""
        rows = (self.order[:steps * self.B] if self.order is not None
                else torch.arange(steps * self.B, device=self.X.device) % self.X.shape[0])
        return self.Y[rows]

    def prologue_args(self, xb, yd, grad, bump=None):
        """Argument tail of ``dn_lstm_pack_gather`` (the prologue riding in the weight pack)."""
        return [self.X.data_ptr(), self._mode(xb), self.row,
                self.Y.data_ptr(), _lib.ptr(self.order), self.nb, self.cursor.data_ptr(),
                self.B, xb.data_ptr(), yd.data_ptr(), grad.data_ptr(), grad.numel(),
                _lib.ptr(bump)]


_STEP_RECORD = None


def _step_record_type():
    """The ctypes layout of ``optim.hip StepRecord``, checked against the library once."""
    global _STEP_RECORD
    if _STEP_RECORD is None:
        import ctypes

        class _Rec(ctypes.Structure):
            _fields_ = [("out", ctypes.c_void_p), ("ld", ctypes.c_long), ("col", ctypes.c_int),
                        ("B", ctypes.c_int), ("loss", ctypes.c_void_p), ("rs", ctypes.c_void_p),
                        ("rl", ctypes.c_void_p), ("n", ctypes.c_long), ("cursor", ctypes.c_void_p),
                        ("pred", ctypes.c_void_p)]
        L = _lib.lib()
        L.dn_step_record_size.restype = ctypes.c_long
        if ctypes.sizeof(_Rec) != L.dn_step_record_size():
            raise RuntimeError("step record layout mismatch with the kernel library")
        _STEP_RECORD = _Rec
    return _STEP_RECORD


class StepRecorder:
    """Per-step train records of device-fed steps (``runtime.feed.DeviceFeed``): ring slot
    ``c mod n`` of batch cursor ``c`` holds the step's score column ``out[:, col]`` (``[B]``; ICA:
    ``prob[:, 1]``, the reference's train-AUC input, ``comps/icalstm/__init__.py:64-65``; ``col``
    < 0: the predicted class, FS's hard-label scores, ``comps/fs/__init__.py:57-59``) and its
    loss (``:67-68``).  The write rides in the packing Adam launch (one more workgroup,
    ``optim.hip adam_pack_kernel``) or is a one-workgroup launch of its own (``dn_step_record``)
    after an update that already advanced the cursor; either way K-step graph replays keep exact
    per-sample train metrics with no host work between steps."""

    def __init__(self, n: int, B: int, cursor: torch.Tensor, col: int = 1):
        self.n, self.B, self.col = int(n), int(B), int(col)
        dev = cursor.device
        self.scores = torch.zeros(self.n, self.B, dtype=torch.float32, device=dev)
        self.losses = torch.zeros(self.n, dtype=torch.float32, device=dev)
        self.cursor = cursor
        self._cache: Dict[tuple, object] = {}

    def args(self, out: torch.Tensor, loss: torch.Tensor, pred: Optional[torch.Tensor] = None):
        """The ``StepRecord`` struct for a step whose outputs are ``out`` [B, C] / ``loss`` []
        (/ ``pred`` [B] int64, needed when ``col`` < 0).  Cached per output set: a multi-site
        step issued from the host every step asks for the same static buffers' struct each time
        (no per-step class or library query)."""
        if self.col < 0 and (pred is None or pred.dtype != torch.int64 or pred.numel() != self.B
                             or not pred.is_contiguous()):
            raise ValueError("StepRecorder(col < 0) records the predicted class: pass pred [B] int64")
        pp = pred.data_ptr() if (self.col < 0 and pred is not None) else None
        key = (out.data_ptr(), loss.data_ptr(), tuple(out.shape), pp)
        rec = self._cache.get(key)
        if rec is not None:
            return rec
        if (out.dim() != 2 or out.shape[0] != self.B or out.dtype != torch.float32
                or not out.is_contiguous() or loss.dtype != torch.float32 or loss.numel() != 1):
            raise ValueError("StepRecorder: out must be contiguous fp32 [B, C], loss fp32 scalar")
        rec = _step_record_type()(out.data_ptr(), out.shape[1], self.col, self.B, loss.data_ptr(),
                                  self.scores.data_ptr(), self.losses.data_ptr(), self.n,
                                  self.cursor.data_ptr(), pp)
        if len(self._cache) > 64:
            self._cache.clear()
        self._cache[key] = rec
        return rec

    def record(self, out: torch.Tensor, loss: torch.Tensor, cofs: int = -1,
               pred: Optional[torch.Tensor] = None):
        """Standalone record into slot ``(cursor + cofs) mod n``."""
        if out.is_cuda:
            rec = self.args(out, loss, pred)  # (held: the launcher reads it through its address)
            _lib.call("dn_step_record", ctypes_addr(rec), int(cofs), _lib.stream())
            return
        c = (int(self.cursor.item()) + cofs) % self.n
        self.scores[c].copy_((pred if self.col < 0 else out[:, self.col]).float())
        self.losses[c] = loss.detach().float()

    def reset(self):
        self.scores.zero_()
        self.losses.zero_()
