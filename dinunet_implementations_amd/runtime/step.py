"""The training step of one site: forward, loss, backward, aggregation, optimizer.

Everything launch-bound (encoder GEMM, persistent LSTM, classifier, loss head, full backward) is
captured into HIP graphs and replayed.  With one site the fused Adam update is captured too (its
step number and bias corrections live on the device): a host-fed step is one prologue launch +
one replay, and device-fed runs (``bind`` / ``run``) replay graphs of K whole steps with no host
work between them.

Before each host-fed replay ONE prologue launch converts the batch into the graph's static
(bf16) input, copies the labels and zeroes the flat gradient.

Across sites (``comm_graph``, default) the engine's collectives are captured in the same graph:
the two backward parts, the bucket exchanges between them, the engine's reduction and the fused
Adam form ONE captured step, and device-fed runs replay K-step graphs exactly as at one site.  An
engine says whether its site-means can be captured (``Engine.capturable``): always with the peer
exchange (``parallel/peer.py``, kernels on the step's stream, any process-group backend), with
RCCL for the all-reduce; host collectives (gloo all-reduce) and RCCL's all-to-all exchange
cannot, and those steps (or ``DINUNET_CAPTURE_COMM=0``) replay two graphs A / B with the
collectives and the update issued from the host between and after the replays.

Split backward (across sites): the model's ``stem`` (ICA: the encoder) produces the LAST
gradients of the backward, so the backward is issued in two parts cut at the LSTM input
projection when the model provides ``proj_stem`` (part A ends with every LSTM and head gradient
final; part B = the input-gradient GEMM + the encoder's weight gradients), else at the stem
output.  The exchange of every non-stem gradient starts between the parts (RCCL: on its own
stream; peer: the push, whose data cross the links while part B runs) and only the small stem
bucket's exchange is exposed.
"""
from __future__ import annotations

import contextlib
import os
from typing import Callable, Optional

import torch

from .. import ops
from ..ops import _lib
from ..ops.lstm import defer_pack, ride_pack, run_deferred_pack, use_persistent
from .timers import NULL, PhaseTimer, enabled_by_env


def ica_forward_loss(model, x, y):
    return model.forward_loss(x, y)


def fs_forward_loss(model, x, y):
    return model.forward_loss(x, y)


HEADS = {"ica": ica_forward_loss, "fs": fs_forward_loss}

# Capture in thread-local mode: RCCL's process-group watchdog thread polls the events of
# finished collectives (hipEventQuery) at any time, and under the default global mode such a
# query from another thread while this thread captures invalidates the capture and kills the
# watchdog (hipErrorStreamCaptureUnsupported -> abort).
CAPTURE_MODE = "thread_local"


def _engine_capturable(engine) -> bool:
    cap = getattr(engine, "capturable", None)
    if cap is None:  # an engine without the property: RCCL collectives capture, host ones not
        return engine.group.backend == "nccl"
    return bool(cap)


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def _quiesce_collectives(group) -> None:
    """Before a capture on an RCCL group: every eager collective issued so far has finished on
    the device AND the process group's watchdog has retired it.  The watchdog polls the
    completion event of every eager collective it holds; one it still held when a capture
    re-recorded that event aborted the process (hipErrorCapturedEvent, ``profiles/
    r6_captured_event_abort.txt``: right after eager collectives, e.g. the warm-up steps or
    dsgd_collective=calibrate).  ``ProcessGroup._wait_for_pending_works`` returns once the
    watchdog's list is empty -- a condition, not a guessed delay (the round-5 form slept 0.3 s).
    ``init_sites`` also turns off torch's completion-event cache
    (``TORCH_NCCL_CUDA_EVENT_CACHE=0``), so no pooled event is shared between works."""
    if getattr(group, "distributed", False) and getattr(group, "backend", None) == "nccl":
        torch.cuda.synchronize()
        pg = getattr(group, "pg", None)
        if pg is not None and hasattr(pg, "_wait_for_pending_works"):
            pg._wait_for_pending_works()


# The LSTM weight repack leaves the graph and rides in the step prologue's launch
# (DINUNET_DEFER_PACK=0 keeps it captured)
DEFER_PACK = os.environ.get("DINUNET_DEFER_PACK", "1") != "0"

# Split capture (dSGD across sites) cuts at the LSTM input projection when the model allows
# (DINUNET_SPLIT_AT=stem keeps the encoder-output cut): graph B is then the input-gradient GEMM +
# the encoder's weight gradients, ~25 us at the headline step instead of ~10
SPLIT_AT_PROJECTION = os.environ.get("DINUNET_SPLIT_AT", "projection") != "stem"

# Device-fed steps with the Adam-emitted pack read the batch IN PLACE from the HBM-resident
# dataset at large batch: the Adam writes the next batch's subject indices instead of copying
# the batch (B*S*C*W bf16: 400 MB at B=2048), and the two GEMMs that consume it -- the encoder
# forward (A rows) and the encoder weight gradient (B's k rows) -- gather the rows through them
# (ops.gemm.rows_from, gemm.hip RowGather).  DINUNET_ROWS_FEED=1 / 0 forces it on / off; auto
# from 256 samples per step
ROWS_FEED = os.environ.get("DINUNET_ROWS_FEED", "auto")
ROWS_FEED_MIN_B = 256

# Device-fed single-site steps: the fused Adam rewrites the packed LSTM / encoder operand images
# from the parameters it updates, zeroes the gradient and gathers the next batch (one launch
# instead of Adam + a pack/gather launch per step); DINUNET_ADAM_PACK=0 keeps the pack launch
ADAM_PACK = os.environ.get("DINUNET_ADAM_PACK", "1") != "0"

# Multi-site steps over RCCL capture the engine's collectives inside the step graph
# (DINUNET_CAPTURE_COMM=0 keeps host-issued collectives between two graph replays)
CAPTURE_COMM = os.environ.get("DINUNET_CAPTURE_COMM", "1") != "0"


class _NoDefer:
    records: list = []

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class TrainStep:
    def __init__(self, model, flat, opt, engine, task: str = "ica", use_graph: bool = True,
                 eager_warmup: int = 3, forward_loss: Optional[Callable] = None,
                 timers: Optional[PhaseTimer] = None, split: Optional[bool] = None,
                 accum: int = 1):
        self.model = model
        # gradient accumulation (``local_iterations``): a step is ``accum`` calls; the first
        # zeroes the gradient, every call backpropagates d(loss)/accum (the reference's
        # (loss / local_iterations).backward()), the last one reduces and updates
        self.accum = max(1, int(accum))
        self.flat = flat
        self.opt = opt
        self.engine = engine
        self.forward_loss = forward_loss or HEADS[task]
        # graph-capturable engines: dSGD, and rank-dAD in gradient space (its local
        # factorisation joins the captured region via pre_reduce)
        self.use_graph = (use_graph and flat.data.is_cuda
                          and (engine.name == "dSGD" or getattr(engine, "fast", False)))
        # the local factorisation (rank-dAD / PowerSGD pre_reduce) is captured only when every
        # replay is a whole step: with accumulation it must run once, after the LAST micro-batch
        # (PowerSGD's error feedback and rank-dAD's warm start would otherwise be applied to
        # every partial gradient), so it then runs eagerly inside engine.reduce()
        pre = getattr(engine, "pre_reduce", None) if engine.name != "dSGD" else None
        if not getattr(engine, "pre_capturable", True):
            pre = None  # (engine.reduce() runs it after the replay)
        self._pre_reduce = pre if self.accum == 1 else None
        self._pre_any = pre  # device-fed accumulated steps capture it after the last micro-batch
        self.eager_warmup = eager_warmup
        self.calls = 0
        self.graph = None
        self.static = None
        self.last_loss = torch.zeros(())
        self.last_out = None
        self.last_pred = None
        self.timers = timers if timers is not None else (PhaseTimer() if enabled_by_env() else NULL)
        # split capture: needs a stem/body model, the default loss, and sites to overlap with
        can_split = (self.use_graph and forward_loss is None and hasattr(model, "stem")
                     and hasattr(model, "body_loss") and hasattr(model, "stem_parameters")
                     and hasattr(engine, "split_buckets"))
        if split is None:
            env = os.environ.get("DINUNET_SPLIT_GRAPH", "")
            split = can_split and ((engine.group.distributed
                                    and getattr(engine, "prefers_split", True))
                                   if env == "" else env == "1")
        self.split = bool(split and can_split)
        # collectives inside the captured step: the engine says whether its site-means can be
        # captured (the peer exchange on any backend, RCCL's all-reduce; not host collectives)
        grp = engine.group
        self.comm_graph = bool(CAPTURE_COMM and self.use_graph and grp.distributed
                               and self.accum == 1 and _engine_capturable(engine))
        self.split_at = None  # "projection" | "stem", set at capture
        self._first_buckets = engine.split_buckets(list(model.stem_parameters())) if self.split else []
        self.graph_b = None
        self._one = None
        self.graph_opt = False
        self._prebump = False
        self._cap_lr = None
        self._bf16_in = False
        self._packs: list = []  # LSTM repacks deferred out of the captured graph
        self.src = None  # device-fed batches (bind)
        self.rec = None  # device-side train records of device-fed steps (bind)

    def _grad_one(self, device, dtype=torch.float32):
        # a persistent d(loss)/d(loss) = 1: loss.backward() would launch a fill kernel for it
        # inside every replay
        one = self._one
        if one is None or one.device != device or one.dtype != dtype:
            one = self._one = torch.full((), 1.0 / self.accum, dtype=dtype, device=device)
        return one

    def _backward(self, loss):
        torch.autograd.backward(loss, self._grad_one(loss.device, loss.dtype))

    def _fwd_bwd(self, x, y):
        with self.engine.step_context():
            # the step backpropagates exactly this tensor: fused ops may start their backward
            # inside the forward (ops.head.loss_grad_hint)
            hint = self._grad_one(x.device) if x.is_cuda else None
            with ops.head.loss_grad_hint(hint):
                out, loss, pred = self.forward_loss(self.model, x, y)
            self._backward(loss)
        return out, loss, pred

    def _eager(self, x, y, first: bool = True, last: bool = True):
        T = self.timers
        sync = getattr(self.engine, "sync_enabled", None)
        with T.phase("fwd_bwd"):
            if first:
                self.flat.zero_grad()
            if sync is not None:
                self.engine.sync_enabled = last  # collectives only with the last micro-batch
            out, loss, pred = self._fwd_bwd(x, y)
        if last:
            with T.phase("reduce"):
                scale = self.engine.reduce()
            with T.phase("optim"):
                self.opt.step(grad_scale=scale)
        self.last_out, self.last_loss, self.last_pred = out.detach(), loss.detach(), pred
        return loss

    def _static_inputs(self, x, y):
        # bf16 static input when the model takes it: the step prologue converts while copying
        # (bit-identical: the GEMMs round their operands to bf16 while staging anyway)
        bf = (x.dtype == torch.float32 and getattr(self.model, "accepts_bf16_input", False)
              and x.numel() % 8 == 0 and y.dtype == torch.int64 and self.flat.grad.numel() % 4 == 0)
        sx = torch.empty_like(x, dtype=torch.bfloat16 if bf else x.dtype)
        sy = torch.empty_like(y)
        self._bf16_in = bf
        return sx, sy

    def _feed(self, x, y, sx, sy, zero: bool = True):
        """Before a replay, in ONE launch when possible: inputs into the static buffers, the
        gradient buffer zeroed (the graphs no longer contain the zeroing; not for the later
        micro-batches of an accumulated step), the LSTM weight repack the capture deferred out
        of the graph (``ops.lstm.defer_pack``) and, when the update is captured
        (``_prebump``), the advance of Adam's device step counter."""
        bump = self.opt.device_step() if (self.graph_opt and self._prebump) else None
        g = self.flat.grad if zero else self.flat.grad[:0]
        if self._packs:
            if self._bf16_in:
                run_deferred_pack(self._packs, (x, sx, y, sy, g), bump)
                return
            run_deferred_pack(self._packs)
        if self._bf16_in:
            ops.step_prologue(x, sx, y, sy, g, bump)
            return
        if sx.data_ptr() != x.data_ptr():
            sx.copy_(x, non_blocking=True)
        if y.dtype == torch.int64 and self.flat.grad.numel() % 4 == 0:
            ops.step_prologue(x, None, y, sy, g, bump)
        else:
            if sy.data_ptr() != y.data_ptr():
                sy.copy_(y, non_blocking=True)
            if zero:
                self.flat.grad.zero_()

    def _dev_graph_opt_ok(self) -> bool:
        """Can a device-fed replay hold whole steps (update inside)?  With accumulation a
        device-fed body is a whole step of ``accum`` micro-batches (:meth:`_dev_body_accum`),
        so unlike a host-fed replay it may hold the reduction and the update too."""
        if self.accum == 1:
            return self._graph_opt_ok()
        g = self.engine.group
        comm = (not g.distributed) or (CAPTURE_COMM and _engine_capturable(self.engine))
        return comm and isinstance(self.opt, ops.FusedAdam) and self.flat.data.is_cuda

    def _graph_opt_ok(self) -> bool:
        # the optimizer joins the graph when every collective between backward and update is
        # captured too (one site: none) and every replay is a whole step (no accumulation)
        return ((not self.engine.group.distributed or self.comm_graph)
                and isinstance(self.opt, ops.FusedAdam) and self.flat.data.is_cuda
                and self.accum == 1)

    def _reduce_after_replay(self):
        if self._pre_reduce is not None:
            return self.engine.reduce(factorized=True)
        return self.engine.reduce()

    def _capture(self, x, y):
        _quiesce_collectives(self.engine.group)
        sx, sy = self._static_inputs(x, y)
        g = torch.cuda.CUDAGraph()
        prev = getattr(self.engine, "sync_enabled", None)
        if prev is not None:
            self.engine.sync_enabled = False  # no collectives inside the captured region
        self.graph_opt = self._graph_opt_ok()
        # the feed before each replay always launches a step prologue on this path, and that
        # launch advances Adam's device step counter: no one-thread bump node in the graph
        self._prebump = self.graph_opt and (
            self._bf16_in or (y.dtype == torch.int64 and self.flat.grad.numel() % 4 == 0))
        if self.graph_opt:
            self.opt.sync_device_step()
            self._cap_lr = self.opt.lr
        try:
            with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE), self._defer_pack() as dp:
                if self.split:  # comm_graph: both backward parts, the buckets launched between
                    out, loss, pred = self._split_backward(sx, sy)
                else:
                    out, loss, pred = self._fwd_bwd(sx, sy)
                if self._pre_reduce is not None:
                    self._pre_reduce()
                if self.graph_opt:
                    scale = (self.engine.reduce(factorized=True) if self._pre_reduce is not None
                             else self.engine.reduce())
                    self.opt.step_graphable(grad_scale=scale, prebumped=self._prebump)
        finally:
            if prev is not None:
                self.engine.sync_enabled = prev
        self.graph = g
        self.static = (sx, sy, out, loss, pred)
        self._packs = dp.records

    def _defer_pack(self):
        return defer_pack() if DEFER_PACK else _NoDefer()

    def _split_fwd_bwd(self, sx, sy):
        """Graph A of a split step: forward, loss and the backward of everything after the cut
        (returns the cut tensor ``h``, its detached twin ``hd`` holding d loss / d h, and the
        step outputs).  The cut is the LSTM input projection when the model has the fused path
        (``proj_stem``: every LSTM / head gradient is then final in graph A and only the input
        gradient + encoder gradients remain for graph B), else the stem (encoder) output."""
        at_proj = (SPLIT_AT_PROJECTION and hasattr(self.model, "proj_stem")
                   and self.model.split_at_projection(sx))
        self.split_at = "projection" if at_proj else "stem"
        with self.engine.step_context():
            h = self.model.proj_stem(sx) if at_proj else self.model.stem(sx)
            hd = h.detach().requires_grad_(h.requires_grad)
            with ops.head.loss_grad_hint(self._grad_one(sx.device)):
                body = self.model.proj_body_loss if at_proj else self.model.body_loss
                out, loss, pred = body(hd, sy)
            self._backward(loss)
        return h, hd, out, loss, pred

    def _split_backward(self, sx, sy, fwd_ctx=None):
        """Both parts of a split step issued into the current stream, the non-stem buckets'
        collectives launched between them (captured: a branch on RCCL's stream).  ``fwd_ctx``:
        the context the forward runs in (device-fed prologue / Adam-emitted pack)."""
        with (fwd_ctx if fwd_ctx is not None else _NoDefer()) as rp:
            h, hd, out, loss, pred = self._split_fwd_bwd(sx, sy)
        if isinstance(rp, ride_pack) and not rp.consumed:
            raise RuntimeError("device-fed prologue was not absorbed by the model's weight pack")
        for b in self._first_buckets:  # all-reduce under the stem backward
            self.engine.launch_bucket(b)
        if h.requires_grad:
            torch.autograd.backward(h, hd.grad)
        self._keep = (h, hd)
        return out, loss, pred

    def _capture_split(self, x, y):
        sx, sy = self._static_inputs(x, y)
        ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        self.engine.sync_enabled = False
        self.graph_opt = False
        try:
            with torch.cuda.graph(ga, capture_error_mode=CAPTURE_MODE), self._defer_pack() as dp:
                h, hd, out, loss, pred = self._split_fwd_bwd(sx, sy)
            with torch.cuda.graph(gb, pool=ga.pool(), capture_error_mode=CAPTURE_MODE):
                if h.requires_grad:
                    torch.autograd.backward(h, hd.grad)
        finally:
            self.engine.sync_enabled = True
        self.graph, self.graph_b = ga, gb
        self.static = (sx, sy, out, loss, pred)
        self._packs = dp.records
        self._keep = (h, hd)  # the graphs replay into these buffers

    def __call__(self, x, y, first: bool = True, last: bool = True):
        """One micro-batch; ``first`` / ``last`` delimit an accumulated step (``accum`` > 1)."""
        self.calls += 1
        if not self.use_graph:
            return self._eager(x, y, first, last)
        if self.graph is not None and self.graph_opt and self.opt.lr != self._cap_lr:
            self.graph = None  # the learning rate is baked into the captured update
        if self.graph is None:
            if self.calls <= self.eager_warmup * self.accum:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    loss = self._eager(x, y, first, last)
                torch.cuda.current_stream().wait_stream(s)
                return loss
            (self._capture_split if (self.split and not self.comm_graph) else self._capture)(x, y)
        sx, sy, out, loss, pred = self.static
        if sx.shape != x.shape or sy.shape != y.shape:  # e.g. a ragged last batch
            loss = self._eager(x, y, first, last)
            if self.graph_opt:
                # the eager update advanced only the host step count: the captured update reads
                # the device counter
                self.opt.sync_device_step()
            return loss
        T = self.timers
        with T.phase("fwd_bwd"):
            self._feed(x, y, sx, sy, zero=first)
            self.graph.replay()
            if self.graph_b is not None:
                if last:
                    for b in self._first_buckets:  # all-reduce under the stem backward
                        self.engine.launch_bucket(b)
                self.graph_b.replay()
        if not last:
            self.last_out, self.last_loss, self.last_pred = out, loss, pred
            return loss
        if hasattr(self.engine, "sync_enabled"):
            self.engine.sync_enabled = True
        if self.graph_opt:
            self.opt.step_count += 1  # the replay ran the update
        else:
            with T.phase("reduce"):
                scale = self._reduce_after_replay()
            with T.phase("optim"):
                self.opt.step(grad_scale=scale)
        self.last_out, self.last_loss, self.last_pred = out, loss, pred
        return loss

    # ---- device-fed steps ---------------------------------------------------------------------
    def bind(self, src, steps_per_graph: int = 8, recorder=None):
        """Train from an ``ops.DeviceSource`` (batches resident in HBM, gathered on the device).

        Every step is then device-only: its first launch gathers the batch at the source's cursor
        into the static input (riding in the LSTM weight pack when the model allows,
        ``ops.lstm.ride_pack``), zeroes the gradient and advances Adam's counter; its Adam
        launch advances the cursor.  With one site (the update inside the graph) ``run``
        replays graphs holding ``steps_per_graph`` whole steps, so there is no host work and no
        graph boundary between them.  ``recorder`` (``ops.StepRecorder`` on the source's cursor):
        every step also writes its score column and loss into the recorder's rings (inside the
        packing Adam launch when there is one), so the train metrics of an epoch are exact without
        a host round trip per step (``runtime.feed.DeviceFeed``)."""
        bf = src.X.dtype == torch.bfloat16
        if bf and not getattr(self.model, "accepts_bf16_input", False):
            raise ValueError("TrainStep.bind: a bf16 dataset needs a model that takes a bf16 batch")
        if not isinstance(self.opt, ops.FusedAdam):
            raise ValueError("TrainStep.bind: device-fed steps need the fused Adam")
        self.src = src
        self.rec = recorder
        if recorder is not None and recorder.cursor.data_ptr() != src.cursor.data_ptr():
            raise ValueError("TrainStep.bind: the recorder must index by the source's cursor")
        self.opt.cursor = src.cursor
        dev = src.X.device
        # the static input the prologue gathers into (bf16, or the fp32 rows of an fp32
        # dataset such as FS features: exact), and what the model reads of it
        self._dsx = torch.empty((src.B,) + src.sample_shape,
                                dtype=torch.bfloat16 if bf else torch.float32, device=dev)
        self._dsxf = src.view(self._dsx)
        self._dsy = torch.empty(src.B, dtype=torch.int64, device=dev)
        self._dK = (max(1, int(steps_per_graph)) if (self.use_graph and self._dev_graph_opt_ok())
                    else 1)
        self._dgraphs = {}
        self._dcalls = 0
        # the Adam-emitted operand pack (ADAM_PACK): every replayed step then runs encoder GEMM
        # (which advances Adam's step counter and the cursor) ... Adam (update + images + zeroed
        # gradient + NEXT batch); the eager warm-up steps keep the pack launch
        self._apack = None
        self._dsubj = None
        self._rows = None
        from ..ops.gemm import PLAIN_BLAS
        # (across sites the update runs after the replays, eagerly: the same launch then)
        # (one gather per step: not with accumulation, whose micro-batches gather each)
        if (ADAM_PACK and self.accum == 1 and self.use_graph and (self._graph_opt_ok() or self.split)
                and not PLAIN_BLAS and self._rides() and hasattr(self.model, "persistent_pack")):
            pp = self.model.persistent_pack(dev)
            if pp is not None:
                rows = self._rows_feed_ok(src)
                if rows:
                    # [B + 1]: a K tile's second subject index may be read one past the batch
                    self._dsubj = torch.zeros(src.B + 1, dtype=torch.int64, device=dev)
                    S = src.sample_shape[0]
                    self._rows = (self._dsx.view(src.B * S, -1),
                                  src.X.view(src.X.shape[0] * S, -1), self._dsubj, S)
                self.opt.attach_pack(pp, src, self._dsx, self._dsy,
                                     sd=self._dsubj if rows else None, copy_x=not rows)
                # the device step counter must exist before any capture: created inside one, its
                # allocation and initial fill would become nodes of the graph, resetting the
                # counter at every replay
                self.opt.sync_device_step()
                self._apack = pp

    def _rows_feed_ok(self, src) -> bool:
        """Read the batch in place (``ROWS_FEED``)?  A bf16 [N, S, ...] dataset with S >= 64
        windows per subject (at most two subjects per 64-row K tile) and 16-B window rows."""
        shp = src.sample_shape
        ok = (src.X.dtype == torch.bfloat16 and len(shp) >= 2 and shp[0] >= 64
              and (src.row // shp[0]) % 8 == 0)
        if ROWS_FEED == "1":
            if not ok:
                raise ValueError("DINUNET_ROWS_FEED=1: the dataset cannot be read in place")
            return True
        return ok and ROWS_FEED == "auto" and src.B >= ROWS_FEED_MIN_B

    def _rides(self) -> bool:
        fn = getattr(self.model, "prologue_rides_pack", None)
        return bool(fn is not None and fn(self._dsx))

    def _dev_prologue(self, bump, grad: Optional[torch.Tensor] = None):
        """The device-fed prologue of one step: riding in the model's first launch when it can
        (returns the context to run the forward in), else as a launch of its own.  ``grad``:
        the gradient range it zeroes (default all; empty for the later micro-batches of an
        accumulated step)."""
        grad = self.flat.grad if grad is None else grad
        if self._rides():
            tail = self.src.prologue_args(self._dsx, self._dsy, grad, bump)
            return ride_pack(tail)
        self.src.gather(self._dsx, self._dsy, grad, bump)
        return _NoDefer()

    def _dev_body_accum(self, graph_opt: bool):
        """One whole device-fed step of ``accum`` micro-batches (``local_iterations``; the
        reference's ``(loss / local_iterations).backward()`` per micro-batch and one update,
        ``/root/reference/compspec.json:88-95``): each micro-batch gathers its batch at the
        cursor and backpropagates d(loss)/accum into the gradient the first one zeroed; the
        cursor advances per micro-batch (the last one through the update) and every micro-batch
        is recorded; then, once, the local factorisation (rank-dAD / PowerSGD), the reduction and
        the update.  Eager (``graph_opt`` false), the collectives ride the last micro-batch's
        backward and the caller reduces and updates."""
        sx, sy = self._dsxf, self._dsy
        A = self.accum
        sync = getattr(self.engine, "sync_enabled", None)
        for k in range(A):
            bump = self.opt.device_step() if (graph_opt and k == 0) else None
            grad = self.flat.grad if k == 0 else self.flat.grad[:0]
            if sync is not None and not graph_opt and not _capturing():
                # eager only: a captured body without the update keeps the collectives off
                # (_dev_capture disabled them) and the engine's reduction after the replay
                # launches every bucket -- enabling them here would issue host or uncapturable
                # collectives inside the capture
                self.engine.sync_enabled = k == A - 1
            with self._dev_prologue(bump, grad) as rp:
                out, loss, pred = self._fwd_bwd(sx, sy)
            if isinstance(rp, ride_pack) and not rp.consumed:
                raise RuntimeError("device-fed prologue was not absorbed by the model's weight pack")
            if k < A - 1:
                self.src.cursor.add_(1)
                self._record(out, loss, pred)
        if graph_opt:
            if self._pre_any is not None:
                self._pre_any()
            scale = (self.engine.reduce(factorized=True) if self._pre_any is not None
                     else self.engine.reduce())
            self.opt.step_graphable(grad_scale=scale, prebumped=True)
            self._record(out, loss, pred)
        return out, loss, pred

    @contextlib.contextmanager
    def _apack_forward(self):
        """The forward of a step whose operands the previous step's Adam (or
        :meth:`_apack_prime`) already packed and gathered: its encoder GEMM advances Adam's device
        step counter and the batch cursor (``dn_gemm_arm_bump``)."""
        _lib.call("dn_gemm_arm_bump", self.opt.device_step().data_ptr(), self.src.cursor.data_ptr())
        self._apack.used = False
        try:
            with use_persistent(self._apack):
                yield
        finally:
            armed = int(_lib.lib().dn_gemm_bump_armed())
            _lib.call("dn_gemm_arm_bump", None, None)  # never leaks into a later launch
        if armed or not self._apack.used:
            raise RuntimeError("Adam-emitted pack: the forward did not start with the encoder GEMM "
                               "on the persistent operand images")

    def _rows_ctx(self):
        """The in-place batch rows (``ROWS_FEED``) for every GEMM issued inside -- the encoder
        forward AND its weight gradient, which a split step issues after the forward context."""
        from ..ops.gemm import rows_from
        return rows_from(*self._rows) if self._rows is not None else _NoDefer()

    def _dev_body_apack(self):
        """One whole device-fed step in the Adam-emitted-pack form (single site)."""
        sx, sy = self._dsxf, self._dsy
        with self._rows_ctx(), self._apack_forward():
            out, loss, pred = self._fwd_bwd(sx, sy)
        if self._pre_reduce is not None:
            self._pre_reduce()
        scale = (self.engine.reduce(factorized=True) if self._pre_reduce is not None
                 else self.engine.reduce())
        self.opt.step_pack(grad_scale=scale, record=self._rec_args(out, loss, pred))
        return out, loss, pred

    def _rec_args(self, out, loss, pred=None):
        return self.rec.args(out, loss, pred) if self.rec is not None else None

    def _record(self, out, loss, pred=None):
        """The standalone record of a step whose update already advanced the cursor."""
        if self.rec is not None:
            self.rec.record(out, loss, cofs=-1, pred=pred)

    def _apack_prime(self):
        """Before the first replay of a run: the persistent images from the current parameters,
        the gradient zeroed and the batch at the cursor gathered (one launch); the cursor steps
        back one, so the first step's encoder GEMM brings it back (see :meth:`_apack_unprime`)."""
        self.opt.sync_device_step()
        self.opt.step_pack(update=False, gofs=0)
        self.src.cursor.sub_(1)

    def _apack_unprime(self):
        # after the last replay: the cursor names the NEXT batch again (the eager convention)
        self.src.cursor.add_(1)

    def _dev_body_split(self):
        """One whole multi-site device-fed step with its collectives (``comm_graph``): prologue
        (or the Adam-emitted pack's forward), the split backward with the non-stem buckets'
        all-reduce between its parts, the reduction, and the update that also emits the next
        step's operands -- everything a replay needs, so K such steps form one graph."""
        if self._apack is not None:
            with self._rows_ctx():
                out, loss, pred = self._split_backward(self._dsxf, self._dsy,
                                                       self._apack_forward())
        else:
            out, loss, pred = self._split_backward(self._dsxf, self._dsy,
                                                   self._dev_prologue(self.opt.device_step()))
        scale = self._reduce_after_replay()
        if self._apack is not None:
            self.opt.step_pack(grad_scale=scale, record=self._rec_args(out, loss, pred))
        else:
            self.opt.step_graphable(grad_scale=scale, prebumped=True)
            self._record(out, loss, pred)
        return out, loss, pred

    def _dev_body(self, graph_opt: bool):
        """One whole device-fed step as issued into the current stream (eager or captured)."""
        if self.accum > 1:
            return self._dev_body_accum(graph_opt)
        if self.split and self.comm_graph and graph_opt:
            return self._dev_body_split()
        if self._apack is not None and graph_opt:
            return self._dev_body_apack()
        bump = self.opt.device_step() if graph_opt else None
        sx, sy = self._dsxf, self._dsy
        with self._dev_prologue(bump) as rp:
            out, loss, pred = self._fwd_bwd(sx, sy)
        if isinstance(rp, ride_pack) and not rp.consumed:
            raise RuntimeError("device-fed prologue was not absorbed by the model's weight pack")
        if self._pre_reduce is not None and graph_opt:
            self._pre_reduce()
        if graph_opt:
            scale = (self.engine.reduce(factorized=True) if self._pre_reduce is not None
                     else self.engine.reduce())
            self.opt.step_graphable(grad_scale=scale, prebumped=True)
            self._record(out, loss, pred)
        return out, loss, pred

    def _dev_capture(self, k: int):
        _quiesce_collectives(self.engine.group)
        g = torch.cuda.CUDAGraph()
        prev = getattr(self.engine, "sync_enabled", None)
        if prev is not None:
            self.engine.sync_enabled = False
        graph_opt = self._dK > 1 or self._dev_graph_opt_ok()
        if graph_opt:
            self.opt.sync_device_step()
            self._cap_lr = self.opt.lr
        try:
            with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
                for _ in range(k):
                    res = self._dev_body(graph_opt)
        finally:
            if prev is not None:
                self.engine.sync_enabled = prev
        self._dgraphs[k] = (g, res, graph_opt)

    def _dev_capture_split(self):
        """Device-fed form of :meth:`_capture_split`: graph A = prologue + forward + backward
        down to the cut (:meth:`_split_fwd_bwd`), graph B = the rest (the all-reduce of every
        non-stem gradient runs between the two replays)."""
        _quiesce_collectives(self.engine.group)
        ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        sx, sy = self._dsxf, self._dsy
        self.engine.sync_enabled = False
        try:
            with self._rows_ctx():
                with torch.cuda.graph(ga, capture_error_mode=CAPTURE_MODE):
                    with (self._apack_forward() if self._apack is not None
                          else self._dev_prologue(None)) as rp:
                        h, hd, out, loss, pred = self._split_fwd_bwd(sx, sy)
                    if isinstance(rp, ride_pack) and not rp.consumed:
                        raise RuntimeError("device-fed prologue was not absorbed by the weight "
                                           "pack")
                with torch.cuda.graph(gb, pool=ga.pool(), capture_error_mode=CAPTURE_MODE):
                    if h.requires_grad:
                        torch.autograd.backward(h, hd.grad)
        finally:
            self.engine.sync_enabled = True
        self._dgraphs["split"] = (ga, gb, (out, loss, pred), (h, hd))

    def _dev_eager(self):
        T = self.timers
        sync = getattr(self.engine, "sync_enabled", None)
        with T.phase("fwd_bwd"):
            if sync is not None:
                self.engine.sync_enabled = True
            out, loss, pred = self._dev_body(False)
        with T.phase("reduce"):
            scale = self.engine.reduce()
        with T.phase("optim"):
            self.opt.step(grad_scale=scale)  # advances the source cursor too
            self._record(out, loss, pred)
        self.last_out, self.last_loss, self.last_pred = out.detach(), loss.detach(), pred
        return loss

    def run(self, n: int):
        """``n`` device-fed training steps (``bind`` first); returns the last step's loss."""
        if self.src is None:
            raise RuntimeError("TrainStep.run: bind a DeviceSource first")
        loss = self.last_loss
        done = 0
        primed = False
        try:
            while done < n:
                loss, done, primed = self._run_one(n, done, loss, primed)
        finally:
            if primed:
                self._apack_unprime()
        return loss

    def _run_one(self, n: int, done: int, loss, primed: bool):
        """One eager step, one split-graph step or one K-step replay of :meth:`run`; returns
        ``(loss, done, primed)``."""
        self._dcalls += 1
        if not self.use_graph or self._dcalls <= self.eager_warmup:
            if primed:  # (never: warm-up steps precede every replay)
                self._apack_unprime()
                primed = False
            if self.use_graph:  # warm-up off the capture stream, like __call__
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    loss = self._dev_eager()
                torch.cuda.current_stream().wait_stream(s)
            else:
                loss = self._dev_eager()
            return loss, done + 1, primed
        if self._dgraphs and self.opt.lr != self._cap_lr and any(
                v[2] is True for v in self._dgraphs.values()):
            self._dgraphs = {}  # the learning rate is baked into the captured update
        if self.split and not self.comm_graph and self.accum == 1:
            if "split" not in self._dgraphs:
                self._dev_capture_split()
            ga, gb, (out, loss, pred), _ = self._dgraphs["split"]
            if self._apack is not None and not primed:
                self._apack_prime()
                primed = True
            with self.timers.phase("fwd_bwd"):
                ga.replay()
                for b in self._first_buckets:  # all-reduce under the stem backward
                    self.engine.launch_bucket(b)
                gb.replay()
            self.engine.sync_enabled = True
            with self.timers.phase("reduce"):
                scale = self._reduce_after_replay()
            with self.timers.phase("optim"):
                if self._apack is not None:
                    # + next operands and batch (+ this step's train record)
                    self.opt.step_pack(grad_scale=scale, record=self._rec_args(out, loss, pred))
                    self.opt.step_count += 1
                else:
                    self.opt.step(grad_scale=scale)
                    self._record(out, loss, pred)
            self.last_out, self.last_loss, self.last_pred = out, loss, pred
            return loss, done + 1, primed
        k = min(self._dK, n - done)
        if k not in self._dgraphs:
            self._dev_capture(k)
        g, (out, loss, pred), graph_opt = self._dgraphs[k]
        if self._apack is not None and graph_opt and not primed:
            self._apack_prime()
            primed = True
        with self.timers.phase("fwd_bwd"):
            g.replay()
        if graph_opt:
            self.opt.step_count += k
        else:
            with self.timers.phase("reduce"):
                # the replay holds no local factorisation here (_dev_body captures pre_reduce
                # only with the update): the engine's full reduction runs it
                scale = self.engine.reduce()
            with self.timers.phase("optim"):
                self.opt.step(grad_scale=scale)
                self._record(out, loss, pred)
        self.last_out, self.last_loss, self.last_pred = out, loss, pred
        return loss, done + k, primed

    def prepare(self, n: int = 0):
        """Capture (without running) every graph a following ``run(n)`` will replay, so a timed
        region never includes a capture.  Call after the eager warm-up steps."""
        if self.src is None or not self.use_graph or self._dcalls < self.eager_warmup:
            return
        if self.split and not self.comm_graph and self.accum == 1:
            if "split" not in self._dgraphs:
                self._dev_capture_split()
            return
        for k in ({self._dK} if n <= 0 else {min(self._dK, n), n % self._dK} - {0}):
            if k not in self._dgraphs:
                self._dev_capture(k)

    @property
    def last_labels(self):
        """Labels of the last device-fed step.  With the Adam-emitted pack the static label
        buffer already holds the NEXT batch's labels, so they are looked up at the cursor."""
        if self._apack is not None and self._dgraphs:
            return self.src.batch(int(self.src.cursor.item()) - 1)[1]
        return self._dsy
