"""Gradient-aggregation engines: dSGD, rank-dAD, PowerSGD (reference ``comps/__init__.py:13-16``).

Each engine turns every site's local gradient (living in the flat grad buffer of
``ops.FlatParams``) into the *global* update all sites apply with their own optimizer, so
replicas stay identical:

* ``dSGD``     mean of site gradients — one (bucketed, backward-overlapped) RCCL all-reduce.
* ``rankDAD``  for every ``nn.Linear``: rank-r factors of ``Delta^T A`` from a structured power
  iteration (``lowrank.dad_factors``), all-gathered (a few KB per layer), reconstructed as
  ``mean_s P_s Q_s^T``; exact dAD (raw ``A``, ``Delta`` exchange) when r covers the full rank.
  Every other parameter (biases, BatchNorm) falls back to the dSGD mean.
* ``powerSGD`` rank-r ``P = M Q`` / ``Q = M^T P`` with two all-reduces, warm-started ``Q`` and
  per-site error feedback (Vogels et al. 2019); vectors use the dSGD mean.

Every engine also exposes the three pieces the COINSTAC file transport needs
(``payload`` on a site, ``aggregate`` on the remote, ``apply`` back on the site) with the same
arithmetic as the collective path (``compat/``).

``reduce()`` returns the scale the optimizer must apply to the flat gradient (dSGD leaves the
all-reduce SUM in place and folds ``1/world`` into the fused Adam launch).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops import _grad as _gradreg
from ..ops import _lib
from ..ops import capture as _cap
from ..ops.optim import FlatParams
from .collective import (PAYLOAD_TYPES, SB, DirectMean, from_payload, launch_on, payload_name,
                         payload_numel, to_payload)
from .group import SiteGroup
from .lowrank import EPS as EPS_MGS
from .lowrank import LowRankTable, _mgs_torch_, dad_factors, orthonormalize_

Tensor = torch.Tensor


COLLECTIVES = ("auto", "allreduce", "direct", "peer", "calibrate")


class Engine:
    name = "base"

    def __init__(self, model: nn.Module, flat: FlatParams, group: SiteGroup, cfg: Optional[dict] = None):
        self.model = model
        self.flat = flat
        self.group = group
        self.cfg = dict(cfg or {})
        # wire type of every site-mean (collective.payload_name): fp16 at precision_bits=16 like
        # the reference, or the explicit ``payload_dtype``; always accumulated in fp32
        self.wire = payload_name(self.cfg)
        self.half = self.wire != "fp32"
        self.comm_bytes = 0  # payload bytes this site sent in the last reduce (observability)
        self._means: Dict[Tuple[int, int], DirectMean] = {}
        # ``dsgd_collective``: the site-mean form of every engine -- "allreduce" (RCCL / gloo),
        # "direct" (all-to-all + fp32 sum + all-gather through the process group), "peer" (the
        # IPC-mapped HBM exchange of parallel/peer.py: kernels only, captured in the step's
        # graph on any backend), "auto" (peer for 16-bit wires on GPU sites -- the fp32-sum form
        # the reference's 16-bit payloads need, captured -- else all-reduce), "calibrate"
        # (dSGD: measured; the low-rank engines take auto's choice)
        coll = str(self.cfg.get("dsgd_collective", "auto"))
        if coll not in COLLECTIVES:
            raise ValueError(f"dsgd_collective {coll!r}: expected one of {', '.join(COLLECTIVES)}")
        self.collective = coll
        self.peer = self._want_peer(coll)

    def _peer_ok(self) -> bool:
        from . import peer as _peer
        return _peer.available(self.group, self.flat.grad.device)

    def _want_peer(self, coll: str) -> bool:
        if not self.group.distributed:
            return False
        if coll == "peer":
            if not self._peer_ok():
                raise ValueError("dsgd_collective='peer' needs GPU sites and the kernel library "
                                 f"(at most 16 sites); device {self.flat.grad.device}")
            return True
        return coll in ("auto", "calibrate") and self.half and self._peer_ok()

    # collective path -------------------------------------------------------------------------
    @property
    def capturable(self) -> bool:
        """Can the step capture this engine's collectives in its HIP graph
        (``runtime.step.TrainStep.comm_graph``)?  Always with the peer exchange (its kernels are
        ordinary launches on the step's stream, whatever the process group); with RCCL for the
        fp32 all-reduce; not for host collectives (gloo) nor for RCCL's all-to-all exchange
        (captured from the exchange's own stream it crashed at capture end,
        ``tools/diag/capture_collectives.py`` a2a_side, RCCL 2.26.6)."""
        if not self.group.distributed or self.peer:
            return True
        return self.group.backend == "nccl" and not self.half

    @property
    def pre_capturable(self) -> bool:
        """May the step capture :meth:`pre_reduce` (the local factorisation) in its graph?  Not
        when it starts with a collective of its own (rank-dAD's site mean over several GPUs per
        site, a host-issued collective on gloo): the step then runs it after the replay."""
        return True

    def _peer_mean(self, tag, n: int):
        from . import peer as _peer
        return _peer.mean(self.group, self.flat.grad.device, n, self.wire, (self.name,) + tuple(tag))

    def step_context(self):
        return contextlib.nullcontext()

    def reduce(self) -> float:
        raise NotImplementedError

    # resume ------------------------------------------------------------------------------------
    def state_dict(self) -> Dict[str, object]:
        """Engine state a resumed run needs to continue the same curve (warm-started factors,
        error feedback); empty for stateless engines."""
        return {}

    def load_state_dict(self, sd: Dict[str, object]):
        pass

    # file-transport path (COINSTAC compat) ---------------------------------------------------
    def payload(self) -> Dict[str, Tensor]:
        raise NotImplementedError

    @classmethod
    def aggregate(cls, payloads: Sequence[Dict[str, Tensor]], cfg: Optional[dict] = None) -> Dict[str, Tensor]:
        raise NotImplementedError

    def apply(self, agg: Dict[str, Tensor]) -> float:
        raise NotImplementedError

    # helpers ---------------------------------------------------------------------------------
    def _direct(self, key, n: int, device) -> DirectMean:
        dm = self._means.get(key)
        if dm is None or dm.n != n:
            dm = self._means[key] = DirectMean(self.group, n, self.wire, device)
        return dm

    def _allreduce_mean_(self, buf: Tensor, tag=("mean",)):
        """In-place mean over sites, honouring ``precision_bits`` / ``payload_dtype``: the peer
        exchange when selected (``tag`` names the exchange region: exchanges that may be in
        flight together need their own), else a 16-bit payload goes through the direct exchange
        (fp32 accumulation, collective.DirectMean) and fp32 through the all-reduce."""
        g = self.group
        if not g.distributed:
            return
        if self.peer:
            self.comm_bytes += self._peer_mean(tag, buf.numel()).run_(buf)
        elif self.half:
            self.comm_bytes += self._direct(("mean", buf.numel()), buf.numel(), buf.device).run_(buf)
        else:
            g.all_reduce(buf)
            buf.mul_(1.0 / g.world)
            self.comm_bytes += buf.numel() * 4


class _PeerWork:
    """``Work``-like handle of a pushed peer exchange: ``wait()`` issues its reduce + unpack on
    the current stream."""

    def __init__(self, pm, view: Tensor, scale: float = 1.0):
        self.pm, self.view, self.scale = pm, view, scale

    def wait(self):
        self.pm.finish(self.view, self.scale)


# =============================================================================================
# dSGD
# =============================================================================================
class DSGDEngine(Engine):
    """Bucketed all-reduce of the flat gradient, overlapped with the backward pass.

    Buckets are contiguous ranges of the flat buffer formed in REVERSE parameter order (the
    order gradients become ready: classifier, then LSTM, then encoder for ICA).  A bucket's
    all-reduce is launched from the post-accumulate-grad hook of its last parameter, on RCCL's
    own stream, while autograd keeps computing earlier layers.
    """
    name = "dSGD"

    def __init__(self, model, flat, group, cfg=None, bucket_mb: Optional[float] = None,
                 overlap: bool = True):
        super().__init__(model, flat, group, cfg)
        self.overlap = overlap and group.distributed and bool(self.cfg.get("dsgd_overlap", True))
        self.sync_enabled = True
        if bucket_mb is None:
            bucket_mb = float(self.cfg.get("dsgd_bucket_mb", 4.0))
        cap = int(bucket_mb * (1 << 20) / 4)
        self.buckets: List[Tuple[int, int]] = []
        self._param_bucket: Dict[int, int] = {}
        cur_end, cur_start = None, None
        segs = list(flat.segments())
        for p, o, n in reversed(segs):
            end = o + ((n + 3) // 4) * 4
            if cur_end is None:
                cur_end, cur_start = end, o
            elif cur_end - o > cap and cur_end - cur_start > 0:
                self.buckets.append((cur_start, cur_end))
                cur_end, cur_start = cur_start, o
            else:
                cur_start = o
            self._param_bucket[id(p)] = len(self.buckets)
        if cur_end is not None:
            self.buckets.append((cur_start, cur_end))
        self._pending = [0] * len(self.buckets)
        self._expected = [0] * len(self.buckets)
        for p, _, _ in segs:
            self._expected[self._param_bucket[id(p)]] += 1
        self._handles: Dict[int, object] = {}
        self._half_bufs: Dict[int, Tensor] = {}
        # ``dsgd_collective``: "peer" = the IPC-mapped HBM exchange (peer.py: push / fp32 sum /
        # push back, captured in the step graph); "direct" = all_to_all + fp32 sum + all_gather
        # (collective.py) on a comm stream of its own; "allreduce" = one RCCL all-reduce per
        # bucket (a 16-bit payload is then SUMMED in 16 bits inside RCCL); "auto" = peer for
        # 16-bit payloads on GPU sites (direct off the GPU), all-reduce for fp32; "calibrate" =
        # whichever captured form measures faster on this job's buckets and links
        coll = self.collective
        self.calibration: Optional[dict] = None
        if coll == "calibrate":
            coll = self._calibrate()
            self.peer = coll == "peer"
        self.direct = (not self.peer) and (coll == "direct" or (coll == "auto" and self.half))
        if self.half and not self.direct and not self.peer and self.wire == "fp16":
            # RCCL sums an all-reduce buffer in its own type: unscaled fp16 would flush
            # gradients below ~6e-8 and overflow past 65504 in the sum over sites, and a
            # per-site block scale cannot be summed.  The 16-bit all-reduce therefore ships
            # bf16 (fp32's range); the fp16 wire needs the direct exchange (fp32 sum).
            import warnings
            warnings.warn("dsgd_collective='allreduce' with an fp16 payload: sending bf16 "
                          "(RCCL would sum unscaled fp16); use dsgd_collective='direct' for an "
                          "fp16 wire", RuntimeWarning, stacklevel=2)
            self.wire = "bf16"
        self._comm_stream = (torch.cuda.Stream(device=flat.grad.device)
                             if self.direct and group.distributed and flat.grad.is_cuda else None)
        # the peer exchange takes the whole gradient as ONE exchange after the backward, and the
        # step keeps its backward in one piece (``prefers_split``, runtime.step): the split's
        # extra launches (a second grouped weight-gradient launch and split-K reduce, ~15 us) and a
        # second exchange's three launches cost more than pushing the body bucket early hides
        # (loopback fp16 step: profiles/r6_peer_unsplit_ab.jsonl).  The RCCL all-reduce keeps the
        # split: its buckets run on RCCL's own stream, truly under the encoder backward.
        self.prefers_split = not self.peer
        if self.peer and len(self.buckets) > 1 and bool(self.cfg.get("peer_one_bucket", True)):
            self._set_buckets([(self.buckets[-1][0], self.buckets[0][1])])
        self._peer_build()
        self._hooks = []
        self._delivered = set()
        if self.peer:
            # no pushes from autograd's gradient hooks: they run in the autograd thread, on a
            # stream that need not be the step's, and the peer exchange reuses its slots safely
            # only when every push is stream-ordered after the previous exchange's finish
            # (replicas diverged with hook-issued pushes in eager side-stream steps).  The
            # captured step pushes the body bucket between its backward parts itself
            # (launch_bucket); eager steps push every bucket in reduce().
            self.overlap = False
        if self.overlap:
            # autograd fires a parameter's post-accumulate hook even when its producer returned
            # no gradient for it -- which is what the fused ops do: they accumulate into .grad
            # themselves, possibly later (deferred grouped GEMM at the end of the backward), and
            # notify through ops._grad.  A tensor hook sees whether a real gradient arrived, and
            # only then does the post-accumulate hook count the parameter as ready.
            for p, _, _ in segs:
                self._hooks.append(p.register_hook(self._marker(id(p))))
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_accumulated))
            _gradreg.register(self._on_grad)  # fused ops write .grad directly and notify
        self._reset()

    @property
    def capturable(self) -> bool:
        # the peer exchange always; RCCL all-reduce buckets (fp32, or the 16-bit all-reduce)
        if not self.group.distributed or self.peer:
            return True
        return self.group.backend == "nccl" and not self.direct

    def _calibrate(self) -> str:
        """``dsgd_collective="calibrate"``: time the site-mean forms the step can run on THIS
        job's buckets and links and keep the faster -- the choice the link model of
        ``profiles/r4_comm_model.md`` could only predict (per-hop latency and link rates).

        Each candidate is timed in the form the step will run it: the bucket sequence captured
        in a HIP graph and replayed (``TrainStep.comm_graph`` captures the collectives into the
        step), except an all-reduce over a host backend (gloo), which the step issues from the
        host and which is timed so.  Candidates: the all-reduce and the peer exchange
        (``parallel.peer``, GPU sites).  Only forms with the SAME arithmetic compete: a 16-bit
        wire takes the fp32-sum exchange without a race (peer on GPU sites, else direct) --
        RCCL's all-reduce would sum 16-bit partials, so a timing could change the training
        numerics.  The per-form times are max-reduced over the sites, so every site takes the
        same decision from the same numbers; the record lands in ``self.calibration``
        (``logs.json`` ``dsgd_collective``).  ``dsgd_calibrate_reps`` (default 10) timed
        replays."""
        import time as _time
        g = self.group
        sizes = [e - s for s, e in self.buckets]
        if not g.distributed:
            self.calibration = {"choice": "allreduce", "reason": "one site: no collective"}
            return "allreduce"
        peer_ok = self._peer_ok()
        dev = self.flat.grad.device
        cuda = dev.type == "cuda"
        reps = max(1, int(self.cfg.get("dsgd_calibrate_reps", 10)))
        sync = torch.cuda.synchronize if cuda else (lambda: None)
        bufs = [torch.zeros(n, dtype=torch.float32, device=dev) for n in sizes]
        if self.half:
            note = None
            if peer_ok:
                prange = [(self.buckets[-1][0], self.buckets[0][1])]
                peer_ok, note = self._peer_verify(
                    [torch.zeros(prange[0][1] - prange[0][0], dtype=torch.float32, device=dev)],
                    prange)
            choice = "peer" if peer_ok else "direct"
            self.calibration = {"choice": choice, "wire": self.wire,
                                "reason": "16-bit wire: only the exchange sums in fp32"
                                          + (f"; peer {note}" if note else "")}
            return choice

        def allreduce():
            for b in bufs:
                g.all_reduce(b)

        # the peer exchange as the step would run it: ONE exchange of the whole gradient
        prange = [(self.buckets[-1][0], self.buckets[0][1])]
        pbufs = [torch.zeros(prange[0][1] - prange[0][0], dtype=torch.float32, device=dev)]

        def peer():
            for (s, e), b in zip(prange, pbufs):
                self._peer_mean(("bucket", s, e), e - s).run_(b)

        def host_timed(fn):
            for _ in range(2):
                fn()
            sync()
            g.barrier()
            t0 = _time.perf_counter()
            for _ in range(reps):
                fn()
            sync()
            return (_time.perf_counter() - t0) / reps * 1e6

        def graph_timed(fn):
            fn()  # eager once (RCCL communicator / peer regions set up outside the capture)
            from ..runtime.step import _quiesce_collectives
            _quiesce_collectives(g)  # every eager collective retired by the watchdog first
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, capture_error_mode="thread_local"):
                fn()
            gr.replay()
            sync()
            g.barrier()
            t0 = _time.perf_counter()
            for _ in range(reps):
                gr.replay()
            sync()
            t = (_time.perf_counter() - t0) / reps * 1e6
            g.barrier()
            del gr
            return t

        rccl_graph = cuda and g.backend == "nccl"
        peer_note = None
        if peer_ok:
            peer_ok, peer_note = self._peer_verify(pbufs, prange)
        times = [graph_timed(allreduce) if rccl_graph else host_timed(allreduce),
                 graph_timed(peer) if peer_ok else float("inf")]
        t = torch.tensor(times, dtype=torch.float64, device=dev if g.backend == "nccl" else "cpu")
        g.all_reduce(t, op=dist.ReduceOp.MAX)
        t_ar, t_peer = (float(v) for v in t.cpu())
        choice = "peer" if t_peer < t_ar else "allreduce"
        self.calibration = {"choice": choice, "allreduce_us": round(t_ar, 2),
                            "peer_us": round(t_peer, 2) if peer_ok else None,
                            "allreduce_form": "captured" if rccl_graph else "host-issued",
                            "peer_form": "captured" if peer_ok else (peer_note or "unavailable"),
                            "bucket_elems": sizes, "sites": g.world, "reps": reps,
                            "wire": self.wire}
        return choice

    def _peer_verify(self, bufs, ranges) -> Tuple[bool, Optional[str]]:
        """Before the peer exchange may compete in ``calibrate``: run it once on every bucket with
        known values (site r sends (r + 1) * v, v small integers: every sum exact) under a short
        wait limit and check the mean and the error words on EVERY site -- a machine whose IPC
        mapping or cross-GPU flags misbehave keeps the all-reduce instead of training on a broken
        exchange.  Returns (usable, reason when not)."""
        from . import peer as _peer
        g = self.group
        note = None
        ok = True
        _lib.call("dn_peer_set_timeout_ms", 2000)
        try:
            for (s, e), b in zip(ranges, bufs):
                v = (torch.arange(e - s, device=b.device, dtype=torch.float32) % 7) + 1.0
                b.copy_(v * float(g.rank + 1))
                self._peer_mean(("bucket", s, e), e - s).run_(b)
            torch.cuda.synchronize()
            want = (g.world + 1) / 2.0
            for (s, e), b in zip(ranges, bufs):
                v = (torch.arange(e - s, device=b.device, dtype=torch.float32) % 7) + 1.0
                if not torch.allclose(b, v * want, rtol=1e-6, atol=0):
                    ok, note = False, "failed verification (wrong mean)"
            errs = _peer.errors()
            if errs:
                ok, note = False, f"failed verification (wait timed out: {errs[0][2]})"
        except RuntimeError as ex:  # e.g. the IPC mapping refused
            ok, note = False, f"failed verification ({type(ex).__name__}: {ex})"[:200]
        finally:
            ms = os.environ.get("DINUNET_PEER_TIMEOUT_MS")
            _lib.call("dn_peer_set_timeout_ms", int(ms) if ms else -1)
        flag = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64,
                            device=self.flat.grad.device if g.backend == "nccl" else "cpu")
        g.all_reduce(flag, op=dist.ReduceOp.MIN)  # one site's failure disqualifies it everywhere
        if flag.item() < 0.5 and ok:
            ok, note = False, "failed verification on another site"
        for b in bufs:
            b.zero_()
        return ok, note

    def _marker(self, pid: int):
        def hook(g):
            if g is not None:
                self._delivered.add(pid)
        return hook

    def _on_accumulated(self, p):
        if id(p) in self._delivered:
            self._delivered.discard(id(p))
            self._on_grad(p)

    def _reset(self):
        self._pending = list(self._expected)
        self._handles.clear()
        self._ready = [False] * len(self.buckets)
        self._next = 0
        self._seen = set()

    def _drain(self):
        """Launch ready buckets strictly in bucket order.  Every rank then issues the same
        collective sequence whatever path produced its gradients: an eager step (autograd hooks,
        e.g. a ragged last batch), a graph replay (``launch_bucket`` / ``reduce``), or a split
        replay.  Out-of-order launches across ranks would pair different buckets in RCCL."""
        while self._next < len(self.buckets) and self._ready[self._next]:
            if self._next not in self._handles:
                self._launch(self._next)
            self._next += 1

    def split_buckets(self, stem_params) -> List[int]:
        """Re-bucket for a step whose backward is replayed in two parts (``TrainStep`` split
        capture): every gradient outside ``stem_params`` first (ready when the first part ends),
        then the stem's.  Returns the bucket ids of the first group; the caller launches them
        with :meth:`launch_bucket` between the two parts, ``reduce()`` launches the rest."""
        ids = {id(p) for p in stem_params}
        segs = list(self.flat.segments())
        stem = [(o, o + ((n + 3) // 4) * 4) for p, o, n in segs if id(p) in ids]
        if not stem:
            raise ValueError("stem parameters are not in the flat buffer")
        s0, s1 = min(a for a, _ in stem), max(b for _, b in stem)
        if sum(b - a for a, b in stem) != s1 - s0 or any(s0 <= o < s1 and id(p) not in ids
                                                        for p, o, _ in segs):
            raise ValueError("stem parameters must occupy one contiguous flat range")
        body = [r for r in ((s1, self.flat.numel), (0, s0)) if r[1] > r[0]]
        self._set_buckets(body + [(s0, s1)])
        self._peer_build()
        return list(range(len(body)))

    def _set_buckets(self, ranges):
        """New contiguous bucket ranges (covering every parameter); per-parameter bookkeeping
        rebuilt to match."""
        segs = list(self.flat.segments())
        self.buckets = list(ranges)
        self._param_bucket = {}
        for p, o, _ in segs:
            self._param_bucket[id(p)] = next(i for i, (a, b) in enumerate(self.buckets) if a <= o < b)
        self._expected = [0] * len(self.buckets)
        for p, _, _ in segs:
            self._expected[self._param_bucket[id(p)]] += 1
        self._half_bufs.clear()
        self._reset()

    def _peer_build(self):
        """The peer exchange of every bucket, built now (arena regions and the IPC handle
        exchange are host work, never inside a capture; every site builds in the same order)."""
        if self.peer:
            for s, e in self.buckets:
                self._peer_mean(("bucket", s, e), e - s)

    def launch_bucket(self, b: int):
        """Mark bucket ``b`` ready and start every ready bucket up to it, in order (RCCL stream
        ordered after the current stream)."""
        if self.group.distributed:
            self._ready[b] = True
            self._drain()

    def _launch(self, b: int):
        if not self._handles:  # first bucket of this step
            self.comm_bytes = 0
        s, e = self.buckets[b]
        view = self.flat.grad[s:e]
        if self.peer:
            # push now (no wait: the peers' data travel under the rest of the backward), reduce
            # + unpack when reduce() waits, in bucket order
            pm = self._peer_mean(("bucket", s, e), e - s)
            pm.start(view)
            self._handles[b] = _PeerWork(pm, view)
            self.comm_bytes += pm.bytes_sent
        elif self.direct:
            dm = self._direct((s, e), e - s, view.device)
            self._handles[b] = launch_on(self._comm_stream, lambda: dm.run_(view))
            self.comm_bytes += dm.n * dm.send.element_size()
        elif self.half:
            buf = self._half_bufs.get(b)
            if buf is None:
                dt = PAYLOAD_TYPES[self.wire][1]  # one unscaled block: headers sum to 0
                buf = self._half_bufs[b] = torch.zeros(payload_numel(e - s), dtype=dt,
                                                       device=view.device)
            to_payload(view, buf, 1, -(-(e - s) // SB) * SB)
            self._handles[b] = self.group.all_reduce(buf, async_op=True)
            self.comm_bytes += (e - s) * buf.element_size()
        else:
            self._handles[b] = self.group.all_reduce(view, async_op=True)
            self.comm_bytes += view.numel() * 4

    def _on_grad(self, p):
        if not self.sync_enabled:
            return
        b = self._param_bucket.get(id(p))
        if b is None or id(p) in self._seen:  # each parameter counts once per step
            return
        self._seen.add(id(p))
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._ready[b] = True
            self._drain()

    def reduce(self) -> float:
        g = self.group
        if not g.distributed:
            self._reset()
            return 1.0
        self._ready = [True] * len(self.buckets)
        self._drain()
        if self.peer:  # every pushed bucket's reduce + unpack, in bucket order, fused launches
            from . import peer as _peer
            _peer.finish_many([(h.pm, h.view, h.scale) for h in self._handles.values()])
            self._handles.clear()
        for b, h in self._handles.items():
            h.wait()
            if self.half and not self.direct and not self.peer:
                s, e = self.buckets[b]
                buf = self._half_bufs[b]
                from_payload(buf, self.flat.grad[s:e])
        self._reset()
        # the exchanges leave the mean, the all-reduce the sum
        self.last_scale = 1.0 if (self.direct or self.peer) else 1.0 / g.world
        return self.last_scale

    def close(self):
        for h in self._hooks:
            h.remove()
        self._hooks.clear()
        _gradreg.unregister(self._on_grad)

    # file transport
    def payload(self):
        g = self.flat.grad
        return {"grad": g.to(PAYLOAD_TYPES[self.wire][1]) if self.half else g.clone()}

    @classmethod
    def aggregate(cls, payloads, cfg=None):
        acc = None
        for p in payloads:
            v = p["grad"].float()
            acc = v.clone() if acc is None else acc.add_(v)
        return {"grad": acc / len(payloads)}

    def apply(self, agg):
        self.flat.grad.copy_(agg["grad"].to(self.flat.grad.device, torch.float32))
        return 1.0


# =============================================================================================
# rank-dAD
# =============================================================================================
class RankDADEngine(Engine):
    name = "rankDAD"

    def __init__(self, model, flat, group, cfg=None):
        super().__init__(model, flat, group, cfg)
        self.rank = int(self.cfg.get("dad_reduction_rank", 10))
        self.iters = int(self.cfg.get("dad_num_pow_iters", 5))
        self.tol = float(self.cfg.get("dad_tol", 1e-3))
        self.linears: List[nn.Linear] = [m for m in model.modules() if isinstance(m, nn.Linear)]
        self._weight_ids = {id(m.weight) for m in self.linears}
        self.dense_segs = [(o, n) for p, o, n in flat.segments() if id(p) not in self._weight_ids]
        self._cap: Optional[_cap.DADCapture] = None
        self._gen = None
        # GPU: factorise in GRADIENT space.  The fused kernels already produce each site's
        # G_s = Delta_s^T A_s in the flat grad buffer, and the structured iteration
        # P <- orth(Delta^T (A Q)), Q <- A^T (Delta P) is exactly the power iteration on G_s:
        # running it on G_s ([out, in], a few hundred KB) instead of the [B*S, .] activation /
        # delta factors gives the same factors without capturing them, with no host sync (the
        # dad_tol early stop is a device-side mask), so it is captured in the step's HIP graph.
        self.fast = bool(flat.data.is_cuda and self.cfg.get("dad_gradient_space", True))
        # the one-launch power iteration spins on per-layer barriers, so all of a launch's
        # workgroups must be resident together: never when several site processes share one GPU
        # (the gloo rehearsal), whose persistent launches could then hold each other's CUs
        shared = getattr(group, "gpu_shared", None)
        if shared is None:  # a group built by hand: assume sharing when ranks outnumber GPUs
            shared = group.distributed and group.world > max(1, torch.cuda.device_count())
        self._persist_ok = bool(self.fast and not shared)
        if self.fast:
            self._init_fast()

    # ---- gradient-space path ---------------------------------------------------------------
    @property
    def pre_capturable(self) -> bool:
        return self.group.replicas <= 1

    @property
    def capturable(self) -> bool:
        # the site mean of several GPUs per site runs in reduce(), outside the graph
        return self.group.replicas <= 1 and Engine.capturable.fget(self)

    def _init_fast(self):
        """Device tables of the factorisation kernels (csrc/kernels/lowrank.hip): per large
        Linear, its gradient view, the warm-start / candidate Q, and the P and Q slots of the
        send buffer that the factor all-gather ships."""
        import ctypes
        segs = {id(p): o for p, o, _ in self.flat.segments()}
        dev = self.flat.data.device
        gen = torch.Generator(device="cpu").manual_seed(int(self.cfg.get("seed", 0)) + 777)
        r = max(1, min(self.rank, 16))
        self.fast_layers = []  # (module, flat offset, out, in, r, send offset of P, of Q)
        off = 0
        for m in self.linears:
            out_f, in_f = m.weight.shape
            if self.rank >= min(out_f, in_f):
                continue  # exact mode: the dense mean of G (== sum_s Delta_s^T A_s / W)
            self.fast_layers.append((m, segs[id(m.weight)], out_f, in_f, r, off, off + out_f * r))
            off += (out_f + in_f) * r
        low = {id(l[0].weight) for l in self.fast_layers}
        self.fast_dense = [(o, n) for p, o, n in self.flat.segments() if id(p) not in low]
        # the dense (dSGD-mean) part: adjacent segments merged; one index gather / scatter when
        # they are not one range (no per-segment copies)
        merged: List[List[int]] = []
        for o, n in sorted(self.fast_dense):
            if merged and merged[-1][1] == o:
                merged[-1][1] = o + n
            else:
                merged.append([o, o + n])
        self._dense_ranges = [(a, b) for a, b in merged]
        self._dense_idx = (torch.cat([torch.arange(a, b) for a, b in self._dense_ranges]).to(dev)
                           if len(self._dense_ranges) > 1 else None)
        self._dense_buf = (torch.empty(self._dense_idx.numel(), dtype=torch.float32, device=dev)
                           if self._dense_idx is not None else None)
        # the send slot is also the per-rank stride of the gather: 16-byte multiple, whole payload
        # sub-blocks when the factors travel in 16 bits
        pad = SB if (self.half and self.group.distributed) else 8
        self._send = torch.zeros(-(-max(off, 1) // pad) * pad, dtype=torch.float32, device=dev)
        n = len(self.fast_layers)
        if not n:
            return
        W = self.group.world
        self._gathered = (torch.zeros(W * self._send.numel(), dtype=torch.float32, device=dev)
                          if self.group.distributed else self._send)
        if self.half and self.group.distributed:
            dt = PAYLOAD_TYPES[self.wire][1]
            self._send16 = torch.zeros(payload_numel(self._send.numel()), dtype=dt, device=dev)
            self._gathered16 = torch.zeros(W * self._send16.numel(), dtype=dt, device=dev)
        layers = []
        self._praw = []
        for _, o, out_f, in_f, rr, po, qo in self.fast_layers:
            q = torch.randn(in_f, rr, generator=gen)  # identical on every site (same seed)
            _mgs_torch_(q)
            qsend = self._send[qo:qo + in_f * rr].view(in_f, rr)
            qsend.copy_(q.to(dev))  # the send slot doubles as the next step's warm start
            praw = torch.empty(out_f, rr, dtype=torch.float32, device=dev)
            self._praw.append(praw)
            G = self.flat.grad[o:o + out_f * in_f].view(out_f, in_f)
            layers.append((G, None, praw, self._send[po:po + out_f * rr].view(out_f, rr), qsend))
        self._table = LowRankTable(layers, dev)
        if self.peer:  # the exchanges, built outside any capture (peer.PeerArena)
            from . import peer as _peer
            if self._dense_ranges:
                self._peer_mean(("dense",), sum(b - a for a, b in self._dense_ranges))
            _peer.gather(self.group, dev, self._send.numel(), self.wire, ("rankDAD", "factors"))

        class PiRecon(ctypes.Structure):
            _fields_ = [("G", ctypes.c_void_p), ("P", ctypes.c_void_p), ("Q", ctypes.c_void_p),
                        ("out", ctypes.c_int), ("inn", ctypes.c_int), ("r", ctypes.c_int),
                        ("start", ctypes.c_long)]
        L = _lib.lib()
        L.dn_pi_recon_size.restype = ctypes.c_long
        if ctypes.sizeof(PiRecon) != L.dn_pi_recon_size():
            raise RuntimeError("reconstruction table layout mismatch with the kernel library")
        rec = (PiRecon * n)()
        start = 0
        G0, gat0 = self.flat.grad.data_ptr(), self._gathered.data_ptr()
        for i, (_, o, out_f, in_f, rr, po, qo) in enumerate(self.fast_layers):
            c = rec[i]
            c.G, c.P, c.Q = G0 + 4 * o, gat0 + 4 * po, gat0 + 4 * qo
            c.out, c.inn, c.r, c.start = out_f, in_f, rr, start
            start += out_f * in_f
        self._recon_total = start
        self._rec_host = rec  # (the launcher reads the tile prefix from the host copy)
        self._rec = torch.frombuffer(bytearray(bytes(rec)), dtype=torch.uint8).to(dev)

    def state_dict(self):
        if self.fast and getattr(self, "fast_layers", None):
            return {"send": self._send.detach().cpu().clone()}  # holds every warm-start Q
        return {}

    def load_state_dict(self, sd):
        if "send" in sd and getattr(self, "fast_layers", None):
            self._send.copy_(sd["send"].to(self._send.device))

    def pre_reduce(self):
        """Local rank-r factors of every large Linear's gradient into the send buffer: two
        launches per power iteration for all layers (``G Q``; fp64-Gram Cholesky QR + ``G^T P``), the
        ``dad_tol`` stop decided on the device: no host sync, HIP-graph capturable."""
        if not self.fast or not self.fast_layers:
            return
        # several GPUs per site: the site's gradient (mean over its replicas) is what the site
        # factorises; its replicas then compute identical factors
        self.group.site_mean_(self.flat.grad)
        self._dense_start()  # (peer) the dense part travels under the power iteration
        if self._persist_ok and self._table.persist(max(1, self.iters), self.tol):
            return  # every iteration in one launch (lr_persist_kernel)
        for it in range(max(1, self.iters)):
            self._table.gq(it, self.tol)
            self._table.orth_gtp(it)

    def _dense_view(self) -> Tensor:
        """The dense (dSGD-mean) part of the gradient as one contiguous fp32 range: the flat
        range itself, or gathered into ``_dense_buf`` (scatter back with ``_dense_back``)."""
        grad = self.flat.grad
        if self._dense_idx is None:
            a, b = self._dense_ranges[0]
            return grad[a:b]
        torch.index_select(grad, 0, self._dense_idx, out=self._dense_buf)
        return self._dense_buf

    def _dense_back(self, buf: Tensor):
        if self._dense_idx is not None:
            self.flat.grad.index_copy_(0, self._dense_idx, buf)

    def _dense_start(self):
        """Peer exchange: push the dense part right after the backward (no wait), so it crosses
        the links while the power iteration runs; ``_fast_reduce`` finishes it."""
        self._dense_pending = None
        if not (self.peer and self.group.distributed and self._dense_ranges):
            return
        buf = self._dense_view()
        pm = self._peer_mean(("dense",), buf.numel())
        pm.start(buf)
        self._dense_pending = (pm, buf)

    def power_iterations(self) -> Optional[List[int]]:
        """Cumulative power iterations each factorised layer ran on the device (``dad_tol``
        stops a layer early; ``dad_num_pow_iters`` bounds it), or None off the device path."""
        if not (self.fast and getattr(self, "fast_layers", None)):
            return None
        return self._table.iterations()

    def _fast_reduce(self) -> float:
        g = self.group
        W = g.world
        self.comm_bytes = 0
        # (not consumed: a pre_reduce captured in a graph pushes at every replay, and every
        # reduction after it finishes that push)
        pend = getattr(self, "_dense_pending", None)
        if pend is not None:  # pushed before the power iteration (peer)
            pm, buf = pend
            pm.finish(buf)
            self._dense_back(buf)
            self.comm_bytes += pm.bytes_sent
        elif g.distributed and self._dense_ranges:
            buf = self._dense_view()
            self._allreduce_mean_(buf, tag=("dense",))
            self._dense_back(buf)
        if not self.fast_layers:
            return 1.0
        if g.distributed:
            if self.peer:  # one-sided writes into every site's gather slot (fp32 out)
                from . import peer as _peer
                pg = _peer.gather(g, self.flat.grad.device, self._send.numel(), self.wire,
                                  ("rankDAD", "factors"))
                self.comm_bytes += pg.run(self._send, self._gathered, self._send.numel())
            elif self.half:  # factors on the wire in the payload type, reconstructed in fp32
                n = self._send.numel()
                to_payload(self._send, self._send16, 1, n)
                g.all_gather_into(self._gathered16, self._send16)
                from_payload(self._gathered16, self._gathered)
                self.comm_bytes += self._send16.numel() * self._send16.element_size()
            else:
                g.all_gather_into(self._gathered, self._send)
                self.comm_bytes += self._send.numel() * 4
        # every layer's G = [P_1..P_W][Q_1..Q_W]^T / W in one launch
        _lib.call("dn_pi_reconstruct", self._rec.data_ptr(), ctypes.addressof(self._rec_host),
                  len(self.fast_layers),
                  self._recon_total, self._send.numel(), W if g.distributed else 1, _lib.stream())
        return 1.0

    def step_context(self):
        if self.fast:
            return contextlib.nullcontext()
        self._cap = _cap.DADCapture(modules=self.linears)
        return self._cap

    def _dense_pack(self) -> Tensor:
        g = self.flat.grad
        return torch.cat([g[o:o + n] for o, n in self.dense_segs]) if self.dense_segs else g[:0].clone()

    def _dense_unpack(self, buf: Tensor):
        g = self.flat.grad
        off = 0
        for o, n in self.dense_segs:
            g[o:o + n].copy_(buf[off:off + n])
            off += n

    def _layer_inputs(self):
        """Per captured Linear: concatenated ``(A [N, in], Delta [N, out])``."""
        recs = self._cap.records if self._cap is not None else {}
        out = []
        for m in self.linears:
            r = recs.get(m)
            if not r:
                continue
            A = torch.cat([a.reshape(-1, a.shape[-1]) for a, _ in r]).float()
            D = torch.cat([d.reshape(-1, d.shape[-1]) for _, d in r]).float()
            out.append((m, A, D))
        return out

    def _exact(self, A: Tensor, D: Tensor) -> bool:
        # decided from the layer shape only, so every site picks the same mode (the collective
        # layouts must agree); at r >= rank(G) the power iteration is exact anyway
        return self.rank >= min(A.shape[1], D.shape[1])

    def local_factors(self):
        """[(module, mode, X, Y)] with mode 'exact' (X=Delta, Y=A) or 'lowrank' (X=P, Y=Q)."""
        res = []
        k = self.group.replicas
        for m, A, D in self._layer_inputs():
            if self._exact(A, D):
                res.append((m, "exact", D, A))
            else:
                if k > 1:  # the site's gradient: its replicas' rows, G = sum_r D_r^T A_r / k
                    D = self.group.site_all_gather_varlen(D) / k
                    A = self.group.site_all_gather_varlen(A)
                P, Q = dad_factors(D, A, self.rank, self.iters, self.tol)
                res.append((m, "lowrank", P, Q))
        return res

    def reduce(self, factorized: bool = False) -> float:
        """``factorized``: :meth:`pre_reduce` already ran (inside the captured step)."""
        if self.fast:
            if not factorized:
                self.pre_reduce()
            return self._fast_reduce()
        g = self.group
        self.comm_bytes = 0
        dense = self._dense_pack()
        self._allreduce_mean_(dense)
        self._dense_unpack(dense)
        facs = self.local_factors()
        W = g.world
        low = [(m, X, Y) for m, mode, X, Y in facs if mode == "lowrank"]
        if low:
            flat = torch.cat([torch.cat([X.reshape(-1), Y.reshape(-1)]) for _, X, Y in low])
            if self.half:
                flat = flat.to(PAYLOAD_TYPES[self.wire][1])
            gathered = torch.empty(W * flat.numel(), dtype=flat.dtype, device=flat.device)
            g.all_gather_into(gathered, flat)
            self.comm_bytes += flat.numel() * flat.element_size()
            gathered = gathered.view(W, -1).float()
            off = 0
            for m, X, Y in low:
                nx, ny = X.numel(), Y.numel()
                Ps = gathered[:, off:off + nx].reshape(W, *X.shape)
                Qs = gathered[:, off + nx:off + nx + ny].reshape(W, *Y.shape)
                off += nx + ny
                # mean_s P_s Q_s^T  ==  [P_1..P_W] [Q_1..Q_W]^T / W  (one GEMM)
                Pc = Ps.permute(1, 0, 2).reshape(X.shape[0], -1)
                Qc = Qs.permute(1, 0, 2).reshape(Y.shape[0], -1)
                m.weight.grad.copy_((Pc @ Qc.t()).div_(W).view_as(m.weight))
        for m, mode, D, A in facs:
            if mode != "exact":
                continue
            Dc = g.all_gather_varlen(D)
            Ac = g.all_gather_varlen(A)
            self.comm_bytes += (D.numel() + A.numel()) * 4
            m.weight.grad.copy_((Dc.t() @ Ac).div_(W).view_as(m.weight))
        if self._cap is not None:
            self._cap.clear()
        return 1.0

    # file transport
    def payload(self):
        out = {"dense": self._dense_pack()}
        facs = self.local_factors()
        self._captured_order = [m for m, _, _, _ in facs]
        for i, (m, mode, X, Y) in enumerate(facs):
            out[f"L{i:03d}.{mode}.X"] = X
            out[f"L{i:03d}.{mode}.Y"] = Y
        if self._cap is not None:
            self._cap.clear()
        return out

    @classmethod
    def aggregate(cls, payloads, cfg=None):
        W = len(payloads)
        agg = {"dense": sum(p["dense"].float() for p in payloads) / W}
        keys = sorted({k.rsplit(".", 1)[0] for p in payloads for k in p if k != "dense"})
        for k in keys:
            X = torch.cat([p[k + ".X"].float() for p in payloads], 1 if ".lowrank" in k else 0)
            Y = torch.cat([p[k + ".Y"].float() for p in payloads], 1 if ".lowrank" in k else 0)
            agg[k] = (X @ Y.t() / W) if ".lowrank" in k else (X.t() @ Y / W)
        return agg

    def apply(self, agg):
        self._dense_unpack(agg["dense"].to(self.flat.grad.device))
        by_layer = {int(k.split(".")[0][1:]): k for k in agg if k != "dense"}
        for i, k in sorted(by_layer.items()):
            m = self._captured_order[i]
            m.weight.grad.copy_(agg[k].to(m.weight.grad.device).view_as(m.weight))
        return 1.0


# =============================================================================================
# PowerSGD
# =============================================================================================
class PowerSGDEngine(Engine):
    name = "powerSGD"

    def __init__(self, model, flat, group, cfg=None):
        super().__init__(model, flat, group, cfg)
        self.rank = int(self.cfg.get("powersgd_rank", 4))
        self.warm = bool(self.cfg.get("powersgd_warm_start", True))
        self.mats = []   # (param, n, m, r)
        dense = []
        for p, o, n in flat.segments():
            if p.dim() >= 2:
                rows, cols = p.shape[0], p.numel() // p.shape[0]
                r = min(self.rank, rows, cols)
                if (rows + cols) * r < rows * cols:
                    self.mats.append((p, rows, cols, r))
                    continue
            dense.append((o, n))
        self.dense_segs = dense
        gen = torch.Generator(device="cpu").manual_seed(int(self.cfg.get("seed", 0)) + 12345)
        dev = flat.data.device
        # GPU: every matrix of the model per launch (csrc/kernels/lowrank.hip): P = M Q with
        # M = G + err formed in the same pass, Cholesky QR (fp64 Gram) + Q = M^T P, then G = P Q^T and the
        # error feedback -- three launches and two all-reduces per step, no host sync
        self.fast = bool(flat.data.is_cuda and self.warm and _lib.native_available()
                         and self.cfg.get("powersgd_device", True) and self.mats)
        qs = [torch.randn(c, r, generator=gen) for _, _, c, r in self.mats]
        if not self.fast:
            self.Q = [q.to(dev) for q in qs]
            self.err = [torch.zeros(rw, c, device=dev) for _, rw, c, _ in self.mats]
            return
        seg = {id(p): o for p, o, _ in flat.segments()}
        rows_r = sum(rw * r for _, rw, _, r in self.mats)
        self._qbuf = torch.cat([q.reshape(-1) for q in qs]).to(dev)  # Q: warm start + Q all-reduce
        self._pbuf = torch.zeros(rows_r, dtype=torch.float32, device=dev)   # raw P: all-reduce
        self._psend = torch.zeros(rows_r, dtype=torch.float32, device=dev)  # orthonormal P
        self._ebuf = torch.zeros(sum(rw * c for _, rw, c, _ in self.mats), dtype=torch.float32,
                                 device=dev)
        self.Q, self.err, layers = [], [], []
        po = qo = eo = 0
        for p, rw, c, r in self.mats:
            Q = self._qbuf[qo:qo + c * r].view(c, r)
            E = self._ebuf[eo:eo + rw * c].view(rw, c)
            P = self._pbuf[po:po + rw * r].view(rw, r)
            Ps = self._psend[po:po + rw * r].view(rw, r)
            G = flat.grad[seg[id(p)]:seg[id(p)] + rw * c].view(rw, c)
            self.Q.append(Q)
            self.err.append(E)
            layers.append((G, E, P, Ps, Q))
            po, qo, eo = po + rw * r, qo + c * r, eo + rw * c
        self._table = LowRankTable(layers, dev)
        if self.peer:  # the exchanges, built outside any capture (peer.PeerArena)
            nd = sum(n for _, n in self.dense_segs)
            if nd:
                self._peer_mean(("dense",), nd)
            self._peer_mean(("P",), self._pbuf.numel())
            self._peer_mean(("Q",), self._qbuf.numel())

    def pre_reduce(self):
        """M = G + err and the local P = M Q of every matrix (one launch, graph-capturable)."""
        if self.fast:
            self._table.gq(0)

    def state_dict(self):
        return {"Q": [q.detach().cpu().clone() for q in self.Q],
                "err": [e.detach().cpu().clone() for e in self.err]}

    def load_state_dict(self, sd):
        for dst, key in ((self.Q, "Q"), (self.err, "err")):
            for t, v in zip(dst, sd.get(key, [])):
                t.copy_(v.to(t.device))

    def _dense_pack(self):
        g = self.flat.grad
        return torch.cat([g[o:o + n] for o, n in self.dense_segs]) if self.dense_segs else g[:0].clone()

    def _dense_unpack(self, buf):
        g = self.flat.grad
        off = 0
        for o, n in self.dense_segs:
            g[o:o + n].copy_(buf[off:off + n])
            off += n

    def reduce(self, factorized: bool = False) -> float:
        """``factorized``: :meth:`pre_reduce` already ran (inside the captured step)."""
        g = self.group
        W = g.world
        self.comm_bytes = 0
        dense_pm = None
        if g.distributed:
            dense = self._dense_pack()
            if self.peer and self.fast and self.mats and dense.numel():
                # the peer exchange: push the dense part now, finish it after the P / Q rounds
                dense_pm = self._peer_mean(("dense",), dense.numel())
                dense_pm.start(dense)
            else:
                self._allreduce_mean_(dense, tag=("dense",))
                self._dense_unpack(dense)
        if not self.mats:
            return 1.0
        if self.fast:
            if not factorized:
                self.pre_reduce()
            self._allreduce_mean_(self._pbuf, tag=("P",))  # round 1: P (mean over sites)
            self._table.orth_gtp(0)                         # orthonormalise P, Q = M^T P
            self._allreduce_mean_(self._qbuf, tag=("Q",))  # round 2: Q (mean); next warm start
            self._table.recon_ef()                          # G = P Q^T, err = M - G
            if dense_pm is not None:
                dense_pm.finish(dense)
                self._dense_unpack(dense)
                self.comm_bytes += dense_pm.bytes_sent
            return 1.0
        Ms = []
        for (p, rows, cols, r), e in zip(self.mats, self.err):
            M = p.grad.reshape(rows, cols) + e
            Ms.append(M)
        if not self.warm:
            for q in self.Q:
                q.normal_()
        Ps = [M @ q for M, q in zip(Ms, self.Q)]
        pbuf = torch.cat([P.reshape(-1) for P in Ps])
        if g.distributed:
            g.all_reduce(pbuf)
            pbuf.div_(W)
            self.comm_bytes += pbuf.numel() * 4
        off = 0
        for i, P in enumerate(Ps):
            Ps[i] = pbuf[off:off + P.numel()].view_as(P)
            off += P.numel()
        orthonormalize_(Ps)
        Qs = [M.t() @ P for M, P in zip(Ms, Ps)]
        qbuf = torch.cat([Q.reshape(-1) for Q in Qs])
        if g.distributed:
            g.all_reduce(qbuf)
            qbuf.div_(W)
            self.comm_bytes += qbuf.numel() * 4
        off = 0
        for i, (Q, M, P) in enumerate(zip(Qs, Ms, Ps)):
            Qn = qbuf[off:off + Q.numel()].view_as(Q)
            off += Q.numel()
            self.Q[i].copy_(Qn)
            Mh = P @ Qn.t()
            self.err[i].copy_(M - Mh)
            p = self.mats[i][0]
            p.grad.copy_(Mh.view_as(p))
        return 1.0

    # file transport: two rounds (P then Q) are modelled as one call sequence by the compat layer
    def payload_p(self):
        self._Ms = [p.grad.reshape(rw, c) + e for (p, rw, c, _), e in zip(self.mats, self.err)]
        return {"dense": self._dense_pack(), **{f"P{i}": M @ q for i, (M, q) in enumerate(zip(self._Ms, self.Q))}}

    def payload_q(self, agg_p):
        Ps = [agg_p[f"P{i}"].to(self.flat.data.device).clone() for i in range(len(self.mats))]
        orthonormalize_(Ps)
        self._Ps = Ps
        return {f"Q{i}": M.t() @ P for i, (M, P) in enumerate(zip(self._Ms, Ps))}

    def apply_pq(self, agg_p, agg_q):
        self._dense_unpack(agg_p["dense"].to(self.flat.grad.device))
        for i, ((p, rw, c, _), P) in enumerate(zip(self.mats, self._Ps)):
            Qn = agg_q[f"Q{i}"].to(P.device)
            self.Q[i].copy_(Qn)
            Mh = P @ Qn.t()
            self.err[i].copy_(self._Ms[i] - Mh)
            p.grad.copy_(Mh.view_as(p))
        return 1.0

    @classmethod
    def aggregate(cls, payloads, cfg=None):
        W = len(payloads)
        return {k: sum(p[k].float() for p in payloads) / W for k in payloads[0]}


ENGINES = {"dSGD": DSGDEngine, "rankDAD": RankDADEngine, "powerSGD": PowerSGDEngine}


def make_engine(name: str, model: nn.Module, flat: FlatParams, group: SiteGroup, cfg: dict) -> Engine:
    try:
        cls = ENGINES[name]
    except KeyError:
        raise ValueError(f"unknown agg_engine {name!r}; expected one of {sorted(ENGINES)}")
    return cls(model, flat, group, cfg)
