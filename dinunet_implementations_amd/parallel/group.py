"""Site group: one process per GPU, each GPU plays one COINSTAC site (rank == site index), or --
a site input listing several GPUs (``gpus: [0, 1]``) -- ``replicas`` consecutive ranks share one
site (rank = site * replicas + replica).

The reference routes every update through a remote aggregator over files + JSON (star topology,
SURVEY.md §2.4).  Here all sites form one ``torch.distributed`` process group — backend ``nccl``
(= RCCL on ROCm, point-to-point xGMI between the 8 MI355X of a node) on GPUs, ``gloo`` on CPU for
tests — and every "remote" reduction is a collective whose result every rank holds.  Decisions
the remote used to make (best epoch, early stop) are computed redundantly and identically on all
ranks from collectively-reduced inputs.

Intra-site data parallelism (the reference GUI's "GPU IDs to use, e.g. [0, 1]",
``datasets/icalstm/inputspec.json:6-10``): the replicas of a site hold disjoint shards of the
site's splits (``runtime.site.FederatedSite``) and each trains on ``batch_size / replicas`` rows of
every batch.  Every site has the same replica count, so the engines' mean over ALL ranks is the
mean over sites of each site's full-batch gradient (dSGD exactly: equal shard sizes); rank-dAD
first forms the site gradient on ``site_pg`` (``SiteGroup.site_mean_``) so that each site factorises
its own gradient, and its replicas contribute identical factors.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Any, List, Optional

import torch
import torch.distributed as dist


@dataclass
class SiteGroup:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: Optional[str] = None
    pg: Any = None
    # does another site process use this rank's GPU? (init_sites: all-gathered (host, device);
    # None = unknown).  Launches whose workgroups wait on each other are only safe when not.
    gpu_shared: Optional[bool] = None
    # a one-rank RCCL group that still takes every collective code path (``init_sites(loopback=
    # True)``, ``bench.py --loopback-rccl``): times the N > 1 step on one GPU
    loopback: bool = False
    # processes (GPUs) per site and this process's index among its site's; site_pg = the
    # process group of this site's replicas (None at one replica)
    replicas: int = 1
    replica: int = 0
    site_pg: Any = None

    @property
    def distributed(self) -> bool:
        return self.world > 1 or self.loopback

    @property
    def is_master(self) -> bool:
        return self.rank == 0

    @property
    def site(self) -> int:
        """This process's site index (the data directory ``local<site>``)."""
        return self.rank // max(1, self.replicas)

    @property
    def sites(self) -> int:
        return self.world // max(1, self.replicas)

    def site_mean_(self, t: torch.Tensor) -> torch.Tensor:
        """In place: the mean of ``t`` over this site's replicas (identity at one replica)."""
        if self.replicas > 1 and self.site_pg is not None:
            dist.all_reduce(t, group=self.site_pg)
            t.div_(self.replicas)
        return t

    def site_all_gather_varlen(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate variable-length tensors over this site's replicas (replica order)."""
        if self.replicas <= 1 or self.site_pg is None:
            return t
        n = torch.tensor([t.shape[0]], device=t.device, dtype=torch.long)
        ns = [torch.empty_like(n) for _ in range(self.replicas)]
        dist.all_gather(ns, n, group=self.site_pg)
        sizes = [int(v.item()) for v in ns]
        mx = max(sizes)
        pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if t.shape[0]:
            pad[:t.shape[0]] = t
        parts = [torch.empty_like(pad) for _ in range(self.replicas)]
        dist.all_gather(parts, pad, group=self.site_pg)
        return torch.cat([p[:s] for p, s in zip(parts, sizes)], 0)

    # ---- thin collective helpers (no-ops at world 1) ----------------------------------------
    def barrier(self):
        if self.distributed:
            if self.backend == "nccl":
                dist.barrier(group=self.pg, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.pg)

    def all_reduce(self, t: torch.Tensor, op=dist.ReduceOp.SUM, async_op: bool = False):
        if not self.distributed:
            return None
        return dist.all_reduce(t, op=op, group=self.pg, async_op=async_op)

    def broadcast(self, t: torch.Tensor, src: int = 0, async_op: bool = False):
        if not self.distributed:
            return None
        return dist.broadcast(t, src=src, group=self.pg, async_op=async_op)

    def all_gather(self, t: torch.Tensor) -> List[torch.Tensor]:
        if not self.distributed:
            return [t]
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t.contiguous(), group=self.pg)
        return out

    def all_gather_into(self, out: torch.Tensor, t: torch.Tensor, async_op: bool = False):
        """Gather equal-size tensors into one flat ``[world * numel]`` buffer (one collective)."""
        if not self.distributed:
            out.copy_(t.reshape(-1))
            return None
        if self.backend == "gloo" and t.is_cuda:
            # gloo has no device all_gather_into_tensor: stage through the host (multi-site
            # rehearsal on one GPU only; production GPU runs use RCCL)
            parts = self.all_gather(t.detach().reshape(-1).cpu())
            out.copy_(torch.cat(parts).to(out.device))
            return None
        return dist.all_gather_into_tensor(out, t.contiguous().reshape(-1), group=self.pg,
                                           async_op=async_op)

    def all_gather_object(self, obj) -> List[Any]:
        if not self.distributed:
            return [obj]
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self.pg)
        return out

    def broadcast_object(self, obj, src: int = 0):
        if not self.distributed:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src, group=self.pg)
        return box[0]

    def all_gather_varlen(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate variable-length 1-D/2-D tensors from all ranks (rank order)."""
        if not self.distributed:
            return t
        n = torch.tensor([t.shape[0]], device=t.device, dtype=torch.long)
        sizes = [int(s.item()) for s in self.all_gather(n)]
        mx = max(sizes) if sizes else 0
        pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if t.shape[0]:
            pad[:t.shape[0]] = t
        parts = self.all_gather(pad)
        return torch.cat([p[:s] for p, s in zip(parts, sizes)], 0)


_GROUP: Optional[SiteGroup] = None


def resolve_device(gpus=None, local_rank: int = 0, world: int = 1, backend: Optional[str] = None,
                   n_devices: Optional[int] = None, replica: int = 0,
                   replicas: int = 1) -> torch.device:
    """The device of a site from its ``gpus`` input (the reference's "GPU IDs to use",
    ``datasets/icalstm/inputspec.json:6-10``: site 0 -> ``[0]``, site 1 -> ``[1]``;
    ``datasets/test_fsl/inputspec.json:15-17``: ``[]`` = CPU-only FreeSurfer sites).

    * ``None`` (not given): this rank's GPU (``LOCAL_RANK``) when one exists, else the CPU;
    * ``[]``: the CPU, as the reference;
    * ``[k, ...]``: GPU ``k`` -- with ``replicas`` processes per site, replica ``i`` takes
      ``ids[i]`` (a site's data-parallel replicas, one process per GPU); ids beyond the replicas
      are not used (warned).  With RCCL every process needs its own GPU, so the id must equal
      ``LOCAL_RANK``; a site listing another GPU is a configuration conflict and raises."""
    if n_devices is None:
        n_devices = torch.cuda.device_count() if torch.cuda.is_available() else 0
    if gpus is None:
        return torch.device("cuda", local_rank % n_devices) if n_devices else torch.device("cpu")
    if isinstance(gpus, int):
        gpus = [gpus]
    ids = [int(g) for g in gpus]
    if not ids:
        return torch.device("cpu")
    replicas = max(1, int(replicas))
    if replicas > 1 and len(ids) < replicas:
        # (run.py --site-gpus k over site inputs that list one GPU each): every process of the
        # site takes its own GPU, as without a list
        import warnings
        warnings.warn(f"gpus={ids} lists fewer GPUs than the site's {replicas} processes: each "
                      f"process uses its own GPU (LOCAL_RANK)", RuntimeWarning)
        return torch.device("cuda", local_rank % n_devices) if n_devices else torch.device("cpu")
    k = ids[replica] if replica < len(ids) else ids[0]
    if len(ids) > replicas:
        # the reference's GUI offers "GPU IDs to use Eg. [0], [0, 1]" (assets/coinstac-gui.png):
        # a site uses one GPU per replica process (run.py --site-gpus / a uniform gpus length),
        # so ids beyond the replicas are not used -- say so instead of dropping them silently
        import warnings
        warnings.warn(f"gpus={ids}: a site runs on {replicas} GPU(s) ({ids[:replicas]}, one "
                      f"process each); the other ids {ids[replicas:]} are not used "
                      f"(launch {len(ids)} processes per site to use them)", RuntimeWarning)
    if not n_devices:
        import warnings
        warnings.warn(f"gpus={ids} but no GPU is visible: the site runs on the CPU", RuntimeWarning)
        return torch.device("cpu")
    if not 0 <= k < n_devices:
        if backend == "nccl":
            raise ValueError(f"gpus={ids}: GPU {k} does not exist ({n_devices} visible)")
        # several sites rehearsed on fewer GPUs (gloo, the in-process simulator): wrap around
        import warnings
        warnings.warn(f"gpus={ids}: GPU {k} does not exist ({n_devices} visible); using GPU "
                      f"{k % n_devices}", RuntimeWarning)
        k %= n_devices
    if world > 1 and backend == "nccl" and k != local_rank:
        raise ValueError(f"gpus={ids} conflicts with LOCAL_RANK={local_rank}: with RCCL each "
                         f"site's process owns GPU LOCAL_RANK (site r -> gpus [r])")
    return torch.device("cuda", k)


def init_sites(backend: Optional[str] = None, device: Optional[str] = None,
               timeout_s: Optional[int] = None, gpus=None, loopback: bool = False,
               replicas: int = 1) -> SiteGroup:
    """Initialise from torchrun-style env vars; world 1 when they are absent.

    ``replicas``: processes per site (intra-site data parallelism, see the module docstring):
    ranks ``s * replicas .. s * replicas + replicas - 1`` are site ``s``; WORLD_SIZE must be a
    multiple.  Each site's replicas get their own process group (``site_pg``).

    ``loopback`` (world 1 only): build a one-rank process group anyway (RCCL on a GPU) and mark
    the group distributed, so every collective of the multi-site step runs -- and is captured --
    exactly as at N > 1 (``bench.py --loopback-rccl``).

    ``timeout_s`` (default ``DINUNET_PG_TIMEOUT``, else 1800 s) bounds every collective: a site
    that dies or hangs makes the survivors' next collective fail (gloo: at once when the peer's
    socket closes; RCCL: the process-group watchdog after the timeout) instead of waiting
    forever; ``run.py`` then reports the failure and exits non-zero."""
    global _GROUP
    if timeout_s is None:
        timeout_s = int(os.environ.get("DINUNET_PG_TIMEOUT", "1800"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    replicas = max(1, int(replicas))
    if world % replicas:
        raise ValueError(f"WORLD_SIZE={world} is not a multiple of the {replicas} processes "
                         f"(GPUs) per site")
    if device == "cpu":
        dev = torch.device("cpu")
    elif device not in (None, "", "auto", "cuda"):
        dev = torch.device(device)  # an explicit device wins over the site input
    else:
        # the site input's `gpus` picks the device (None: this rank's GPU); with RCCL it must
        # be GPU LOCAL_RANK
        be0 = backend or os.environ.get("DINUNET_BACKEND") or "nccl"
        dev = resolve_device(gpus, local, world, be0, replica=rank % replicas, replicas=replicas)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    # DINUNET_BACKEND=gloo rehearses the multi-site GPU path with several ranks on ONE GPU
    # (RCCL needs one device per rank); production multi-GPU runs use nccl (= RCCL)
    be = backend or os.environ.get("DINUNET_BACKEND") or ("nccl" if dev.type == "cuda" else "gloo")
    pg = None
    loopback = bool(loopback and world == 1)
    # every collective's completion events are its own: with torch's event cache a pooled event
    # the process group's watchdog still polls could be re-recorded by a collective inside a
    # graph capture, and the watchdog's next query aborts the process (hipErrorCapturedEvent)
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    if world > 1 or loopback:
        if not dist.is_initialized():
            kw = dict(backend=be, rank=rank, world_size=world,
                      timeout=datetime.timedelta(seconds=timeout_s))
            if loopback:
                kw["store"] = dist.HashStore()  # one rank: an in-process store, no TCP port
            else:
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if be == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(**kw)
        pg = dist.group.WORLD
    site_pg = None
    if replicas > 1 and world > 1:
        # every rank creates every site's group, in site order (new_group is collective)
        for s in range(world // replicas):
            g = dist.new_group(list(range(s * replicas, (s + 1) * replicas)))
            if s == rank // replicas:
                site_pg = g
    _GROUP = SiteGroup(rank=rank, world=world, local_rank=local, device=dev,
                       backend=be if (world > 1 or loopback) else None, pg=pg, loopback=loopback,
                       replicas=replicas if world > 1 else 1, replica=rank % replicas,
                       site_pg=site_pg)
    _GROUP.gpu_shared = _gpu_shared(_GROUP)
    return _GROUP


def _gpu_shared(g: SiteGroup) -> Optional[bool]:
    """Whether several ranks of ``g`` drive the same GPU: decided from the actual (host, device)
    pairs, not from world vs device count -- explicit ``gpus`` lists, a gloo rehearsal with every
    site on GPU 0, or more ranks than inputspec entries can all stack sites on one card, while a
    multi-node run has more ranks than local devices without sharing any."""
    if g.device.type != "cuda":
        return False
    if g.world == 1:
        return False
    import socket
    me = (socket.gethostname(), int(g.device.index or 0))
    return g.all_gather_object(me).count(me) > 1


def current() -> SiteGroup:
    global _GROUP
    if _GROUP is None:
        _GROUP = SiteGroup()
    return _GROUP


def shutdown():
    global _GROUP
    if dist.is_initialized():
        dist.destroy_process_group()
    _GROUP = None
