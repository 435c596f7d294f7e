"""One site of a decentralized run — what ``COINNLocal`` + ``COINNRemote`` did together
(SURVEY.md E2, E3, E13-E16), executed as one rank of a process group.

Phases per fold (``fold_0 .. fold_{k-1}``):

1. list files (plugin ``DataHandle``) -> deterministic per-site split (ratio / k-fold / files)
   -> plugin ``Dataset`` -> ONE preprocessing pass into HBM-resident tensors.
2. model init with a seed shared by all sites + broadcast from rank 0 (identical replicas); or,
   with ``pretrain``, the site holding the most training data trains alone with
   ``pretrain_args`` and its best weights are broadcast as the common init (config 5).
3. training in lockstep: every site contributes a gradient at every step (``steps_per_epoch``
   = max over sites; sites with less data cycle their reshuffled loader), ``local_iterations``
   micro-batches per step, aggregation by the engine (dSGD / rank-dAD / PowerSGD), fused Adam.
4. every ``validation_epochs``: each site scores its validation split, scores+labels are
   all-gathered, the *global* metric (``monitor_metric``, ``metric_direction``) drives the
   best-epoch checkpoint and ``patience`` early stopping identically on every rank (the
   remote's decisions, made redundantly instead of by a separate process).
5. test: reload the best checkpoint, score the test split, write global + local test metrics.

Outputs: ``logs.json`` / ``test_metrics.csv`` per site and for the global "remote" view, remote
results zip, ``checkpoint_best.pt`` / ``checkpoint_last.pt`` (resume with ``resume=True``).
"""
from __future__ import annotations

import copy
import math
import os
import signal
import time
from typing import Any, Dict, List, Optional, Tuple

import torch

from ..config import site_seed
from ..data.loader import DeviceLoader
from ..data.splits import make_splits
from ..parallel import SiteGroup, make_engine
from ..utils import logs as L
from ..utils.metrics import Averages, Metrics, improved, metric_value
from ..ops import FusedAdam
from . import health
from .feed import DeviceFeed
from .step import TrainStep
from .trainer import NNTrainer, set_seed


def _fault_step(rank: int) -> Optional[int]:
    """``DINUNET_FAULT=<rank>:<step>[:raise]``: that rank kills itself (SIGKILL, no cleanup) --
    or, with ``:raise``, raises -- before its <step>-th training step: the dead-site and the
    failing-site cases the failure-path tests exercise."""
    spec = os.environ.get("DINUNET_FAULT", "")
    if not spec:
        return None
    r, _, s = spec.partition(":")
    return int(s.partition(":")[0] or 0) if int(r) == rank else None


def _fault():
    if os.environ.get("DINUNET_FAULT", "").endswith(":raise"):
        raise RuntimeError("DINUNET_FAULT: injected site failure")
    os.kill(os.getpid(), signal.SIGKILL)


class _PretrainSignal:
    """The pretraining site's side of :meth:`FederatedSite._await_pretrain`: a heartbeat counter
    in the process group's store advanced every ``pretrain_heartbeat_s`` by a daemon thread while
    it pretrains, then the done key set to "1", or to "fail: <error>" when pretraining raises
    (the error still propagates)."""

    def __init__(self, group: SiteGroup, tag: str, cfg: Dict[str, Any]):
        self.store = None
        if group.distributed and group.pg is not None:
            import torch.distributed as dist
            self.store = dist.distributed_c10d._get_default_store()
        self.key, self.hb = self.keys(tag)
        self.every = self.period(cfg)
        self._stop = None

    @staticmethod
    def keys(tag: str):
        base = "dinunet/pretrain_done/" + os.path.basename(os.path.normpath(tag))
        return base, base + "/heartbeat"

    @staticmethod
    def period(cfg: Dict[str, Any]) -> float:
        return float(cfg.get("pretrain_heartbeat_s") or
                     min(30.0, max(0.5, float(cfg.get("collective_timeout_s") or 1800) / 4)))

    def done(self, value: str):
        if self.store is not None:
            self.store.set(self.key, value)

    def __enter__(self):
        if self.store is not None:
            import threading
            self._stop = threading.Event()

            def beat():
                while not self._stop.wait(self.every):
                    try:
                        self.store.add(self.hb, 1)
                    except Exception:
                        return
            self.store.add(self.hb, 1)
            threading.Thread(target=beat, daemon=True, name="pretrain-heartbeat").start()
        return self

    def __exit__(self, et, ev, tb):
        if self._stop is not None:
            self._stop.set()
        self.done("1" if et is None else f"fail: {et.__name__}: {ev}"[:500])
        return False


class FederatedSite:
    def __init__(self, cfg: Dict[str, Any], group: SiteGroup, trainer_cls, dataset_cls,
                 datahandle_cls, state: Dict[str, Any], out_dir: str, site_name: Optional[str] = None,
                 verbose: bool = True):
        self.cfg = cfg
        self.group = group
        self.Trainer, self.Dataset, self.DataHandle = trainer_cls, dataset_cls, datahandle_cls
        self.state = state
        self.out_dir = out_dir
        self.site = site_name or f"local{group.site}"
        self.device = group.device
        self.verbose = verbose
        self.task_id = str(cfg.get("task_id"))

    # ---------------------------------------------------------------------------------------
    def log(self, *a):
        if self.verbose and self.group.replica == 0:
            print(f"[{self.site}]", *a, flush=True)

    def _global_max(self, v: int) -> int:
        t = torch.tensor([int(v)], device=self.device)
        self.group.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        return int(t.item())

    def _datasets(self, split: Dict[str, List[Any]]) -> Dict[str, Tuple[torch.Tensor, torch.Tensor]]:
        """The site's splits on this process's device; with several processes per site
        (``group.replicas``) this replica's shard of each: rows ``replica::replicas`` of the
        site's (identically made) splits, so the replicas' shards are disjoint and cover it."""
        cache = self.cfg
        out = {}
        k, r = self.group.replicas, self.group.replica
        for key in ("train", "validation", "test"):
            ds = self.Dataset(cache=cache, state=self.state, mode=key)
            if split.get(key):
                ds.add(split[key])
            X, y = ds.materialize(self.device)
            if k > 1:
                X, y = X[r::k].contiguous(), y[r::k].contiguous()
            out[key] = (X, y)
        return out

    def _batch_size(self, cfg: Dict[str, Any]) -> int:
        """Rows per step on this process: the site's ``batch_size`` split over its replicas."""
        bs = int(cfg.get("batch_size", 16))
        k = self.group.replicas
        if k > 1:
            if bs % k:
                raise ValueError(f"batch_size {bs} does not split over the site's {k} GPUs")
            bs //= k
        return bs

    def _loader(self, X, y, key: str, batch_size: int, seed: int) -> DeviceLoader:
        dl_args = (self.cfg.get("dataloader_args") or {}).get(key, {})
        drop_last = bool(dl_args.get("drop_last", False))
        shuffle = key == "train"
        if drop_last and X.shape[0] < batch_size:
            drop_last = False  # keep at least one batch on tiny splits
        return DeviceLoader(X, y, batch_size, shuffle=shuffle, drop_last=drop_last, seed=seed)

    # ---- global evaluation ------------------------------------------------------------------
    def global_eval(self, trainer: NNTrainer, loader: DeviceLoader):
        res = trainer.evaluate(loader)
        avg: Averages = res["averages"]
        met: Metrics = res["metrics"]
        s, l = met.tensors()
        s = s.to(self.device).float()
        l = l.to(self.device).long()
        S = self.group.all_gather_varlen(s)
        Lb = self.group.all_gather_varlen(l)
        st = avg.to_state()
        tot = torch.tensor([st["sum"], float(st["n"])], device=self.device, dtype=torch.float64)
        self.group.all_reduce(tot)
        gloss = float(tot[0] / tot[1]) if float(tot[1]) > 0 else 0.0
        gm = Metrics.from_tensors(S, Lb, met.num_class)
        return {"loss": gloss, "scores": gm.scores(), "local_loss": avg.average,
                "local_scores": met.scores(), "n": int(tot[1])}

    def _broadcast_model(self, trainer: NNTrainer, src: int = 0):
        if not self.group.distributed:
            return
        self.group.broadcast(trainer.flat.data, src)
        for m in trainer.nn.values():
            for b in m.buffers():
                self.group.broadcast(b, src)

    def _replica_checksum(self, trainer: NNTrainer) -> bool:
        """Debug race/sync check: are all sites' parameters bit-identical?"""
        v = trainer.flat.data.double().sum().reshape(1)
        allv = self.group.all_gather(v)
        return all(bool(torch.equal(x, allv[0])) for x in allv)

    # ---- train loops ------------------------------------------------------------------------
    def _train_epochs(self, trainer: NNTrainer, engine, data, cfg: Dict[str, Any], group: SiteGroup,
                      fold_dir: str, seed: int, logs: Dict[str, Any], tag: str = "",
                      start_epoch: int = 1, best: Optional[Dict[str, Any]] = None,
                      resume: Optional[Dict[str, Any]] = None):
        bs = self._batch_size(cfg)
        li = max(1, int(cfg.get("local_iterations", 1)))
        tr = self._loader(*data["train"], "train", bs, seed)
        va = self._loader(*data["validation"], "validation", bs, seed)
        local_steps = max(1, math.ceil(len(tr) / li)) if tr.num_samples else 0
        if group is self.group:
            steps = self._global_max(local_steps)
        else:
            steps = local_steps
        epochs = int(cfg.get("epochs", 1))
        patience = int(cfg.get("patience", epochs + 1))
        val_every = max(1, int(cfg.get("validation_epochs", 1)))
        monitor = str(cfg.get("monitor_metric", "auc"))
        direction = str(cfg.get("metric_direction", "maximize"))
        if monitor.lower() == "loss":
            direction = "minimize"
        best = best or {"score": None, "epoch": 0, "wait": 0}
        # gradient accumulation runs on the fast path too (TrainStep accum) unless the engine
        # captures per-micro-batch activations (rank-dAD's CPU activation-space form)
        use_fast = trainer.has_fast_path and (li == 1 or getattr(engine, "fast", True)
                                               or engine.name != "rankDAD")
        step = None
        if use_fast:
            use_graph = (bool(cfg.get("use_graph", True)) and self.device.type == "cuda"
                         and not trainer.reference_math)
            sm = trainer.split_module()
            if sm is not None:  # stem/body model: split capture overlaps the all-reduce
                step = TrainStep(sm, trainer.flat, trainer.optimizer, engine, use_graph=use_graph,
                                 accum=li)
            else:
                step = TrainStep(trainer.modules(), trainer.flat, trainer.optimizer, engine,
                                 use_graph=use_graph, accum=li,
                                 forward_loss=lambda m, x, y: trainer.forward_loss(x, y))
        fault_at = _fault_step(self.group.rank)
        feed = self._device_feed(trainer, step, engine, tr, bs, li, steps, cfg, fault_at)
        if resume and resume.get("loader"):
            it = tr.resume_iter(resume["loader"], indices=feed is not None)
        else:
            it = tr.iter_indices() if feed is not None else iter(tr)
        if feed is not None:
            logs[f"{tag}feed"] = "device"
        tl = logs.setdefault(f"{tag}train_log", [])
        vl = logs.setdefault(f"{tag}validation_log", [])
        lvl = logs.setdefault(f"{tag}local_validation_log", [])
        # duration lists per phase (the pretraining pass logs under its own tag, so the
        # federated clock of the pretrain site starts at 0 like every other site's)
        comp = logs.setdefault(f"{tag}time_spent_on_computation", [])
        cum = logs.setdefault(f"{tag}cumulative_total_duration", [])
        itd = logs.setdefault(f"{tag}local_iter_duration", [])
        # only a resumed run continues its clock from the checkpointed total
        t_run = time.time() - (cum[-1] if (resume and cum) else 0.0)
        trainer.train()
        for epoch in range(start_epoch, epochs + 1):
            t0 = time.time()
            avg, met = trainer.new_averages(), trainer.new_metrics()
            nsamp = 0
            if feed is not None:
                # ONE host call per epoch: the epoch's batch order (the loader's own passes),
                # then K-step graph replays with the train records kept on the device
                order = []
                for _ in range(steps * li):  # li batches per step (local_iterations)
                    try:
                        order.append(next(it))
                    except StopIteration:
                        it = tr.iter_indices()
                        order.append(next(it))
                losses, scores, labels = feed.run_epoch(torch.cat(order))
                avg.add(losses.mean(), steps * li * bs)
                met.add(scores.clone(), labels)
                nsamp += steps * li * bs
            for _ in range(steps if feed is None else 0):
                if fault_at is not None:  # failure-path tests (DINUNET_FAULT=<rank>:<step>)
                    fault_at -= 1
                    if fault_at < 0:
                        _fault()
                if step is not None:
                    for k in range(li):
                        try:
                            x, y, _ix = next(it)
                        except StopIteration:
                            it = iter(tr)
                            x, y, _ix = next(it)
                        loss = step(x, y, first=k == 0, last=k == li - 1)
                        avg.add(loss.detach(), len(y))
                        # clone: a graph replay overwrites its static outputs next step
                        met.add(trainer.score(step.last_out, step.last_pred).detach().clone(), y)
                        nsamp += len(y)
                    continue
                trainer.flat.zero_grad()
                if hasattr(engine, "sync_enabled"):
                    engine.sync_enabled = False
                with engine.step_context():
                    for k in range(li):
                        try:
                            x, y, ix = next(it)
                        except StopIteration:
                            it = iter(tr)
                            x, y, ix = next(it)
                        if hasattr(engine, "sync_enabled"):
                            engine.sync_enabled = k == li - 1
                        out = trainer.iteration({"inputs": x, "labels": y, "ix": ix})
                        (out["loss"] / li).backward()
                        avg.accumulate(out["averages"])
                        met.accumulate(out["metrics"])
                        nsamp += len(y)
                scale = engine.reduce()
                trainer.optimizer.step(grad_scale=scale)
            if self.device.type == "cuda":
                torch.cuda.synchronize()
            dt = time.time() - t0
            itd.append(dt / max(steps, 1))
            tl.append([round(avg.average, 6)] + met.get((monitor if monitor != "loss" else "auc",)))
            logs.setdefault(f"{tag}samples_per_sec", []).append(nsamp / dt if dt > 0 else 0.0)
            stop = False
            if epoch % val_every == 0:
                if group is self.group:
                    r = self.global_eval(trainer, va)
                else:
                    res = trainer.evaluate(va)
                    r = {"loss": res["averages"].average, "scores": res["metrics"].scores(),
                         "local_loss": res["averages"].average, "local_scores": res["metrics"].scores()}
                score = r["loss"] if monitor.lower() == "loss" else metric_value(r["scores"], monitor)
                vl.append([round(r["loss"], 6), round(score, 6)])
                lvl.append([round(r["local_loss"], 6),
                            round(r["local_loss"] if monitor.lower() == "loss"
                                  else metric_value(r["local_scores"], monitor), 6)])
                if improved(score, best["score"], direction):
                    best.update(score=score, epoch=epoch, wait=0)
                    trainer.save_checkpoint(os.path.join(fold_dir, f"{tag}checkpoint_best.pt"),
                                            epoch=epoch, best_val_epoch=epoch, best_val_score=score)
                else:
                    best["wait"] += 1
                    if best["wait"] >= patience:
                        stop = True
                self.log(f"{tag}epoch {epoch} train_loss {avg.average:.4f} val_loss {r['loss']:.4f} "
                         f"val_{monitor} {score:.4f} best@{best['epoch']}")
                # a persistent kernel whose in-kernel wait timed out used incomplete data:
                # fail the run instead of training on it (runtime.health)
                health.check(trainer.nn.values(), engine, f"in epoch {epoch}")
                if cfg.get("check_replicas") and group.distributed and engine.name != "dSGD-local":
                    ok = self._replica_checksum(trainer)
                    logs.setdefault("replica_check", []).append(bool(ok))
            comp.append(time.time() - t0)
            cum.append(time.time() - t_run)
            if epoch % val_every == 0 and cfg.get("checkpoint_every_validation", True):
                # everything a resume needs to continue this exact curve:
                # weights + optimizer, best/patience, the log history, every RNG, the train
                # loader's position and the engine's warm-start / error-feedback state
                trainer.save_checkpoint(os.path.join(fold_dir, f"{tag}checkpoint_last.pt"),
                                        epoch=epoch, best=dict(best), logs=copy.deepcopy(logs),
                                        rng=trainer.rng_state(), loader=tr.state(),
                                        engine=engine.state_dict(), stopped=bool(stop))
            if stop:
                logs[f"{tag}stopped_epoch"] = epoch
                break
        if best["score"] is None:  # no validation happened: keep the last model as "best"
            trainer.save_checkpoint(os.path.join(fold_dir, f"{tag}checkpoint_best.pt"),
                                    epoch=epochs, best_val_epoch=epochs, best_val_score=None)
            best["epoch"] = epochs
        health.check(trainer.nn.values(), engine, "in training")
        logs[f"{tag}best_val_epoch"] = best["epoch"]
        logs[f"{tag}best_val_score"] = best["score"]
        if step is not None and step.timers.summary():
            logs[f"{tag}phase_ms"] = step.timers.summary()  # DINUNET_PHASE_TIMERS=1
        return best

    def _device_feed(self, trainer: NNTrainer, step, engine, tr: DeviceLoader, bs: int, li: int,
                     steps: int, cfg: Dict[str, Any], fault_at) -> Optional[DeviceFeed]:
        """The device-fed epoch (``runtime.feed``) when this site's step can take it: a captured
        step on the GPU, a model that takes a bf16 batch, a plugin with a score column, full
        batches, an engine that runs inside the captured step (``local_iterations`` > 1: whole
        accumulated steps per replay, ``TrainStep._dev_body_accum``).  ``device_feed``
        (default on) turns it off; the fault-injection hook keeps the per-step host loop."""
        col = getattr(trainer, "score_column", None)
        if (step is None or not step.use_graph or self.device.type != "cuda" or step.accum != li
                or not cfg.get("device_feed", True) or fault_at is not None or col is None
                or not tr.full_batches or steps < 1
                or not isinstance(trainer.optimizer, FusedAdam)
                or not (engine.name.startswith("dSGD") or getattr(engine, "fast", False))):
            return None
        X = tr.inputs
        bf = bool(getattr(step.model, "accepts_bf16_input", False))
        row = X[0].numel() if X.shape[0] else 0
        copies = (X.dtype != torch.bfloat16) if bf else (X.dtype != torch.float32 or row % 8 != 0)
        if copies:
            # the feed keeps its own copy of the split in HBM next to the loader's (bf16, or
            # fp32 rows padded to 8 features): fall back to the host-fed loop (same trajectory)
            # when it would not fit
            need = X.shape[0] * (2 * row if bf else 4 * (-(-row // 8) * 8)) + tr.labels.numel() * 8
            free, _ = torch.cuda.mem_get_info(self.device)
            if need > 0.9 * free:
                self.log(f"device feed off: its copy of the train split ({need / 2**30:.2f} "
                         f"GiB) does not fit the free HBM ({free / 2**30:.2f} GiB)")
                return None
        return DeviceFeed(step, X, tr.labels, bs, steps, col=col)

    def _pretrain(self, trainer: NNTrainer, data, fold_dir: str, seed: int, logs: Dict[str, Any]):
        if self.group.replicas > 1:
            raise NotImplementedError("pretrain with several GPUs per site: the pretraining "
                                      "site trains alone (one process)")
        sizes = self.group.all_gather_object(int(data["train"][0].shape[0]))
        src = max(range(len(sizes)), key=lambda r: (sizes[r], -r))
        logs["pretrain_site"] = f"local{src}"
        pa = dict(self.cfg.get("pretrain_args") or {})
        if self.group.rank == src and int(pa.get("epochs", 0)) > 0:
            with _PretrainSignal(self.group, fold_dir, self.cfg):
                delay = float(os.environ.get("DINUNET_PRETRAIN_DELAY_S", "0") or 0)
                if delay > 0:  # tests: a pretraining phase longer than the collective timeout
                    time.sleep(delay)
                pcfg = copy.deepcopy(self.cfg)
                pcfg.update(pa)
                from ..parallel import DSGDEngine
                from ..parallel.group import SiteGroup as _SG
                solo = _SG(device=self.device)
                trainer.optimizer.lr = float(pa.get("learning_rate", trainer.optimizer.lr))
                eng = DSGDEngine(trainer.modules(), trainer.flat, solo, pcfg, overlap=False)
                eng.name = "dSGD-local"
                self.log(f"pretraining alone on {sizes[src]} samples for {pa.get('epochs')} epochs")
                b = self._train_epochs(trainer, eng, data, pcfg, solo, fold_dir, seed, logs,
                                       tag="pretrain_")
                trainer.load_checkpoint(os.path.join(fold_dir, "pretrain_checkpoint_best.pt"))
                logs["pretrain_best_val_epoch"] = b["epoch"]
        elif self.group.rank == src:
            _PretrainSignal(self.group, fold_dir, self.cfg).done("1")
        self._await_pretrain(src, fold_dir)
        self._broadcast_model(trainer, src)
        # fresh optimizer state for the federated phase
        trainer._init_optimizer()

    def _await_pretrain(self, src: int, tag: str):
        """The other sites wait for the pretraining site OUTSIDE the collectives: a wait inside
        the weight broadcast would be bounded by ``collective_timeout_s`` (the failure detector's
        clock), so a long pretraining phase would make every idle site time out.  They block on a
        key the pretraining site sets in the process group's store when it is done ("1") or has
        failed ("fail: ..."), bounded by their own deadline (``pretrain_timeout_s``), and they
        watch its heartbeat counter: no beat for ``collective_timeout_s`` means the pretraining
        site is gone (killed, hung), and the wait raises instead of lasting the whole deadline."""
        g = self.group
        if not g.distributed or g.pg is None or g.rank == src:
            return
        if os.environ.get("DINUNET_PRETRAIN_STORE_WAIT", "1") == "0":
            return  # negative control of tests/test_failure.py: wait inside the broadcast
        import datetime
        import torch.distributed as dist
        store = dist.distributed_c10d._get_default_store()
        key, hb = _PretrainSignal.keys(tag)
        deadline = time.time() + float(self.cfg.get("pretrain_timeout_s") or 7 * 86400)
        silence = float(self.cfg.get("collective_timeout_s") or 1800)
        beat, t_beat = store.add(hb, 0), time.time()
        while True:
            slice_s = max(0.05, min(_PretrainSignal.period(self.cfg), deadline - time.time()))
            try:
                store.wait([key], datetime.timedelta(seconds=slice_s))
                break
            except Exception:  # (the store's wait timeout) -- check the heartbeat
                now = time.time()
                b = store.add(hb, 0)
                if b != beat:
                    beat, t_beat = b, now
                elif now - t_beat > silence:
                    raise RuntimeError(f"pretraining site local{src} stopped signalling for "
                                       f"{now - t_beat:.0f} s (collective_timeout_s {silence:g})")
                if now >= deadline:
                    raise RuntimeError(f"pretraining site local{src} did not finish within "
                                       f"pretrain_timeout_s")
        v = store.get(key).decode(errors="replace")
        if v != "1":
            raise RuntimeError(f"pretraining site local{src} failed: {v}")

    # ---- folds ------------------------------------------------------------------------------
    def run_fold(self, fold: int, split: Dict[str, List[Any]]) -> Dict[str, Any]:
        cfg = self.cfg
        t_fold = time.time()
        g = self.group
        # a site's replicas write their own logs / checkpoints (their loaders differ) beside it
        fdir = L.fold_dir(self.out_dir, self.site if g.replica == 0 else
                          f"{self.site}_replica{g.replica}", self.task_id, fold)
        seed = site_seed(cfg, g.site) + 7919 * fold + 104729 * g.replica
        data = self._datasets(split)
        logs: Dict[str, Any] = {
            "task_id": self.task_id, "agg_engine": cfg.get("agg_engine"), "fold": fold,
            "site": self.site, "rank": self.group.rank, "num_sites": self.group.sites,
            "gpus_per_site": self.group.replicas,
            "log_header": cfg.get("log_header"), "mode": cfg.get("mode"),
            "split_sizes": {k: int(v[1].shape[0]) for k, v in data.items()},
            "device": str(self.device),
        }
        trainer = self.Trainer(cache=cfg, state=self.state, device=self.device)
        trainer.init_nn(seed=int(cfg.get("seed", 0) or 0) + fold)  # same init on every site
        self._broadcast_model(trainer, 0)
        start_epoch, best, resume = 1, None, None
        last = os.path.join(fdir, "checkpoint_last.pt")
        if cfg.get("mode") == "test":
            path = cfg.get("pretrained_path") or os.path.join(fdir, "checkpoint_best.pt")
            trainer.load_checkpoint(path)
            best = {"epoch": 0, "score": None}
        else:
            if cfg.get("resume") and os.path.exists(last):
                resume = trainer.load_checkpoint(last, load_optimizer=True)
                start_epoch = int(resume.get("epoch", 0)) + 1
                best = resume.get("best")
                if resume.get("stopped"):  # early stopping had already ended this fold
                    logs["stopped_epoch"] = int(resume.get("epoch", 0))
                    start_epoch = int(cfg.get("epochs", 1)) + 1
                for k, v in (resume.get("logs") or {}).items():
                    logs.setdefault(k, v)
                self.log(f"resuming fold {fold} at epoch {start_epoch}")
            elif cfg.get("pretrain"):
                self._pretrain(trainer, data, fdir, seed, logs)
            engine = make_engine(str(cfg.get("agg_engine", "dSGD")), trainer.modules(), trainer.flat,
                                 self.group, cfg)
            cal = getattr(engine, "calibration", None)
            if cal:  # dsgd_collective="calibrate": what was measured and chosen
                logs["dsgd_collective"] = cal
                self.log(f"dsgd_collective calibrated: {cal}")
            if resume is not None:
                if resume.get("engine"):
                    engine.load_state_dict(resume["engine"])
                if resume.get("rng"):
                    trainer.load_rng_state(resume["rng"])
            best = self._train_epochs(trainer, engine, data, cfg, self.group, fdir, seed, logs,
                                      start_epoch=start_epoch, best=best, resume=resume)
            if hasattr(engine, "close"):
                engine.close()
            trainer.load_checkpoint(os.path.join(fdir, "checkpoint_best.pt"))
        te = self._loader(*data["test"], "test", self._batch_size(cfg), seed)
        r = self.global_eval(trainer, te)
        logs["test_metrics"] = L.test_row(r["loss"], r["scores"])
        logs["local_test_metrics"] = L.test_row(r["local_loss"], r["local_scores"])
        logs["test_scores"] = r["scores"]
        logs["test_header"] = L.TEST_HEADER
        logs["fold_duration"] = time.time() - t_fold
        L.write_logs(fdir, logs)
        L.write_test_metrics(fdir, [logs["local_test_metrics"]])
        if self.group.is_master:
            rdir = L.fold_dir(self.out_dir, "remote", self.task_id, fold)
            rlogs = {k: v for k, v in logs.items() if not k.startswith("local_")}
            rlogs["remote_iter_duration"] = logs.get("local_iter_duration", [])  # NB.ipynb:860
            rlogs["site"] = "remote"
            rlogs["sites"] = [f"local{i}" for i in range(self.group.sites)]
            L.write_logs(rdir, rlogs)
            L.write_test_metrics(rdir, [logs["test_metrics"]])
            L.zip_results(rdir, os.path.join(rdir, f"{self.task_id}_fold_{fold}_results.zip"))
        self.log(f"fold {fold} test: loss {r['loss']:.4f} " +
                 " ".join(f"{k} {v:.4f}" for k, v in r["scores"].items()))
        return logs

    def run(self) -> List[Dict[str, Any]]:
        # replicas of a site make identical splits (explicit site seed), which _datasets then
        # shards; their dropout streams differ
        set_seed(site_seed(self.cfg, self.group.site) + 104729 * self.group.replica)
        handle = self.DataHandle(cache=self.cfg, state=self.state)
        files = handle.list_files()
        splits = make_splits(files, self.cfg, site_seed(self.cfg, self.group.site),
                             base=self.state.get("baseDirectory", "."))
        nfolds = self._global_max(len(splits))
        if nfolds != len(splits):
            raise RuntimeError("all sites must run the same number of folds")
        return [self.run_fold(k, s) for k, s in enumerate(splits)]
