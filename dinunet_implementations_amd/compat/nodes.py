"""COINSTAC-compatible site ("local") and aggregator ("remote") nodes over a FILE transport.

For real multi-institution runs the reference is a COINSTAC computation: every iteration the
COINSTAC runtime calls ``local.run(data)`` on each site and ``remote.run(data)`` on the
aggregator (``entry.py:5``), passing ``data = {'input', 'state'}`` and routing each returned
``{'output': ...}``; bulk tensors travel as files through transfer directories (SURVEY.md E1,
§2.4).  This module re-creates that contract on top of the same engines, trainer, datasets and
metrics as the collective path:

site   : payload = ``engine.payload()`` (precision_bits honoured) -> ``transferDirectory``
remote : ``Engine.aggregate([payloads])`` -> ``transferDirectory`` (mp.Pool of ``num_reducers``
         not needed: the reduction is one vectorised op per tensor)
site   : ``engine.apply(aggregate)`` -> fused optimizer step

Phases (remote-driven):  init_runs -> [pretrain] -> train (computation rounds; PowerSGD uses two
sub-rounds P/Q) -> validation (global metrics, save-best / early-stop decision) -> ... -> test
(global test metrics, remote logs + zip) -> next fold / success.

One node object per site and one remote object persist across calls (the reference keeps state
in a module-global ``CACHE``, ``local.py:15``).
"""
from __future__ import annotations

import copy
import os
import zlib
import time
from typing import Any, Dict, List, Optional

import torch

from ..config import build_config, site_seed
from ..data.loader import DeviceLoader
from ..data.splits import make_splits
from ..parallel.engines import ENGINES
from ..parallel.group import SiteGroup
from ..tasks import get_task
from ..utils import logs as L
from ..utils.metrics import Averages, Metrics, improved, merge_states, metric_value


def _save(obj: Dict[str, torch.Tensor], path: str):
    torch.save({k: v.detach().cpu() for k, v in obj.items()}, path)


def _load(path: str) -> Dict[str, torch.Tensor]:
    return torch.load(path, map_location="cpu", weights_only=True)


class LocalNode:
    """State machine of one site (the ``COINNLocal`` role)."""

    def __init__(self, device: Optional[str] = None, **code_defaults):
        self.code_defaults = code_defaults
        self.cfg: Optional[Dict[str, Any]] = None
        # explicit device, else the site input's `gpus` (resolved in _setup)
        self._device_arg = device
        self.device = torch.device(device) if device else torch.device("cpu")
        self.trainer = None
        self.engine = None
        self.it = None

    # ------------------------------------------------------------------------------------------
    def _setup(self, inp: Dict[str, Any], state: Dict[str, Any]):
        self.state = state
        self.cfg = build_config(site_input=inp, **self.code_defaults)
        if not self._device_arg:
            from ..parallel.group import resolve_device
            self.device = resolve_device(self.cfg.get("gpus"))
        self.site = state.get("clientId", "local0")
        T, D, H = get_task(self.cfg["task_id"])
        self.Trainer, self.Dataset = T, D
        files = H(cache=self.cfg, state=state).list_files()
        self.seed = site_seed(self.cfg, zlib.crc32(self.site.encode()) % 997)  # stable across processes
        self.splits = make_splits(files, self.cfg, self.seed, base=state.get("baseDirectory", "."))
        self.logs: Dict[str, Any] = {}

    def _datasets(self, split):
        out = {}
        for key in ("train", "validation", "test"):
            ds = self.Dataset(cache=self.cfg, state=self.state, mode=key)
            if split.get(key):
                ds.add(split[key])
            out[key] = ds.materialize(self.device)
        return out

    def _init_fold(self, fold: int, seed: int, cfg: Dict[str, Any]):
        self.fold = fold
        self.data = self._datasets(self.splits[fold])
        self.trainer = self.Trainer(cache=self.cfg, state=self.state, device=self.device)
        self.trainer.init_nn(seed=seed)
        # the file transport ships rank-dAD's structured (A, Delta) factors: keep that path
        self.engine = ENGINES[str(cfg.get("agg_engine", "dSGD"))](
            self.trainer.modules(), self.trainer.flat, SiteGroup(device=self.device),
            dict(cfg, dad_gradient_space=False))
        bs = int(cfg.get("batch_size", 16))
        dl = (cfg.get("dataloader_args") or {}).get("train", {})
        Xtr = self.data["train"][0]
        self.train_loader = DeviceLoader(*self.data["train"], bs, shuffle=True,
                                         drop_last=bool(dl.get("drop_last", False)) and Xtr.shape[0] >= bs,
                                         seed=self.seed + fold)
        self.it = iter(self.train_loader)
        self.fold_dir = L.fold_dir(self.state.get("outputDirectory", "."), "", str(self.cfg["task_id"]), fold)
        self.logs = {"task_id": self.cfg["task_id"], "agg_engine": cfg.get("agg_engine"), "fold": fold,
                     "site": self.site, "train_log": [], "validation_log": [],
                     "local_iter_duration": []}
        self.avg, self.met = self.trainer.new_averages(), self.trainer.new_metrics()

    def _next_batch(self):
        try:
            return next(self.it)
        except StopIteration:
            self.it = iter(self.train_loader)
            return next(self.it)

    def _compute_grads(self, cfg):
        li = max(1, int(cfg.get("local_iterations", 1)))
        tr = self.trainer
        tr.train()
        tr.flat.zero_grad()
        with self.engine.step_context():
            for _ in range(li):
                x, y, ix = self._next_batch()
                out = tr.iteration({"inputs": x, "labels": y, "ix": ix})
                (out["loss"] / li).backward()
                self.avg.accumulate(out["averages"])
                self.met.accumulate(out["metrics"])

    def _metric_state(self, split: str):
        bs = int(self.cfg.get("batch_size", 16))
        ld = DeviceLoader(*self.data[split], bs, shuffle=False, drop_last=False)
        res = self.trainer.evaluate(ld)
        return {"averages": res["averages"].to_state(), "metrics": res["metrics"].to_state()}

    # ------------------------------------------------------------------------------------------
    def __call__(self, data: Dict[str, Any]) -> Dict[str, Any]:
        inp, state = data.get("input", {}), data.get("state", {})
        t0 = time.time()
        if self.cfg is None:
            self._setup(inp, state)
            return {"output": {"phase": "init_runs", "task_id": self.cfg["task_id"],
                               "agg_engine": self.cfg["agg_engine"],
                               "num_folds": len(self.splits),
                               "data_size": [len(s["train"]) for s in self.splits],
                               "site_cfg": {k: v for k, v in self.cfg.items() if not str(k).startswith("_")}}}
        self.state = {**self.state, **state}
        cmd = inp.get("command")
        cfg = inp.get("cfg", self.cfg)
        tdir = self.state.get("transferDirectory", ".")
        bdir = self.state.get("baseDirectory", ".")
        if cmd == "init_fold":
            self._init_fold(int(inp["fold"]), int(inp["seed"]), cfg)
            if inp.get("pretrained_file"):
                st = _load(os.path.join(bdir, inp["pretrained_file"]))
                self.trainer.load_state({"models": _unflatten_models(st)})
            return {"output": {"phase": "ready"}}
        if cmd == "pretrain":
            if inp.get("site") != self.site:
                return {"output": {"phase": "waiting"}}
            # this site trains alone, then ships its weights (reference: largest site pretrains)
            pa = dict(inp.get("pretrain_args") or {})
            pcfg = copy.deepcopy(cfg)
            pcfg.update(pa)
            from ..runtime.site import FederatedSite
            fs = FederatedSite(pcfg, SiteGroup(device=self.device), self.Trainer, self.Dataset,
                               None, self.state, self.state.get("outputDirectory", "."), self.site,
                               verbose=False)
            logs = {}
            from ..parallel import DSGDEngine
            eng = DSGDEngine(self.trainer.modules(), self.trainer.flat, SiteGroup(device=self.device),
                             pcfg, overlap=False)
            eng.name = "dSGD-local"
            self.trainer.optimizer.lr = float(pa.get("learning_rate", self.trainer.optimizer.lr))
            fs._train_epochs(self.trainer, eng, self.data, pcfg, SiteGroup(device=self.device),
                             self.fold_dir, self.seed, logs, tag="pretrain_")
            self.trainer.load_checkpoint(os.path.join(self.fold_dir, "pretrain_checkpoint_best.pt"))
            _save(_flatten_models(self.trainer), os.path.join(tdir, "pretrained.pt"))
            return {"output": {"phase": "pretrained", "file": "pretrained.pt"}}
        if cmd == "train_round":
            if inp.get("apply_file"):
                agg = _load(os.path.join(bdir, inp["apply_file"]))
                scale = self.engine.apply({k: v.to(self.device) for k, v in agg.items()})
                self.trainer.optimizer.step(grad_scale=scale)
            if inp.get("epoch_end"):
                self.logs["train_log"].append([round(self.avg.average, 6)] + self.met.get(("auc",)))
                self.avg, self.met = self.trainer.new_averages(), self.trainer.new_metrics()
            if inp.get("stop"):
                return {"output": {"phase": "train_done"}}
            self._compute_grads(cfg)
            if self.engine.name == "powerSGD":
                pay = self.engine.payload_p()
            else:
                pay = self.engine.payload()
            _save(pay, os.path.join(tdir, "payload.pt"))
            self.logs["local_iter_duration"].append(time.time() - t0)
            return {"output": {"phase": "payload", "file": "payload.pt"}}
        if cmd == "powersgd_q":
            aggp = {k: v.to(self.device) for k, v in _load(os.path.join(bdir, inp["p_file"])).items()}
            self._agg_p = aggp
            _save(self.engine.payload_q(aggp), os.path.join(tdir, "payload_q.pt"))
            return {"output": {"phase": "payload_q", "file": "payload_q.pt"}}
        if cmd == "powersgd_apply":
            aggq = {k: v.to(self.device) for k, v in _load(os.path.join(bdir, inp["q_file"])).items()}
            scale = self.engine.apply_pq(self._agg_p, aggq)
            self.trainer.optimizer.step(grad_scale=scale)
            return {"output": {"phase": "applied"}}
        if cmd == "validate":
            if inp.get("apply_file"):
                agg = _load(os.path.join(bdir, inp["apply_file"]))
                scale = self.engine.apply({k: v.to(self.device) for k, v in agg.items()})
                self.trainer.optimizer.step(grad_scale=scale)
            return {"output": {"phase": "validation", **self._metric_state("validation")}}
        if cmd == "decision":
            if inp.get("save_best"):
                self.trainer.save_checkpoint(os.path.join(self.fold_dir, "checkpoint_best.pt"),
                                             epoch=inp.get("epoch"))
            self.logs["validation_log"].append(inp.get("val"))
            return {"output": {"phase": "ready"}}
        if cmd == "test":
            p = os.path.join(self.fold_dir, "checkpoint_best.pt")
            if os.path.exists(p):
                self.trainer.load_checkpoint(p)
            st = self._metric_state("test")
            loc = Metrics.from_state(st["metrics"]).scores()
            lavg = Averages.from_state(st["averages"]).average
            self.logs["local_test_metrics"] = L.test_row(lavg, loc)
            return {"output": {"phase": "test", **st}}
        if cmd == "finish_fold":
            self.logs.update(inp.get("global", {}))
            L.write_logs(self.fold_dir, self.logs)
            L.write_test_metrics(self.fold_dir, [self.logs.get("local_test_metrics", [])])
            return {"output": {"phase": "fold_done"}}
        if cmd == "success":
            return {"output": {"phase": "success"}, "success": True}
        raise ValueError(f"unknown command {cmd!r}")


def _flatten_models(trainer) -> Dict[str, torch.Tensor]:
    out = {}
    for name, m in trainer.nn.items():
        for k, v in m.state_dict().items():
            out[f"{name}::{k}"] = v
    return out


def _unflatten_models(flat: Dict[str, torch.Tensor]) -> Dict[str, Dict[str, torch.Tensor]]:
    out: Dict[str, Dict[str, torch.Tensor]] = {}
    for k, v in flat.items():
        n, key = k.split("::", 1)
        out.setdefault(n, {})[key] = v
    return out


class RemoteNode:
    """Aggregator state machine (the ``COINNRemote`` role): learns the task from site
    messages, aggregates payloads, merges metrics, decides best/stop, sequences folds."""

    def __init__(self):
        self.phase = "start"
        self.cfg = None
        self.sites: List[str] = []

    def _broadcast(self, inp: Dict[str, Any]) -> Dict[str, Any]:
        return {"output": inp}

    def _files(self, state, name):
        base = state.get("baseDirectory", ".")
        return [os.path.join(base, s, name) for s in self.sites]

    def __call__(self, data: Dict[str, Any]) -> Dict[str, Any]:
        inp, state = data.get("input", {}), data.get("state", {})
        msgs = inp  # {site: output}
        tdir = state.get("transferDirectory", ".")
        if self.phase == "start":
            self.sites = sorted(msgs)
            first = msgs[self.sites[0]]
            self.cfg = dict(first["site_cfg"])
            self.task_id = first["task_id"]
            self.engine_cls = ENGINES[str(self.cfg.get("agg_engine", "dSGD"))]
            self.num_folds = min(m["num_folds"] for m in msgs.values())
            self.sizes = {s: msgs[s]["data_size"] for s in self.sites}
            self.fold = 0
            self.t_start = time.time()
            return self._start_fold(state)
        if self.phase == "pretrain_ready":
            self.phase = "pretraining"
            return {"output": {"command": "pretrain", "site": self.pretrain_site, "cfg": self.cfg,
                               "pretrain_args": self.cfg.get("pretrain_args")}}
        if self.phase == "pretraining":
            src = self.pretrain_site
            import shutil
            shutil.copy(os.path.join(state["baseDirectory"], src, msgs[src]["file"]),
                        os.path.join(tdir, "pretrained.pt"))
            self.phase = "init_fold"
            return {"output": {"command": "init_fold", "fold": self.fold, "seed": self.seed,
                               "cfg": self.cfg, "pretrained_file": "pretrained.pt"}}
        if self.phase == "init_fold":
            self.epoch, self.step = 1, 0
            self.best = {"score": None, "epoch": 0, "wait": 0}
            self.rlogs = {"task_id": self.task_id, "agg_engine": self.cfg.get("agg_engine"),
                          "fold": self.fold, "site": "remote", "sites": self.sites,
                          "validation_log": [], "remote_iter_duration": [],
                          "time_spent_on_computation": [], "cumulative_total_duration": []}
            self.phase = "train"
            return {"output": {"command": "train_round", "cfg": self.cfg}}
        if self.phase in ("train", "powersgd_q"):
            t0 = time.time()
            name = "payload_q.pt" if self.phase == "powersgd_q" else "payload.pt"
            pays = [_load(f) for f in self._files(state, name)]
            if self.engine_cls.__name__ == "PowerSGDEngine":
                agg = self.engine_cls.aggregate(pays, self.cfg)
                if self.phase == "train":
                    _save(agg, os.path.join(tdir, "agg_p.pt"))
                    self.phase = "powersgd_q"
                    return {"output": {"command": "powersgd_q", "p_file": "agg_p.pt", "cfg": self.cfg}}
                _save(agg, os.path.join(tdir, "agg_q.pt"))
                self.phase = "powersgd_applied"
                self.rlogs["remote_iter_duration"].append(time.time() - t0)
                return {"output": {"command": "powersgd_apply", "q_file": "agg_q.pt", "cfg": self.cfg}}
            agg = self.engine_cls.aggregate(pays, self.cfg)
            _save(agg, os.path.join(tdir, "agg.pt"))
            self.rlogs["remote_iter_duration"].append(time.time() - t0)
            return self._after_step(apply_file="agg.pt")
        if self.phase == "powersgd_applied":
            self.phase = "train"
            return self._after_step(apply_file=None)
        if self.phase == "validation":
            states = [msgs[s] for s in self.sites]
            m = merge_states([s["metrics"] for s in states])
            tot = sum(s["averages"]["sum"] for s in states)
            n = sum(s["averages"]["n"] for s in states)
            loss = tot / max(n, 1)
            monitor = str(self.cfg.get("monitor_metric", "auc"))
            direction = "minimize" if monitor == "loss" else str(self.cfg.get("metric_direction", "maximize"))
            score = loss if monitor == "loss" else metric_value(m.scores(), monitor)
            save = improved(score, self.best["score"], direction)
            if save:
                self.best.update(score=score, epoch=self.epoch, wait=0)
            else:
                self.best["wait"] += 1
            self.rlogs["validation_log"].append([round(loss, 6), round(score, 6)])
            stop = (self.best["wait"] >= int(self.cfg.get("patience", 10 ** 9))
                    or self.epoch >= int(self.cfg.get("epochs", 1)))
            self.rlogs["cumulative_total_duration"].append(time.time() - self.t_start)
            self.epoch += 1
            self.step = 0
            self.phase = "test" if stop else "train_after_decision"
            return {"output": {"command": "decision", "save_best": save, "epoch": self.epoch - 1,
                               "val": [round(loss, 6), round(score, 6)], "stop": stop}}
        if self.phase == "train_after_decision":
            self.phase = "train"
            return {"output": {"command": "train_round", "cfg": self.cfg, "epoch_end": True}}
        if self.phase == "test":
            self.phase = "test_results"
            return {"output": {"command": "test"}}
        if self.phase == "test_results":
            states = [msgs[s] for s in self.sites]
            m = merge_states([s["metrics"] for s in states])
            tot = sum(s["averages"]["sum"] for s in states)
            n = sum(s["averages"]["n"] for s in states)
            row = L.test_row(tot / max(n, 1), m.scores())
            self.rlogs.update(test_metrics=row, best_val_epoch=self.best["epoch"],
                              best_val_score=self.best["score"], test_scores=m.scores())
            out_dir = state.get("outputDirectory", ".")
            rdir = L.fold_dir(out_dir, "", str(self.task_id), self.fold)
            L.write_logs(rdir, self.rlogs)
            L.write_test_metrics(rdir, [row])
            L.zip_results(rdir, os.path.join(tdir, f"{self.task_id}_fold_{self.fold}_results.zip"))
            self.phase = "fold_done"
            return {"output": {"command": "finish_fold",
                               "global": {"test_metrics": row, "best_val_epoch": self.best["epoch"]}}}
        if self.phase == "fold_done":
            self.fold += 1
            if self.fold < self.num_folds:
                return self._start_fold(state)
            self.phase = "done"
            return {"output": {"command": "success"}, "success": True}
        raise RuntimeError(f"remote in unknown phase {self.phase}")

    def _start_fold(self, state):
        self.seed = int(self.cfg.get("seed", 0) or 0) + self.fold
        if self.cfg.get("pretrain") and int((self.cfg.get("pretrain_args") or {}).get("epochs", 0)) > 0:
            sizes = {s: self.sizes[s][self.fold] for s in self.sites}
            self.pretrain_site = max(self.sites, key=lambda s: (sizes[s], [-ord(c) for c in s]))
            # all sites init the fold first; the chosen site then pretrains
            self.phase = "pretrain_ready"
            return {"output": {"command": "init_fold", "fold": self.fold, "seed": self.seed,
                               "cfg": self.cfg}}
        self.phase = "init_fold"
        return {"output": {"command": "init_fold", "fold": self.fold, "seed": self.seed, "cfg": self.cfg}}

    def _after_step(self, apply_file: Optional[str]):
        self.step += 1
        steps = max(self.steps_per_epoch, 1)
        if self.step >= steps:
            # validation every `validation_epochs` epochs (compspec.json:149-160), the same rule
            # as the collective runtime (runtime/site.py); patience counts validations
            ve = max(1, int(self.cfg.get("validation_epochs", 1)))
            if self.epoch % ve == 0:
                self.phase = "validation"
                return {"output": {"command": "validate", "apply_file": apply_file, "cfg": self.cfg}}
            last = self.epoch >= int(self.cfg.get("epochs", 1))
            self.rlogs["cumulative_total_duration"].append(time.time() - self.t_start)
            self.epoch += 1
            self.step = 0
            out = {"command": "train_round", "apply_file": apply_file, "cfg": self.cfg,
                   "epoch_end": True}
            if last:  # sites apply the last update and stop; the next round is the test
                self.phase = "test"
                out["stop"] = True
            return {"output": out}
        return {"output": {"command": "train_round", "apply_file": apply_file, "cfg": self.cfg}}

    @property
    def steps_per_epoch(self) -> int:
        bs = int(self.cfg.get("batch_size", 16))
        li = max(1, int(self.cfg.get("local_iterations", 1)))
        n = max(self.sizes[s][self.fold] for s in self.sites)
        return max(1, (n // bs) // li) if n >= bs else 1
