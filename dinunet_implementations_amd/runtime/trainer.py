"""Trainer base — the ``COINNTrainer`` role.

A task plugin subclasses :class:`NNTrainer` exactly like the reference's
``FreeSurferTrainer(COINNTrainer)`` (``comps/fs/__init__.py:42-63``): it registers modules in
``self.nn`` from ``_init_nn_model`` and implements ``iteration(batch)`` returning
``{'out', 'loss', 'averages', 'metrics', ...}``.  The base owns device placement, the flat
fp32 parameter buffer + fused Adam (``learning_rate``), evaluation, checkpoints with the
reference ``state_dict`` key names, and the fast training step.

Fast path: a plugin that implements ``forward_loss(x, y) -> (out, loss, pred)`` and
``score(out, pred)`` gets the HIP-graph-captured :class:`runtime.step.TrainStep`; any other
plugin trains through ``iteration`` eagerly (still on the fused kernels).
"""
from __future__ import annotations

import os
import random
from typing import Any, Dict, Optional

import numpy as np
import torch
import torch.nn as nn

from ..ops import FlatParams, FusedAdam
from ..utils.metrics import Averages, Metrics


def set_seed(seed: int):
    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)


class NNTrainer:
    def __init__(self, cache: Optional[Dict[str, Any]] = None, state: Optional[Dict[str, Any]] = None,
                 device=None, **kw):
        self.cache = cache if cache is not None else {}
        self.state = state if state is not None else {}
        dev = torch.device(device) if device is not None else torch.device("cpu")
        self.device = {"gpu": dev}
        self.nn: Dict[str, nn.Module] = {}
        self.flat: Optional[FlatParams] = None
        self.optimizer: Optional[FusedAdam] = None

    # ---- plugin hooks ------------------------------------------------------------------------
    def _init_nn_model(self):
        raise NotImplementedError

    def iteration(self, batch) -> Dict[str, Any]:
        """Default iteration for plugins that implement ``forward_loss``."""
        x = batch["inputs"].to(self.device["gpu"], non_blocking=True)
        y = batch["labels"].to(self.device["gpu"], non_blocking=True).long()
        out, loss, pred = self.forward_loss(x, y)
        m = self.new_metrics()
        m.add(self.score(out, pred), y)
        a = self.new_averages()
        a.add(loss.detach(), len(x))
        return {"out": out, "loss": loss, "averages": a, "metrics": m, "prediction": pred,
                "indices": batch.get("ix")}

    def forward_loss(self, x, y):  # pragma: no cover - optional fast path
        raise NotImplementedError

    def split_module(self):
        """A model with ``stem`` / ``body_loss`` / ``stem_parameters`` whose
        ``body_loss(stem(x), y)`` equals :meth:`forward_loss` (enables the split-capture
        training step), or None."""
        return None

    def score(self, out, pred):
        return pred

    # the column of ``out`` that :meth:`score` returns, when it is one (a device-fed epoch then
    # records it on the device every step: ``runtime.feed``); None keeps the host-fed loop
    score_column: Optional[int] = None

    @property
    def reference_math(self) -> bool:
        """``compute_path = "reference"``: every model runs the fp32 oracle math
        (``ops/reference.py``) instead of the fused kernels, on whatever device it lives on."""
        return str(self.cache.get("compute_path", "fused")) == "reference"

    @property
    def has_fast_path(self) -> bool:
        return type(self).forward_loss is not NNTrainer.forward_loss

    # ---- framework -----------------------------------------------------------------------------
    def new_metrics(self) -> Metrics:
        return Metrics(int(self.cache.get("num_class", 2)))

    def new_averages(self) -> Averages:
        return Averages()

    def init_nn(self, init_model: bool = True, init_optimizer: bool = True, seed: Optional[int] = None):
        if seed is not None:
            set_seed(seed)
        if init_model:
            self.nn = {}
            self._init_nn_model()
            for k in self.nn:
                self.nn[k] = self.nn[k].to(self.device["gpu"])
            if self.reference_math:
                for net in self.nn.values():
                    for m in net.modules():
                        if hasattr(m, "use_fused"):
                            m.use_fused = False
        if init_optimizer:
            self._init_optimizer()

    def parameters(self):
        for k in sorted(self.nn):
            yield from self.nn[k].parameters()

    def _init_optimizer(self, lr: Optional[float] = None):
        self.flat = FlatParams(self.parameters(), device=self.device["gpu"])
        lr = float(lr if lr is not None else self.cache.get("learning_rate", 1e-3))
        self.optimizer = FusedAdam(self.flat, lr=lr, weight_decay=float(self.cache.get("weight_decay", 0.0)))

    def modules(self) -> nn.Module:
        """All registered modules as one container (engines walk ``.modules()``)."""
        return nn.ModuleDict({k: v for k, v in self.nn.items()})

    def train(self):
        for m in self.nn.values():
            m.train()

    def eval(self):
        for m in self.nn.values():
            m.eval()

    @torch.no_grad()
    def evaluate(self, loader) -> Dict[str, Any]:
        """Run ``iteration`` over a loader; returns merged averages/metrics and predictions."""
        self.eval()
        avg, met = self.new_averages(), self.new_metrics()
        outs = []
        for x, y, ix in loader:
            it = self.iteration({"inputs": x, "labels": y, "ix": ix})
            avg.accumulate(it["averages"])
            met.accumulate(it["metrics"])
            outs.append(it["out"].detach())
        self.train()
        return {"averages": avg, "metrics": met, "out": torch.cat(outs) if outs else None}

    # ---- checkpoints (reference state_dict key names) -------------------------
    def checkpoint_state(self, **extra) -> Dict[str, Any]:
        st = {"models": {k: {n: t.detach().cpu() for n, t in v.state_dict().items()}
                         for k, v in self.nn.items()}}
        if self.optimizer is not None:
            st["optimizer"] = self.optimizer.state_dict()
        st.update(extra)
        return st

    # ---- random state (resume continues the same training curve) -------------
    def rng_state(self) -> Dict[str, Any]:
        """Every generator a training step draws from: torch (CPU, and the device's when on a
        GPU), Python ``random``, NumPy, and the device-side dropout counters of fused heads."""
        npst = np.random.get_state()
        st: Dict[str, Any] = {
            "torch": torch.get_rng_state(),
            "python": random.getstate(),
            "numpy": {"keys": torch.from_numpy(npst[1].astype(np.int64)), "pos": int(npst[2]),
                      "has_gauss": int(npst[3]), "cached": float(npst[4])},
        }
        dev = self.device["gpu"]
        if dev.type == "cuda":
            st["cuda"] = torch.cuda.get_rng_state(dev)
        heads = {}
        for k, m in self.nn.items():
            spec = getattr(m, "_head", None)
            if spec is not None and getattr(spec, "_rng", None) is not None:
                heads[k] = spec._rng.detach().cpu().clone()
        st["heads"] = heads
        return st

    def load_rng_state(self, st: Dict[str, Any]):
        torch.set_rng_state(st["torch"])
        py = st["python"]
        random.setstate((py[0], tuple(py[1]), py[2]))
        n = st["numpy"]
        np.random.set_state(("MT19937", n["keys"].numpy().astype(np.uint32), n["pos"],
                             n["has_gauss"], n["cached"]))
        dev = self.device["gpu"]
        if dev.type == "cuda" and "cuda" in st:
            torch.cuda.set_rng_state(st["cuda"], dev)
        for k, t in (st.get("heads") or {}).items():
            spec = getattr(self.nn.get(k), "head_spec", None)
            if spec is not None:
                spec().rng(dev).copy_(t.to(dev))

    def save_checkpoint(self, path: str, **extra):
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        tmp = path + ".tmp"
        torch.save(self.checkpoint_state(**extra), tmp)
        os.replace(tmp, path)

    def load_checkpoint(self, path: str, load_optimizer: bool = False) -> Dict[str, Any]:
        st = torch.load(path, map_location="cpu", weights_only=True)
        self.load_state(st, load_optimizer)
        return st

    def load_state(self, st: Dict[str, Any], load_optimizer: bool = False):
        models = st.get("models", st)
        for k, sd in models.items():
            if k in self.nn:
                self.nn[k].load_state_dict(sd)
        if load_optimizer and self.optimizer is not None and "optimizer" in st:
            self.optimizer.load_state_dict(st["optimizer"])
