"""Per-phase step timers on HIP events (fwd/bwd, comm, optimizer).

Events are recorded on the current stream around each phase and resolved lazily (one
synchronize when a summary is requested), so timing does not serialize the step.  Enabled by
``DINUNET_PHASE_TIMERS=1`` or ``TrainStep(..., timers=PhaseTimer())``; the site runtime copies
``summary()`` into ``logs.json`` under ``phase_ms``.
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, List, Tuple

import torch


def enabled_by_env() -> bool:
    return os.environ.get("DINUNET_PHASE_TIMERS", "0") == "1"


class PhaseTimer:
    def __init__(self, max_pending: int = 4096):
        self._pending: List[Tuple[str, "torch.cuda.Event", "torch.cuda.Event"]] = []
        self._tot: Dict[str, float] = {}
        self._cnt: Dict[str, int] = {}
        self.max_pending = max_pending

    @contextlib.contextmanager
    def phase(self, name: str):
        if not torch.cuda.is_available():
            yield
            return
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        try:
            yield
        finally:
            b.record()
            self._pending.append((name, a, b))
            if len(self._pending) >= self.max_pending:
                self._resolve()

    def _resolve(self):
        if not self._pending:
            return
        self._pending[-1][2].synchronize()
        for name, a, b in self._pending:
            self._tot[name] = self._tot.get(name, 0.0) + a.elapsed_time(b)
            self._cnt[name] = self._cnt.get(name, 0) + 1
        self._pending.clear()

    def summary(self) -> Dict[str, Dict[str, float]]:
        """``{phase: {"mean_ms": ..., "total_ms": ..., "count": ...}}``"""
        self._resolve()
        return {k: {"mean_ms": self._tot[k] / self._cnt[k], "total_ms": self._tot[k],
                     "count": self._cnt[k]} for k in self._tot}

    def reset(self):
        self._pending.clear()
        self._tot.clear()
        self._cnt.clear()


class _NullTimer:
    @contextlib.contextmanager
    def phase(self, name: str):
        yield

    def summary(self):
        return {}

    def reset(self):
        pass


NULL = _NullTimer()
