"""Loss averages and classification metrics that merge across sites.

The reference trainers call ``new_averages().add(loss.item(), n)`` and
``new_metrics().add(pred_or_score, labels)`` (``comps/fs/__init__.py:58-61``,
``comps/icalstm/__init__.py:64-68``); the remote then computes *global* scores from merged
per-site state, not by averaging site AUCs.  Here both objects keep device tensors (no per-batch
``.item()`` host sync), serialise to plain dicts, and merge exactly:

* :class:`Averages`  weighted running mean (sum, count).
* :class:`Metrics`   confusion counts for accuracy / precision / recall / F1 + the raw
  ``(score, label)`` pairs for an exact global ROC-AUC.  FS feeds hard argmax labels (its AUC is
  the hard-label AUC, quirk A10), ICA feeds ``prob[:, 1]``.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch


class Averages:
    def __init__(self):
        self._sum = 0.0
        self._n = 0
        self._dev_sum: Optional[torch.Tensor] = None

    def add(self, value, n: int = 1):
        if isinstance(value, torch.Tensor):
            v = value.detach().float() * n
            self._dev_sum = v if self._dev_sum is None else self._dev_sum + v
        else:
            self._sum += float(value) * n
        self._n += int(n)
        return self

    def accumulate(self, other: "Averages"):
        self._flush()
        other._flush()
        self._sum += other._sum
        self._n += other._n
        return self

    def _flush(self):
        if self._dev_sum is not None:
            self._sum += float(self._dev_sum)
            self._dev_sum = None

    @property
    def count(self) -> int:
        return self._n

    @property
    def average(self) -> float:
        self._flush()
        return self._sum / self._n if self._n else 0.0

    def get(self) -> List[float]:
        return [round(self.average, 6)]

    def to_state(self) -> Dict:
        self._flush()
        return {"sum": self._sum, "n": self._n}

    @classmethod
    def from_state(cls, st: Dict) -> "Averages":
        a = cls()
        a._sum, a._n = float(st["sum"]), int(st["n"])
        return a

    def reset(self):
        self.__init__()


def roc_auc(scores: np.ndarray, labels: np.ndarray) -> float:
    """Exact ROC-AUC (Mann-Whitney U with average ranks for ties).  0.5 if one class is absent.
    Runs in the C++ host library when built (``data/native.py``); this Python body is the
    fallback and the test oracle (:func:`roc_auc_py`)."""
    from ..data import native
    v = native.roc_auc(scores, labels)
    return v if v is not None else roc_auc_py(scores, labels)


def roc_auc_py(scores: np.ndarray, labels: np.ndarray) -> float:
    scores = np.asarray(scores, dtype=np.float64).ravel()
    labels = np.asarray(labels).ravel().astype(np.int64)
    pos = labels == 1
    n_pos = int(pos.sum())
    n_neg = int(labels.size - n_pos)
    if n_pos == 0 or n_neg == 0:
        return 0.5
    order = np.argsort(scores, kind="mergesort")
    s = scores[order]
    ranks = np.empty(s.size, dtype=np.float64)
    i = 0
    while i < s.size:
        j = i
        while j + 1 < s.size and s[j + 1] == s[i]:
            j += 1
        ranks[i:j + 1] = 0.5 * (i + j) + 1.0
        i = j + 1
    r = np.empty_like(ranks)
    r[order] = ranks
    return float((r[pos].sum() - n_pos * (n_pos + 1) / 2.0) / (n_pos * n_neg))


class Metrics:
    """Binary (or multiclass hard-label) classification metrics with exact merge."""

    def __init__(self, num_class: int = 2, threshold: float = 0.5):
        self.num_class = num_class
        self.threshold = threshold
        self._scores: List[torch.Tensor] = []
        self._labels: List[torch.Tensor] = []

    def add(self, pred_or_score: torch.Tensor, labels: torch.Tensor):
        s = pred_or_score.detach().reshape(-1)
        self._scores.append(s.float() if s.is_floating_point() else s.long().float())
        self._labels.append(labels.detach().reshape(-1).long())
        return self

    def accumulate(self, other: "Metrics"):
        self._scores.extend(other._scores)
        self._labels.extend(other._labels)
        return self

    # raw tensors (device) — what sites all-gather for the global score
    def tensors(self):
        if not self._scores:
            return torch.zeros(0), torch.zeros(0, dtype=torch.long)
        return torch.cat(self._scores), torch.cat(self._labels)

    @classmethod
    def from_tensors(cls, scores: torch.Tensor, labels: torch.Tensor, num_class: int = 2):
        m = cls(num_class)
        m._scores = [scores.detach()]
        m._labels = [labels.detach().long()]
        return m

    def _np(self):
        s, l = self.tensors()
        return s.cpu().numpy(), l.cpu().numpy()

    def _hard(self, s: np.ndarray) -> np.ndarray:
        if self.num_class == 2:
            return (s >= self.threshold).astype(np.int64) if not np.all(np.mod(s, 1) == 0) \
                else s.astype(np.int64)
        return s.astype(np.int64)

    def confusion(self):
        s, l = self._np()
        p = self._hard(s)
        tp = int(((p == 1) & (l == 1)).sum())
        tn = int(((p == 0) & (l == 0)).sum())
        fp = int(((p == 1) & (l == 0)).sum())
        fn = int(((p == 0) & (l == 1)).sum())
        return tp, fp, tn, fn

    def scores(self) -> Dict[str, float]:
        s, l = self._np()
        if s.size == 0:
            return {"accuracy": 0.0, "precision": 0.0, "recall": 0.0, "f1": 0.0, "auc": 0.5}
        tp, fp, tn, fn = self.confusion()
        acc = (tp + tn) / max(tp + tn + fp + fn, 1)
        prec = tp / (tp + fp) if tp + fp else 0.0
        rec = tp / (tp + fn) if tp + fn else 0.0
        f1 = 2 * prec * rec / (prec + rec) if prec + rec else 0.0
        return {"accuracy": acc, "precision": prec, "recall": rec, "f1": f1,
                "auc": roc_auc(s, l)}

    @property
    def auc(self):
        return self.scores()["auc"]

    def get(self, keys: Sequence[str] = ("auc",)) -> List[float]:
        sc = self.scores()
        return [round(sc[k], 6) for k in keys]

    def to_state(self) -> Dict:
        s, l = self._np()
        return {"scores": s.tolist(), "labels": l.tolist(), "num_class": self.num_class}

    @classmethod
    def from_state(cls, st: Dict) -> "Metrics":
        return cls.from_tensors(torch.tensor(st["scores"], dtype=torch.float32),
                                torch.tensor(st["labels"], dtype=torch.long),
                                int(st.get("num_class", 2)))

    def reset(self):
        self._scores.clear()
        self._labels.clear()


def merge_states(states: Sequence[Dict]) -> Metrics:
    m = Metrics(int(states[0].get("num_class", 2)) if states else 2)
    for st in states:
        m.accumulate(Metrics.from_state(st))
    return m


def metric_value(scores: Dict[str, float], name: str) -> float:
    name = name.lower()
    aliases = {"acc": "accuracy", "f1_score": "f1", "auroc": "auc", "roc_auc": "auc"}
    return float(scores[aliases.get(name, name)])


def improved(new: float, best: Optional[float], direction: str = "maximize", eps: float = 1e-9) -> bool:
    if best is None:
        return True
    return new > best + eps if direction.startswith("max") else new < best - eps
