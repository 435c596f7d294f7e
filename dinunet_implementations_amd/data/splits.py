"""Deterministic per-site splits: ratio, k-fold, or user split files.

* ``split_ratio`` (``compspec.json:205-216``): shuffled with the site seed, cut into
  train/validation/test (2 entries -> train/validation, no test).
* ``num_folds`` (``compspec.json:217-224``): k folds; fold i uses fold i as test, fold (i+1) % k
  as validation and the rest as train.  Runs are sequential ``fold_0 .. fold_{k-1}``.
* ``split_files``: JSON files ``{"train": [...], "validation": [...], "test": [...]}`` (the
  reference's ``split_files`` key); entries are sample ids as returned by ``list_files``.
"""
from __future__ import annotations

import json
import os
import random
from typing import Any, Dict, List, Sequence


def _shuffled(items: Sequence[Any], seed: int) -> List[Any]:
    it = list(items)
    random.Random(seed).shuffle(it)
    return it


def ratio_split(items: Sequence[Any], ratio: Sequence[float], seed: int = 0) -> Dict[str, List[Any]]:
    it = _shuffled(items, seed)
    n = len(it)
    r = list(ratio)
    n_tr = int(round(r[0] * n))
    n_va = int(round(r[1] * n)) if len(r) > 1 else 0
    if len(r) == 2:
        n_va = n - n_tr
    n_tr = min(n_tr, n)
    n_va = min(n_va, n - n_tr)
    return {"train": it[:n_tr], "validation": it[n_tr:n_tr + n_va], "test": it[n_tr + n_va:]}


def kfold_splits(items: Sequence[Any], k: int, seed: int = 0) -> List[Dict[str, List[Any]]]:
    if k < 3:
        # fold i is the test set and fold i+1 the validation set: with k=2 nothing is left to
        # train on
        raise ValueError("num_folds must be >= 3")
    it = _shuffled(items, seed)
    folds = [it[i::k] for i in range(k)]
    out = []
    for i in range(k):
        te, va = folds[i], folds[(i + 1) % k]
        tr = [x for j, f in enumerate(folds) if j not in (i, (i + 1) % k) for x in f]
        out.append({"train": tr, "validation": va, "test": te})
    return out


def load_split_files(paths: Sequence[str], base: str = ".") -> List[Dict[str, List[Any]]]:
    res = []
    for p in paths:
        fp = p if os.path.isabs(p) else os.path.join(base, p)
        with open(fp) as f:
            d = json.load(f)
        res.append({"train": list(d.get("train", [])),
                    "validation": list(d.get("validation", d.get("val", []))),
                    "test": list(d.get("test", []))})
    return res


def make_splits(items: Sequence[Any], cfg: Dict[str, Any], seed: int, base: str = ".") -> List[Dict[str, List[Any]]]:
    if cfg.get("split_files"):
        return load_split_files(cfg["split_files"], base)
    if cfg.get("num_folds"):
        return kfold_splits(items, int(cfg["num_folds"]), seed)
    return [ratio_split(items, cfg.get("split_ratio") or [0.8, 0.1, 0.1], seed)]
