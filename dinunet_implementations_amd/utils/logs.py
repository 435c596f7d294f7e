"""Run outputs with the reference layout and keys.

``<out>/<site>/<task_id>/fold_k/logs.json`` per site (``local0`` .. ``localN-1``) and
``<out>/remote/<task_id>/fold_k/logs.json`` for the aggregated view (what the reference's
remote wrote, ``NB.ipynb:851,885``), plus ``test_metrics.csv`` (columns read by the reference
notebook as Accuracy / F1 at ``NB.ipynb:99-100``) and a zip of the remote results
(``nnlogs.ipynb:77-84``).  Durations follow ``coinstac_dinunet.utils.duration``: lists of
seconds appended per iteration under ``time_spent_on_computation`` /
``cumulative_total_duration`` (``local.py:51-52``).
"""
from __future__ import annotations

import csv
import json
import os
import time
import zipfile
from typing import Any, Dict, List, Optional

TEST_HEADER = ["Loss", "Accuracy", "F1", "Precision", "Recall", "AUC"]


def duration(cache: Dict[str, Any], t0: float, key: str) -> float:
    """Reference ``coinstac_dinunet.utils.duration``: append elapsed seconds to ``cache[key]``."""
    dt = time.time() - t0
    cache.setdefault(key, []).append(dt)
    return dt


def fold_dir(out_dir: str, site: str, task_id: str, fold: int) -> str:
    d = os.path.join(out_dir, site, str(task_id), f"fold_{fold}")
    os.makedirs(d, exist_ok=True)
    return d


def _jsonable(v):
    if isinstance(v, dict):
        return {k: _jsonable(x) for k, x in v.items() if not str(k).startswith("_")}
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    try:
        return float(v)
    except Exception:
        return str(v)


def write_logs(d: str, logs: Dict[str, Any]) -> str:
    p = os.path.join(d, "logs.json")
    tmp = p + ".tmp"
    with open(tmp, "w") as f:
        json.dump(_jsonable(logs), f, indent=1)
    os.replace(tmp, p)
    return p


def write_test_metrics(d: str, rows: List[List[float]], header: Optional[List[str]] = None) -> str:
    p = os.path.join(d, "test_metrics.csv")
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header or TEST_HEADER)
        for r in rows:
            w.writerow([round(float(x), 6) for x in r])
    return p


def test_row(loss: float, scores: Dict[str, float]) -> List[float]:
    return [loss, scores["accuracy"], scores["f1"], scores["precision"], scores["recall"],
            scores["auc"]]


def zip_results(src_dir: str, zip_path: str) -> str:
    with zipfile.ZipFile(zip_path, "w", zipfile.ZIP_DEFLATED) as z:
        for root, _, files in os.walk(src_dir):
            for fn in files:
                full = os.path.join(root, fn)
                if os.path.abspath(full) == os.path.abspath(zip_path):
                    continue
                z.write(full, os.path.relpath(full, src_dir))
    return zip_path
