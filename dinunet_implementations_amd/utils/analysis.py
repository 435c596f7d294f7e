"""Result analysis over run outputs (the reference's notebooks as a library + CLI).

The reference analyses its runs by hand in two notebooks; this module computes the same numbers
from the ``logs.json`` / ``test_metrics.csv`` tree this framework (or the COINSTAC simulator
adapter) writes:

* ``engine_report``   - per run: aggregation engine, global test loss / AUC, cumulative and
                        compute-only wall time of sites and remote (``nnlogs.ipynb:64-92``).
* ``fold_report``     - per fold: best-validation (stopping) epoch and test metrics; summary
                        statistics (mean / median / quartiles / range) of Accuracy, F1 and the
                        stopping epoch across folds - the numbers behind the committed box
                        plots (``NB.ipynb:95-209``, ``assets/perf_box.png``, ``pretrain_box.png``).
* ``iteration_report``- mean per-iteration duration per site and for the remote
                        (``NB.ipynb:851-912``).
* ``compare``         - two fold reports side by side (scratch vs pretrain, ``NB.ipynb:188-209``).

CLI: ``python -m dinunet_implementations_amd.utils.analysis <out_dir> [<out_dir_b>]``
"""
from __future__ import annotations

import csv
import glob
import json
import os
import statistics
import sys
import zipfile
from typing import Any, Dict, List, Optional


def _load(path: str) -> Dict[str, Any]:
    with open(path) as f:
        return json.load(f)


def find_logs(out_dir: str, site: Optional[str] = None) -> List[str]:
    """All ``logs.json`` under ``out_dir`` (optionally of one site: ``local0`` / ``remote``)."""
    pat = os.path.join(out_dir, site or "*", "**", "logs.json")
    return sorted(glob.glob(pat, recursive=True))


def _fold_of(path: str) -> int:
    for part in reversed(path.split(os.sep)):
        if part.startswith("fold_"):
            try:
                return int(part[5:])
            except ValueError:
                pass
    return 0


def _site_of(out_dir: str, path: str) -> str:
    rel = os.path.relpath(path, out_dir).split(os.sep)
    return rel[0] if rel else "?"


def summarize(values: List[float]) -> Dict[str, float]:
    v = sorted(float(x) for x in values if x is not None)
    if not v:
        return {}
    q = statistics.quantiles(v, n=4) if len(v) >= 2 else [v[0], v[0], v[0]]
    return {"n": len(v), "mean": statistics.fmean(v), "median": statistics.median(v),
            "q1": q[0], "q3": q[2], "min": v[0], "max": v[-1]}


def _test_metrics(fold_dir: str, logs: Dict[str, Any]) -> Dict[str, float]:
    p = os.path.join(fold_dir, "test_metrics.csv")
    if os.path.exists(p):
        with open(p, newline="") as f:
            rows = list(csv.reader(f))
        if len(rows) >= 2:
            return {h: float(x) for h, x in zip(rows[0], rows[1])}
    header = logs.get("test_header") or ["Loss", "Accuracy", "F1", "Precision", "Recall", "AUC"]
    vals = logs.get("test_metrics") or []
    return {h: float(x) for h, x in zip(header, vals)}


def fold_report(out_dir: str, site: str = "remote") -> Dict[str, Any]:
    """Per-fold stopping epoch + test metrics of one site (default: the global/remote view)."""
    folds = []
    for p in find_logs(out_dir, site):
        logs = _load(p)
        m = _test_metrics(os.path.dirname(p), logs)
        folds.append({"fold": _fold_of(p), "best_val_epoch": logs.get("best_val_epoch"),
                      "pretrain_best_val_epoch": logs.get("pretrain_best_val_epoch"), **m})
    folds.sort(key=lambda r: r["fold"])
    summary = {k: summarize([f.get(k) for f in folds])
               for k in ("Accuracy", "F1", "AUC", "Loss", "best_val_epoch")}
    return {"site": site, "folds": folds, "summary": summary}


def engine_report(out_dir: str) -> List[Dict[str, Any]]:
    """One row per (site, fold): engine, test loss/AUC, cumulative and compute seconds."""
    rows = []
    for p in find_logs(out_dir):
        d = os.path.dirname(p)
        logs = _load(p)
        m = _test_metrics(d, logs)
        rows.append({
            "site": _site_of(out_dir, p), "fold": _fold_of(p), "agg_engine": logs.get("agg_engine"),
            "test_loss": m.get("Loss"), "test_auc": m.get("AUC"),
            "cumulative_total_s": sum(logs.get("cumulative_total_duration", []) or []),
            "computation_s": sum(logs.get("time_spent_on_computation", []) or []),
            "fold_duration_s": logs.get("fold_duration"),
        })
    return rows


def iteration_report(out_dir: str) -> Dict[str, Dict[str, float]]:
    """Mean / median per-iteration duration (seconds) per site and for the remote."""
    out = {}
    for p in find_logs(out_dir):
        logs = _load(p)
        site = _site_of(out_dir, p)
        key = "remote_iter_duration" if site == "remote" else "local_iter_duration"
        v = logs.get(key) or logs.get("local_iter_duration") or []
        if v:
            out[f"{site}/fold_{_fold_of(p)}"] = summarize(v)
    return out


def extract_zips(out_dir: str) -> List[str]:
    """Unpack the remote results zips next to themselves (``nnlogs.ipynb:77-84``)."""
    done = []
    for z in glob.glob(os.path.join(out_dir, "**", "*.zip"), recursive=True):
        dst = os.path.join(os.path.dirname(z), "GLOBAL_res")
        os.makedirs(dst, exist_ok=True)
        with zipfile.ZipFile(z) as f:
            for name in f.namelist():
                target = os.path.realpath(os.path.join(dst, name))
                if not target.startswith(os.path.realpath(dst) + os.sep):
                    raise ValueError(f"unsafe path in {z}: {name}")
            f.extractall(dst)
        done.append(dst)
    return done


def compare(out_a: str, out_b: str, site: str = "remote") -> Dict[str, Any]:
    a, b = fold_report(out_a, site), fold_report(out_b, site)
    return {"a": a["summary"], "b": b["summary"]}


def _fmt_summary(s: Dict[str, Dict[str, float]]) -> str:
    lines = ["| metric | n | mean | median | q1 | q3 | min | max |", "|---|---:|---:|---:|---:|---:|---:|---:|"]
    for k, v in s.items():
        if v:
            lines.append(f"| {k} | {v['n']} | {v['mean']:.4f} | {v['median']:.4f} | {v['q1']:.4f} | "
                         f"{v['q3']:.4f} | {v['min']:.4f} | {v['max']:.4f} |")
    return "\n".join(lines)


def report_markdown(out_dir: str) -> str:
    parts = [f"# Run report: `{out_dir}`", ""]
    fr = fold_report(out_dir)
    if fr["folds"]:
        parts += ["## Folds (global view)", "", "| fold | best_val_epoch | Loss | Accuracy | F1 | AUC |",
                  "|---:|---:|---:|---:|---:|---:|"]
        for f in fr["folds"]:
            parts.append(f"| {f['fold']} | {f.get('best_val_epoch')} | {f.get('Loss', float('nan')):.4f} | "
                         f"{f.get('Accuracy', float('nan')):.4f} | {f.get('F1', float('nan')):.4f} | "
                         f"{f.get('AUC', float('nan')):.4f} |")
        parts += ["", _fmt_summary(fr["summary"]), ""]
    er = engine_report(out_dir)
    if er:
        parts += ["## Engines / time", "", "| site | fold | engine | test loss | test AUC | cumulative s | compute s |",
                  "|---|---:|---|---:|---:|---:|---:|"]
        for r in er:
            parts.append(f"| {r['site']} | {r['fold']} | {r['agg_engine']} | {r['test_loss']} | {r['test_auc']} | "
                         f"{r['cumulative_total_s']:.2f} | {r['computation_s']:.2f} |")
        parts.append("")
    ir = iteration_report(out_dir)
    if ir:
        parts += ["## Per-iteration duration (s)", "", "| site/fold | n | mean | median |", "|---|---:|---:|---:|"]
        for k, v in ir.items():
            parts.append(f"| {k} | {v['n']} | {v['mean']:.5f} | {v['median']:.5f} |")
    return "\n".join(parts) + "\n"


def plot_boxes(experiments: Dict[str, List[Dict[str, Any]]], perf_png: str, epoch_png: str,
               scores=("Accuracy", "F1")) -> None:
    """The reference notebook's two figures (``NB.ipynb:131-189`` -> ``assets/perf_box.png`` /
    ``assets/pretrain_box.png``) from per-fold tables (``fold_report(...)["folds"]``), one entry
    per experiment label (e.g. ``{"scratch": ..., "pretrain": ...}``): test scores per
    experiment as box plots with means, and the stopping (best-validation) epoch per experiment.
    matplotlib only (the notebook used seaborn)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    labels = list(experiments)
    fig, ax = plt.subplots(figsize=(10, 6))
    width = 0.8 / max(len(scores), 1)
    for si, sc in enumerate(scores):
        data = [[f[sc] for f in experiments[e] if f.get(sc) is not None] for e in labels]
        pos = [i + (si - (len(scores) - 1) / 2) * width for i in range(len(labels))]
        bp = ax.boxplot(data, positions=pos, widths=width * 0.8, showmeans=True,
                        patch_artist=True)
        for b in bp["boxes"]:
            b.set_facecolor(f"C{si}")
            b.set_alpha(0.6)
        ax.plot([], [], color=f"C{si}", linewidth=8, alpha=0.6, label=sc)
    ax.set_xticks(range(len(labels)))
    ax.set_xticklabels(labels)
    ax.set_ylabel("Value")
    ax.legend()
    ax.set_title("Test performance, scratch vs with pre-training, per-fold box plot (higher is better)")
    fig.tight_layout()
    fig.savefig(perf_png)
    plt.close(fig)
    fig, ax = plt.subplots(figsize=(8, 6))
    data = [[f["best_val_epoch"] for f in experiments[e] if f.get("best_val_epoch") is not None]
            for e in labels]
    ax.boxplot(data, widths=0.3, showmeans=True)
    ax.set_xticks(range(1, len(labels) + 1))
    ax.set_xticklabels(labels)
    ax.set_ylabel("Stopped on epoch")
    ax.set_title("Train from scratch vs with pre-training, per-fold box plot (lower is better)")
    fig.tight_layout()
    fig.savefig(epoch_png)
    plt.close(fig)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        print(__doc__)
        return 2
    if len(argv) >= 2:
        c = compare(argv[0], argv[1])
        print("# A:", argv[0])
        print(_fmt_summary(c["a"]))
        print("\n# B:", argv[1])
        print(_fmt_summary(c["b"]))
        return 0
    print(report_markdown(argv[0]))
    return 0


if __name__ == "__main__":
    sys.exit(main())
