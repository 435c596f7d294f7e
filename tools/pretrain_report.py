#!/usr/bin/env python3
"""Aggregate the per-run JSONs of ``tools/ica_pretrain_study.py`` (several GPU calls, one or more
seeds each) into one report: per run the test metrics, the federated best-validation (stopping)
epoch and the epochs to validation-AUC targets; per mode the mean +- sd stopping epoch next to
the reference's 68.5 / 42.7 (``/root/reference/NB.ipynb:200,209``), with a two-sided
Mann-Whitney U test of scratch vs pretrain.

    python tools/pretrain_report.py --tag r5_ica_pretrain [--dir profiles] [--out profiles/r5_ica_pretrain.md]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def epochs_to(curve, target):
    for i, v in enumerate(curve or []):
        if v is not None and v >= target:
            return i + 1
    return None


def msd(xs):
    xs = [float(x) for x in xs]
    if not xs:
        return "-"
    sd = statistics.stdev(xs) if len(xs) > 1 else 0.0
    return f"{statistics.mean(xs):.1f} ± {sd:.1f}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r5_ica_pretrain")
    ap.add_argument("--dir", default=os.path.join(ROOT, "profiles"))
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    runs = []
    for p in sorted(glob.glob(os.path.join(a.dir, f"{a.tag}_*_s*.json"))):
        with open(p) as f:
            r = json.load(f)
        if r.get("rc"):
            continue
        runs.append(r)
    if not runs:
        print("no runs", file=sys.stderr)
        return 1
    targets = (0.65, 0.70, 0.75)
    cfg = runs[0].get("config", {})
    md = [f"# ICA-LSTM pretrain -> finetune vs scratch: stopping epochs with a usable validation "
          f"set ({runs[0].get('sites')} sites, {runs[0].get('engine')}, {runs[0].get('device')})",
          "",
          f"Data: {runs[0].get('data')}.  Federated phase: batch {cfg.get('batch_size')}, up to "
          f"{cfg.get('epochs')} epochs, patience {cfg.get('patience')}, learning rate "
          f"{cfg.get('learning_rate')}.  Pretraining (largest site alone): batch "
          f"{next((r['config'].get('pretrain_batch_size') for r in runs if r['mode'] == 'pretrain'), '-')}, "
          f"learning rate "
          f"{next((r['config'].get('pretrain_learning_rate') for r in runs if r['mode'] == 'pretrain'), '-')}.  "
          "Every site holds >= 1,024 validation subjects (the global validation set is their "
          "union), so the validation AUC curve an early stop reads is not the ~190-subject one of "
          "round 4 (`profiles/r4_ica_pretrain.md`).",
          "",
          "| seed | mode | test AUC | test acc | test F1 | best-val (stopping) epoch | stopped at | "
          "pretrain best epoch | max val AUC | epochs to " + " / ".join(f"{t:.2f}" for t in targets)
          + " | wall s |",
          "|---:|---|---:|---:|---:|---:|---:|---:|---:|---|---:|"]
    for r in sorted(runs, key=lambda r: (r["seed"], r["mode"])):
        t = r["test"]
        cur = r.get("validation_auc_curve") or []
        et = " / ".join(str(epochs_to(cur, x) or "-") for x in targets)
        md.append(f"| {r['seed']} | {r['mode']} | {t['AUC']:.3f} | {t['Accuracy']:.3f} | "
                  f"{t['F1']:.3f} | {r['best_val_epoch']} | {r.get('stopped_epoch') or '-'} | "
                  f"{r.get('pretrain_best_val_epoch') or '-'} | {max(cur) if cur else float('nan'):.3f} | "
                  f"{et} | {r.get('wall_s')} |")
    md += ["", "| mode | runs | best-val (stopping) epoch, mean ± sd | median | test AUC, mean ± sd | "
               "reference mean stopping epoch (FS, `NB.ipynb:200,209`) |",
           "|---|---:|---:|---:|---:|---:|"]
    by = {}
    for r in runs:
        by.setdefault(r["mode"], []).append(r)
    refs = {"scratch": "68.5", "pretrain": "42.7"}
    for mode in ("scratch", "pretrain"):
        rs = by.get(mode, [])
        if not rs:
            continue
        ep = [r["best_val_epoch"] for r in rs]
        auc = [r["test"]["AUC"] for r in rs]
        sd = statistics.stdev(auc) if len(auc) > 1 else 0.0
        md.append(f"| {mode} | {len(rs)} | {msd(ep)} | {statistics.median(ep)} | "
                  f"{statistics.mean(auc):.3f} ± {sd:.3f} | {refs[mode]} |")
    if by.get("scratch") and by.get("pretrain"):
        try:
            from scipy.stats import mannwhitneyu
            a_ = [r["best_val_epoch"] for r in by["scratch"]]
            b_ = [r["best_val_epoch"] for r in by["pretrain"]]
            u = mannwhitneyu(a_, b_, alternative="two-sided")
            md += ["", f"Mann-Whitney U (stopping epoch, scratch vs pretrain): U = {u.statistic:.1f}, "
                       f"two-sided p = {u.pvalue:.3g} over {len(a_)} + {len(b_)} runs."]
        except Exception as e:  # scipy missing / degenerate samples
            md += ["", f"(no U test: {e})"]
    text = "\n".join(md) + "\n"
    out = a.out or os.path.join(a.dir, f"{a.tag}.md")
    with open(out, "w") as f:
        f.write(text)
    print(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
