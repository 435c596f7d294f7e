"""Reproduce the reference's published FreeSurfer numbers on its own shipped data (BASELINE config 1).

Runs ``datasets/test_fsl`` (the reference's 5-site simulator data, read-only) through
``python -m dinunet_implementations_amd.run`` as one gloo process per site on the CPU, for every
aggregation engine, 10-fold, from scratch and with ``pretrain=true``, with the compspec defaults
(epochs 101, patience 35, batch 16, lr 1e-3).  Per run it writes
``profiles/fs_parity_<S>site_<engine>_<mode>.json`` (global fold table + summary from
``utils/analysis.fold_report``) and a combined ``profiles/fs_parity.md`` next to the reference's
numbers:

* test AUC per engine, fold 0 of run ``fs-lstm_2S``: powerSGD 0.907, rankDAD 0.854, dSGD 0.814
  (``/root/reference/nnlogs.ipynb:48,52,56``);
* mean stopping (best-validation) epoch over 10 folds: scratch 68.5, pretrain 42.7
  (``/root/reference/NB.ipynb:200,209``);
* 10-fold test accuracy / F1 box plots (``assets/perf_box.png``, medians ~0.917 / ~0.92-0.93).

Usage: ``python tools/fs_parity.py [--sites 2 5] [--engines dSGD rankDAD powerSGD]
[--modes scratch pretrain] [--folds 10] [--pretrain-epochs 51]``
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dinunet_implementations_amd.utils import analysis  # noqa: E402

REF = {
    "auc_fold0": {"powerSGD": 0.90702, "rankDAD": 0.85351, "dSGD": 0.81404},
    "stop_epoch_mean": {"scratch": 68.5, "pretrain": 42.7},
    "accuracy_median": {"scratch": 0.917, "pretrain": 0.917},
    "f1_median": {"scratch": 0.92, "pretrain": 0.93},
}
DATA = "/root/reference/datasets/test_fsl"


def run_one(sites, engine, mode, folds, pre_epochs, out, port, extra=()):
    sets = [f"agg_engine={engine}", f"num_folds={folds}"]
    if mode == "pretrain":
        sets += ["pretrain=true", json.dumps({"epochs": pre_epochs, "learning_rate": 1e-3,
                                              "batch_size": 16, "patience": 51,
                                              "validation_epochs": 1}).join(["pretrain_args=", ""])]
    sets += list(extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           str(sites), "--master-addr", "127.0.0.1", "--master-port", str(port),
           "-m", "dinunet_implementations_amd.run", "--data-path", DATA, "--out", out,
           "--device", "cpu"]
    for s in sets:
        cmd += ["--set", s]
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    t0 = time.time()
    with open(out + ".log", "w") as f:
        rc = subprocess.call(cmd, stdout=f, stderr=subprocess.STDOUT, env=env)
    return rc, time.time() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sites", type=int, nargs="+", default=[2, 5])
    ap.add_argument("--engines", nargs="+", default=["dSGD", "rankDAD", "powerSGD"])
    ap.add_argument("--modes", nargs="+", default=["scratch", "pretrain"])
    ap.add_argument("--folds", type=int, default=10)
    ap.add_argument("--pretrain-epochs", type=int, default=51)
    ap.add_argument("--work", default="/tmp/fs_parity")
    ap.add_argument("--profiles", default=os.path.join(ROOT, "profiles"))
    a = ap.parse_args()
    os.makedirs(a.work, exist_ok=True)
    rows = []
    port = 29700
    for S in a.sites:
        for eng in a.engines:
            for mode in a.modes:
                out = os.path.join(a.work, f"{S}site_{eng}_{mode}")
                subprocess.call(["rm", "-rf", out])
                port += 1
                rc, wall = run_one(S, eng, mode, a.folds, a.pretrain_epochs, out, port)
                if rc != 0:
                    print(f"FAILED {out} rc={rc}; see {out}.log", flush=True)
                    rows.append({"sites": S, "engine": eng, "mode": mode, "rc": rc})
                    continue
                fr = analysis.fold_report(out)
                fold0 = next((f for f in fr["folds"] if f["fold"] == 0), {})
                pre = [f.get("pretrain_best_val_epoch") for f in analysis.fold_report(out, "local0")["folds"]]
                rec = {"sites": S, "engine": eng, "mode": mode, "folds": a.folds, "rc": rc,
                       "wall_s": round(wall, 1), "data": DATA + " (reference's shipped FS data)",
                       "config": {"epochs": 101, "patience": 35, "batch_size": 16,
                                  "learning_rate": 1e-3, "split": f"{a.folds}-fold",
                                  "pretrain_epochs": a.pretrain_epochs if mode == "pretrain" else 0},
                       "fold0_test_auc": fold0.get("AUC"), "summary": fr["summary"],
                       "folds_table": fr["folds"],
                       "reference": {"fold0_test_auc": REF["auc_fold0"].get(eng),
                                     "stop_epoch_mean": REF["stop_epoch_mean"][mode]}}
                if mode == "pretrain":
                    rec["pretrain_best_val_epochs"] = pre
                with open(os.path.join(a.profiles, f"fs_parity_{S}site_{eng}_{mode}.json"), "w") as f:
                    json.dump(rec, f, indent=1)
                s = fr["summary"]
                print(f"{S} sites {eng:8s} {mode:8s} fold0 AUC {fold0.get('AUC', float('nan')):.4f} "
                      f"mean AUC {s['AUC']['mean']:.4f} acc med {s['Accuracy']['median']:.4f} "
                      f"F1 med {s['F1']['median']:.4f} stop epoch mean {s['best_val_epoch']['mean']:.1f} "
                      f"({wall:.0f} s)", flush=True)
                rows.append(rec)
    md = ["# FS-Classification parity on the reference's `datasets/test_fsl` (CPU, gloo, 1 process/site)", "",
          "Reference: fold-0 test AUC powerSGD 0.907 / rankDAD 0.854 / dSGD 0.814 (`nnlogs.ipynb:48,52,56`, "
          "run `fs-lstm_2S`, data unstated); mean stopping epoch 10-fold scratch 68.5 / pretrain 42.7 "
          "(`NB.ipynb:200,209`); accuracy median ~0.917, F1 median ~0.92 / 0.93 (`assets/perf_box.png`).", "",
          "| sites | engine | mode | fold-0 AUC (ref) | mean AUC | median acc | median F1 | mean stop epoch (ref) | wall s |",
          "|---:|---|---|---:|---:|---:|---:|---:|---:|"]
    for r in rows:
        if r.get("rc"):
            md.append(f"| {r['sites']} | {r['engine']} | {r['mode']} | FAILED rc={r['rc']} | | | | | |")
            continue
        s = r["summary"]
        md.append(f"| {r['sites']} | {r['engine']} | {r['mode']} | {r['fold0_test_auc']:.3f} "
                  f"({r['reference']['fold0_test_auc']}) | {s['AUC']['mean']:.3f} | "
                  f"{s['Accuracy']['median']:.3f} | {s['F1']['median']:.3f} | "
                  f"{s['best_val_epoch']['mean']:.1f} ({r['reference']['stop_epoch_mean']}) | {r['wall_s']} |")
    with open(os.path.join(a.profiles, "fs_parity.md"), "w") as f:
        f.write("\n".join(md) + "\n")
    print("\n".join(md))
    return 0 if all(not r.get("rc") for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
