#!/usr/bin/env python3
"""BASELINE config 5: ICA-LSTM pretrain -> finetune vs from scratch, many sites, large-batch
pretraining (reference ``compspec.json:120-148``: ``pretrain`` + ``pretrain_args``).

Generates a site-shifted hard ICA cohort (``data.synthetic.ica_cohort_hard``) in the reference
site layout -- one large site (the pretraining site) and ``--sites - 1`` small ones -- then runs the
production launcher (``python -m dinunet_implementations_amd.run``, one process per site) twice:

* ``scratch``: federated training from a common random init;
* ``pretrain``: the largest site first trains alone with ``pretrain_args`` (large batch), its best
  weights become the common init, then the same federated training.

Per mode it records the global test AUC / accuracy / F1, the federated best-validation
(stopping) epoch, the pretraining epochs, and wall time, as
``profiles/ica_pretrain_<mode>.json`` plus ``profiles/ica_pretrain.md``.  On one GPU the site
processes share it over gloo (``DINUNET_BACKEND=gloo``): epoch counts and AUCs are what this
measures; the per-epoch wall time includes host-staged gloo collectives, not RCCL over xGMI.

    python tools/ica_pretrain_study.py --sites 8 --big 4096 --small 256 --device cuda
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dinunet_implementations_amd.data.synthetic import make_ica_sites  # noqa: E402
from dinunet_implementations_amd.utils import analysis  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sites", type=int, default=8)
    ap.add_argument("--big", type=int, default=4096, help="subjects at the pretraining site")
    ap.add_argument("--small", type=int, default=256, help="subjects at every other site")
    ap.add_argument("--signal", type=float, default=0.35)
    ap.add_argument("--label-noise", type=float, default=0.1)
    ap.add_argument("--engine", default="dSGD")
    ap.add_argument("--modes", nargs="+", default=["scratch", "pretrain"])
    ap.add_argument("--epochs", type=int, default=40)
    ap.add_argument("--patience", type=int, default=12)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--pretrain-batch", type=int, default=512)
    ap.add_argument("--pretrain-epochs", type=int, default=60)
    ap.add_argument("--pretrain-patience", type=int, default=15)
    ap.add_argument("--hidden", type=int, default=384)
    ap.add_argument("--input-size", type=int, default=256)
    ap.add_argument("--comps", type=int, default=100)
    ap.add_argument("--temporal", type=int, default=980)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--work", default="/tmp/ica_pretrain")
    ap.add_argument("--profiles", default=os.path.join(ROOT, "profiles"))
    ap.add_argument("--tag", default="ica_pretrain")
    ap.add_argument("--logdir", default=None, help="per-mode launcher logs (default: --work)")
    ap.add_argument("--set", action="append", default=[], help="extra run.py --set items")
    ap.add_argument("--lr", type=float, default=1e-3, help="federated learning_rate")
    ap.add_argument("--pretrain-lr", type=float, default=1e-3)
    ap.add_argument("--split", default="0.8,0.1,0.1", help="train,validation,test ratios")
    ap.add_argument("--seeds", default="11", help="comma-separated run seeds (init + splits)")
    a = ap.parse_args()
    seeds = [int(x) for x in str(a.seeds).split(",") if x.strip()]
    split = [float(x) for x in a.split.split(",")]

    shutil.rmtree(a.work, ignore_errors=True)
    data = os.path.join(a.work, "data")
    t0 = time.time()
    make_ica_sites(data, sites=a.sites, subjects=[a.big] + [a.small] * (a.sites - 1),
                   comps=a.comps, T=a.temporal, seed=3, hidden_size=a.hidden,
                   input_size=a.input_size, cohort="hard", signal=a.signal,
                   label_noise=a.label_noise)
    print(f"# data generated in {time.time() - t0:.1f} s", flush=True)
    rows = []
    port = 29810
    for seed, mode in [(sd, md) for sd in seeds for md in a.modes]:
        out = os.path.join(a.work, f"{mode}_s{seed}")
        sets = [f"agg_engine={a.engine}", f"epochs={a.epochs}", f"patience={a.patience}",
                f"batch_size={a.batch}", f"seed={seed}", f"learning_rate={a.lr}",
                "split_ratio=" + json.dumps(split)] + list(a.set)
        if mode == "pretrain":
            sets += ["pretrain=true", "pretrain_args=" + json.dumps({
                "epochs": a.pretrain_epochs, "learning_rate": a.pretrain_lr,
                "batch_size": a.pretrain_batch, "local_iterations": 1, "validation_epochs": 1,
                "patience": a.pretrain_patience})]
        port += 1
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
               str(a.sites), "--master-addr", "127.0.0.1", "--master-port", str(port),
               "-m", "dinunet_implementations_amd.run", "--data-path", data, "--out", out,
               "--device", a.device]
        for s in sets:
            cmd += ["--set", s]
        env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
        env.setdefault("DINUNET_BACKEND", "gloo")
        t1 = time.time()
        logp = os.path.join(a.logdir or a.work, f"{mode}_s{seed}.log")
        os.makedirs(os.path.dirname(logp), exist_ok=True)
        with open(logp, "w") as f:
            rc = subprocess.call(cmd, stdout=f, stderr=subprocess.STDOUT, env=env)
        wall = time.time() - t1
        if rc != 0:
            print(f"FAILED {mode} rc={rc}; see {logp}", flush=True)
            rows.append({"mode": mode, "seed": seed, "rc": rc})
            continue
        fr = analysis.fold_report(out)
        loc0 = analysis.fold_report(out, "local0")["folds"]
        f0 = fr["folds"][0] if fr["folds"] else {}
        with open(analysis.find_logs(out, "remote")[0]) as f:
            rlogs = json.load(f)
        rec = {"mode": mode, "seed": seed, "rc": rc, "wall_s": round(wall, 1), "sites": a.sites,
               "engine": a.engine, "device": a.device,
               "data": (f"synthetic hard ICA cohort (signal {a.signal}, label noise "
                        f"{a.label_noise}); site 0: {a.big} subjects, sites 1..{a.sites - 1}: "
                        f"{a.small} each; split {a.split}"),
               "config": {"epochs": a.epochs, "patience": a.patience, "batch_size": a.batch,
                          "learning_rate": a.lr,
                          "pretrain_learning_rate": a.pretrain_lr if mode == "pretrain" else None,
                          "pretrain_batch_size": a.pretrain_batch if mode == "pretrain" else None,
                          "pretrain_epochs": a.pretrain_epochs if mode == "pretrain" else None,
                          "hidden_size": a.hidden, "input_size": a.input_size,
                          "num_components": a.comps, "temporal_size": a.temporal},
               "test": {k: f0.get(k) for k in ("AUC", "Accuracy", "F1", "Loss")},
               "best_val_epoch": f0.get("best_val_epoch"),
               "stopped_epoch": rlogs.get("stopped_epoch"),
               "pretrain_best_val_epoch": (loc0[0].get("pretrain_best_val_epoch")
                                           if loc0 else None),
               "validation_auc_curve": [round(float(r[-1]), 4) if isinstance(r, list) else r
                                        for r in rlogs.get("validation_log", [])]}
        rows.append(rec)
        with open(os.path.join(a.profiles, f"{a.tag}_{mode}_s{seed}.json"), "w") as f:
            json.dump(rec, f, indent=1)
        print(f"seed {seed} {mode:8s} test AUC {rec['test']['AUC']} best val epoch "
              f"{rec['best_val_epoch']} pretrain best epoch {rec['pretrain_best_val_epoch']} "
              f"({wall:.0f} s)", flush=True)
    md = [f"# ICA-LSTM pretrain -> finetune vs scratch ({a.sites} sites, {a.engine}, "
          f"{a.device}; BASELINE config 5)", "",
          f"Data: {rows[0].get('data', '') if rows else ''}.  Federated phase: batch {a.batch}, "
          f"up to {a.epochs} epochs, patience {a.patience}.  Pretraining (largest site alone): "
          f"batch {a.pretrain_batch}, up to {a.pretrain_epochs} epochs, patience "
          f"{a.pretrain_patience}.  Learning rate {a.lr} (pretraining {a.pretrain_lr}).  "
          f"Reference (FS, `NB.ipynb:200,209`): mean stopping epoch 68.5 scratch vs 42.7 "
          f"pretrain.", "",
          "| seed | mode | test AUC | test acc | test F1 | federated best-val epoch | stopped at | pretrain best epoch | wall s |",
          "|---:|---|---:|---:|---:|---:|---:|---:|---:|"]
    for r in rows:
        if r.get("rc"):
            md.append(f"| {r.get('seed')} | {r['mode']} | FAILED rc={r['rc']} | | | | | | |")
            continue
        t = r["test"]
        md.append(f"| {r['seed']} | {r['mode']} | {t['AUC']:.3f} | {t['Accuracy']:.3f} | "
                  f"{t['F1']:.3f} | {r['best_val_epoch']} | {r.get('stopped_epoch') or '-'} | "
                  f"{r['pretrain_best_val_epoch'] or '-'} | {r['wall_s']} |")
    import statistics
    md += ["", "| mode | runs | mean best-val (stopping) epoch | median | mean test AUC |",
           "|---|---:|---:|---:|---:|"]
    for mode in a.modes:
        ok = [r for r in rows if r["mode"] == mode and not r.get("rc")]
        if not ok:
            continue
        ep = [r["best_val_epoch"] for r in ok]
        md.append(f"| {mode} | {len(ok)} | {statistics.mean(ep):.1f} | {statistics.median(ep)} | "
                  f"{statistics.mean(r['test']['AUC'] for r in ok):.3f} |")
    with open(os.path.join(a.profiles, f"{a.tag}.md"), "w") as f:
        f.write("\n".join(md) + "\n")
    print("\n".join(md), flush=True)
    return 0 if all(not r.get("rc") for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
