#!/usr/bin/env python3
"""The production launcher's own throughput at the headline config: writes a
synthetic hard ICA cohort in the reference site layout (``data.synthetic.make_ica_sites``, one
site, C=100 components x T=980 -> S=98 windows of 10), runs ``python -m
dinunet_implementations_amd.run`` on it (B=32, H=384, I=256, dSGD, one GPU), and reports the
``samples_per_sec`` that ``runtime.site.FederatedSite`` logged to ``logs.json`` per epoch (median
of the epochs after the first, which holds the warm-up and graph captures), next to a
``bench.py`` run of the same build for comparison.

    python tools/runpy_rate.py --subjects 2560 --epochs 6 [--out profiles/r4_runpy_rate.json]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--subjects", type=int, default=2560)
    ap.add_argument("--epochs", type=int, default=6)
    ap.add_argument("--work", default="/tmp/dinunet_runpy_rate")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r4_runpy_rate.json"))
    ap.add_argument("--bench", type=int, default=1, help="also run bench.py for the comparison")
    ap.add_argument("--li", type=int, default=1, help="local_iterations (gradient accumulation)")
    a = ap.parse_args()
    from dinunet_implementations_amd.data.synthetic import make_ica_sites
    from dinunet_implementations_amd.utils import analysis
    shutil.rmtree(a.work, ignore_errors=True)
    data = os.path.join(a.work, "data")
    make_ica_sites(data, sites=1, subjects=[a.subjects], comps=100, T=980, seed=5,
                   hidden_size=384, input_size=256, cohort="hard", signal=0.35, label_noise=0.1)
    out = os.path.join(a.work, "out")
    sets = ["agg_engine=dSGD", "batch_size=32", f"epochs={a.epochs}", f"patience={a.epochs}",
            "split_ratio=[0.8, 0.1, 0.1]", "learning_rate=0.001", "seed=11",
            f"local_iterations={a.li}"]
    cmd = [sys.executable, "-m", "dinunet_implementations_amd.run", "--data-path", data,
           "--out", out, "--device", "cuda"]
    for s in sets:
        cmd += ["--set", s]
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    wall = time.time() - t0
    if r.returncode != 0:
        print(r.stdout[-2000:], r.stderr[-4000:], file=sys.stderr)
        return r.returncode
    logp = analysis.find_logs(out, "local0")
    with open(logp[0]) as f:
        logs = json.load(f)
    sps = logs.get("samples_per_sec", [])
    rec = {"what": "python -m dinunet_implementations_amd.run, 1 site, synthetic hard ICA cohort "
                   f"({a.subjects} subjects, C=100, T=980 -> S=98, split 0.8/0.1/0.1), B=32, "
                   "H=384, I=256, dSGD, bf16, 1 MI355X",
           "feed": logs.get("feed", "host"), "epochs": a.epochs, "local_iterations": a.li,
           "samples_per_sec_per_epoch": [round(v, 1) for v in sps],
           "runpy_samples_per_sec": round(statistics.median(sps[1:] or sps), 1) if sps else None,
           "runpy_wall_s": round(wall, 1),
           "train_samples": int(logs["split_sizes"]["train"]),
           "test_auc": logs.get("test_metrics", [None])[-1]}
    if a.bench:
        b = subprocess.run([sys.executable, "bench.py", "--steps", "200", "--warmup", "20",
                            "--site-loop", "0"], cwd=ROOT, capture_output=True, text=True)
        line = [ln for ln in b.stdout.splitlines() if ln.startswith("{")]
        if line:
            bj = json.loads(line[-1])
            rec["bench_samples_per_sec"] = bj["value"]
            rec["bench_ms_per_step"] = bj["ms_per_step"]
            if rec["runpy_samples_per_sec"]:
                rec["runpy_vs_bench"] = round(rec["runpy_samples_per_sec"] / bj["value"], 4)
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))
    shutil.rmtree(a.work, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
