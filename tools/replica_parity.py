#!/usr/bin/env python3
"""Several GPUs per site vs one GPU per site, end to end (run.py, dSGD, the hard synthetic ICA
cohort, full model size): 2 sites x 1 process vs 2 sites x 2 processes (--site-gpus 2, each on
batch_size / 2), every process sharing this machine's GPU over gloo (a rehearsal of the layout).
Prints the global test metrics and best validation epoch of both runs per seed, as JSON lines."""
import json
import os
import socket
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run(data, out, nproc, k, seed, epochs):
    env = dict(os.environ, DINUNET_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           str(nproc), "--master-addr", "127.0.0.1", "--master-port", str(port()), "-m",
           "dinunet_implementations_amd.run", "--data-path", data, "--out", out, "--site-gpus",
           str(k), "--set", f"epochs={epochs}", "--set", "batch_size=32", "--set", f"seed={seed}",
           "--set", "validation_epochs=1"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    if r.returncode:
        raise SystemExit(r.stderr[-3000:])
    f = next(os.path.join(d, x) for d, _, fs in os.walk(os.path.join(out, "remote"))
             for x in fs if x == "logs.json")
    with open(f) as fh:
        lg = json.load(fh)
    return {"test": lg["test_metrics"], "best_val_epoch": lg.get("best_val_epoch"),
            "val_curve": [v[1] for v in lg.get("validation_log", [])]}


def main():
    from dinunet_implementations_amd.data.synthetic import make_ica_sites
    epochs = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    seeds = [int(s) for s in (sys.argv[2] if len(sys.argv) > 2 else "0,1").split(",")]
    tmp = tempfile.mkdtemp()
    data = make_ica_sites(os.path.join(tmp, "ica"), sites=2, subjects=(320, 320), cohort="hard")
    for seed in seeds:
        one = run(data, os.path.join(tmp, f"one{seed}"), 2, 1, seed, epochs)
        two = run(data, os.path.join(tmp, f"two{seed}"), 4, 2, seed, epochs)
        print(json.dumps({"seed": seed, "epochs": epochs, "one_gpu_per_site": one,
                          "two_gpus_per_site": two}), flush=True)


if __name__ == "__main__":
    main()
