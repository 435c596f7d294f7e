#!/usr/bin/env python3
"""FreeSurfer MSANNet training-step throughput (BASELINE config 1's model).

The reference model (``comps/fs/models.py:4-31``: 66 -> 256 -> 128 -> 64 -> 32 -> 2 with
BatchNorm + ReLU, log-softmax + NLL) at the compspec batch (16) through the production
TrainStep: on a GPU the whole network is the fused head kernels (csrc/kernels/mlp_head.hip,
head_big.hip for batches > 64) plus the fused Adam, replayed as a HIP graph; on the CPU (config 1
is CPU/gloo) the reference math.  One JSON line per batch size:

    python tools/bench_fs.py [--device cuda|cpu] [--batch 16 256 2048] [--steps 200]
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        tools/bench_fs.py --device cpu        # 2 sites, dSGD over gloo
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--batch", type=int, nargs="+", default=[16])
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--engine", default="dSGD")
    a = ap.parse_args()
    if a.device == "cpu":
        os.environ.setdefault("DINUNET_BACKEND", "gloo")
    from dinunet_implementations_amd.models import MSANNet
    from dinunet_implementations_amd.ops import FlatParams, FusedAdam
    from dinunet_implementations_amd.parallel import init_sites, make_engine, shutdown
    from dinunet_implementations_amd.runtime.step import TrainStep

    grp = init_sites(device=a.device)
    dev = grp.device
    for B in a.batch:
        torch.manual_seed(0)
        m = MSANNet(66, [256, 128, 64, 32], 2).to(dev).train()
        flat = FlatParams(m.parameters())
        grp.broadcast(flat.data, 0)
        opt = FusedAdam(flat, lr=1e-3)
        eng = make_engine(a.engine, m, flat, grp, {"precision_bits": "32", "seed": 0})
        step = TrainStep(m, flat, opt, eng, task="fs", use_graph=dev.type == "cuda")
        g = torch.Generator(device=dev).manual_seed(100 + grp.rank)
        xs = torch.rand(8, B, 66, device=dev, generator=g)
        ys = torch.randint(0, 2, (8, B), device=dev, generator=g)
        for i in range(a.warmup):
            step(xs[i % 8], ys[i % 8])
        if dev.type == "cuda":
            torch.cuda.synchronize()
        grp.barrier()
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(xs[i % 8], ys[i % 8])
        if dev.type == "cuda":
            torch.cuda.synchronize()
        grp.barrier()
        dt = time.perf_counter() - t0
        if grp.is_master:
            print(json.dumps({
                "metric": f"samples/sec FS MSANNet training step ({a.engine})",
                "value": round(grp.world * B * a.steps / dt, 1),
                "unit": "samples/s (sum over sites)", "ms_per_step": round(1000 * dt / a.steps, 4),
                "n_sites": grp.world, "batch_per_site": B, "device": dev.type,
                "hip_graph": bool(step.graph is not None), "steps": a.steps, "warmup": a.warmup,
                "data": "synthetic [B, 66] volumes",
                "final_loss": round(float(step.last_loss.detach()), 5),
            }), flush=True)
    shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
