#!/usr/bin/env python3
"""Headline benchmark: ICA-LSTM dSGD training throughput, one site per GPU.

BASELINE.json metric: "samples/sec/site ICA-LSTM dSGD at 1/2/4/8 sites".  Config = the
reference's ICA single-site runner (``comps/icalstm/site_run.py:6-8``: batch_size 32) on the
inputspec geometry (``datasets/icalstm/inputspec.json``: C=100 components, T=980, W=10 -> S=98
windows) with the compspec hidden size 384 (``compspec.json:251-281``), input_size 256.  Each
timed step is a complete training step: fused encoder GEMM, persistent bi-LSTM forward,
classifier + softmax-CE, full backward, dSGD all-reduce (RCCL over xGMI for N>1), fused Adam.
Synthetic data (the ICA dataset is not shipped, ``.gitignore:123``) and random-init weights.

Launch: ``python bench.py`` (1 GPU) or ``python -m torch.distributed.run --nproc-per-node N
--master-addr 127.0.0.1 bench.py --gpus N``.  Rank 0 prints ONE JSON line; ``value`` is the
whole-job aggregate (samples/s summed over all sites), ``per_site`` the per-GPU rate.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

# reference CPU throughput of the same step (172.7 samples/s, B=32, H=384)
BASELINE_SAMPLES_PER_SEC_PER_SITE = 172.7
BASELINE_METRIC = "samples/sec/site ICA-LSTM dSGD at 1/2/4/8 sites; wall-clock to target AUC"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32, help="per-site batch (reference site_run: 32)")
    ap.add_argument("--engine", default="dSGD", choices=["dSGD", "rankDAD", "powerSGD"])
    ap.add_argument("--hidden", type=int, default=384)
    ap.add_argument("--input-size", type=int, default=256)
    ap.add_argument("--comps", type=int, default=100)
    ap.add_argument("--window", type=int, default=10)
    ap.add_argument("--temporal", type=int, default=980)
    ap.add_argument("--precision-bits", default="32", choices=["16", "32"])
    ap.add_argument("--graph", type=int, default=1, help="capture fwd+bwd(+opt) in a HIP graph")
    ap.add_argument("--pool", type=int, default=8, help="distinct synthetic batches resident in HBM")
    ap.add_argument("--feed", default="device", choices=["device", "host"],
                    help="device: the site dataset lives in HBM as bf16 and every step gathers its "
                         "batch on the device (K whole steps per HIP graph); host: each step is fed "
                         "a batch tensor by the host loop")
    ap.add_argument("--graph-steps", type=int, default=0,
                    help="steps per HIP graph in device-feed mode (0: the largest divisor of "
                         "--steps up to 10)")
    return ap.parse_args()


def main():
    args = parse()
    from dinunet_implementations_amd.parallel import init_sites, make_engine
    from dinunet_implementations_amd.runtime.step import TrainStep
    from dinunet_implementations_amd.models import ICALstm
    from dinunet_implementations_amd.ops import FlatParams, FusedAdam

    grp = init_sites()
    dev = grp.device
    if dev.type != "cuda":
        print("bench.py needs a GPU", file=sys.stderr)
        return 2
    torch.manual_seed(1234)
    S = args.temporal // args.window
    model = ICALstm(input_size=args.input_size, hidden_size=args.hidden, num_comps=args.comps,
                    window_size=args.window, num_cls=2).to(dev).train()
    flat = FlatParams(model.parameters())
    grp.broadcast(flat.data, 0)
    opt = FusedAdam(flat, lr=1e-3)
    cfg = {"precision_bits": args.precision_bits, "seed": 0}
    engine = make_engine(args.engine, model, flat, grp, cfg)
    step = TrainStep(model, flat, opt, engine, task="ica", use_graph=bool(args.graph))

    g = torch.Generator(device=dev).manual_seed(100 + grp.rank)
    xs = torch.randn(args.pool, args.batch, S, args.comps, args.window, device=dev, generator=g)
    ys = torch.randint(0, 2, (args.pool, args.batch), device=dev, generator=g)

    pi, it0 = getattr(engine, "power_iterations", None), None
    if args.feed == "device":
        # the site's (synthetic) dataset resident in HBM as bf16, batches gathered on the device
        # by the step's first launch; the timed steps run as replays of K-step graphs
        from dinunet_implementations_amd.ops import DeviceSource
        src = DeviceSource(xs.view(args.pool * args.batch, S, args.comps, args.window)
                           .to(torch.bfloat16), ys.view(-1), args.batch)
        del xs
        K = args.graph_steps or max(d for d in range(1, 11) if args.steps % d == 0)
        step.bind(src, steps_per_graph=K)
        step.run(args.warmup)
        step.prepare(args.steps)
        it0 = pi() if pi else None
        torch.cuda.synchronize()
        grp.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step.run(args.steps)
        torch.cuda.synchronize()
        grp.barrier()
        torch.cuda.synchronize()
    else:
        for i in range(args.warmup):
            step(xs[i % args.pool], ys[i % args.pool])
        torch.cuda.synchronize()
        grp.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(xs[i % args.pool], ys[i % args.pool])
        torch.cuda.synchronize()
        grp.barrier()
        torch.cuda.synchronize()
    dt = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    iters = None
    if it0 is not None:
        # rank-dAD: power iterations actually run per timed step (mean over the factorised
        # layers; dad_tol may stop a layer before dad_num_pow_iters)
        it1 = pi()
        iters = round(sum(b - a for a, b in zip(it0, it1)) / max(1, len(it0)) / args.steps, 3)
    grp.all_reduce(dt, op=torch.distributed.ReduceOp.MAX)
    dt = float(dt.item())
    loss = float(step.last_loss.detach())
    n = grp.world
    total = n * args.batch * args.steps / dt
    if grp.is_master:
        rec = {
            # the headline metric names dSGD; other engines report the same quantity under
            # their own name (never mistaken for the dSGD headline)
            "metric": BASELINE_METRIC.replace("dSGD", args.engine),
            "value": round(total, 2),
            "unit": "samples/s (whole job: sum over the N sites)",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * dt / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(total / BASELINE_SAMPLES_PER_SEC_PER_SITE, 2),
            "dtype": "bf16",
            "data": "synthetic",
            "config": {"model": f"ICA-LSTM (C={args.comps}, W={args.window}, S={S}, "
                                f"I={args.input_size}, H={args.hidden}, bi-dir)",
                       "global_batch": args.batch * n, "seq_len": S,
                       "parallelism": f"dp{n}", "engine": args.engine,
                       "precision_bits": args.precision_bits, "hip_graph": bool(args.graph),
                       "feed": args.feed},
            "per_site": round(total / n, 2),
            "vs_baseline_per_site": round((total / n) / BASELINE_SAMPLES_PER_SEC_PER_SITE, 2),
            "baseline_note": "vs_baseline = value / 172.7 samples/s (BASELINE.md: the reference "
                             "model's step, B=32, H=384, measured on CPU; the reference publishes "
                             "no throughput); per-site rate in per_site",
            "final_loss": round(loss, 5),
            **({"dad_iters_per_step": iters} if iters is not None else {}),
            # HBM high-water mark of the run (allocator view: model, optimizer state, activations,
            # graph pools and the resident synthetic dataset of --pool batches)
            "peak_hbm_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 3),
            "dataset_hbm_gib": round(args.pool * args.batch * S * args.comps * args.window
                                     * (2 if args.feed == "device" else 4) / 2**30, 3),
        }
        print(json.dumps(rec), flush=True)
    from dinunet_implementations_amd.parallel import shutdown
    shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
