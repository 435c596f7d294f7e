#!/usr/bin/env python3
"""Headline benchmark: ICA-LSTM dSGD training throughput, one site per GPU.

BASELINE.json metric: "samples/sec/site ICA-LSTM dSGD at 1/2/4/8 sites".  Config = the
reference's ICA single-site runner (``comps/icalstm/site_run.py:6-8``: batch_size 32) on the
inputspec geometry (``datasets/icalstm/inputspec.json``: C=100 components, T=980, W=10 -> S=98
windows) with the compspec hidden size 384 (``compspec.json:251-281``), input_size 256.  Each
timed step is a complete training step: fused encoder GEMM, persistent bi-LSTM forward,
classifier + softmax-CE, full backward, dSGD all-reduce (RCCL over xGMI for N>1), fused Adam.
Synthetic data (the ICA dataset is not shipped, ``.gitignore:123``) and random-init weights.

The timed steps run through ``runtime.feed.DeviceFeed`` -- the object the production site loop
(``runtime.site.FederatedSite``) trains its epochs with, per-step train records included.  At one
site the run then trains a synthetic hard cohort through ``FederatedSite`` itself and adds the
second half of the BASELINE metric, wall-clock to the target validation AUC
(``time_to_auc_s``), and the site loop's own logged throughput (``site_loop_samples_per_sec``).

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
    ap.add_argument("--site-loop", default="auto", choices=["auto", "0", "1"],
                    help="after the timed steps, train a synthetic hard ICA cohort through the "
                         "production site loop (runtime.site.FederatedSite: device-fed epochs, "
                         "validation, early stopping, checkpoints) and report its wall-clock to "
                         "the target validation AUC and its logged samples/s (auto: N == 1)")
    ap.add_argument("--target-auc", type=float, default=0.75)
    ap.add_argument("--tta-subjects", type=int, default=2560,
                    help="site-loop cohort size (split 0.8/0.1/0.1)")
    ap.add_argument("--tta-epochs", type=int, default=30)
    ap.add_argument("--collective", default="calibrate",
                    choices=["auto", "allreduce", "direct", "peer", "calibrate"],
                    help="site-mean form (dsgd_collective): RCCL all-reduce, RCCL all-to-all "
                         "exchange, the IPC peer exchange (parallel/peer.py), or calibrate = time "
                         "the captured all-reduce and peer exchange, keep the faster")
    ap.add_argument("--loopback-rccl", action="store_true",
                    help="one GPU, but through a one-rank RCCL group marked distributed: the "
                         "N > 1 step (split backward, bucketed all-reduce, captured collectives) "
                         "timed on one GPU")
    return ap.parse_args()


def site_loop(grp, args):
    """Wall-clock to the target validation AUC through the production runtime: this rank's site
    gets a synthetic hard ICA cohort (``data.synthetic.ica_cohort_hard``: connectivity labels,
    site shift, 10% label noise) written in the reference layout (``[N, C, T]`` npy + labels
    CSV), and ``FederatedSite.run`` trains it exactly as ``python -m
    dinunet_implementations_amd.run`` would (device-fed epochs, global validation AUC, best /
    last checkpoints, logs.json).  Returns the clock of the first epoch whose global validation
    AUC reached the target (``cumulative_total_duration``, reference ``local.py:52``) and the
    steady-state train throughput the site logged (``samples_per_sec``, epochs after the first)."""
    import csv
    import shutil
    import statistics
    import tempfile

    import numpy as np
    from dinunet_implementations_amd.config import build_config
    from dinunet_implementations_amd.data.synthetic import ica_cohort_hard
    from dinunet_implementations_amd.runtime.site import FederatedSite
    from dinunet_implementations_amd.tasks import get_task

    root = tempfile.mkdtemp(prefix=f"dinunet_bench_{grp.rank}_")
    try:
        base = os.path.join(root, "input", f"local{grp.rank}", "simulatorRun")
        os.makedirs(base)
        x, y = ica_cohort_hard(args.tta_subjects, args.comps, args.temporal, seed=300 + grp.rank,
                               site=grp.rank, signal=0.35, label_noise=0.1)
        np.save(os.path.join(base, "ica_data.npy"), x)
        del x
        with open(os.path.join(base, "labels.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["data_index", "label"])
            w.writerows([[i, int(v)] for i, v in enumerate(y)])
        cfg = build_config(overrides={
            "task_id": "ICA-Classification", "agg_engine": args.engine,
            "precision_bits": args.precision_bits, "batch_size": args.batch,
            "epochs": args.tta_epochs, "patience": args.tta_epochs, "split_ratio": [0.8, 0.1, 0.1],
            "data_file": "ica_data.npy", "labels_file": "labels.csv",
            "input_size": args.input_size, "hidden_size": args.hidden,
            "window_size": args.window, "window_stride": args.window,
            "temporal_size": args.temporal, "num_components": args.comps, "num_class": 2,
            "learning_rate": 1e-3, "seed": 11})
        T, D, H = get_task(cfg["task_id"])
        site = FederatedSite(cfg, grp, T, D, H, {"baseDirectory": base, "clientId": f"local{grp.rank}"},
                             os.path.join(root, "out"), site_name=f"local{grp.rank}", verbose=False)
        logs = site.run()[0]
    finally:
        shutil.rmtree(root, ignore_errors=True)
    val = [float(r[-1]) for r in logs.get("validation_log", [])]
    cum = logs.get("cumulative_total_duration", [])
    hit = next((i for i, a in enumerate(val) if a >= args.target_auc), None)
    sps = logs.get("samples_per_sec", [])
    return {
        "time_to_auc_s": round(cum[hit], 3) if hit is not None else None,
        "target_auc": args.target_auc,
        "epochs_to_auc": hit + 1 if hit is not None else None,
        "steps_per_epoch": int(logs["split_sizes"]["train"]) // args.batch,
        "best_val_auc": round(max(val), 4) if val else None,
        "test_auc": round(float(logs["test_metrics"][-1]), 4) if logs.get("test_metrics") else None,
        "site_loop_samples_per_sec": round(statistics.median(sps[1:] or sps), 1) if sps else None,
        "site_loop_feed": logs.get("feed", "host"),
        "tta_data": (f"synthetic hard ICA cohort, {args.tta_subjects} subjects/site "
                     "(signal 0.35, label noise 0.1), split 0.8/0.1/0.1"),
    }


def main():
    args = parse()
    from dinunet_implementations_amd.parallel import init_sites, make_engine
    from dinunet_implementations_amd.runtime.step import TrainStep
    from dinunet_implementations_amd.models import ICALstm
    from dinunet_implementations_amd.ops import FlatParams, FusedAdam

    grp = init_sites(loopback=args.loopback_rccl)
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
    cfg = {"precision_bits": args.precision_bits, "seed": 0, "dsgd_collective": args.collective}
    engine = make_engine(args.engine, model, flat, grp, cfg)
    step = TrainStep(model, flat, opt, engine, task="ica", use_graph=bool(args.graph))

    g = torch.Generator(device=dev).manual_seed(100 + grp.rank)
    xs = torch.randn(args.pool, args.batch, S, args.comps, args.window, device=dev, generator=g)
    ys = torch.randint(0, 2, (args.pool, args.batch), device=dev, generator=g)

    pi, it0 = getattr(engine, "power_iterations", None), None
    if args.feed == "device":
        # the site's (synthetic) dataset resident in HBM as bf16, batches gathered on the device
        # by the step's first launch, per-step train records kept on the device: the same
        # runtime object (runtime.feed.DeviceFeed) FederatedSite trains its epochs with
        from dinunet_implementations_amd.runtime.feed import DeviceFeed
        K = args.graph_steps or max(d for d in range(1, 11) if args.steps % d == 0)
        feed = DeviceFeed(step, xs.view(args.pool * args.batch, S, args.comps, args.window),
                          ys.view(-1), args.batch, nb=args.pool, col=1, steps_per_graph=K)
        del xs
        feed.run(args.warmup)
        feed.prepare(args.steps)
        it0 = pi() if pi else None
        torch.cuda.synchronize()
        grp.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        feed.run(args.steps)
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
    peak = torch.cuda.max_memory_allocated(dev)
    tta = None
    if args.site_loop == "1" or (args.site_loop == "auto" and n == 1 and not grp.loopback):
        try:
            tta = site_loop(grp, args)
        except Exception as e:  # never lose the throughput line to the study
            tta = {"time_to_auc_s": None, "site_loop_error": f"{type(e).__name__}: {e}"}
    else:
        tta = {"time_to_auc_s": None,
               "site_loop": "not run (default at N > 1; --site-loop 1 runs it on every site)"}
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
                       "parallelism": f"dp{n}" + ("-loopback-rccl" if grp.loopback else ""),
                       "engine": args.engine,
                       "precision_bits": args.precision_bits, "hip_graph": bool(args.graph),
                       "feed": args.feed},
            "per_site": round(total / n, 2),
            "vs_baseline_per_site": round((total / n) / BASELINE_SAMPLES_PER_SEC_PER_SITE, 2),
            "baseline_note": "vs_baseline = value / 172.7 samples/s (BASELINE.md: the reference "
                             "model's step, B=32, H=384, measured on CPU; the reference publishes "
                             "no throughput); per-site rate in per_site",
            "final_loss": round(loss, 5),
            # N > 1 code path: collectives captured inside the K-step graphs (runtime.step)
            "comm_graph": bool(getattr(step, "comm_graph", False)),
            "collective": (getattr(engine, "calibration", None)
                           or ("peer" if engine.peer else
                               "direct" if getattr(engine, "direct", False) else "allreduce")),
            "split_backward": bool(getattr(step, "split", False)),
            **({"dad_iters_per_step": iters} if iters is not None else {}),
            # HBM high-water mark of the run (allocator view: model, optimizer state, activations,
            # graph pools and the resident synthetic dataset of --pool batches)
            "peak_hbm_gib": round(peak / 2**30, 3),
            "dataset_hbm_gib": round(args.pool * args.batch * S * args.comps * args.window
                                     * (2 if args.feed == "device" else 4) / 2**30, 3),
        }
        if tta is not None:
            rec.update(tta)
        print(json.dumps(rec), flush=True)
    from dinunet_implementations_amd.parallel import shutdown
    shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
