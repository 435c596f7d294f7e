#!/usr/bin/env python3
"""Wall-clock to a target validation AUC: ICA-LSTM dSGD (BASELINE.json metric, second half).

Each rank is one site holding a private synthetic ICA cohort (``data.synthetic.ica_timecourses``:
label-dependent oscillations in 10% of 100 components, T=980, windows of 10 -> S=98) resident in
HBM.  Training runs the same fused step as ``bench.py`` (dSGD all-reduce for N>1) and, every
``--eval-every`` steps, the GLOBAL validation AUC (scores gathered from every site) is computed;
the clock stops when it reaches ``--target``.  Prints one JSON line (rank 0).

    python tools/bench_time_to_auc.py [--target 0.9]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        tools/bench_time_to_auc.py

``--cohort hard`` (``data.synthetic.ica_cohort_hard``: connectivity labels, site shifts, label
noise) is the cohort that separates engines / precisions; ``--compute-path reference`` runs the
fp32 oracle math (``ops/reference.py``, no fused kernels, eager) on the same device as the
bf16-fidelity baseline.  The JSON line carries the whole validation-AUC curve.
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
    ap.add_argument("--target", type=float, default=0.9)
    ap.add_argument("--subjects", type=int, default=512, help="training subjects per site")
    ap.add_argument("--val", type=int, default=256, help="validation subjects per site")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--eval-every", type=int, default=16)
    ap.add_argument("--max-steps", type=int, default=4000)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--effect", "--signal", dest="signal", type=float, default=0.6,
                    help="class-signal amplitude (--effect under torchrun: --signal is ambiguous there)")
    ap.add_argument("--engine", default="dSGD", choices=["dSGD", "rankDAD", "powerSGD"])
    ap.add_argument("--cohort", default="easy", choices=["easy", "hard"])
    ap.add_argument("--label-noise", type=float, default=0.1, help="hard cohort")
    ap.add_argument("--compute-path", default="fused", choices=["fused", "reference"])
    ap.add_argument("--seed", type=int, default=0, help="model init / batch order")
    ap.add_argument("--full", action="store_true", help="run max-steps even after the target")
    a = ap.parse_args()

    from dinunet_implementations_amd.data.synthetic import ica_cohort_hard, ica_timecourses
    from dinunet_implementations_amd.models import ICALstm
    from dinunet_implementations_amd.ops import FlatParams, FusedAdam
    from dinunet_implementations_amd.ops.reference import ica_windows
    from dinunet_implementations_amd.parallel import init_sites, make_engine, shutdown
    from dinunet_implementations_amd.runtime.step import TrainStep
    from dinunet_implementations_amd.utils.metrics import roc_auc

    grp = init_sites()
    dev = grp.device
    C, T, W = 100, 980, 10
    if a.cohort == "hard":
        x, y = ica_cohort_hard(a.subjects + a.val, C, T, seed=1000 + grp.rank, site=grp.rank,
                               signal=a.signal, label_noise=a.label_noise)
    else:
        x, y = ica_timecourses(a.subjects + a.val, C, T, seed=1000 + grp.rank, signal=a.signal)
    xw = ica_windows(torch.from_numpy(x), W, W, T)  # [N, S, C, W]
    X = xw.to(dev)
    Y = torch.from_numpy(y).to(dev)
    Xtr, Ytr, Xva, Yva = X[:a.subjects], Y[:a.subjects], X[a.subjects:], Y[a.subjects:]

    torch.manual_seed(a.seed)  # same init everywhere
    model = ICALstm(input_size=256, hidden_size=384, num_comps=C, window_size=W).to(dev).train()
    ref_math = a.compute_path == "reference"
    if ref_math:
        for m in model.modules():
            if hasattr(m, "use_fused"):
                m.use_fused = False
    flat = FlatParams(model.parameters())
    grp.broadcast(flat.data, 0)
    opt = FusedAdam(flat, lr=a.lr)
    engine = make_engine(a.engine, model, flat, grp, {"precision_bits": "32", "seed": 0})
    step = TrainStep(model, flat, opt, engine, task="ica",
                     use_graph=dev.type == "cuda" and not ref_math)
    g = torch.Generator(device=dev).manual_seed(7 + grp.rank + 100 * a.seed)

    def global_auc():
        model.eval()
        with torch.no_grad():
            probs = []
            for i in range(0, len(Xva), 64):
                out, _, _ = model.forward_loss(Xva[i:i + 64], Yva[i:i + 64])
                probs.append(out[:, 1].float())
            p = torch.cat(probs)
        model.train()
        p_all = grp.all_gather_varlen(p) if grp.distributed else p
        y_all = grp.all_gather_varlen(Yva.float()) if grp.distributed else Yva.float()
        return float(roc_auc(p_all.cpu().numpy(), y_all.cpu().numpy()))

    if dev.type == "cuda":
        torch.cuda.synchronize()
    grp.barrier()
    t0 = time.perf_counter()
    auc, steps = 0.5, 0
    curve = []
    t_hit, s_hit = None, None
    while steps < a.max_steps:
        idx = torch.randint(0, len(Xtr), (a.batch,), device=dev, generator=g)
        step(Xtr[idx], Ytr[idx])
        steps += 1
        if steps % a.eval_every == 0:
            auc = global_auc()
            curve.append([steps, round(auc, 4)])
            if auc >= a.target and t_hit is None:
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                t_hit, s_hit = time.perf_counter() - t0, steps
                if not a.full:
                    break
            if grp.is_master and steps % (a.eval_every * 16) == 0:
                print(f"# step {steps} auc {auc:.4f}", file=sys.stderr, flush=True)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    grp.barrier()
    dt = time.perf_counter() - t0 if t_hit is None else t_hit
    if grp.is_master:
        print(json.dumps({
            "metric": "wall-clock to target validation AUC, ICA-LSTM " + a.engine,
            "value": round(dt, 3), "unit": "s", "higher_is_better": False,
            "target_auc": a.target, "reached": t_hit is not None,
            "steps": s_hit if s_hit is not None else steps,
            "samples_per_site": (s_hit if s_hit is not None else steps) * a.batch,
            "final_auc": round(auc, 4), "best_auc": max([c[1] for c in curve] or [0.5]),
            "n_sites": grp.world, "seed": a.seed, "engine": a.engine,
            "data": ("synthetic ICA cohort %s (signal=%g%s)" % (
                a.cohort, a.signal,
                ", label_noise=%g" % a.label_noise if a.cohort == "hard" else "")),
            "compute_path": a.compute_path,
            "dtype": "fp32" if ref_math else "bf16",
            "curve": curve,
        }), flush=True)
    shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
