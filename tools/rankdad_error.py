#!/usr/bin/env python3
"""rank-dAD reconstruction error over a training run (is the accuracy gap to
dSGD a defect of the factorisation or the rank-r loss itself?).

One process, one GPU, ``--sites`` simulated sites, each with its own hard synthetic ICA cohort
(``data.synthetic.ica_cohort_hard``) and batch stream.  Every step computes each site's local
gradient G_s with the fused kernels, then runs the REAL rank-dAD factorisation of the engine
(``RankDADEngine.pre_reduce``: the device power iteration on G_s, warm-started from that site's
previous Q, ``dad_tol`` stop on the device) with one engine instance per site (its own warm-start
state), and records per factorised Linear

    err_engine = || mean_s P_s Q_s^T - mean_s G_s || / || mean_s G_s ||

and, every ``--svd-every`` steps, the same error for the OPTIMAL rank-r factors of each site
(truncated SVD of G_s, the best any rank-r per-site compression can do) and each site's energy
beyond rank r.  ``err_engine`` close to ``err_svd`` means the power iteration delivers what rank r
allows and the remaining gap is rank-r loss; ``err_engine`` far above it means a defect (too few
iterations, a bad warm start, an early ``dad_tol`` stop).

Trajectories (``--modes``), all from the same init and the same site batches:
  dsgd      the exact mean (the dSGD update);
  rankdad   the engine's reconstruction for every factorised Linear, dense mean elsewhere;
  rankdad_tol0  the same with every power iteration run (``dad_tol`` 0: no early stop);
  svd       mean of the per-site truncated SVDs (the rank-r optimum) -- accuracy of ideal rank r.
Global validation AUC every ``--eval-every`` steps.  Prints one JSON line.

(Differences from a real multi-process run: one BatchNorm running-stat buffer sees every site's
batches in turn instead of one replica per site; the factorisation and the update are the
production kernels.)
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
    ap.add_argument("--sites", type=int, default=8)
    ap.add_argument("--subjects", type=int, default=384, help="training subjects per site")
    ap.add_argument("--val", type=int, default=128)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--eval-every", type=int, default=50)
    ap.add_argument("--svd-every", type=int, default=25)
    ap.add_argument("--rank", type=int, default=10)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--tol", type=float, default=1e-3)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--effect", type=float, default=0.35)
    ap.add_argument("--modes", default="dsgd,rankdad,rankdad_tol0,svd")
    a = ap.parse_args()

    from dinunet_implementations_amd.data.synthetic import ica_cohort_hard
    from dinunet_implementations_amd.models import ICALstm
    from dinunet_implementations_amd.ops import FlatParams, FusedAdam
    from dinunet_implementations_amd.ops.reference import ica_windows
    from dinunet_implementations_amd.parallel import make_engine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    from dinunet_implementations_amd.utils.metrics import roc_auc

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    C, T, Wn = 100, 980, 10
    sites = []
    for s in range(a.sites):
        x, y = ica_cohort_hard(a.subjects + a.val, C, T, seed=1000 + s, site=s, signal=a.effect,
                               label_noise=0.1)
        X = ica_windows(torch.from_numpy(x), Wn, Wn, T).to(dev)
        Y = torch.from_numpy(y).to(dev)
        sites.append((X[:a.subjects], Y[:a.subjects], X[a.subjects:], Y[a.subjects:]))
        del x
    cfg = {"precision_bits": "32", "seed": 0, "dad_reduction_rank": a.rank,
           "dad_num_pow_iters": a.iters, "dad_tol": a.tol}

    def run(mode):
        mcfg = dict(cfg)
        if mode == "rankdad_tol0":  # every power iteration, no dad_tol early stop
            mcfg["dad_tol"] = 0.0
        torch.manual_seed(a.seed)
        model = ICALstm(input_size=256, hidden_size=384, num_comps=C, window_size=Wn).to(dev).train()
        flat = FlatParams(model.parameters())
        opt = FusedAdam(flat, lr=a.lr)
        grp = SiteGroup(device=dev)
        engs = [make_engine("rankDAD", model, flat, grp, dict(mcfg)) for _ in range(a.sites)]
        layers = engs[0].fast_layers  # (module, flat offset, out, in, r, send P off, send Q off)
        names = {id(m): n for n, m in model.named_modules()}
        gens = [torch.Generator(device=dev).manual_seed(7 + s + 100 * a.seed) for s in range(a.sites)]
        err_hist = {names[id(l[0])]: [] for l in layers}
        svd_hist = {names[id(l[0])]: [] for l in layers}
        tail_hist = {names[id(l[0])]: [] for l in layers}
        curve = []

        def val_auc():
            model.eval()
            ps, ys = [], []
            with torch.no_grad():
                for _, _, Xv, Yv in sites:
                    for i in range(0, len(Xv), 64):
                        out, _, _ = model.forward_loss(Xv[i:i + 64], Yv[i:i + 64])
                        ps.append(out[:, 1].float())
                    ys.append(Yv.float())
            model.train()
            return float(roc_auc(torch.cat(ps).cpu().numpy(), torch.cat(ys).cpu().numpy()))

        t0 = time.perf_counter()
        for step in range(1, a.steps + 1):
            gs = []
            for s, (Xt, Yt, _, _) in enumerate(sites):
                idx = torch.randint(0, len(Xt), (a.batch,), device=dev, generator=gens[s])
                flat.zero_grad()
                _, loss, _ = model.forward_loss(Xt[idx], Yt[idx])
                loss.backward()
                if mode.startswith("rankdad") or step % a.svd_every == 0:
                    engs[s].pre_reduce()  # the production power iteration on this site's G_s
                gs.append(flat.grad.clone())
            gmean = torch.stack(gs).mean(0)
            upd = gmean.clone()
            analyse = step % a.svd_every == 0
            for m, o, out_f, in_f, r, po, qo in layers:
                name = names[id(m)]
                exact = gmean[o:o + out_f * in_f].view(out_f, in_f).double()
                need_engine = mode.startswith("rankdad") or analyse
                if need_engine:
                    rec = torch.zeros_like(exact)
                    for e in engs:
                        P = e._send[po:po + out_f * r].view(out_f, r).double()
                        Q = e._send[qo:qo + in_f * r].view(in_f, r).double()
                        rec += P @ Q.t()
                    rec /= a.sites
                    if mode.startswith("rankdad"):
                        upd[o:o + out_f * in_f] = rec.reshape(-1).float()
                    err_hist[name].append(float((rec - exact).norm() / exact.norm().clamp_min(1e-30)))
                if mode == "svd" or analyse:
                    # every site's G at once (batched SVD), the truncation in fp64
                    Gs = torch.stack([g[o:o + out_f * in_f].view(out_f, in_f) for g in gs])
                    U, S, Vh = torch.linalg.svd(Gs, full_matrices=False)
                    U, S, Vh = U.double(), S.double(), Vh.double()
                    rec2 = torch.einsum("sik,sk,skj->ij", U[:, :, :r], S[:, :r], Vh[:, :r]) / a.sites
                    tails = ((S[:, r:] ** 2).sum(1) / (S ** 2).sum(1).clamp_min(1e-300)).tolist()
                    if mode == "svd":
                        upd[o:o + out_f * in_f] = rec2.reshape(-1).float()
                    if analyse:
                        svd_hist[name].append(float((rec2 - exact).norm() / exact.norm().clamp_min(1e-30)))
                        tail_hist[name].append(sum(tails) / len(tails))
            flat.grad.copy_(upd)
            opt.step()
            if step % a.eval_every == 0:
                curve.append([step, round(val_auc(), 4)])
                print(f"# {mode} step {step} auc {curve[-1][1]}", file=sys.stderr, flush=True)
        iters = engs[0].power_iterations()

        def summ(h):
            return {k: {"mean": round(sum(v) / len(v), 4), "first": round(v[0], 4),
                        "last": round(v[-1], 4)} for k, v in h.items() if v}
        return {"final_auc": curve[-1][1] if curve else None,
                "best_auc": max(c[1] for c in curve) if curve else None,
                "curve": curve, "wall_s": round(time.perf_counter() - t0, 1),
                "err_engine": summ(err_hist), "err_svd_opt": summ(svd_hist),
                "energy_beyond_rank": summ(tail_hist),
                "engine_iters_site0": iters}

    res = {"sites": a.sites, "rank": a.rank, "iters": a.iters, "tol": a.tol, "steps": a.steps,
           "seed": a.seed, "batch": a.batch, "subjects": a.subjects, "val": a.val}
    for mode in a.modes.split(","):
        res[mode] = run(mode)
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
