#!/usr/bin/env python3
"""Multi-site replica check on ONE GPU: N ranks (torch.distributed.run, ``DINUNET_BACKEND=gloo``,
every rank on cuda:0) train the ICA-LSTM through the production TrainStep (HIP-graph replay,
split capture with the all-reduce between the replays for dSGD) on rank-specific data, then
compare every rank's flat parameters bit for bit.  Replicas of a synchronous engine must stay
identical; any divergence means two ranks applied different updates.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        tools/multirank_check.py --engine dSGD --precision 16 --ragged --accum 2

Prints one JSON line (rank 0); exit status 0 iff all ranks are bit-identical (and, with
``--oracle``, the N-rank result matches the single-process oracle).

``--oracle``: rank 0 also replays the whole run in-process as the reference semantics of dSGD
(SURVEY.md E10): for every step it computes EACH site's gradient on that site's batches (the same
generators, the same ragged batch), averages them in fp64 in site order, and applies the same
fused Adam.  Agreement is judged on the parameter UPDATE (final - initial): the relative L2 error
of the N-rank update against the oracle's is reported (``update_rel_err``) and, at
``--precision 32``, must stay below ``--oracle-tol``; at 16 bits it measures what the payload
precision costs after Adam (which turns the sign of every near-zero mean gradient into a full
``lr`` step, so it amplifies payload rounding).  For every engine the first step's reduced
gradient is also compared with the oracle's (``grad_rel_err``, bounded by ``--grad-tol``): the
payload's own error for dSGD, and for rank-dAD / PowerSGD the distance between the engine's
reconstruction and the fp64 replay of the same factorisation.  (Bit-identical replicas alone would also pass if every rank applied the same
WRONG update.)
"""
import argparse
import json
import os
import sys

os.environ.setdefault("DINUNET_BACKEND", "gloo")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _orth(P):
    """Orthonormal basis of span(P) (fp64 Householder QR; the kernels use Cholesky QR -- the
    reconstruction P P^T G does not depend on which basis of the span)."""
    import torch
    return torch.linalg.qr(P, mode="reduced")[0]


def oracle_reducer(engine, model, flat, cfg, world, dev):
    """``reduce(site_grads) -> mean gradient`` in fp64: the reference semantics of each engine
    (SURVEY.md E10-E12), replayed from every site's own local gradient with the engine's own
    initial state (warm-start Q, error feedback) kept per site.

    * dSGD: the mean of the site gradients.
    * rank-dAD (gradient space, fixed ``dad_num_pow_iters``: run with ``--dad-tol 0``): per large
      Linear, site s runs its power iteration on its own G_s from its own warm start
      (P = orth(G_s Q); Q = G_s^T P; the last Q warm-starts its next step) and the layer
      gradient is mean_s P_s Q_s^T; every other parameter is the dSGD mean.
    * PowerSGD (Vogels et al. 2019, warm start): M_s = G_s + e_s; P = orth(mean_s M_s Q);
      Q = mean_s M_s^T P (the next warm start); G = P Q^T; e_s = M_s - G; vectors: mean."""
    import torch
    from dinunet_implementations_amd.parallel import make_engine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    if engine == "dSGD":
        return lambda gs: sum(gs) / len(gs)
    tmpl = make_engine(engine, model, flat, SiteGroup(device=dev), dict(cfg))  # initial state
    seg = {id(p): (o, n) for p, o, n in flat.segments()}
    if engine == "rankDAD":
        iters = max(1, tmpl.iters)
        layers = []  # (offset, out, in, [per-site warm Q])
        for m, o, out_f, in_f, r, po, qo in tmpl.fast_layers:
            q0 = tmpl._send[qo:qo + in_f * r].view(in_f, r).double().clone()
            layers.append((o, out_f, in_f, [q0.clone() for _ in range(world)]))

        def red(gs):
            g = sum(gs) / len(gs)
            for o, out_f, in_f, qs in layers:
                acc = torch.zeros(out_f, in_f, dtype=torch.float64, device=dev)
                for s, gsite in enumerate(gs):
                    G = gsite[o:o + out_f * in_f].view(out_f, in_f)
                    Q = qs[s]
                    for _ in range(iters):
                        P = _orth(G @ Q)
                        Q = G.t() @ P
                    qs[s] = Q
                    acc += P @ Q.t()
                g[o:o + out_f * in_f] = (acc / len(gs)).reshape(-1)
            return g
        return red
    if engine == "powerSGD":
        mats = []  # (offset, rows, cols, Q, [per-site error])
        for (p, rows, cols, r), q in zip(tmpl.mats, tmpl.Q):
            o = seg[id(p)][0]
            mats.append([o, rows, cols, q.double().clone(),
                         [torch.zeros(rows, cols, dtype=torch.float64, device=dev)
                          for _ in range(world)]])

        def red(gs):
            g = sum(gs) / len(gs)
            for mt in mats:
                o, rows, cols, Q, errs = mt
                Ms = [gsite[o:o + rows * cols].view(rows, cols) + e for gsite, e in zip(gs, errs)]
                P = _orth(sum(M @ Q for M in Ms) / len(Ms))
                Qn = sum(M.t() @ P for M in Ms) / len(Ms)
                Gh = P @ Qn.t()
                mt[3] = Qn
                mt[4] = [M - Gh for M in Ms]
                g[o:o + rows * cols] = Gh.reshape(-1)
            return g
        return red
    raise SystemExit(f"--oracle: no oracle for engine {engine}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engine", default="dSGD")
    ap.add_argument("--precision", default="32")
    ap.add_argument("--accum", type=int, default=1)
    ap.add_argument("--ragged", action="store_true",
                    help="rank 1 feeds one short batch mid-run (eager fallback beside replays)")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=24)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--overlap", type=int, default=1, help="dSGD all-reduce under the backward")
    ap.add_argument("--diag", action="store_true", help="report dSGD gradient-ready counts")
    ap.add_argument("--split", type=int, default=-1, help="-1: TrainStep's default")
    ap.add_argument("--oracle", action="store_true", help="compare with the fp64-mean oracle")
    ap.add_argument("--oracle-tol", type=float, default=1e-3)
    ap.add_argument("--payload", default=None, help="payload_dtype (fp16 | bf16 | fp32)")
    ap.add_argument("--collective", default="auto",
                    help="dsgd_collective (auto | direct | allreduce | peer | calibrate)")
    ap.add_argument("--dad-tol", type=float, default=None,
                    help="dad_tol (the rank-dAD oracle replays a fixed iteration count: pass 0)")
    ap.add_argument("--grad-tol", type=float, default=None,
                    help="bound on the first step's reduced-gradient error vs the fp64 oracle "
                         "(dSGD; default: 1e-6 at 32 bits, 2e-3 at 16)")
    ap.add_argument("--feed", default="host", choices=["host", "device"],
                    help="device: each site's batches resident in HBM (bf16), TrainStep.bind/run "
                         "(the bench path: split capture across sites, Adam-emitted operand pack)")
    a = ap.parse_args()

    import torch
    from dinunet_implementations_amd.models import ICALstm
    from dinunet_implementations_amd.ops import FlatParams, FusedAdam
    from dinunet_implementations_amd.parallel import init_sites, make_engine, shutdown
    from dinunet_implementations_amd.runtime.step import TrainStep

    grp = init_sites()
    dev = grp.device
    torch.manual_seed(1234)  # identical init on every site
    m = ICALstm(input_size=128, hidden_size=384, num_comps=50, window_size=10).to(dev).train()
    m.classifier[0].p = 0.0
    flat = FlatParams(m.parameters())
    init = flat.data.detach().clone()
    opt = FusedAdam(flat, lr=1e-3)
    cfg = {"precision_bits": a.precision, "dad_reduction_rank": 8, "powersgd_rank": 4, "seed": 5,
           "dsgd_overlap": bool(a.overlap), "dsgd_collective": a.collective}
    if a.payload:
        cfg["payload_dtype"] = a.payload
    if a.dad_tol is not None:
        cfg["dad_tol"] = a.dad_tol
    eng = make_engine(a.engine, m, flat, grp, cfg)
    counts = {}
    if a.diag and hasattr(eng, "_on_grad"):
        names = {id(p): n for n, p in m.named_parameters()}
        orig = eng._on_grad

        def spy(p):
            if eng.sync_enabled:
                counts[names.get(id(p), "?")] = counts.get(names.get(id(p), "?"), 0) + 1
            return orig(p)
        eng._on_grad = spy
        import dinunet_implementations_amd.ops._grad as _gr
        _gr.unregister(orig)
        _gr.register(spy)
        for h in eng._hooks:
            h.remove()
        eng._hooks = [p.register_post_accumulate_grad_hook(spy) for p in m.parameters()]
    step = TrainStep(m, flat, opt, eng, task="ica", use_graph=bool(a.graph), accum=a.accum,
                     split=None if a.split < 0 else bool(a.split))
    n_micro = a.steps * a.accum
    ragged_at = (n_micro // 2) // a.accum * a.accum + a.accum - 1  # a last micro-batch

    def site_batches(rank):
        """The micro-batches site ``rank`` trains on, in order (its own generator)."""
        g = torch.Generator(device=dev).manual_seed(100 + rank)  # site-specific data
        for i in range(n_micro):
            B = a.batch - 5 if (a.ragged and rank == 1 and i == ragged_at) else a.batch
            x = torch.randn(B, a.seq, 50, 10, device=dev, generator=g)
            y = torch.randint(0, 2, (B,), device=dev, generator=g)
            yield i, x, y

    g_first = None
    if a.feed == "device":
        if a.ragged:
            raise SystemExit("--feed device does not take --ragged")
        from dinunet_implementations_amd.ops import DeviceSource
        xs, ys = zip(*[(x, y) for _, x, y in site_batches(grp.rank)])
        src = DeviceSource(torch.cat(xs).to(torch.bfloat16), torch.cat(ys), a.batch)
        step.bind(src, steps_per_graph=2)
        step.run(a.steps)
    for i, x, y in (site_batches(grp.rank) if a.feed == "host" else ()):
        step(x, y, first=i % a.accum == 0, last=i % a.accum == a.accum - 1)
        if i == a.accum - 1:  # the first reduced gradient (every engine writes it to flat.grad)
            g_first = (flat.grad.double() * getattr(eng, "last_scale", 1.0)).clone()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    if getattr(eng, "peer", False):  # a timed-out wait of the peer exchange (sticky error words)
        from dinunet_implementations_amd.parallel import peer as _peer
        errs = grp.all_gather_object([(a.me, a.error()) for a in _peer.arenas()])
        if any(code for site in errs for _, code in site):  # which flags were left set
            dump = [(str(k), _peer.flag_state(ex)) for a_ in _peer.arenas()
                    for k, ex in a_._cache.items()]
            for r_, d_ in enumerate(grp.all_gather_object(dump)):
                if grp.rank == 0:
                    print(f"# site {r_} flags: {d_}", file=sys.stderr, flush=True)
    else:
        errs = None
    mine = flat.data.detach().cpu()
    allp = grp.all_gather(mine)
    same = all(torch.equal(p, allp[0]) for p in allp)
    if errs is not None and any(code for site in errs for _, code in site):
        same = False  # a timed-out wait: that step used incomplete data
    maxdiff = max(float((p - allp[0]).abs().max()) for p in allp)
    res = {"ok": bool(same), "world": grp.world, "engine": a.engine, "precision": a.precision,
           "payload": eng.wire, "collective": a.collective,
           "accum": a.accum, "ragged": a.ragged, "graph": step.graph is not None or bool(getattr(step, "_dgraphs", None)),
           "split": bool(step.split), "steps": opt.step_count, "max_abs_diff": maxdiff,
           "feed": a.feed, "adam_pack": getattr(step, "_apack", None) is not None,
           "peer": bool(getattr(eng, "peer", False)), "comm_graph": bool(step.comm_graph),
           "captured_update": bool(step.graph_opt or any(
               v[2] is True for v in getattr(step, "_dgraphs", {}).values()
               if isinstance(v, tuple) and len(v) == 3)),
           "param_sum": float(mine.double().sum()), "peer_errors": errs}
    if a.oracle:
        ok_o = torch.zeros(1, dtype=torch.float64, device=dev)
        if grp.rank == 0:
            torch.manual_seed(1234)
            mo = ICALstm(input_size=128, hidden_size=384, num_comps=50, window_size=10).to(dev).train()
            mo.classifier[0].p = 0.0
            fo = FlatParams(mo.parameters())
            oo = FusedAdam(fo, lr=1e-3)
            assert torch.equal(fo.data, init)
            reducer = oracle_reducer(a.engine, mo, fo, cfg, grp.world, dev)
            sites = [site_batches(r) for r in range(grp.world)]
            for s_i in range(a.steps):
                gs = []
                for r in range(grp.world):
                    fo.zero_grad()
                    for _k in range(a.accum):
                        _, x, y = next(sites[r])
                        _, loss, _ = mo.forward_loss(x, y)
                        (loss / a.accum).backward()
                    gs.append(fo.grad.double().clone())
                gm = reducer(gs)  # what the engine's reduction means, in fp64
                if s_i == 0 and g_first is not None:
                    res["grad_rel_err"] = float((g_first - gm).norm() / gm.norm().clamp_min(1e-30))
                    res["grad_max_abs_err"] = float((g_first - gm).abs().max())
                fo.grad.copy_(gm.float())
                oo.step()
            d_n = (flat.data - init).double()
            d_o = (fo.data - init).double()
            err = float((d_n - d_o).norm() / d_o.norm().clamp_min(1e-30))
            res["update_rel_err"] = err
            res["update_max_abs_err"] = float((d_n - d_o).abs().max())
            res["update_norm"] = float(d_o.norm())
            good = err <= a.oracle_tol
            if "grad_rel_err" in res:
                gt = a.grad_tol if a.grad_tol is not None else (1e-6 if a.precision == "32" else 2e-3)
                res["grad_tol"] = gt
                good = good and res["grad_rel_err"] <= gt
            res["oracle_tol"] = a.oracle_tol
            res["oracle_ok"] = bool(good)
            ok_o.fill_(1.0 if good else 0.0)
        grp.broadcast(ok_o, 0)
        same = same and bool(ok_o.item() > 0.5)
    if a.diag:
        res["notify_counts_per_param"] = {k: v / n_micro for k, v in counts.items() if v != n_micro}
        res["params_never_notified"] = [n for n, _ in m.named_parameters() if n not in counts]
    if grp.rank == 0:
        print(json.dumps(res), flush=True)
    shutdown()
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
