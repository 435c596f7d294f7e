#!/usr/bin/env python3
"""Peer exchange check on ONE GPU: N site processes (``torch.distributed.run``, gloo group for
the IPC-handle exchange only, every rank on cuda:0) run ``parallel.peer.PeerMean`` /
``PeerGather`` -- real cross-process device traffic through IPC-mapped HBM -- eagerly and inside a
captured HIP graph replayed several times with fresh data, and compare with an fp64 reference.

    python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 \\
        tools/peer_check.py --wire fp16

Prints one JSON line (rank 0): per wire, the max relative error of the mean against fp64, whether
every rank holds bit-identical means, the gather's exactness, and the device time per exchange.
Exit status 0 iff every check passes.
"""
import argparse
import json
import os
import sys

os.environ.setdefault("DINUNET_BACKEND", "gloo")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# relative error bounds of the mean vs fp64: fp32 wire = one fp32 rounding per add; bf16 / fp16 =
# the site value and the mean rounded once each to the wire type (fp16 block-scaled: 11 bits)
TOL = {"fp32": 1e-6, "bf16": 1.6e-2, "fp16": 2e-3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--wire", default="all", help="fp32 | bf16 | fp16 | all")
    ap.add_argument("--n", type=int, default=1_063_106, help="elements (default: the ICA model)")
    ap.add_argument("--reps", type=int, default=4, help="graph replays with fresh data")
    ap.add_argument("--time", type=int, default=20, help="timed graph replays")
    a = ap.parse_args()

    import torch
    from dinunet_implementations_amd.parallel import init_sites, shutdown
    from dinunet_implementations_amd.parallel import peer

    grp = init_sites()
    dev = grp.device
    W, me = grp.world, grp.rank
    wires = ["fp32", "bf16", "fp16"] if a.wire == "all" else [a.wire]
    res = {"world": W, "n": a.n, "ok": True}

    def site_data(step, rank, n):
        g = torch.Generator(device="cpu").manual_seed(1000 * step + rank)
        # gradient-like: a wide dynamic range (tiny and large blocks)
        x = torch.randn(n, generator=g) * torch.exp2(torch.randint(-30, 4, (n // 4096 + 1,),
                                                                    generator=g).float()
                                                      ).repeat_interleave(4096)[:n]
        return x

    for wire in wires:
        pm = peer.mean(grp, dev, a.n, wire, ("check", wire))
        pg = peer.gather(grp, dev, 5003, wire, ("check", wire))
        x = torch.empty(a.n, dtype=torch.float32, device=dev)
        gsrc = torch.empty(5003, dtype=torch.float32, device=dev)
        gdst = torch.empty(W * 5008, dtype=torch.float32, device=dev)
        worst, same, gerr = 0.0, True, 0.0

        def check(step, out, gout):
            nonlocal worst, same, gerr
            xs_ = [site_data(step, r, a.n).double() for r in range(W)]
            ref = sum(xs_) / W
            mag = sum(v.abs() for v in xs_) / W  # the scale every rounding is relative to
            o = out.detach().cpu().double()
            err = float(((o - ref).abs() / mag.clamp_min(1e-38)).max())
            worst = max(worst, err)
            outs = grp.all_gather(out.detach().cpu())
            same = same and all(torch.equal(t, outs[0]) for t in outs)
            for r in range(W):
                want = site_data(step, r, 5003).double()
                got = gout.cpu().view(W, 5008)[r, :5003].double()
                e = float(((got - want).abs() / want.abs().clamp_min(1e-30))
                          [want.abs() > want.abs().max() * 2 ** -12].max())
                gerr = max(gerr, e)

        # eager
        x.copy_(site_data(0, me, a.n))
        gsrc.copy_(site_data(0, me, 5003))
        pm.run_(x)
        pg.run(gsrc, gdst, 5008)
        torch.cuda.synchronize()
        check(0, x, gdst)
        # captured: the exchange is a graph of ordinary kernels, replayed with fresh data
        xs = torch.empty_like(x)
        gs = torch.empty_like(gsrc)
        gr = torch.cuda.CUDAGraph()
        grp.barrier()
        with torch.cuda.graph(gr):
            x.copy_(xs)
            pm.run_(x)
            pg.run(gs, gdst, 5008)
        for step in range(1, 1 + a.reps):
            xs.copy_(site_data(step, me, a.n))
            gs.copy_(site_data(step, me, 5003))
            gr.replay()
            torch.cuda.synchronize()
            check(step, x, gdst)
        # device time per exchange (mean + gather; replays back to back, every rank together)
        grp.barrier()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(a.time):
            gr.replay()
        t1.record()
        torch.cuda.synchronize()
        us = t0.elapsed_time(t1) * 1e3 / max(1, a.time)
        # two exchanges pushed back to back, then finished together (peer.finish_many)
        n2 = a.n // 3 + 77
        pm2 = peer.mean(grp, dev, n2, wire, ("check2", wire))
        y1, y2 = torch.empty(a.n, device=dev), torch.empty(n2, device=dev)
        y1.copy_(site_data(11, me, a.n))
        y2.copy_(site_data(12, me, n2))
        pm.start(y1)
        pm2.start(y2)
        peer.finish_many([(pm, y1, 1.0), (pm2, y2, 1.0)])
        torch.cuda.synchronize()
        for step_, out_, n_ in ((11, y1, a.n), (12, y2, n2)):
            xs_ = [site_data(step_, r, n_).double() for r in range(W)]
            ref = sum(xs_) / W
            mag = sum(v.abs() for v in xs_) / W
            worst = max(worst, float(((out_.cpu().double() - ref).abs() / mag.clamp_min(1e-38)).max()))
            outs = grp.all_gather(out_.cpu())
            same = same and all(torch.equal(t, outs[0]) for t in outs)
        err_word = pm.ar.error()
        ok = worst <= TOL[wire] and same and gerr <= TOL[wire] and err_word == 0
        res[wire] = {"mean_rel_err": worst, "replicas_identical": same, "gather_rel_err": gerr,
                     "us_per_exchange": round(us, 1), "error_word": err_word, "ok": ok}
        res["ok"] = res["ok"] and ok
    flags = torch.tensor([1.0 if res["ok"] else 0.0])
    grp.all_reduce(flags, op=torch.distributed.ReduceOp.MIN)
    res["ok"] = bool(flags.item() > 0.5)
    if me == 0:
        print(json.dumps(res), flush=True)
    grp.barrier()
    shutdown()
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
