#!/usr/bin/env python3
"""Sweep tile shape x split-K for every GEMM of the ICA-LSTM step (exact layouts / dtypes /
epilogues of ``ops.lstm`` and ``ops.linear``), timing 20 back-to-back launches with HIP events
(per-launch time incl. the split-K reduce).  Prints the best (tile, splits) per shape.

usage: python tools/bench_gemm_sweep.py [--B 32]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TILES = {0: "64x64", 1: "128x128"}


def t_loop(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / reps)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    args = ap.parse_args()
    from dinunet_implementations_amd.ops.gemm import mm, mm_grouped, choose_tiling
    dev = "cuda"
    N_ = args.B * 98
    bf = torch.bfloat16
    x = torch.randn(N_, 1000, device=dev)
    we = torch.randn(256, 1000, device=dev) * 0.03
    be = torch.randn(256, device=dev)
    enc = torch.randn(N_, 256, device=dev).to(bf)
    wih = (torch.randn(1536, 256, device=dev) * 0.05).to(bf)
    xp = torch.empty(N_, 1536, device=dev)
    hprev = torch.randn(2, N_, 192, device=dev).to(bf)
    whh = (torch.randn(2, 768, 192, device=dev) * 0.05).to(bf)
    bias = torch.randn(1536, device=dev)
    dpre = torch.randn(N_, 1536, device=dev).to(bf)
    gwih = torch.zeros(2, 768, 256, device=dev)
    gwhh = torch.zeros(2, 768, 192, device=dev)
    rmap = torch.randperm(768, device=dev).to(torch.int32)
    denc = torch.randn(N_, 256, device=dev).to(bf)
    gwe = torch.zeros(256, 1000, device=dev)

    cases = {
        "enc fwd  x W^T +b relu ->bf16": lambda t, s: mm(x, we, trans_b=True, bias=be, relu=True,
                                                         out_dtype=bf, tile=t, splits=s),
        "xp  enc Wih^T ->f32": lambda t, s: mm(enc, wih, trans_b=True, out=xp, tile=t, splits=s),
        "pre grouped h Whh^T +=": lambda t, s: mm_grouped(
            [dict(a=hprev[d], b=whh[d], out=xp[:, d * 768:(d + 1) * 768], beta=1.0,
                  bias=bias[d * 768:(d + 1) * 768]) for d in range(2)], trans_b=True, tile=t,
            splits=s),
        "dx  dpre Wih ->bf16": lambda t, s: mm(dpre, wih, out_dtype=bf, tile=t, splits=s),
        "dW grouped ih+hh (4 probs)": lambda t, s: mm_grouped(
            [p for d in range(2) for p in (
                dict(a=dpre[:, d * 768:(d + 1) * 768], b=enc, out=gwih[d], beta=1.0, row_map=rmap),
                dict(a=dpre[:, d * 768:(d + 1) * 768], b=hprev[d], out=gwhh[d], beta=1.0,
                     row_map=rmap))], trans_a=True, tile=t, splits=s),
        "dWe denc^T X": lambda t, s: mm(denc, x, trans_a=True, out=gwe, beta=1.0, tile=t, splits=s),
    }
    for name, fn in cases.items():
        res = []
        for t in TILES:
            for s in (1, 2, 3, 4, 6, 8):
                try:
                    us = t_loop(lambda: fn(t, s))
                except Exception as e:  # noqa: BLE001
                    print(f"  {name}: tile {t} splits {s} failed: {e}")
                    continue
                res.append((us, t, s))
        res.sort()
        auto = t_loop(lambda: fn(None, None))
        top = ", ".join(f"{TILES[t]}/s{s}: {us:.1f}" for us, t, s in res[:5])
        print(f"{name:32s} auto {auto:6.1f} us | best {top}", flush=True)


if __name__ == "__main__":
    main()
