#!/usr/bin/env python3
"""GEMM shapes of the ICA-LSTM step: hand-written MFMA kernel vs hipBLASLt (torch.mm), CUDA events.

usage: python tools/bench_gemm.py [--rows 3136] [--tiles 0 1] [--splits 1 2 4 8]
(--rows = B*S: 3136 is the B=32 bench step, 200704 the B=2048 one)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


INNER = 10  # launches between the two events: per-launch host overhead overlaps GPU work


def t_us(fn, reps=15):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(INNER):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / INNER)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=3136)
    ap.add_argument("--tiles", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--out-bf16", action="store_true", help="bf16 outputs (the step's xp / enc)")
    args = ap.parse_args()
    from dinunet_implementations_amd.ops import mm
    from dinunet_implementations_amd.ops.gemm import choose_tiling
    dev = "cuda"
    N_ = args.rows
    # (name, M, N, K, ta, tb, a_dtype)
    shapes = [
        ("enc fwd  x[N,1000] W^T", N_, 256, 1000, False, True, torch.bfloat16),
        ("xp   enc[N,256] Wih^T", N_, 1536, 256, False, True, torch.bfloat16),
        ("pre  h[N,192] Whh^T", N_, 768, 192, False, True, torch.bfloat16),
        ("dx   dpre[N,1536] Wih", N_, 256, 1536, False, False, torch.bfloat16),
        ("dWih dpre^T x", 768, 256, N_, True, False, torch.bfloat16),
        ("dWhh dpre^T h", 768, 192, N_, True, False, torch.bfloat16),
        ("dWe  denc^T X", 256, 1000, N_, True, False, torch.bfloat16),
    ]
    print(f"{'shape':28s} {'M':>5} {'N':>5} {'K':>5}  {'ours us':>8} {'TF':>6}  {'hipBLASLt us':>12} {'TF':>6}  tiling")
    for name, M, N, K, ta, tb, dt in shapes:
        a = (torch.randn(K, M, device=dev) if ta else torch.randn(M, K, device=dev)).to(dt)
        b = (torch.randn(N, K, device=dev) if tb else torch.randn(K, N, device=dev)).to(torch.bfloat16)
        fl = 2.0 * M * N * K
        odt = torch.bfloat16 if args.out_bf16 else torch.float32
        ours = t_us(lambda: mm(a, b, trans_a=ta, trans_b=tb, out_dtype=odt))
        A = (a.t() if ta else a).to(torch.bfloat16)
        B = b.t() if tb else b
        lt = t_us(lambda: torch.mm(A, B, out_dtype=odt) if odt != torch.bfloat16 else torch.mm(A, B))
        print(f"{name:28s} {M:5d} {N:5d} {K:5d}  {ours:8.1f} {fl / ours / 1e6:6.0f}  {lt:12.1f} {fl / lt / 1e6:6.0f}  {choose_tiling(M, N, K)}")
        for tl in args.tiles:
            for sp in args.splits:
                o = t_us(lambda: mm(a, b, trans_a=ta, trans_b=tb, splits=sp, tile=tl, out_dtype=odt))
                print(f"      tile={tl} splits={sp}: {o:9.1f} us {fl / o / 1e6:6.0f} TF", flush=True)


if __name__ == "__main__":
    main()
