#!/usr/bin/env python3
"""GEMM shapes of the ICA-LSTM step: hand-written MFMA kernel vs hipBLASLt (torch.mm), CUDA events.

usage: python tools/bench_gemm.py [--splits ...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t_us(fn, reps=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    from dinunet_implementations_amd.ops import mm
    from dinunet_implementations_amd.ops.gemm import choose_tiling
    dev = "cuda"
    N_ = 3136
    # (name, M, N, K, ta, tb, a_dtype)
    shapes = [
        ("enc fwd  x[N,1000] W^T", N_, 256, 1000, False, True, torch.float32),
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
        ours = t_us(lambda: mm(a, b, trans_a=ta, trans_b=tb))
        A = (a.t() if ta else a).to(torch.bfloat16)
        B = b.t() if tb else b
        lt = t_us(lambda: torch.mm(A, B))
        print(f"{name:28s} {M:5d} {N:5d} {K:5d}  {ours:8.1f} {fl / ours / 1e6:6.0f}  {lt:12.1f} {fl / lt / 1e6:6.0f}  {choose_tiling(M, N, K)}")
        for sp in (1, 2, 4, 8):
            o = t_us(lambda: mm(a, b, trans_a=ta, trans_b=tb, splits=sp))
            print(f"      splits={sp}: {o:7.1f} us")


if __name__ == "__main__":
    main()
