#!/usr/bin/env python3
"""Per-op timing of the ICA-LSTM hot path on one GPU (CUDA events, median of N reps).

usage: python tools/bench_ops.py [--batch 32] [--reps 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000.0)
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--hidden", type=int, default=384)
    a = ap.parse_args()
    from dinunet_implementations_amd.ops import _lib, mm
    from dinunet_implementations_amd.ops.lstm import bilstm
    dev = "cuda"
    B, S, C, W, I, H = a.batch, 98, 100, 10, 256, a.hidden
    Hd = H // 2
    res = {}
    x = torch.randn(B * S, C * W, device=dev)
    we = torch.randn(I, C * W, device=dev) * 0.03
    be = torch.randn(I, device=dev)
    res["enc_gemm_bias_relu"] = timeit(lambda: mm(x, we, trans_b=True, bias=be, relu=True,
                                                  out_dtype=torch.bfloat16), a.reps)
    enc = torch.randn(B, S, I, device=dev).to(torch.bfloat16)
    ps = []
    for _ in range(2):
        ps.append(tuple((torch.randn(*s, device=dev) * 0.1).requires_grad_() for s in
                        [(4 * Hd, I), (4 * Hd,), (4 * Hd, Hd), (4 * Hd,)]))
    encg = enc.clone().requires_grad_()

    def fwd():
        return bilstm(encg, ps, reduce="mean")

    res["lstm_fwd_total"] = timeit(fwd, a.reps)
    out, _ = fwd()
    g = torch.randn_like(out)

    def fwdbwd():
        o, _ = bilstm(encg, ps, reduce="mean")
        o.backward(g)

    res["lstm_fwd_bwd_total"] = timeit(fwdbwd, a.reps)
    # kernel-only timings via a profiler pass
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(10):
            fwdbwd()
        torch.cuda.synchronize()
    kt = {}
    for ev in prof.key_averages():
        if ev.device_time_total > 0:
            kt[ev.key[:90]] = (round(ev.device_time_total / max(ev.count, 1), 1), ev.count)
    out = {k: [round(v[0], 1), round(v[1], 1)] for k, v in res.items()}
    print(json.dumps({"batch": B, "median_min_us": out}, indent=1))
    for k, v in sorted(kt.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
        print(f"{v[0]:9.1f} us x{v[1]:4d}  {k}")


if __name__ == "__main__":
    main()
