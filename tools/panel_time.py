#!/usr/bin/env python3
"""Time the LSTM input projection C = A W^T (bf16) at the ICA shapes: the row-panel kernel
(csrc/kernels/panel.hip, every column-group width) against the 256 x 256 / 64 x 64 tile kernels.
Prints one JSON line per batch size."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from dinunet_implementations_amd.ops import _lib
    from dinunet_implementations_amd.ops import gemm as G
    dev = torch.device("cuda", 0)
    K, N = 256, 1536
    for B in [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "32,512,2048,4096").split(",")]:
        M = B * 98
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.1).to(torch.bfloat16)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

        def timed(fn, reps=20):
            for _ in range(3):
                fn()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0.record()
            for _ in range(reps):
                fn()
            t1.record()
            torch.cuda.synchronize()
            return round(t0.elapsed_time(t1) * 1e3 / reps, 1)

        res = {"B": B, "M": M}
        tile = 2 if M >= 65536 else 0
        res["tile_us"] = timed(lambda: G.mm(a, w, trans_b=True, out_dtype=torch.bfloat16, tile=tile))
        ref = G.mm(a, w, trans_b=True, out_dtype=torch.bfloat16, tile=tile)
        for ncol in (0, 128, 256, 384, 512):
            fn = lambda: _lib.lib().dn_panel_gemm(a.data_ptr(), K, w.data_ptr(), K, c.data_ptr(), N,
                                                  M, N, K, ncol, _lib.stream())
            res[f"panel{ncol}_us"] = timed(fn)
            fn()
            torch.cuda.synchronize()
            res[f"panel{ncol}_equal"] = bool(torch.equal(c, ref))
        bytes_ = M * K * 2 + M * N * 2
        res["panel_best_TBps"] = round(bytes_ / min(v for k, v in res.items() if k.startswith("panel") and k.endswith("_us")) / 1e6, 2)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
