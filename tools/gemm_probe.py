#!/usr/bin/env python3
"""Probe where a GEMM's time goes: vary K / output dtype / shape for the xp GEMM geometry."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench_gemm_sweep import t_loop  # noqa: E402


def main():
    from dinunet_implementations_amd.ops.gemm import mm
    dev, bf = "cuda", torch.bfloat16
    for (M, N, K, od) in [(3136, 1536, 256, torch.float32), (3136, 1536, 256, bf),
                          (3136, 1536, 32, torch.float32), (3136, 1536, 32, bf),
                          (3136, 1536, 1024, bf), (3136, 256, 1024, bf), (3136, 256, 64, bf),
                          (64, 64, 64, bf), (64, 64, 1024, bf), (256, 256, 256, bf),
                          (1024, 1024, 256, bf), (2048, 2048, 256, bf)]:
        a = torch.randn(M, K, device=dev).to(bf)
        b = torch.randn(N, K, device=dev).to(bf)
        us = t_loop(lambda: mm(a, b, trans_b=True, out_dtype=od, splits=1, tile=0))
        print(f"M={M:5d} N={N:5d} K={K:5d} out={str(od)[6:]:9s} {us:7.1f} us  "
              f"{2 * M * N * K / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
