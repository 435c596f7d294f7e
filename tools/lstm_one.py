#!/usr/bin/env python3
"""Bench-shape fused bi-LSTM forward + backward, N times (for rocprofv3 --pmc passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dinunet_implementations_amd.ops.lstm import bilstm  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
B, S, I, Hd = 32, 98, 256, 192
ps = []
for d in range(2):
    ps.append(tuple((torch.randn(*s, device="cuda") * 0.1).requires_grad_() for s in
                    ((4 * Hd, I), (4 * Hd,), (4 * Hd, Hd), (4 * Hd,))))
x = torch.randn(B, S, I, device="cuda").to(torch.bfloat16).requires_grad_()
for _ in range(n):
    out, _ = bilstm(x, ps, reduce="mean")
    out.sum().backward()
torch.cuda.synchronize()
print("ok")
