#!/usr/bin/env python3
"""Encoder GEMM candidates at the bench shape (rocprofv3 --stats gives the kernel times):
hand-written bias+ReLU GEMM vs hipBLASLt (torch._addmm_activation, fused RELU_BIAS epilogue)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dinunet_implementations_amd.ops.gemm import mm  # noqa: E402

M, K, N = 3136, 1000, 256
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = torch.randn(N, K, device="cuda") * 0.03
b = torch.randn(N, device="cuda")
wb, bb = w.to(torch.bfloat16), b.to(torch.bfloat16)
for _ in range(50):
    y0 = mm(x, w, trans_b=True, bias=b, relu=True, out_dtype=torch.bfloat16)
    y1 = torch._addmm_activation(bb, x, wb.t())
    y2 = torch.relu(torch.addmm(bb, x, wb.t()))
torch.cuda.synchronize()
ref = torch.relu(x.float() @ wb.float().t() + b)
print("err hand", ((y0.float() - ref).norm() / ref.norm()).item(),
      "err lt", ((y1.float() - ref).norm() / ref.norm()).item())
