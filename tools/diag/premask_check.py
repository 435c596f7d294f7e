#!/usr/bin/env python3
"""Which kernel-library entry points does one eager ICA training step call?  (Checks that the
encoder's ReLU mask rides in the LSTM dX GEMM: no dn_relu_bwd call.)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dinunet_implementations_amd.models import ICALstm  # noqa: E402
from dinunet_implementations_amd.ops import _lib  # noqa: E402

calls = []
orig = _lib.call


def spy(name, *a):
    calls.append(name)
    return orig(name, *a)


_lib.call = spy
import dinunet_implementations_amd.ops.linear as lin  # noqa: E402
import dinunet_implementations_amd.ops.lstm as lstm  # noqa: E402
import dinunet_implementations_amd.ops.gemm as gemm  # noqa: E402
for m in (lin, lstm, gemm):
    if hasattr(m, "_lib"):
        m._lib.call = spy
torch.manual_seed(0)
m = ICALstm(input_size=256, hidden_size=384, num_comps=100, window_size=10).cuda().train()
x = torch.randn(32, 98, 100, 10, device="cuda")
y = torch.randint(0, 2, (32,), device="cuda")
enc = m.stem(x)
_, loss, _ = m.body_loss(enc, y)
loss.backward()
torch.cuda.synchronize()
print("calls:", calls)
print("relu_bwd launched:", "dn_relu_bwd" in calls)
