#!/usr/bin/env python3
"""Device-fed (Adam-emitted pack -> replicated head) vs host-fed per-step losses (diagnostic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
from test_step_gpu import _batches, _trainer  # noqa: E402
from dinunet_implementations_amd.ops import head as H  # noqa: E402
from dinunet_implementations_amd.runtime.feed import DeviceFeed  # noqa: E402

xs, ys = _batches(n=8)
B = xs.shape[1]
X = xs.reshape(-1, *xs.shape[2:]).to(torch.bfloat16)
Y = ys.reshape(-1)
_, fh, sh = _trainer(0, use_graph=True)
_, fd, sd = _trainer(0, use_graph=True)
feed = DeviceFeed(sd, X, Y, B, 8, col=1, steps_per_graph=4)
hl = []
for c in range(8):
    xb, yb = feed.src.batch(c)
    hl.append(float(sh(xb.float(), yb)))
n0 = H.REP_LAUNCHES
losses, scores, labels = feed.run_epoch(torch.arange(64, device="cuda"))
torch.cuda.synchronize()
print("rep launches", H.REP_LAUNCHES - n0)
print("host  ", [round(v, 5) for v in hl])
print("device", [round(v, 5) for v in losses.tolist()])
print("last_loss host", float(sh.last_loss), "device", float(sd.last_loss))
print("param max diff", float((fh.data - fd.data).abs().max()))
