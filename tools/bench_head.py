#!/usr/bin/env python3
"""Fused MLP head fwd / bwd latency (CUDA events), ICA classifier and FS network shapes."""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dinunet_implementations_amd.ops.head import head_loss  # noqa: E402


def t_us(fn, reps=50):
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
    from dinunet_implementations_amd.models import MSANNet
    from dinunet_implementations_amd.ops.head import HeadSpec
    dev = "cuda"
    cases = [
        ("ICA head B=32 p=0", nn.Sequential(nn.Dropout(0.0), nn.Linear(384, 256), nn.BatchNorm1d(256),
                                         nn.ReLU(), nn.Linear(256, 64), nn.ReLU(), nn.Linear(64, 2)), 32, 384, False),
        ("ICA head B=32", nn.Sequential(nn.Dropout(0.25), nn.Linear(384, 256), nn.BatchNorm1d(256),
                                         nn.ReLU(), nn.Linear(256, 64), nn.ReLU(), nn.Linear(64, 2)), 32, 384, False),
        ("ICA head B=64", nn.Sequential(nn.Dropout(0.25), nn.Linear(384, 256), nn.BatchNorm1d(256),
                                         nn.ReLU(), nn.Linear(256, 64), nn.ReLU(), nn.Linear(64, 2)), 64, 384, False),
    ]
    fs = MSANNet(66, [256, 128, 64, 32], 2)
    cases.append(("FS MSANNet B=16", nn.Sequential(*[m for blk in fs.layers for m in blk], fs.fc_out), 16, 66, True))
    for name, mods, B, D, log_out in cases:
        mods = mods.to(dev).train()
        spec = HeadSpec(list(mods))
        x = torch.randn(B, D, device=dev, requires_grad=True)
        y = torch.randint(0, 2, (B,), device=dev)
        holder = {}

        def fwd():
            holder["r"] = head_loss(x, spec, y, log_out=log_out)

        def fwd_bwd():
            _, loss, _ = head_loss(x, spec, y, log_out=log_out)
            loss.backward()

        def ref():
            z = x
            for m in mods:
                z = m(z)
            loss = torch.nn.functional.cross_entropy(z, y)
            loss.backward()

        f = t_us(fwd)
        fb = t_us(fwd_bwd)
        r = t_us(ref)
        kf, kb = kernel_us(spec, x, y, log_out)
        stamps(spec, x, y, log_out)
        print(f"{name:18s} kernels: fwd {kf:6.1f} us  bwd {kb:6.1f} us | wall (python+launch): fused "
              f"fwd {f:6.1f}  fwd+bwd {fb:6.1f}  torch modules fwd+bwd {r:6.1f} us")


def stamps(spec, x, y, log_out):
    """Phase timestamps (s_memrealtime, 10 ns ticks) of one fwd + one bwd launch."""
    import ctypes
    from dinunet_implementations_amd.ops import _lib
    buf = torch.zeros(64, dtype=torch.int64, device=x.device)
    L = _lib.lib()
    L.dn_head_set_stamps.argtypes = [ctypes.c_void_p]
    L.dn_head_set_stamps(buf.data_ptr())
    xf = x.detach().clone().requires_grad_()
    _, loss, _ = head_loss(xf, spec, y, log_out=log_out)
    loss.backward()
    torch.cuda.synchronize()
    L.dn_head_set_stamps(None)
    b = buf.cpu().tolist()

    def show(tag, v):
        idx = [i for i, t in enumerate(v) if t]
        t0 = v[0]
        print(f"   {tag}: " + " ".join(f"{i}:{(v[i] - t0) / 100:.1f}" for i in idx) + " us")
    show("fwd (0-2 fwd0, 3-12 fwd1)", b[:16])
    show("bwd (16-21 bwd1, 24 bwd0 start)", b[16:32])
    # the training step's path: fwd1 + bwd1 fused in one launch (d loss known at forward time)
    from dinunet_implementations_amd.ops.head import loss_grad_hint
    buf.zero_()
    L.dn_head_set_stamps(buf.data_ptr())
    xf = x.detach().clone().requires_grad_()
    one = torch.ones((), device=x.device)
    with loss_grad_hint(one):
        _, loss, _ = head_loss(xf, spec, y, log_out=log_out)
    torch.autograd.backward(loss, one)
    torch.cuda.synchronize()
    L.dn_head_set_stamps(None)
    b = buf.cpu().tolist()
    t0 = b[0]
    idx = [i for i, t in enumerate(b) if t]
    print("   fused (0-2 fwd0, 3-12 fwd1, 16-21 bwd1, 24 bwd0): "
          + " ".join(f"{i}:{(b[i] - t0) / 100:.1f}" for i in idx) + " us")


def kernel_us(spec, x, y, log_out, n=20):
    """Pure GPU time per launch: n launches captured in a HIP graph, replayed."""
    from dinunet_implementations_amd.ops import _lib
    B = x.shape[0]
    lay = spec.layout(B)
    ws = torch.empty(lay[0], dtype=torch.uint8, device=x.device)
    out = torch.empty(B, spec.dims[-1], device=x.device)
    loss = torch.empty((), device=x.device)
    pred = torch.empty(B, dtype=torch.long, device=x.device)
    dx = torch.empty_like(x)
    one = torch.ones((), device=x.device)
    rng = spec.rng(x.device)
    pf, pb = spec.ptrs(False), spec.ptrs(True)
    xd = x.detach()

    def f():
        _lib.call("dn_head_fwd", spec.nl, spec._dims, spec._flags, spec._drops, spec._bnp, pf,
                  xd.data_ptr(), xd.stride(0), B, y.data_ptr(), out.data_ptr(), loss.data_ptr(),
                  pred.data_ptr(), rng.data_ptr(), ws.data_ptr(), 1, int(log_out), _lib.stream())

    def b():
        _lib.call("dn_head_bwd", spec.nl, spec._dims, spec._flags, spec._drops, spec._bnp, pb, B,
                  ws.data_ptr(), one.data_ptr(), dx.data_ptr(), x.shape[1], _lib.stream())

    res = []
    for fn in (f, b):
        f()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(n):
                fn()
        res.append(t_us(g.replay, reps=20) / n)
    return res

if __name__ == "__main__":
    main()
