#!/usr/bin/env python3
"""Phase stamps of the replicated-forward head (csrc/kernels/head_rep.hip, s_memrealtime, 100 MHz),
workgroup 0, in us from its start: 1 W0 rows requested, 2 prologue (image, narrow weights,
parameters) in LDS, 3 layer 0 + A1, 4 narrow forward, 5 loss, 6 output-gradient chain, 7 dZ0,
8 dW tiles written, 9 dX written; prologue detail 10 labels stored, 11 input image stored, 12
narrow weight images stored, 13 parameter vectors stored (wave 0; the barrier after 13 waits for
the slowest wave); plus the launch time by HIP events (python included).

usage: python tools/head_rep_stamps.py [B] [dropout]"""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dinunet_implementations_amd.ops import _lib  # noqa: E402
from dinunet_implementations_amd.ops import head as H  # noqa: E402

_lib.register("dn_head_rep_set_stamps", [_lib.c_void_p])


def main():
    dev = "cuda"
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    p = float(sys.argv[2]) if len(sys.argv) > 2 else 0.25
    mods = nn.Sequential(nn.Dropout(p), nn.Linear(384, 256), nn.BatchNorm1d(256), nn.ReLU(),
                         nn.Linear(256, 64), nn.ReLU(), nn.Linear(64, 2)).to(dev).train()
    spec = H.HeadSpec(list(mods))
    x = torch.randn(B, 384, device=dev, requires_grad=True)
    y = torch.randint(0, 2, (B,), device=dev)
    one = torch.ones((), device=dev)

    from dinunet_implementations_amd.ops.lstm import use_persistent

    class Imgs:  # the fused Adam's bf16 weight images (ops.lstm.PersistentPack.bf16_of)
        used = False
        m = {id(mm.weight): mm.weight.detach().to(torch.bfloat16).contiguous()
             for mm in mods if isinstance(mm, nn.Linear)}

        def bf16_of(self, t):
            return self.m.get(id(t))

    imgs = Imgs()

    def run():
        with H.loss_grad_hint(one), use_persistent(imgs):
            _, loss, _ = H.head_loss(x, spec, y, log_out=False)
        torch.autograd.backward(loss, one)

    for _ in range(5):
        run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        run()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    st = torch.zeros(16, dtype=torch.int64, device=dev)
    _lib.lib().dn_head_rep_set_stamps(st.data_ptr())
    rows = []
    for _ in range(10):
        st.zero_()
        run()
        torch.cuda.synchronize()
        v = st.tolist()
        rows.append({k: (v[k] - v[0]) / 100.0 for k in range(16) if v[k]})
    _lib.lib().dn_head_rep_set_stamps(None)
    med = {k: sorted(r[k] for r in rows)[len(rows) // 2] for k in rows[0]}
    print(f"head_rep B={B} p={p}: launch (events incl. python) median {ts[len(ts)//2]:.1f} us")
    print("stamps (us, median of 10): " + " ".join(f"{k}:{t:.2f}" for k, t in sorted(med.items())))


if __name__ == "__main__":
    main()
