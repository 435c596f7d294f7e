#!/usr/bin/env python3
"""Diagnostic: per-phase cycle shares of the persistent LSTM kernels (s_memtime stamps).

Builds csrc/kernels/lstm.hip with -DDN_STAMPS into a separate .so (the production library is
untouched), runs fwd + bwd at the bench shape and prints, per wave, the average cycles per time
step spent in (a) the recurrent MFMA phase (until the first accumulator is consumed), (b) the
gate/elementwise phase, (c) the workgroup barrier.  Read the SHARES, not the absolute lengths
(stamps serialize the scheduler).
"""
import ctypes
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SRC = os.path.join(ROOT, "dinunet_implementations_amd", "csrc", "kernels", "lstm.hip")
OUT = os.path.join(ROOT, "tools", "_stamps", "libdn_lstm_stamps.so")


def build():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-fno-slp-vectorize",
                           "-DDN_STAMPS", "-I", os.path.dirname(SRC), SRC, "-o", OUT])


def main():
    if not os.path.exists(OUT):
        build()
    from dinunet_implementations_amd.ops import mm, _lib
    from dinunet_implementations_amd.ops.lstm import padded_hidden
    lib = ctypes.CDLL(OUT)
    V, I_, F, L = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_long
    lib.dn_lstm_pack.argtypes = [V] * 8 + [I_] * 3 + [V] * 4 + [I_, V, V, V, V]
    lib.dn_lstm_fwd.argtypes = [V, V, V, I_, I_, I_, I_, V, V, V, V, F, V, V, V, I_, I_, V]
    lib.dn_lstm_bwd.argtypes = [V, V, V, V, L, L, F, V, V, I_, I_, I_, I_, V, I_, I_, V]
    lib.dn_set_stamp_buf.argtypes = [V]
    dev = "cuda"
    B, S, I, H = int(os.environ.get("B", 32)), 98, 256, 384
    Hd = H // 2
    HD = padded_hidden(Hd)
    ndir = 2
    GP = 4 * HD
    BR = int(_lib.lib().dn_lstm_rows_per_wg(B, Hd)); Bp = (B + BR - 1) // BR * BR
    torch.manual_seed(0)
    ps = []
    for _ in range(ndir):
        ps += [torch.randn(4 * Hd, I, device=dev) * 0.1, torch.randn(4 * Hd, device=dev) * 0.1,
               torch.randn(4 * Hd, Hd, device=dev) * 0.1, torch.randn(4 * Hd, device=dev) * 0.1]
    wih_p = torch.empty(ndir * GP, I, dtype=torch.bfloat16, device=dev)
    bias_p = torch.empty(ndir * GP, device=dev)
    whh_p = torch.empty(ndir, GP, HD, dtype=torch.bfloat16, device=dev)
    whhT_p = torch.empty(ndir, HD, GP, dtype=torch.bfloat16, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    lib.dn_lstm_pack(*[p.data_ptr() for p in ps], I, Hd, ndir, wih_p.data_ptr(), bias_p.data_ptr(),
                     whh_p.data_ptr(), whhT_p.data_ptr(), 0, None, None, None, st)
    x = torch.randn(B * S, I, device=dev).to(torch.bfloat16)
    xp = mm(x, wih_p, trans_b=True, out_dtype=torch.bfloat16)  # bf16 projection
    pre = torch.empty(xp.shape, dtype=torch.float32, device=dev)
    c_save = torch.empty(ndir, Bp, S, HD, device=dev)
    hprev = torch.empty(ndir, Bp, S, HD, dtype=torch.bfloat16, device=dev)
    hmean = torch.empty(B, ndir * Hd, device=dev)
    hT = torch.empty_like(hmean)
    cT = torch.empty_like(hmean)
    buf = torch.zeros(512 * 4, dtype=torch.int64, device=dev)
    lib.dn_set_stamp_buf(ctypes.c_void_p(buf.data_ptr()))
    dout = torch.randn(B, ndir * Hd, device=dev)
    dpre = torch.empty(Bp * S, ndir * GP, dtype=torch.bfloat16, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for it in range(3):
        ev[0].record()
        lib.dn_lstm_fwd(xp.data_ptr(), bias_p.data_ptr(), whh_p.data_ptr(), B, S, Hd, ndir,
                        c_save.data_ptr(), hprev.data_ptr(), None, hmean.data_ptr(), 1.0 / S,
                        hT.data_ptr(), cT.data_ptr(), pre.data_ptr(), 0, 0, st)
        ev[1].record()
        ev[2].record()
        lib.dn_lstm_bwd(pre.data_ptr(), c_save.data_ptr(), whhT_p.data_ptr(), dout.data_ptr(),
                        ndir * Hd, 0, 1.0 / S, None, None, B, S, Hd, ndir, dpre.data_ptr(), Bp, 0, st)
        ev[3].record()
        torch.cuda.synchronize()
    fwd_us = ev[0].elapsed_time(ev[1]) * 1000
    bwd_us = ev[2].elapsed_time(ev[3]) * 1000
    b = buf.view(512, 4).cpu()
    print(f"stamped build: fwd {fwd_us:.1f} us ({fwd_us / S:.2f} us/step), bwd {bwd_us:.1f} us "
          f"({bwd_us / S:.2f} us/step)")
    for name, base in (("fwd", 0), ("bwd", 256)):
        rows = b[base:base + 64 * ndir]
        rows = rows[rows[:, 3] > 0]
        if len(rows) == 0:
            continue
        per = rows[:, :3].double() / rows[:, 3:4].double()
        tot = per.sum(1)
        print(f"{name}: waves={len(rows)}  cycles/step  mfma {per[:, 0].mean():7.0f}  "
              f"gates {per[:, 1].mean():7.0f}  barrier {per[:, 2].mean():7.0f}  total {tot.mean():7.0f}"
              f"   (min/max total {tot.min():.0f}/{tot.max():.0f})")
        for w in (0, len(rows) // 2, len(rows) - 1):
            print(f"   wave {w:2d}: {per[w, 0]:6.0f} {per[w, 1]:6.0f} {per[w, 2]:6.0f}")


if __name__ == "__main__":
    main()
