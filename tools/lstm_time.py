#!/usr/bin/env python3
"""Wall time of the persistent LSTM kernels at the bench shape (B=32, S=98, H=384, bi-dir),
for A/B runs of kernel-library variants (``tools/build_variant.py``):

    python tools/lstm_time.py [lib.so ...]      # default: the in-tree library

Per library: median over 50 launches of dn_lstm_fwd and dn_lstm_bwd (HIP events), in us and
us per time step.
"""
import ctypes
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def time_lib(path, B=32, S=98, I=256, H=384, reps=50):
    from dinunet_implementations_amd.ops import mm
    lib = ctypes.CDLL(path)
    V, I_, F, L = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_long
    lib.dn_lstm_pack.argtypes = [V] * 8 + [I_] * 3 + [V] * 4 + [I_, V, V, V, V]
    lib.dn_lstm_fwd.argtypes = [V, V, V, I_, I_, I_, I_, V, V, V, V, F, V, V, V, I_, I_, V]
    lib.dn_lstm_bwd.argtypes = [V, V, V, V, L, L, F, V, V, I_, I_, I_, I_, V, I_, I_, V]
    lib.dn_lstm_rows_per_wg.argtypes = [I_, I_]
    lib.dn_lstm_padded_hidden.argtypes = [I_]
    dev = "cuda"
    Hd = H // 2
    HD = lib.dn_lstm_padded_hidden(Hd)
    ndir, GP = 2, 4 * HD
    BR = lib.dn_lstm_rows_per_wg(B, Hd)
    Bp = (B + BR - 1) // BR * BR
    g = torch.Generator(device=dev).manual_seed(0)
    ps = []
    for _ in range(ndir):
        ps += [torch.randn(4 * Hd, I, device=dev, generator=g) * 0.1,
               torch.randn(4 * Hd, device=dev, generator=g) * 0.1,
               torch.randn(4 * Hd, Hd, device=dev, generator=g) * 0.1,
               torch.randn(4 * Hd, device=dev, generator=g) * 0.1]
    wih_p = torch.empty(ndir * GP, I, dtype=torch.bfloat16, device=dev)
    bias_p = torch.empty(ndir * GP, device=dev)
    whh_p = torch.empty(ndir, GP, HD, dtype=torch.bfloat16, device=dev)
    whhT_p = torch.empty(ndir, HD, GP, dtype=torch.bfloat16, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    rc = lib.dn_lstm_pack(*[p.data_ptr() for p in ps], I, Hd, ndir, wih_p.data_ptr(),
                          bias_p.data_ptr(), whh_p.data_ptr(), whhT_p.data_ptr(), 0, None, None,
                          None, st)
    assert rc == 0, rc
    x = torch.randn(B * S, I, device=dev, generator=g).to(torch.bfloat16)
    xp = mm(x, wih_p, trans_b=True, out_dtype=torch.bfloat16)  # bf16 projection
    pre = torch.empty(xp.shape, dtype=torch.float32, device=dev)
    c_save = torch.empty(ndir, Bp, S, HD, device=dev)
    hprev = torch.empty(ndir, Bp, S, HD, dtype=torch.bfloat16, device=dev)
    hmean = torch.empty(B, ndir * Hd, device=dev)
    hT = torch.empty_like(hmean)
    cT = torch.empty_like(hmean)
    dout = torch.randn(B, ndir * Hd, device=dev, generator=g)
    dpre = torch.empty(Bp * S, ndir * GP, dtype=torch.bfloat16, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    tf, tb = [], []
    for it in range(reps + 5):
        ev[0].record()
        rc = lib.dn_lstm_fwd(xp.data_ptr(), bias_p.data_ptr(), whh_p.data_ptr(), B, S, Hd, ndir,
                             c_save.data_ptr(), hprev.data_ptr(), None, hmean.data_ptr(), 1.0 / S,
                             hT.data_ptr(), cT.data_ptr(), pre.data_ptr(), 0, 0, st)
        ev[1].record()
        assert rc == 0, rc
        ev[2].record()
        rc = lib.dn_lstm_bwd(pre.data_ptr(), c_save.data_ptr(), whhT_p.data_ptr(), dout.data_ptr(),
                             ndir * Hd, 0, 1.0 / S, None, None, B, S, Hd, ndir, dpre.data_ptr(), Bp, 0, st)
        ev[3].record()
        assert rc == 0, rc
        torch.cuda.synchronize()
        if it >= 5:
            tf.append(ev[0].elapsed_time(ev[1]) * 1000)
            tb.append(ev[2].elapsed_time(ev[3]) * 1000)
    f, b = statistics.median(tf), statistics.median(tb)
    chk = float(hmean.double().abs().sum()), float(dpre.float().abs().sum())
    return f, b, chk


def main():
    from dinunet_implementations_amd.ops import _lib
    libs = sys.argv[1:] or [_lib.LIB_PATH]
    for p in libs:
        f, b, chk = time_lib(p)
        print(f"{os.path.relpath(p, ROOT):70s} fwd {f:6.1f} us ({f / 98:.3f}/step)  bwd {b:6.1f} us "
              f"({b / 98:.3f}/step)  chk {chk[0]:.4f} {chk[1]:.2f}", flush=True)


if __name__ == "__main__":
    main()
