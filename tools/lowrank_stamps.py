#!/usr/bin/env python3
"""Phase timestamps (shader clock, s_memtime) of lr_gtp, per ICA layer, from a diagnostic
build: ``python tools/build_variant.py lrst -DLR_STAMPS`` then on the GPU
``DINUNET_KERNEL_LIB=dinunet_implementations_amd/_native/variants/lrst/libdinunet_kernels.so
python tools/lowrank_stamps.py``.  Phases: 0 start, 1 P staged (G loads issued), 2 Gram
partials, 3 G^T P partials, 4 merged, 5 Cholesky (wave 0), 6 Q solved + committed, 7 norms."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from dinunet_implementations_amd.ops import _lib  # noqa: E402
from lowrank_bench import ICA, table  # noqa: E402


def main():
    t, _ = table(ICA)
    L = _lib.lib()
    buf = torch.zeros(8 * len(ICA), dtype=torch.int64, device="cuda")
    L.dn_lr_set_stamps.argtypes = [ctypes.c_void_p]
    assert L.dn_lr_set_stamps(buf.data_ptr()) == 0
    st = _lib.stream

    def stage(s_, it):
        _lib.call("dn_lr_stage", t.table.data_ptr(), t.host_table(), t.n, s_, it, 0.0, st())
    acc = torch.zeros(len(ICA), 7, dtype=torch.float64)
    reps = 20
    for k in range(reps + 3):
        stage(0, 0)
        stage(1, 0)
        torch.cuda.synchronize()
        if k >= 3:
            v = buf.view(len(ICA), 8).cpu().double()
            acc += v[:, 1:] - v[:, :-1]
    acc /= reps
    names = ["P staged", "Gram", "G^T P", "merge", "Cholesky", "Q solve+commit", "norms"]
    print("cycles per phase (last column block of each layer, mean of %d launches)" % reps)
    print(f"{'layer':10s} " + " ".join(f"{n:>13s}" for n in names) + "        total")
    for i, nm in enumerate(ICA):
        print(f"{nm:10s} " + " ".join(f"{x:13.0f}" for x in acc[i].tolist())
              + f" {acc[i].sum().item():12.0f}")
    L.dn_lr_set_stamps(None)


if __name__ == "__main__":
    main()
