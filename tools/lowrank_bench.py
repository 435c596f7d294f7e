#!/usr/bin/env python3
"""Per-launch times of the low-rank factorisation kernels (csrc/kernels/lowrank.hip) on the ICA
model's large Linear gradients (rank 10), all layers per table and each layer alone:

    python tools/lowrank_bench.py
"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dinunet_implementations_amd.ops import _lib  # noqa: E402
from dinunet_implementations_amd.parallel.lowrank import LowRankTable  # noqa: E402

SHAPES = {"encoder": (256, 1000), "i2h": (768, 256), "h2h": (768, 192), "cls1": (256, 384),
          "cls4": (64, 256)}
ICA = ["encoder", "i2h", "i2h", "h2h", "h2h", "cls1", "cls4"]


def table(names, r=10, dev="cuda", err=False):
    g = torch.Generator(device=dev).manual_seed(0)
    layers = []
    for nme in names:
        o, i = SHAPES[nme]
        G = torch.randn(o, i, device=dev, generator=g)
        Q = torch.linalg.qr(torch.randn(i, r, device=dev, generator=g))[0].contiguous()
        E = torch.randn(o, i, device=dev, generator=g) * 0.1 if err else None
        layers.append((G, E, torch.empty(o, r, device=dev), torch.empty(o, r, device=dev), Q))
    return LowRankTable(layers, dev), layers


def timeit(fn, reps=50):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for k in range(reps + 5):
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        if k >= 5:
            ts.append(ev[0].elapsed_time(ev[1]) * 1000)
    return statistics.median(ts)


def main():
    st = _lib.stream
    tiny = torch.zeros(4, device="cuda")
    print(f"floor (one tiny torch launch) {timeit(lambda: tiny.add_(0)):6.1f} us", flush=True)
    r = int(os.environ.get("LR_RANK", "10"))
    err = os.environ.get("LR_ERR", "0") == "1"  # PowerSGD: error feedback + recon timed too
    print(f"rank {r}, error feedback {err}", flush=True)
    for label, names in [("ICA (all 7)", ICA)] + [(n, [n]) for n in SHAPES]:
        t, _ = table(names, r=r, err=err)
        L = _lib.lib()
        stage = lambda s_, it: _lib.call("dn_lr_stage", t.table.data_ptr(), t.host_table(),
                                         t.n, s_, it, 0.0, st())
        stage(0, 0)
        stage(1, 0)
        t_gq = timeit(lambda: stage(0, 0))
        t_gt = timeit(lambda: stage(1, 0))
        t_iter = timeit(lambda: (stage(0, 0), stage(1, 0)))
        t_rc = timeit(t.recon_ef) if err else float("nan")
        print(f"{label:14s} gq {t_gq:6.1f}  gtp (Gram Cholesky + P R^-1 + G^T Pn) {t_gt:6.1f}"
              f"  iteration {t_iter:6.1f}  recon {t_rc:6.1f} us   blocks {t.blocks1}/{t.blocks3}",
              flush=True)


if __name__ == "__main__":
    main()
