#!/usr/bin/env python3
"""Run ONE ICA-step GEMM shape N times (for rocprofv3 --pmc passes), and print its CUDA-event time.
usage: python tools/gemm_one.py {enc,xp,dx,dw,dwstep} [reps] [rows = B*S, default 3136]

``dwstep`` is the training step's whole end-of-backward weight-gradient launch: LSTM dW_ih and
dW_hh of both directions with the bias column sums requested beside dW_hh, and the encoder dW with
its bias column sum (ops.gemm._place_colsums decides fold or separate problem;
DINUNET_COLSUM_FOLD=0 forces separate)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from dinunet_implementations_amd.ops.gemm import mm, mm_grouped
    which = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    N_ = int(sys.argv[3]) if len(sys.argv) > 3 else 3136
    dev, bf = "cuda", torch.bfloat16
    x = torch.randn(N_, 1000, device=dev).to(bf)
    we = torch.randn(256, 1000, device=dev) * 0.03
    be = torch.randn(256, device=dev)
    enc = torch.randn(N_, 256, device=dev).to(bf)
    wih = (torch.randn(1536, 256, device=dev) * 0.05).to(bf)
    xp = torch.empty(N_, 1536, device=dev)
    dpre = torch.randn(N_, 1536, device=dev).to(bf)
    hprev = torch.randn(2, N_, 192, device=dev).to(bf)
    denc = torch.randn(N_, 256, device=dev).to(bf)
    gwih = torch.zeros(2, 768, 256, device=dev)
    gwhh = torch.zeros(2, 768, 192, device=dev)
    gb = torch.zeros(2, 2, 768, device=dev)
    gwe = torch.zeros(256, 1000, device=dev)
    gbe = torch.zeros(256, device=dev)
    fns = {
        "enc": lambda: mm(x, we, trans_b=True, bias=be, relu=True, out_dtype=bf),
        "xp": lambda: mm(enc, wih, trans_b=True, out=xp),
        "dx": lambda: mm(dpre, wih, out_dtype=bf),
        "dw": lambda: mm_grouped([p for d in range(2) for p in (
            dict(a=dpre[:, d * 768:(d + 1) * 768], b=enc, out=gwih[d], beta=1.0),
            dict(a=dpre[:, d * 768:(d + 1) * 768], b=hprev[d], out=gwhh[d], beta=1.0))],
            trans_a=True),
        "dwstep": lambda: mm_grouped([p for d in range(2) for p in (
            dict(a=dpre[:, d * 768:(d + 1) * 768], b=enc, out=gwih[d], beta=1.0),
            dict(a=dpre[:, d * 768:(d + 1) * 768], b=hprev[d], out=gwhh[d], beta=1.0,
                 colsum=(gb[d, 0], gb[d, 1])))]
            + [dict(a=denc, b=x, out=gwe, beta=1.0, colsum=(gbe,))], trans_a=True),
    }
    for _ in range(3):
        fns[which]()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fns[which]()
    b.record()
    b.synchronize()
    print(f"ok {which} rows={N_} {a.elapsed_time(b) * 1e3 / reps:.1f} us/launch "
          f"(fold={os.environ.get('DINUNET_COLSUM_FOLD', '1')})")


if __name__ == "__main__":
    main()
