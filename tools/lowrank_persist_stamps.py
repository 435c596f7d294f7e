#!/usr/bin/env python3
"""Phase stamps (s_memrealtime, 100 MHz) of the one-launch rank-dAD power iteration
(lowrank.hip lr_persist_kernel), member 0 of every layer, ICA-LSTM headline geometry; plus the
launch time by events.  Per iteration: A = Q staged + P = G Q, pub = P / Gram partials published,
bar1 = first barrier, gram = partial sums + P staged, chol+H = Cholesky + G^T P, solve = Q rows /
Psend published (hsum: the G^T P partial sums of the column blocks first), bar2 = second
barrier (us)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from dinunet_implementations_amd.models import ICALstm
    from dinunet_implementations_amd.ops import FlatParams, _lib
    from dinunet_implementations_amd.parallel import make_engine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    torch.manual_seed(0)
    m = ICALstm(input_size=256, hidden_size=384, num_comps=100, window_size=10).cuda()
    flat = FlatParams(m.parameters())
    eng = make_engine("rankDAD", m, flat, SiteGroup(device=torch.device("cuda")),
                      {"dad_reduction_rank": 10, "dad_num_pow_iters": 5, "dad_tol": 0.0})
    flat.grad.normal_()
    t = eng._table
    for _ in range(5):
        t.persist(5, 0.0)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(20):
        ev[0].record()
        t.persist(5, 0.0)
        ev[1].record()
        ev[1].synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
    ts.sort()
    st = torch.zeros(8 * 64, dtype=torch.int64, device="cuda")
    L = _lib.lib()
    L.dn_lr_persist_set_stamps(ctypes.c_void_p(st.data_ptr()))
    t.persist(5, 0.0)
    torch.cuda.synchronize()
    L.dn_lr_persist_set_stamps(ctypes.c_void_p(None))
    v = st.view(8, 64).tolist()
    print(f"persistent launch (5 iterations, {t.n} layers): median {ts[len(ts)//2]:.1f} us by events")
    for l in range(t.n):
        row = v[l]
        base = row[0]
        out = [f"layer {l}: G load {(row[1] - base) / 100:.2f}"]
        for it in range(5):
            sb = 1 + 10 * it
            d = lambda a_, b_: (row[sb + b_] - row[sb + a_]) / 100  # noqa: E731
            out.append(f"it{it} A={d(0, 1):.2f} pub={d(1, 2):.2f} bar1={d(2, 3):.2f} "
                       f"gram={d(3, 4):.2f} chol={d(4, 8):.2f} H={d(8, 5):.2f} "
                       f"hsum={d(5, 9):.2f} solve={d(9, 6):.2f} bar2={d(6, 7):.2f}")
        print(" | ".join(out))
    # whole-launch span on the global clock: first member-0 entry to last member-0 exit, and
    # per layer entry -> stamp 0 (argument loads, G load issue) and last barrier -> exit
    ent = [v[l][60] for l in range(t.n)]
    ext = [v[l][61] for l in range(t.n)]
    print(f"member-0 span: entries within {(max(ent) - min(ent)) / 100:.2f} us, first entry -> "
          f"last exit {(max(ext) - min(ent)) / 100:.2f} us; per layer entry->stamp0 " +
          " ".join(f"{(v[l][0] - v[l][60]) / 100:.2f}" for l in range(t.n)) +
          "; last bar2->exit " + " ".join(f"{(v[l][61] - v[l][48]) / 100:.2f}" for l in range(t.n)))


if __name__ == "__main__":
    main()
