#!/usr/bin/env python3
"""Split-capture device-fed steps with and without the Adam-emitted pack, one site (split
forced), compared step by step: parameters, Adam's device counter, the cursor, and the persistent
operand images against a fresh pack of the same parameters."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from dinunet_implementations_amd.models import ICALstm
    from dinunet_implementations_amd.ops import DeviceSource, FlatParams, FusedAdam
    from dinunet_implementations_amd.ops.lstm import pack_params
    from dinunet_implementations_amd.parallel import make_engine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    from dinunet_implementations_amd.runtime import step as step_mod
    g = torch.Generator(device="cuda").manual_seed(7)
    X = torch.randn(64, 24, 50, 10, device="cuda", generator=g).to(torch.bfloat16)
    Y = torch.randint(0, 2, (64,), device="cuda", generator=g)
    runs = {}
    for ap in (False, True):
        step_mod.ADAM_PACK = ap
        torch.manual_seed(1234)
        m = ICALstm(input_size=128, hidden_size=384, num_comps=50, window_size=10).cuda().train()
        m.classifier[0].p = 0.0
        flat = FlatParams(m.parameters())
        opt = FusedAdam(flat, lr=1e-3)
        eng = make_engine("dSGD", m, flat, SiteGroup(device=torch.device("cuda")),
                          {"precision_bits": "32"})
        st = step_mod.TrainStep(m, flat, opt, eng, task="ica", split=True)
        src = DeviceSource(X, Y, 8)
        st.bind(src, steps_per_graph=1)
        hist = []
        for i in range(7):
            st.run(1)
            torch.cuda.synchronize()
            rec = {"data": flat.data.clone(), "cursor": int(src.cursor.item()),
                   "count": opt.step_count,
                   "tdev": int(opt._tdev.item()) if opt._tdev is not None else None,
                   "loss": float(st.last_loss)}
            if ap and st._apack is not None:
                pp = st._apack
                lin = m.encoder[0]
                params = [t for cell in m.lstm.lstms for t in cell.params()]
                casts = []
                w, b, h, hT, _ = pack_params(params, m.lstm.input_size, flat.data.device,
                                             casts=(lin.weight, lin.bias), cast_out=casts)
                torch.cuda.synchronize()
                n = b.numel()
                rec["img"] = [bool(torch.equal(pp.wih_p, w)), bool(torch.equal(pp.whh_p, h)),
                              bool(torch.equal(pp.whhT_p, hT)),
                              float((pp.bias_p[:n] + pp.bias_p[n:] - b).abs().max()),
                              bool(torch.equal(pp.casts[0], casts[0]))]
            hist.append(rec)
        runs[ap] = (hist, st)
    for i, (a, b) in enumerate(zip(runs[False][0], runs[True][0])):
        d = float((a["data"] - b["data"]).abs().max())
        print(f"step {i + 1}: maxdiff {d:.3e}  cursor {a['cursor']}/{b['cursor']}  count "
              f"{a['count']}/{b['count']}  tdev {a['tdev']}/{b['tdev']}  loss {a['loss']:.6f}/"
              f"{b['loss']:.6f}  images(after) {b.get('img')}", flush=True)


if __name__ == "__main__":
    main()
