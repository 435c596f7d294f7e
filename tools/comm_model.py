#!/usr/bin/env python3
"""Exposed-communication model of the multi-site dSGD step.

No multi-GPU run is available to this builder, so this does NOT claim a scaling curve.  It
measures on ONE MI355X what the N > 1 step is made of and combines it with a stated link model:

* the split step's two graphs at the headline config (``runtime.step.TrainStep`` split capture):
  graph A (forward + backward down to the cut) and graph B (what remains after the cut, under
  which the LSTM + head gradient bucket is all-reduced), for the cut at the LSTM input projection
  (default) and at the encoder output (``DINUNET_SPLIT_AT=stem``, the round-3 cut);
* the local kernels of the direct exchange (``parallel.collective.DirectMean``: pack, fp32 rowsum,
  unpack) at the bucket sizes and world sizes 2 / 4 / 8 (what the fp16 / bf16 wire costs on top
  of the transfers);
* the transfer itself from a link model (xGMI, fully connected 8-GPU node): ring all-reduce
  ``2 (N-1)/N * bytes / (c * b) + 2 (N-1) * alpha`` with ``c`` rings on distinct links, direct
  exchange ``2 * (bytes / N / b + alpha)`` (all-to-all + all-gather, every peer on its own link).
  ``b`` (per-link, one direction) and ``alpha`` (per-hop latency) are parameters, printed with
  the result.

Exposed communication per step = max(0, T(body bucket) - T(graph B)) + T(stem bucket): the body
bucket's collective starts between the replays, the stem (encoder) bucket after graph B.

    python tools/comm_model.py [--b-link-gbs 64] [--alpha-us 6] [--rings 4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _time(fn, iters: int = 50, warm: int = 5) -> float:
    import torch
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters  # us


def split_graphs(at: str):
    """(graph A us, graph B us, body bucket bytes, stem bucket bytes) of the headline step."""
    import torch
    from dinunet_implementations_amd.models import ICALstm
    from dinunet_implementations_amd.ops import FlatParams, FusedAdam
    from dinunet_implementations_amd.parallel import make_engine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    from dinunet_implementations_amd.runtime import step as S
    S.SPLIT_AT_PROJECTION = at == "projection"
    torch.manual_seed(0)
    m = ICALstm(input_size=256, hidden_size=384, num_comps=100, window_size=10).cuda().train()
    flat = FlatParams(m.parameters())
    opt = FusedAdam(flat, lr=1e-3)
    eng = make_engine("dSGD", m, flat, SiteGroup(device=torch.device("cuda")), {})
    st = S.TrainStep(m, flat, opt, eng, task="ica", split=True)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(32, 98, 100, 10, device="cuda", generator=g)
    y = torch.randint(0, 2, (32,), device="cuda", generator=g)
    for _ in range(5):  # eager warm-up + capture
        st(x, y)
    torch.cuda.synchronize()
    assert st.graph is not None and st.graph_b is not None and st.split_at == at, st.split_at
    ta = _time(st.graph.replay)
    tb = _time(st.graph_b.replay)
    body = sum(e - s for i, (s, e) in enumerate(eng.buckets) if i in st._first_buckets) * 4
    stem = sum(e - s for i, (s, e) in enumerate(eng.buckets) if i not in st._first_buckets) * 4
    return ta, tb, body, stem


def direct_kernels(n: int, world: int, payload: str) -> float:
    """pack + rowsum + unpack of one DirectMean exchange of ``n`` fp32 elements (us)."""
    import torch
    from dinunet_implementations_amd.parallel import collective as C
    code, dt = C.PAYLOAD_TYPES[payload]
    chunk = max(8, -(-n // (8 * world)) * 8)
    x = torch.randn(n, device="cuda")
    send = torch.zeros(C.blocks_numel(world, chunk), dtype=dt, device="cuda")
    mine = torch.zeros(C.HDR + chunk, dtype=dt, device="cuda")
    amax = torch.zeros(1, dtype=torch.int32, device="cuda") if dt == torch.float16 else None

    def run():
        C.to_payload(x, send, world, chunk, amax=amax)
        C.rowsum(send, mine, world, chunk, 1.0 / world)
        C.from_payload(send, x, world, chunk, 1.0, amax=amax)
    return _time(run)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b-link-gbs", type=float, default=64.0,
                    help="effective per-link one-direction xGMI bandwidth an RCCL channel gets")
    ap.add_argument("--alpha-us", type=float, default=6.0, help="per-hop / per-phase latency")
    ap.add_argument("--rings", type=int, default=4, help="concurrent rings (channels) of RCCL")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r4_comm_model.md"))
    a = ap.parse_args()
    b = a.b_link_gbs * 1e3  # bytes per us
    res = {}
    for at in ("projection", "stem"):
        res[at] = split_graphs(at)
    ta, tb, body, stem = res["projection"]
    rows = []
    lines = ["# Multi-site dSGD step: exposed-communication model (1 MI355X measured + link model)",
             "",
             "Measured on one MI355X (`tools/comm_model.py`): the split step's graphs at the "
             "headline config (ICA-LSTM B=32, S=98, H=384).  Link model (NOT measured: no multi-GPU "
             f"run is available to the builder): per-link one-direction bandwidth {a.b_link_gbs} "
             f"GB/s, per-phase latency {a.alpha_us} us, RCCL ring all-reduce over {a.rings} "
             "concurrent rings; direct exchange = all-to-all + all-gather with every peer on its "
             "own link.  No scaling curve is claimed.", "",
             "| cut | graph A us | graph B us (hides the body bucket) | body bucket MB | stem bucket MB |",
             "|---|---:|---:|---:|---:|"]
    for at, (xa, xb, bb, sb) in res.items():
        lines.append(f"| {at} | {xa:.1f} | {xb:.1f} | {bb / 2**20:.2f} | {sb / 2**20:.2f} |")
    lines += ["", "| N | wire | collective | T(body) us | T(stem) us | local kernels us | exposed us (cut: projection) | exposed us (cut: stem) |",
              "|---:|---|---|---:|---:|---:|---:|---:|"]
    for N in (2, 4, 8):
        for wire, coll in (("fp32", "ring all-reduce"), ("fp32", "direct"), ("fp16", "direct"),
                           ("bf16", "direct")):
            es = 4 if wire == "fp32" else 2
            nb, ns = body / 4 * es, stem / 4 * es
            if coll == "ring all-reduce":
                t = lambda by: 2 * (N - 1) / N * by / (a.rings * b) + 2 * (N - 1) * a.alpha_us
                loc = 0.0
            else:
                t = lambda by: 2 * (by / N / b + a.alpha_us)
                loc = direct_kernels(int(body // 4), N, wire)
            tbody, tstem = t(nb) + loc, t(ns)
            exp_p = max(0.0, tbody - res["projection"][1]) + tstem
            exp_s = max(0.0, tbody - res["stem"][1]) + tstem
            rows.append({"N": N, "wire": wire, "collective": coll, "t_body_us": tbody,
                         "t_stem_us": tstem, "local_us": loc, "exposed_projection_us": exp_p,
                         "exposed_stem_us": exp_s})
            lines.append(f"| {N} | {wire} | {coll} | {tbody:.1f} | {tstem:.1f} | {loc:.1f} | "
                         f"{exp_p:.1f} | {exp_s:.1f} |")
    lines += ["", "Exposed = max(0, T(body) - T(graph B)) + T(stem): the body (LSTM + head) bucket's "
              "collective runs between the replays under graph B; the stem (encoder) bucket's after "
              "it.  Local kernels = the direct exchange's pack + fp32 rowsum + unpack, measured "
              "(they run on the comm stream, inside T(body))."]
    with open(a.out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))
    print(json.dumps({"graphs": {k: list(v) for k, v in res.items()}, "rows": rows}))


if __name__ == "__main__":
    sys.exit(main())
