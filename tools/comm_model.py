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

    python tools/comm_model.py [--b-link-gbs 64] [--alpha-us 2 6] [--rings 4] [--from-json F]
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
    """pack + rowsum + unpack of one DirectMean exchange of ``n`` fp32 elements: (device us as a
    graph replay, us per exchange issued eagerly from Python)."""
    import torch
    from dinunet_implementations_amd.parallel import collective as C
    code, dt = C.PAYLOAD_TYPES[payload]
    chunk = C.chunk_for(n, world)
    x = torch.randn(n, device="cuda")
    send = torch.zeros(C.blocks_numel(world, chunk), dtype=dt, device="cuda")
    mine = torch.zeros(C.payload_numel(chunk), dtype=dt, device="cuda")

    def run():
        C.to_payload(x, send, world, chunk)
        C.rowsum(send, mine, world, chunk, 1.0 / world)
        C.from_payload(send, x, world, chunk, 1.0)
    # device time of the kernels (a graph replay), and separately what issuing them from Python
    # costs per exchange (ctypes launches: the host side of the eager exchange)
    run()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        run()
    return _time(gr.replay), _time(run)


def measure() -> dict:
    """The GPU-measured inputs of the model (see the module docstring)."""
    res = {at: split_graphs(at) for at in ("projection", "stem")}
    body = res["projection"][2]
    local, host = {}, {}
    for N in (2, 4, 8):
        for w in ("fp32", "fp16", "bf16"):
            local[f"{N}/{w}"], host[f"{N}/{w}"] = direct_kernels(int(body // 4), N, w)
    return {"graphs": {k: list(v) for k, v in res.items()}, "local_us": local,
            "local_eager_us": host}


def model(meas: dict, b_gbs: float, alpha: float, rings: int):
    """Rows of the exposed-communication table for one link-model parameter set."""
    b = b_gbs * 1e3  # bytes per us
    g = meas["graphs"]
    body, stem = g["projection"][2], g["projection"][3]
    rows = []
    for N in (2, 4, 8):
        for wire, coll in (("fp32", "ring all-reduce"), ("fp32", "direct"), ("fp16", "direct"),
                           ("bf16", "direct")):
            es = 4 if wire == "fp32" else 2
            nb, ns = body / 4 * es, stem / 4 * es
            if coll == "ring all-reduce":
                def t(by):
                    return 2 * (N - 1) / N * by / (rings * b) + 2 * (N - 1) * alpha
                loc = 0.0
            else:
                def t(by):
                    return 2 * (by / N / b + alpha)
                loc = meas["local_us"][f"{N}/{wire}"]
            tbody, tstem = t(nb) + loc, t(ns)
            rows.append({"N": N, "wire": wire, "collective": coll, "t_body_us": tbody,
                         "t_stem_us": tstem, "local_us": loc,
                         "exposed_projection_us": max(0.0, tbody - g["projection"][1]) + tstem,
                         "exposed_stem_us": max(0.0, tbody - g["stem"][1]) + tstem})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b-link-gbs", type=float, default=64.0,
                    help="effective per-link one-direction xGMI bandwidth an RCCL channel gets")
    ap.add_argument("--alpha-us", type=float, nargs="+", default=[2.0, 6.0],
                    help="per-hop / per-phase latencies to tabulate")
    ap.add_argument("--rings", type=int, default=4, help="concurrent rings (channels) of RCCL")
    ap.add_argument("--from-json", default=None,
                    help="model from a previous run's measurements (the JSON line it printed)")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r4_comm_model.md"))
    a = ap.parse_args()
    if a.from_json:
        with open(a.from_json) as f:
            meas = json.loads(f.read().strip().splitlines()[-1])
        meas.setdefault("local_us", {f"{r['N']}/{r['wire']}": r["local_us"] for r in meas.get("rows", [])
                                     if r["collective"] == "direct"})
    else:
        meas = measure()
    g = meas["graphs"]
    lines = ["# Multi-site dSGD step: exposed-communication model (1 MI355X measured + link model)",
             "",
             "Measured on one MI355X (`tools/comm_model.py`): the split step's two graphs at the "
             "headline config (ICA-LSTM B=32, S=98, H=384) and the direct exchange's local kernels "
             "(pack + fp32 rowsum + unpack of the body bucket).  The transfers come from a link "
             "model, NOT a measurement (no multi-GPU run is available to the builder): per-link "
             f"one-direction bandwidth {a.b_link_gbs} GB/s, RCCL ring all-reduce over {a.rings} "
             "concurrent rings `2(N-1)/N * bytes / (rings * b) + 2(N-1) * alpha`, direct exchange "
             "`2 * (bytes / N / b + alpha)` (all-to-all + all-gather, every peer on its own link).  "
             "No scaling curve is claimed.", "",
             "| cut | graph A us | graph B us (hides the body bucket) | body bucket MB | stem bucket MB |",
             "|---|---:|---:|---:|---:|"]
    for at, (xa, xb, bb, sb) in g.items():
        lines.append(f"| {at} | {xa:.1f} | {xb:.1f} | {bb / 2**20:.2f} | {sb / 2**20:.2f} |")
    for alpha in a.alpha_us:
        lines += ["", f"alpha = {alpha} us:", "",
                  "| N | wire | collective | T(body) us | T(stem) us | local kernels us | exposed us (cut: projection) | exposed us (cut: stem) |",
                  "|---:|---|---|---:|---:|---:|---:|---:|"]
        for r in model(meas, a.b_link_gbs, alpha, a.rings):
            lines.append(f"| {r['N']} | {r['wire']} | {r['collective']} | {r['t_body_us']:.1f} | "
                         f"{r['t_stem_us']:.1f} | {r['local_us']:.1f} | "
                         f"{r['exposed_projection_us']:.1f} | {r['exposed_stem_us']:.1f} |")
    lines += ["", "Exposed = max(0, T(body) - T(graph B)) + T(stem): the body (LSTM + head) bucket's "
              "collective runs between the replays under graph B; the stem (encoder) bucket's after "
              "it.  Local kernels (device time of pack + rowsum + unpack, graph replay) run on the "
              "comm stream inside T(body); issued eagerly from Python the same three launches "
              "take the `local_eager_us` of the JSON line (host-bound)."]
    with open(a.out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))
    print(json.dumps(meas))


if __name__ == "__main__":
    sys.exit(main())
