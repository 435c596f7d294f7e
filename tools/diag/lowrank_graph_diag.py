"""Diagnostic: low-rank engine TrainStep determinism (eager vs eager, graph vs graph, eager vs
graph) with per-parameter max differences."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
from test_step_gpu import _batches, _run, _trainer  # noqa: E402

engine = sys.argv[1] if len(sys.argv) > 1 else "rankDAD"
xs, ys = _batches()
res = {}
for tag, g in (("e1", False), ("e2", False), ("g1", True), ("g2", True)):
    m, f, s = _trainer(0, engine=engine, use_graph=g)
    _run(s, xs, ys)
    res[tag] = (m, f)
names = [n for n, _ in res["e1"][0].named_parameters()]
for a, b in (("e1", "e2"), ("g1", "g2"), ("e1", "g1")):
    fa, fb = res[a][1], res[b][1]
    print(a, b, "max", float((fa.data - fb.data).abs().max()))
    for (n, pa), (_, pb) in zip(res[a][0].named_parameters(), res[b][0].named_parameters()):
        d = float((pa.detach() - pb.detach()).abs().max())
        if d > 1e-5:
            print("   ", n, d)
