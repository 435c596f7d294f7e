"""Diagnostic: eager vs HIP-graph TrainStep losses (tests/test_step_gpu.py setup) under the
current environment switches (DINUNET_HEAD_STEP, DINUNET_SPLITK_REDUCE, ...)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from tests.test_step_gpu import _batches, _trainer  # noqa: E402


def main():
    xs, ys = _batches()
    _, fe, se = _trainer(0, use_graph=False)
    _, fg, sg = _trainer(0, use_graph=True)
    le, lg = [], []
    for i in range(xs.shape[0]):
        le.append(float(se(xs[i], ys[i]).detach()))
        lg.append(float(sg(xs[i], ys[i]).detach()))
        torch.cuda.synchronize()
        d = (fe.data - fg.data).abs().max().item()
        print(f"step {i}: eager {le[-1]:.6f} graph {lg[-1]:.6f} max|dparam| {d:.3e}", flush=True)


if __name__ == "__main__":
    main()
