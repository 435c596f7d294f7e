"""Device-fed training epochs: the step the benchmark times is the step the site loop runs.

The reference trains by iterating a DataLoader on the host and calling ``iteration(batch)`` per
batch (``/root/reference/local.py:49`` -> ``comps/icalstm/__init__.py:56-70``), with a
``loss.item()`` host sync per step (``:67-68``).  Here a site's train split is resident in HBM as
bf16 (:class:`ops.DeviceSource`), and an epoch is ONE host call:

* the epoch's batch order is drawn on the host by the train loader's own pass logic
  (``data.loader.DeviceLoader.iter_indices``: same per-pass shuffles, ``drop_last``
  (``local.py:29``), cycling for sites with fewer batches than the global step count, resume
  position), and copied into the source's order buffer in place;
* ``TrainStep.run`` replays graphs of K whole steps: batch gather, forward, backward, engine
  reduction, fused Adam that also emits the next step's operands, with no host work between
  steps;
* every step writes its ``prob[:, 1]`` column and its loss into device rings
  (:class:`ops.StepRecorder`), so the per-epoch train loss and train AUC are exact
  (``comps/icalstm/__init__.py:64-68``) and cost one device-to-host read per epoch.

``bench.py`` drives the same object (``DeviceFeed.run``) for the timed steps, and
``runtime.site.FederatedSite`` drives it per epoch (``run_epoch``).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ..ops import DeviceSource, StepRecorder


def default_graph_steps(steps: int, cap: int = 10) -> int:
    """Steps per HIP graph: the largest divisor of ``steps`` up to ``cap`` when that is at least
    half the cap (no remainder graph), else ``cap`` (one remainder graph)."""
    steps = max(1, int(steps))
    d = max(k for k in range(1, min(cap, steps) + 1) if steps % k == 0)
    return d if 2 * d >= min(cap, steps) else min(cap, steps)


class DeviceFeed:
    """``nb`` device-fed steps per pass over a resident ``(X, Y)`` with per-step train records.

    ``step``: a :class:`runtime.step.TrainStep` (bound here); ``X`` ``[N, *sample]`` (any float
    dtype, converted once to bf16 in HBM), ``Y`` ``[N]`` labels; ``batch`` samples per step;
    ``nb`` steps per pass (an epoch's step count); with gradient accumulation
    (``step.accum`` = ``local_iterations`` > 1) a step takes ``accum`` batches, so the order
    buffer holds ``nb * accum * batch`` rows and the records are per batch (micro-batch);
    ``col``: the score column of the step's output the train metric ranks (ICA: 1; -1: the
    predicted class, FS's hard-label scores)."""

    def __init__(self, step, X: torch.Tensor, Y: torch.Tensor, batch: int, nb: int,
                 col: int = 1, steps_per_graph: Optional[int] = None):
        if not X.is_cuda:
            raise ValueError("DeviceFeed: the dataset must live on the GPU")
        self.step = step
        self.B = int(batch)
        self.nb = int(nb)
        if self.nb < 1 or X.shape[0] < 1:
            raise ValueError("DeviceFeed: no steps")
        self.A = max(1, int(getattr(step, "accum", 1)))
        self.nbb = self.nb * self.A  # batches per pass
        # bf16 in HBM for models that take a bf16 batch (ICA: the encoder GEMM rounds its operand
        # anyway); fp32 otherwise (FS features, gathered exactly into an fp32 static input)
        if getattr(step.model, "accepts_bf16_input", False):
            Xb = X if X.dtype == torch.bfloat16 else X.to(torch.bfloat16)
        else:
            Xb = X.float()
        rows = torch.arange(self.nbb * self.B, device=X.device) % X.shape[0]
        self.src = DeviceSource(Xb, Y, self.B, order=rows)
        self.rec = StepRecorder(self.nbb, self.B, self.src.cursor, col=col)
        K = steps_per_graph or default_graph_steps(self.nb)
        step.bind(self.src, steps_per_graph=K, recorder=self.rec)

    # ---- epochs of the site loop --------------------------------------------------------------
    def run_epoch(self, order: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """Train ``nb`` steps on the batches ``order`` (``[nb * accum * batch]`` row indices, the
        epoch's batch sequence); returns the device tensors ``(losses [nb * accum], scores
        [nb * accum * B], labels [nb * accum * B])`` of the epoch's per-batch train records."""
        if order.numel() != self.nbb * self.B:
            raise ValueError(f"DeviceFeed.run_epoch: order of {order.numel()} rows, want "
                             f"{self.nbb * self.B}")
        self.src.set_order(order)
        self.src.cursor.zero_()
        self.step.run(self.nb)
        return self.rec.losses, self.rec.scores.view(-1), self.src.labels_of(self.nbb)

    # ---- free-running steps (bench.py) --------------------------------------------------------
    def run(self, n: int):
        """``n`` steps continuing at the cursor (the pass wraps); returns the last loss."""
        return self.step.run(n)

    def prepare(self, n: int):
        """Capture every graph a following :meth:`run` of ``n`` / :meth:`run_epoch` replays."""
        self.step.prepare(n)
