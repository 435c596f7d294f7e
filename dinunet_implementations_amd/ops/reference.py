"""Pure-PyTorch restatement of the reference math.

This module is the numerics oracle: every HIP kernel is tested against it, and it is the
execution path on CPU (gloo plumbing tests, ``SiteRunner`` on a laptop).  It reproduces the
reference quirks listed in SURVEY.md Appendix A:

* A1  i, f, o gates use sigma(sigma(x)); g = tanh of the last quarter; gate rows ordered
  ``[i|f|o|g]`` (``comps/icalstm/models.py:32-37``).
* A2  per-direction hidden = hidden_size // 2; the reverse direction runs on the time-flipped
  sequence and its outputs stay in processing order (``models.py:55,62-63``).
* A3  ``num_layers`` is ignored (``models.py:52,57``).
* A4  the encoder sees each window flattened C-major then W (``models.py:107``).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


def lstm_cell_seq(x: Tensor, w_ih: Tensor, b_ih: Optional[Tensor], w_hh: Tensor,
                  b_hh: Optional[Tensor], h0: Optional[Tuple[Tensor, Tensor]] = None,
                  cell=None) -> Tuple[Tensor, Tuple[Tensor, Tensor]]:
    """One direction of the reference LSTMCell over a ``[B, S, I]`` sequence.

    Mirrors ``comps/icalstm/models.py:20-45`` (double sigmoid on i/f/o).
    Returns ``hidden_seq [B, S, H]`` and the final ``(h, c)``.
    """
    B, S, _ = x.shape
    H = w_hh.shape[1]
    if h0 is None:
        h = x.new_zeros(B, H)
        c = x.new_zeros(B, H)
    else:
        h, c = h0
    # the input projection is time-parallel: hoist it out of the recurrence
    xp = F.linear(x, w_ih, b_ih)
    outs = []
    hprevs = []
    for t in range(S):
        hprevs.append(h)
        pre = xp[:, t] + F.linear(h, w_hh, b_hh)
        s = pre[:, :3 * H].sigmoid()
        i = torch.sigmoid(s[:, :H])
        f = torch.sigmoid(s[:, H:2 * H])
        o = torch.sigmoid(s[:, 2 * H:3 * H])
        g = torch.tanh(pre[:, 3 * H:])
        c = f * c + i * g
        h = o * torch.tanh(c)
        outs.append(h)
    if cell is not None and xp.requires_grad:
        from . import capture as _cap
        if _cap.active() is not None:
            # rank-dAD capture: d(pre_t) == d(xp_t) == d(h2h out_t) for every t
            a_ih = x.detach().reshape(B * S, -1)
            a_hh = torch.stack(hprevs, 1).detach().reshape(B * S, H)

            def _hook(g, cell=cell, a_ih=a_ih, a_hh=a_hh):
                d = g.detach().reshape(B * S, -1)
                _cap.record(cell.i2h, a_ih, d)
                _cap.record(cell.h2h, a_hh, d)
            xp.register_hook(_hook)
    return torch.stack(outs, 1), (h, c)


def bilstm(x: Tensor, params, bidirectional: bool = True, modules=None):
    """Reference bi-LSTM wrapper (``comps/icalstm/models.py:59-66``).

    ``params`` is a list (one per direction) of ``(w_ih, b_ih, w_hh, b_hh)``.
    """
    mods = list(modules) if modules is not None else [None, None]
    hs, (h, c) = lstm_cell_seq(x, *params[0], cell=mods[0])
    if bidirectional:
        rhs, (rh, rc) = lstm_cell_seq(torch.flip(x, (1,)), *params[1], cell=mods[1])
        hs = torch.cat([hs, rhs], 2)
        h = torch.cat([h, rh], 1)
        c = torch.cat([c, rc], 1)
    return hs, (h, c)


def ica_windows(data: Tensor, window_size: int, window_stride: int, temporal_size: int) -> Tensor:
    """``[N, C, T] -> [N, S, C, W]`` with ``S = int(T / W)`` and offset ``j * stride``.

    Reproduces quirk A9 (``comps/icalstm/__init__.py:28-32``): the window *count* comes from the
    window size, the *offset* from the stride.
    """
    S = int(temporal_size / window_size)
    idx = torch.arange(S).unsqueeze(1) * window_stride + torch.arange(window_size).unsqueeze(0)
    if int(idx.max()) >= data.shape[2]:
        raise ValueError(f"windowing needs {int(idx.max()) + 1} time points, data has "
                         f"{data.shape[2]}")
    # [N, C, S, W] -> [N, S, C, W]
    return data[:, :, idx].permute(0, 2, 1, 3).contiguous()


def softmax_ce(logits: Tensor, labels: Tensor):
    """Reference ICA loss head (``comps/icalstm/__init__.py:60-63``)."""
    prob = torch.softmax(logits, 1)
    loss = F.cross_entropy(logits, labels)
    return prob, loss, prob.argmax(1)


def log_softmax_nll(logits: Tensor, labels: Tensor):
    """Reference FS loss head (``comps/fs/__init__.py:54-57``)."""
    out = F.log_softmax(logits, 1)
    loss = F.nll_loss(out, labels)
    return out, loss, out.argmax(1)


def adam_(params, grads, exp_avg, exp_avg_sq, step: int, lr: float, beta1: float = 0.9,
          beta2: float = 0.999, eps: float = 1e-8, weight_decay: float = 0.0):
    """torch.optim.Adam (non-amsgrad, L2 weight decay) restated on flat fp32 tensors."""
    g = grads if weight_decay == 0 else grads + weight_decay * params
    exp_avg.mul_(beta1).add_(g, alpha=1 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (exp_avg_sq.sqrt() / (bc2 ** 0.5)).add_(eps)
    params.addcdiv_(exp_avg, denom, value=-lr / bc1)
    return params
