"""FreeSurfer MLP (``MSANNet``), reference ``comps/fs/models.py:4-31``.

Per hidden layer ``Linear(bias=False) -> BatchNorm1d(track_running_stats=False) -> ReLU``
(+ ``Dropout(0.5)`` for layer indices listed in ``dropout_in``), then ``fc_out`` with bias.
The BatchNorm never tracks running statistics, so evaluation also uses batch statistics
(SURVEY.md A5).  ``state_dict`` keys are identical to the reference:
``layers.{i}.0.weight``, ``layers.{i}.1.{weight,bias}``, ``fc_out.{weight,bias}``.

On a GPU ``forward_loss`` runs the whole network + log-softmax/NLL as one fused HIP launch
forward and one backward (``ops.head``); the module tree is kept for parameter ownership,
checkpoint compatibility, the CPU oracle path and ``forward`` (logits).
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch
import torch.nn as nn

from .. import ops


class MSANNet(nn.Module):
    def __init__(self, in_size: int, hidden_sizes: Sequence[int], out_size: int,
                 dropout_in: Sequence[int] = (), norm_layer: str = "batch"):
        super().__init__()
        self.in_size = int(in_size)
        self.out_size = int(out_size)
        self.hidden_sizes = [int(h) for h in hidden_sizes]
        self.dropout_in = list(dropout_in or [])
        self.layers = nn.ModuleList()
        d = self.in_size
        if norm_layer not in ("batch", "layer"):
            raise ValueError(f"norm_layer {norm_layer!r}: expected 'batch' or 'layer'")
        for i, h in enumerate(self.hidden_sizes):
            # "layer": the optional LayerNorm on its gfx950 kernels (ops.layernorm) in place of
            # the reference's BatchNorm1d
            norm = (nn.BatchNorm1d(h, track_running_stats=False) if norm_layer == "batch"
                    else ops.LayerNorm(h))
            block = [nn.Linear(d, h, bias=False), norm, nn.ReLU()]
            if i in self.dropout_in:
                block.append(nn.Dropout(p=0.5))
            self.layers.append(nn.Sequential(*block))
            d = h
        self.fc_out = nn.Linear(d, self.out_size)
        self.use_fused = True
        self._head: Optional[ops.HeadSpec] = None

    def head_spec(self) -> "ops.HeadSpec":
        if self._head is None:
            mods = [m for blk in self.layers for m in blk] + [self.fc_out]
            self._head = ops.HeadSpec(mods)
        return self._head

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        for layer in self.layers:
            x = layer(x)
        return self.fc_out(x)

    def forward_loss(self, x: torch.Tensor, y: torch.Tensor):
        """``(log_probs, nll_loss, argmax)`` (reference ``comps/fs/__init__.py:54-57``)."""
        if self.use_fused and x.is_cuda:
            return ops.head_loss(x, self.head_spec(), y, log_out=True)
        logits = self.forward(x)
        return ops.log_softmax_nll(logits, y)
