"""FreeSurfer MLP (``MSANNet``), reference ``comps/fs/models.py:4-31``.

Per hidden layer ``Linear(bias=False) -> BatchNorm1d(track_running_stats=False) -> ReLU``
(+ ``Dropout(0.5)`` for layer indices listed in ``dropout_in``), then ``fc_out`` with bias.
The BatchNorm never tracks running statistics, so evaluation also uses batch statistics
(SURVEY.md A5).  ``state_dict`` keys are identical to the reference:
``layers.{i}.0.weight``, ``layers.{i}.1.{weight,bias}``, ``fc_out.{weight,bias}``.

On a GPU the whole forward+backward of the default 66->256->128->64->32->2 network runs as one
fused HIP kernel per direction (``ops.fs_mlp``); the module tree below is kept for parameter
ownership, checkpoint compatibility and the CPU oracle path.
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.nn as nn

from .. import ops


class MSANNet(nn.Module):
    def __init__(self, in_size: int, hidden_sizes: Sequence[int], out_size: int,
                 dropout_in: Sequence[int] = ()):
        super().__init__()
        self.in_size = int(in_size)
        self.out_size = int(out_size)
        self.hidden_sizes = [int(h) for h in hidden_sizes]
        self.dropout_in = list(dropout_in or [])
        self.layers = nn.ModuleList()
        d = self.in_size
        for i, h in enumerate(self.hidden_sizes):
            block = [nn.Linear(d, h, bias=False), nn.BatchNorm1d(h, track_running_stats=False),
                     nn.ReLU()]
            if i in self.dropout_in:
                block.append(nn.Dropout(p=0.5))
            self.layers.append(nn.Sequential(*block))
            d = h
        self.fc_out = nn.Linear(d, self.out_size)
        self.use_fused = True

    def fused_ok(self, x: torch.Tensor) -> bool:
        return (self.use_fused and x.is_cuda and not self.dropout_in
                and ops.fs_mlp_supported(self.in_size, self.hidden_sizes, self.out_size, x.shape[0]))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.fused_ok(x):
            ws = [blk[0].weight for blk in self.layers]
            gs = [blk[1].weight for blk in self.layers]
            bs = [blk[1].bias for blk in self.layers]
            return ops.fs_mlp(x, ws, gs, bs, self.fc_out.weight, self.fc_out.bias,
                              eps=self.layers[0][1].eps)
        for layer in self.layers:
            x = layer(x)
        return self.fc_out(x)
