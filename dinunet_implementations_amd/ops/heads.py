"""Standalone loss heads (used when the classifier itself is not fused, see ``ops.head``).

``softmax_ce``  : ICA head, reference ``comps/icalstm/__init__.py:59-63``
``log_softmax_nll``: FS head, reference ``comps/fs/__init__.py:54-57``
Both return ``(out, loss, pred)`` where ``out`` is the probability (ICA) or log-probability (FS)
tensor, exactly what the reference trainers hand to their metrics.
"""
from __future__ import annotations

import torch

from . import _lib
from . import reference as ref

_lib.register("dn_softmax_xent", [_lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_int,
                                  _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                                  _lib.c_void_p, _lib.c_void_p])


class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, y, log_out: bool):
        z = z.float().contiguous()
        y = y.long().contiguous()
        B, C = z.shape
        out = torch.empty_like(z)
        dz = torch.empty_like(z)
        loss = torch.empty((), dtype=torch.float32, device=z.device)
        pred = torch.empty(B, dtype=torch.long, device=z.device)
        _lib.call("dn_softmax_xent", z.data_ptr(), y.data_ptr(), B, C, int(log_out),
                  out.data_ptr(), dz.data_ptr(), loss.data_ptr(), pred.data_ptr(), _lib.stream())
        ctx.save_for_backward(dz)
        ctx.mark_non_differentiable(out, pred)
        return out, loss, pred

    @staticmethod
    def backward(ctx, dout, dloss, dpred):
        (dz,) = ctx.saved_tensors
        if dloss is None:
            return None, None, None
        return dz * dloss, None, None


def softmax_ce(logits: torch.Tensor, labels: torch.Tensor):
    if logits.is_cuda:
        return _SoftmaxXent.apply(logits, labels, False)
    return ref.softmax_ce(logits, labels)


def log_softmax_nll(logits: torch.Tensor, labels: torch.Tensor):
    if logits.is_cuda:
        return _SoftmaxXent.apply(logits, labels, True)
    return ref.log_softmax_nll(logits, labels)
