"""Fused ``relu(x W^T + b)`` (the ICA encoder, reference ``comps/icalstm/models.py:87,107``).

Forward is ONE MFMA GEMM with the bias+ReLU epilogue storing bf16 activations: on the training
step the input windows and the weight arrive as bf16 (cast by the LSTM pack launch) and take the
LDS-DMA kernel; otherwise fp32 operands are rounded to bf16 while staging.  Backward
masks the incoming gradient with the stored activations, defers the weight / bias gradient
GEMMs (``dym^T x``, ``dym^T 1``) to the end-of-backward grouped launch (``ops._grad.defer``)
and, only when required, runs the input-gradient GEMM.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from . import _grad
from . import _lib
from . import capture as _cap
from .gemm import PLAIN_BLAS, mm

_lib.register("dn_relu_bwd_colsum", [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                                     _lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_int,
                                     _lib.c_void_p])
_lib.register("dn_relu_bwd", [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_long,
                              _lib.c_void_p])
_RB_SLABS = 64

# The one gradient tensor whose ReLU mask was already applied by the GEMM that produced it (the
# fused LSTM's input-gradient GEMM, ``ops.lstm``): a weak reference, so a freed tensor can never
# match a later one that reuses its memory.  Masking is idempotent, so a miss only costs the
# mask launch.
_PREMASKED = None


def mark_premasked(t: torch.Tensor) -> None:
    global _PREMASKED
    import weakref
    _PREMASKED = weakref.ref(t)


def _take_premasked(dy: torch.Tensor) -> bool:
    global _PREMASKED
    r = _PREMASKED() if _PREMASKED is not None else None
    hit = (r is not None and r.data_ptr() == dy.data_ptr() and r.numel() == dy.numel()
           and r.dtype == dy.dtype and dy.is_contiguous())
    if hit:
        _PREMASKED = None
    return hit


class _LinearBiasReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2d, weight, bias, module, w_bf16=None, b_bf16=None):
        if w_bf16 is not None and PLAIN_BLAS:
            # A/B switch: hipBLASLt with its fused RELU_BIAS epilogue
            y = torch._addmm_activation(b_bf16, x2d, w_bf16.t())
        elif w_bf16 is not None:
            # bf16 input and the bf16 weight copy made by the LSTM pack launch: both operands
            # take the LDS-DMA kernel; bias + ReLU in its epilogue (fp32 bias)
            y = mm(x2d, w_bf16, trans_b=True, bias=bias, relu=True, out_dtype=torch.bfloat16)
        else:
            y = mm(x2d, weight, trans_b=True, bias=bias, relu=True, out_dtype=torch.bfloat16)
        ctx.save_for_backward(x2d, y)
        ctx.weight, ctx.bias = weight, bias
        ctx.module = module
        return y

    @staticmethod
    def backward(ctx, dy):
        return _relu_linear_backward(ctx, dy) + (None, None)


def _relu_linear_backward(ctx, dy):
    x2d, y = ctx.saved_tensors
    weight, bias = ctx.weight, ctx.bias
    N, O = y.shape
    premasked = _take_premasked(dy)
    dy = dy.to(torch.bfloat16).contiguous()
    if (N * O) % 8 == 0:
        # mask only; dW += dym^T x and db += dym^T 1 are deferred into the end-of-backward
        # grouped launch with the LSTM's weight gradients (ops._grad.defer)
        if premasked:
            dym = dy.view(N, O)  # masked in the epilogue of the GEMM that produced it
        else:
            dym = torch.empty_like(dy)
            _lib.call("dn_relu_bwd", dy.data_ptr(), y.data_ptr(), dym.data_ptr(), N * O,
                      _lib.stream())
        defer_linear_grads(x2d, dym, weight, bias)
    else:
        dym = torch.empty_like(dy)
        ws = torch.empty(_RB_SLABS * O, dtype=torch.float32, device=dy.device)
        db = _grad.grad_buffer(bias) if bias is not None else \
            torch.empty(O, dtype=torch.float32, device=dy.device)
        _lib.call("dn_relu_bwd_colsum", dy.data_ptr(), y.data_ptr(), dym.data_ptr(),
                  db.data_ptr(), ws.data_ptr(), N, O, int(bias is not None), _lib.stream())
        mm(dym, x2d, trans_a=True, out=_grad.grad_buffer(weight), beta=1.0)
        _grad.notify([weight] + ([bias] if bias is not None else []))
    dx = None
    if ctx.needs_input_grad[0]:
        dx = mm(dym, weight, out_dtype=x2d.dtype)
    if ctx.module is not None and _cap.active() is not None:
        _cap.record(ctx.module, x2d, dym)
    return dx, None, None, None


def defer_linear_grads(x2d: torch.Tensor, dym: torch.Tensor, weight: torch.Tensor,
                       bias: Optional[torch.Tensor], module: Optional[nn.Module] = None) -> None:
    """Queue ``dW += dym^T x2d`` and ``db += dym^T 1`` (``dym``: the masked output gradient,
    bf16 ``[N, O]``) into the end-of-backward grouped launch (``ops._grad.defer``); record the
    pair for activation capture (rank-dAD) when one is active and ``module`` is given."""
    probs = [dict(a=dym, b=x2d, out=_grad.grad_buffer(weight), beta=1.0,
                  colsum=(_grad.grad_buffer(bias),) if bias is not None else None)]
    _grad.defer(probs, [weight] + ([bias] if bias is not None else []))
    if module is not None and _cap.active() is not None:
        _cap.record(module, x2d, dym)


def linear_bias_relu(x2d: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
                     module: Optional[nn.Module] = None,
                     bf16_params: Optional[tuple] = None) -> torch.Tensor:
    """``relu(x W^T + b)`` -> bf16.  ``bf16_params = (W_bf16, b_bf16)``: rounded copies of the
    parameters made for this step; with a bf16 input the forward then runs on the LDS-DMA MFMA
    GEMM (ops.gemm, bias + ReLU in its epilogue; hipBLASLt only under the PLAIN_BLAS A/B switch)."""
    if not x2d.is_cuda:
        return torch.relu(torch.nn.functional.linear(x2d, weight, bias))
    if not _lib.native_available():
        raise RuntimeError("linear_bias_relu on GPU needs the gfx950 kernel library")
    wb = bb = None
    if bf16_params is not None and bias is not None and x2d.dtype == torch.bfloat16:
        wb, bb = bf16_params
    return _LinearBiasReLU.apply(x2d.contiguous(), weight, bias, module, wb, bb)
