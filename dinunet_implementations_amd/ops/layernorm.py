"""LayerNorm on the gfx950 kernels of ``csrc/kernels/layernorm.hip``.

An optional classifier norm (config ``norm_layer = "layer"``): the reference normalises with
``BatchNorm1d`` only, BASELINE.json's north star lists LayerNorm among the
hand-written kernels.  :class:`LayerNorm` IS an ``nn.LayerNorm`` (same parameters, ``state_dict``
keys and CPU math); on a GPU, for a last-dimension norm of ``D % 4 == 0, D <= 2048`` fp32 elements,
forward and backward run on the fused kernels (one wave per row, statistics in registers,
deterministic parameter-gradient reduction).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib

_lib.register("dn_layernorm_fwd", [_lib.c_void_p] * 6 + [_lib.c_int, _lib.c_int, _lib.c_float,
                                                         _lib.c_void_p])
_lib.register("dn_layernorm_ws", [_lib.c_int, _lib.c_int])
_lib.register("dn_layernorm_bwd", [_lib.c_void_p] * 9 + [_lib.c_int, _lib.c_int, _lib.c_int,
                                                         _lib.c_void_p])


def fused_ok(x: torch.Tensor, D: int) -> bool:
    return (x.is_cuda and x.dtype == torch.float32 and D % 4 == 0 and 0 < D <= 2048
            and x.shape[-1] == D and _lib.native_available())


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps: float):
        D = x.shape[-1]
        x2 = x.reshape(-1, D).contiguous()
        R = x2.shape[0]
        y = torch.empty_like(x2)
        mean = torch.empty(R, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        w = weight.contiguous() if weight is not None else None
        b = bias.contiguous() if bias is not None else None
        _lib.call("dn_layernorm_fwd", x2.data_ptr(), _lib.ptr(w), _lib.ptr(b), y.data_ptr(),
                  mean.data_ptr(), rstd.data_ptr(), R, D, float(eps), _lib.stream())
        ctx.save_for_backward(x2, w, mean, rstd)
        ctx.has_b = bias is not None
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, mean, rstd = ctx.saved_tensors
        R, D = x2.shape
        dy2 = dy.reshape(R, D).contiguous().float()
        dx = torch.empty_like(x2)
        need_w = w is not None and ctx.needs_input_grad[1]
        need_b = ctx.has_b and ctx.needs_input_grad[2]
        dg = torch.empty(D, dtype=torch.float32, device=x2.device) if need_w else None
        db = torch.empty(D, dtype=torch.float32, device=x2.device) if need_b else None
        L = _lib.lib()
        L.dn_layernorm_ws.restype = __import__("ctypes").c_long
        ws = (torch.empty(int(L.dn_layernorm_ws(R, D)), dtype=torch.float32, device=x2.device)
              if (need_w or need_b) else None)
        _lib.call("dn_layernorm_bwd", x2.data_ptr(), dy2.data_ptr(), _lib.ptr(w), mean.data_ptr(),
                  rstd.data_ptr(), dx.data_ptr(), _lib.ptr(dg), _lib.ptr(db), _lib.ptr(ws), 0, R, D,
                  _lib.stream())
        return dx.view(ctx.shape), dg, db, None


def layer_norm(x: torch.Tensor, weight, bias, eps: float = 1e-5) -> torch.Tensor:
    """LayerNorm over the last dimension: the fused kernels when they apply, else torch."""
    D = x.shape[-1]
    if fused_ok(x, D):
        return _LayerNormFn.apply(x, weight, bias, eps)
    return nn.functional.layer_norm(x, (D,), weight, bias, eps)


class LayerNorm(nn.LayerNorm):
    """``nn.LayerNorm`` over the last dimension whose GPU forward / backward are the fused gfx950
    kernels (``layer_norm``); identical parameters, ``state_dict`` and CPU behaviour."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if len(self.normalized_shape) != 1:
            return super().forward(x)
        return layer_norm(x, self.weight, self.bias, self.eps)
