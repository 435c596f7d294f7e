"""Direct gradient accumulation for fused ops.

Fused backward kernels/GEMMs write parameter gradients straight into ``param.grad`` (which is a
view into the flat gradient buffer, ``ops.optim.FlatParams``) with an accumulate epilogue, and
return ``None`` to autograd.  That removes autograd's per-parameter ``AccumulateGrad`` add
kernels; engines that overlap communication with backward are told a gradient is final through
:func:`notify` (the same role ``register_post_accumulate_grad_hook`` plays for ordinary params).
"""
from __future__ import annotations

from typing import Callable, Iterable, List

import torch

_callbacks: List[Callable[[torch.nn.Parameter], None]] = []


def register(cb: Callable[[torch.nn.Parameter], None]) -> None:
    if cb not in _callbacks:
        _callbacks.append(cb)


def unregister(cb) -> None:
    if cb in _callbacks:
        _callbacks.remove(cb)


def grad_buffer(p: torch.Tensor) -> torch.Tensor:
    """The fp32 contiguous ``.grad`` a kernel may accumulate into (created if missing)."""
    if p.grad is None:
        p.grad = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
    g = p.grad
    if g.dtype != torch.float32 or not g.is_contiguous():
        raise RuntimeError("fused ops need fp32 contiguous .grad buffers")
    return g


def notify(params: Iterable[torch.Tensor]) -> None:
    if not _callbacks:
        return
    for p in params:
        for cb in list(_callbacks):
            cb(p)
