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

# deferred weight-gradient GEMM problems of the current backward pass (see :func:`defer`)
_pending: List[dict] = []
_pending_params: List[torch.Tensor] = []

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


def defer(problems: Iterable[dict], params: Iterable[torch.Tensor]) -> None:
    """Queue weight-gradient GEMM problems (``mm_grouped`` dicts, all ``trans_a=True``:
    ``out += a^T @ b``) instead of launching them now.  Every problem queued during one
    backward pass is issued by :func:`flush` as ONE grouped launch (per dtype/layout class) on
    the backward's stream when the pass ends, and only then are ``params`` reported final.

    Why: the ICA step's weight gradients (LSTM dW_ih / dW_hh / biases, encoder dW / bias) are
    long-K (K = B*S) GEMMs of few tiles each; issued separately they either serialise or need a
    side stream, and every cross-stream edge of a HIP graph costs ~5-12 us of signalling.  One
    grouped launch puts all ~280 tiles on the 256 CUs at once.
    """
    first = not _pending
    _pending.extend(problems)
    _pending_params.extend(params)
    if first:
        try:
            torch.autograd.Variable._execution_engine.queue_callback(flush)
        except RuntimeError:  # not inside a backward pass: nothing to batch with
            flush()


def flush() -> None:
    """Issue every deferred gradient GEMM (grouped by operand dtypes / layouts) and notify."""
    if not _pending:
        return
    from .gemm import mm_grouped
    probs, params = list(_pending), list(_pending_params)
    _pending.clear()
    _pending_params.clear()
    groups = {}
    for q in probs:
        key = (q["a"].dtype, q["b"].dtype, q["out"].dtype, q["a"].stride(-1) == 1,
               q["b"].stride(-1) == 1, q["a"].device)
        groups.setdefault(key, []).append(q)
    for g in groups.values():
        mm_grouped(g, trans_a=True)
    notify(params)
