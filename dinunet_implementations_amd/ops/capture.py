"""Activation / output-gradient capture for rank-dAD.

For every ``nn.Linear`` the gradient is ``dW = Delta^T A`` with ``A`` the layer input rows and
``Delta`` the gradient w.r.t. the layer output rows.  rank-dAD ships low-rank factors of
``(A, Delta)`` instead of ``dW``.  Plain ``nn.Linear`` modules are captured with hooks; fused
ops (the persistent LSTM) call :func:`record` from their backward with the tensors they already
hold (the encoder output / ``h_{t-1}`` sequence and the gate gradients), so no extra pass runs.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

# Process-global, NOT thread-local: autograd runs the backward of CUDA tensors on its own
# device thread, and the fused ops record from their backward.
_STACK: List["DADCapture"] = []


class DADCapture:
    """Context manager collecting ``{module: [(A, Delta), ...]}`` during backward."""

    def __init__(self, modules: Optional[List[nn.Module]] = None):
        self.records: Dict[nn.Module, List[Tuple[torch.Tensor, torch.Tensor]]] = {}
        self._inputs: Dict[nn.Module, torch.Tensor] = {}
        self._handles = []
        self.modules = modules or []
        self.fused_modules = set()

    # plain Linear path -------------------------------------------------------------------
    def _fwd_hook(self, mod, inp, out):
        x = inp[0]
        self._inputs[mod] = x.detach().reshape(-1, x.shape[-1])

    def _bwd_hook(self, mod, gin, gout):
        a = self._inputs.get(mod)
        if a is None or gout[0] is None:
            return
        d = gout[0].detach().reshape(-1, gout[0].shape[-1])
        self.records.setdefault(mod, []).append((a, d))

    def __enter__(self):
        for m in self.modules:
            self._handles.append(m.register_forward_hook(self._fwd_hook))
            self._handles.append(m.register_full_backward_hook(self._bwd_hook))
        _STACK.append(self)
        return self

    def __exit__(self, *exc):
        for h in self._handles:
            h.remove()
        self._handles.clear()
        self._inputs.clear()
        _STACK.remove(self)
        return False

    def clear(self):
        self.records.clear()
        self._inputs.clear()


def active() -> Optional[DADCapture]:
    return _STACK[-1] if _STACK else None


def record(module: nn.Module, a: torch.Tensor, delta: torch.Tensor) -> None:
    cap = active()
    if cap is not None:
        cap.fused_modules.add(module)
        cap.records.setdefault(module, []).append((a.detach(), delta.detach()))
