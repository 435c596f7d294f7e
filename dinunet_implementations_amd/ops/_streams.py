"""Side HIP stream for work that can overlap the main stream inside one training step.

Used by the fused LSTM: the time-parallel pre-activation GEMMs run beside the classifier head,
and the weight-gradient GEMMs beside the input-gradient / encoder backward.  Fork/join is by
events, so the same code is valid eagerly and inside HIP-graph capture (a forked capture).
"""
from __future__ import annotations

from typing import Dict, Iterable

import torch

_side: Dict[int, torch.cuda.Stream] = {}


def side_stream(device: torch.device) -> torch.cuda.Stream:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _side.get(idx)
    if s is None:
        s = _side[idx] = torch.cuda.Stream(device=idx)
    return s


def fork(device: torch.device) -> torch.cuda.Stream:
    """Side stream ordered after everything issued so far on the current stream."""
    s = side_stream(device)
    s.wait_stream(torch.cuda.current_stream(device))
    return s


def keep_alive(stream: torch.cuda.Stream, tensors: Iterable[torch.Tensor]) -> None:
    """Tell the caching allocator these tensors are in use on ``stream`` (no early reuse)."""
    for t in tensors:
        if t is not None and t.is_cuda:
            t.record_stream(stream)
