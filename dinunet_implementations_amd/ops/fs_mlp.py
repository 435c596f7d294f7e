"""Fused FreeSurfer MLP (``Linear(no bias) -> BN(batch stats) -> ReLU`` x L, then ``fc_out``).

Placeholder gate until the single-workgroup fused kernel lands: returns False so the module
runs its layer-by-layer path.
"""
from __future__ import annotations


def supported(in_size, hidden, out_size, batch) -> bool:
    return False


def fs_mlp(x, ws, gammas, betas, w_out, b_out, eps):  # pragma: no cover
    raise NotImplementedError
