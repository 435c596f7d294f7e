"""Low-rank numerics shared by the rank-dAD and PowerSGD engines (and their file-transport twins).

* :func:`orthonormalize_` — in-place modified Gram-Schmidt of the columns of ``[n, r]`` matrices.
  On GPU a batch of matrices is handled by ONE HIP launch (``dn_mgs_batched``: one workgroup per
  matrix, columns swept sequentially with wave64 + LDS reductions); on CPU a torch loop.
* :func:`dad_factors` — rank-r factors of a layer gradient ``G = Delta^T A`` computed with the
  structured power iteration of rank-dAD (never forms ``G`` when ``N`` is large):
  ``P <- orth(Delta^T (A Q))``, ``Q <- A^T (Delta P)``, stop after ``num_pow_iters`` or when
  ``||Q - Q_prev|| / ||Q|| < tol`` (compspec ``dad_reduction_rank``, ``dad_num_pow_iters``,
  ``dad_tol``: ``compspec.json:236-238``).  Then ``G ~= P Q^T``.
"""
from __future__ import annotations

from typing import List, Tuple

import torch

from ..ops import _lib

_lib.register("dn_mgs_batched", [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_int,
                                  _lib.c_int, _lib.c_float, _lib.c_void_p])
_lib.register("dn_pi_iterate", [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_int,
                                 _lib.c_int, _lib.c_int, _lib.c_void_p, _lib.c_void_p,
                                 _lib.c_void_p, _lib.c_int, _lib.c_float, _lib.c_int,
                                 _lib.c_void_p])
_lib.register("dn_pi_reconstruct", [_lib.c_void_p, _lib.c_int, _lib.c_long, _lib.c_long,
                                     _lib.c_int, _lib.c_void_p])

EPS = 1e-8


def _mgs_torch_(m: torch.Tensor) -> torch.Tensor:
    n, r = m.shape
    for j in range(r):
        v = m[:, j]
        for i in range(j):
            v -= (m[:, i] @ v) * m[:, i]
        nrm = v.norm()
        m[:, j] = v / (nrm + EPS)
    return m


def orthonormalize_(mats: List[torch.Tensor]) -> None:
    """Orthonormalise the columns of every ``[n_i, r_i]`` fp32 matrix in place."""
    if not mats:
        return
    if mats[0].is_cuda and _lib.native_available():
        dev = mats[0].device
        ptrs = torch.tensor([m.data_ptr() for m in mats], dtype=torch.int64)
        dims = torch.tensor([[m.shape[0], m.shape[1], m.stride(0)] for m in mats], dtype=torch.int32)
        ptrs = ptrs.to(dev, non_blocking=True)
        dims = dims.to(dev, non_blocking=True)
        _lib.call("dn_mgs_batched", ptrs.data_ptr(), dims.data_ptr(), None, len(mats), 0, EPS,
                  _lib.stream())
        return
    for m in mats:
        _mgs_torch_(m)


def dad_factors(delta: torch.Tensor, act: torch.Tensor, rank: int, num_iters: int, tol: float,
                generator: torch.Generator = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Rank-``rank`` factors ``(P [out, r], Q [in, r])`` with ``Delta^T A ~= P Q^T``."""
    delta = delta.float()
    act = act.float()
    out_f, in_f = delta.shape[1], act.shape[1]
    r = max(1, min(rank, out_f, in_f))
    q = torch.randn(in_f, r, device=act.device, generator=generator) if generator is not None \
        else torch.randn(in_f, r, device=act.device)
    orthonormalize_([q])
    p = None
    for _ in range(max(1, num_iters)):
        p = delta.t() @ (act @ q)            # [out, r] = G Q
        orthonormalize_([p])
        q_new = act.t() @ (delta @ p)        # [in, r]  = G^T P
        if tol > 0 and _rel_change(q_new, q) < tol:
            q = q_new
            break
        q = q_new
    return p, q


def _rel_change(a: torch.Tensor, b: torch.Tensor) -> float:
    # a single host sync per iteration only on the convergence check path
    return float((a - b).norm() / (a.norm() + EPS))
