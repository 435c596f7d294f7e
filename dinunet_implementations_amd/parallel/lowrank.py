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
_lib.register("dn_lr_stage", [_lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_int,
                              _lib.c_float, _lib.c_void_p])
_lib.register("dn_lr_recon_ef", [_lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_void_p])
_lib.register("dn_pi_reconstruct", [_lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_long,
                                     _lib.c_long, _lib.c_int, _lib.c_void_p])

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


class LowRankTable:
    """Device-side descriptor table of the ``csrc/kernels/lowrank.hip`` factorisation kernels:
    every large gradient matrix of a model, all handled by each launch.

    ``layers``: ``[(G view [out, in], err [out, in] or None, P [out, r], Psend [out, r],
    Qsend [in, r])]`` (fp32 CUDA tensors, contiguous).  ``Qsend`` holds the committed Q: the
    input of every iteration and the next step's warm start (initialise it).  The
    change norms and an ``active`` flag per layer are allocated here.  One
    power iteration = :meth:`gq` + :meth:`orth_gtp`, one launch each, all layers per launch."""

    def __init__(self, layers, device):
        import ctypes
        L = _lib.lib()
        L.dn_lr_layer_size.restype = ctypes.c_long
        maxr, plds, qlds = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        L.dn_lr_limits(ctypes.byref(maxr), ctypes.byref(plds), ctypes.byref(qlds))

        class LrLayer(ctypes.Structure):
            _fields_ = [(k, ctypes.c_void_p) for k in ("G", "err", "P", "Psend", "Qsend", "norms",
                                                     "active", "iters")] + \
                       [(k, ctypes.c_int) for k in ("out", "in_", "r", "b1", "n1", "b3", "n3")]
        if ctypes.sizeof(LrLayer) != L.dn_lr_layer_size():
            raise RuntimeError("low-rank table layout mismatch with the kernel library")
        n = len(layers)
        if n > 256:
            raise ValueError("at most 256 low-rank layers per table")
        self.n = n
        self._keep = []
        self.active = torch.ones(max(n, 1), dtype=torch.int32, device=device)
        # power iterations each layer actually ran (lr_gq counts them; dad_tol stops early)
        self.iters = torch.zeros(max(n, 1), dtype=torch.int32, device=device)
        tab = (LrLayer * max(n, 1))()
        b1 = b3 = 0
        total = 0
        for i, (G, err, P, ps, qs) in enumerate(layers):
            out_f, in_f = G.shape
            r = P.shape[1]
            if r > maxr.value or out_f * r > plds.value:
                raise ValueError(f"low-rank layer [{out_f}, {in_f}] rank {r} exceeds the kernel "
                                 f"limits (r <= {maxr.value}, out * r <= {plds.value})")
            n1 = -(-out_f // 16)
            n3 = -(-in_f // 16)
            norms = torch.zeros(2 * n3, dtype=torch.float32, device=device)
            self._keep.append(norms)
            t = tab[i]
            t.G, t.err = G.data_ptr(), (err.data_ptr() if err is not None else None)
            t.P, t.Psend, t.Qsend = P.data_ptr(), ps.data_ptr(), qs.data_ptr()
            t.norms = norms.data_ptr()
            t.active = self.active.data_ptr() + 4 * i
            t.iters = self.iters.data_ptr() + 4 * i
            t.out, t.in_, t.r, t.b1, t.n1, t.b3, t.n3 = out_f, in_f, r, b1, n1, b3, n3
            b1 += n1
            b3 += n3
            total += out_f * in_f
        self.blocks1, self.blocks3, self.total = b1, b3, total
        # the persistent launch takes the table by value; the staged launches read their layer
        # index (first block / tile per layer, kernel argument) from it
        self._host_tab = tab
        self.table = torch.frombuffer(bytearray(bytes(tab)), dtype=torch.uint8).to(device)
        # (gram partials, norms, barrier words) of dn_lr_persist: allocated (zeroed) here, never
        # inside a capture
        L.dn_lr_persist_words.restype = ctypes.c_long
        L.dn_lr_persist_maxj.restype = ctypes.c_long
        mj = int(L.dn_lr_persist_maxj())
        self._persist = (torch.zeros(max(n, 1) * mj * 256, dtype=torch.float64, device=device),
                         torch.zeros(max(n, 1) * mj * 2, dtype=torch.float32, device=device),
                         torch.zeros(int(L.dn_lr_persist_words()), dtype=torch.int32, device=device))

    def persist(self, iters: int, tol: float = 0.0) -> bool:
        """ALL ``iters`` power iterations of every layer in ONE launch (``lr_persist_kernel``:
        each layer's G slices stay in registers, members meet at per-layer barriers).  False when
        the table does not fit it (or ``DINUNET_LR_PERSIST=0``): run :meth:`gq` / :meth:`orth_gtp`."""
        import ctypes
        import os
        if not self.n or os.environ.get("DINUNET_LR_PERSIST", "1") == "0":
            return False
        L = _lib.lib()
        gram, norms, sync = self._persist
        rc = L.dn_lr_persist(ctypes.c_void_p(ctypes.addressof(self._host_tab)), ctypes.c_int(self.n),
                             ctypes.c_int(int(iters)), ctypes.c_float(tol),
                             ctypes.c_void_p(gram.data_ptr()), ctypes.c_void_p(norms.data_ptr()),
                             ctypes.c_void_p(sync.data_ptr()), ctypes.c_void_p(_lib.stream()))
        if rc == 3:  # DN_UNSUPPORTED: the staged kernels
            return False
        if rc != 0:
            raise RuntimeError(f"dn_lr_persist failed with status {rc}")
        return True

    def persist_error(self) -> int:
        """Error word of the persistent launch (0: every barrier met; else 0x100 / 0x200 + layer
        of a barrier wait that timed out)."""
        return int(self._persist[2][-1].item())

    def iterations(self) -> list:
        """Cumulative power iterations run per layer (host sync)."""
        return [int(v) for v in self.iters[:self.n].tolist()]

    def host_table(self) -> int:
        """Address of the host copy of the descriptor table."""
        import ctypes
        return ctypes.addressof(self._host_tab)

    def _stage(self, stage: int, it: int, tol: float = 0.0):
        if self.n:
            _lib.call("dn_lr_stage", self.table.data_ptr(), self.host_table(), self.n, stage,
                      int(it), float(tol), _lib.stream())

    def gq(self, it: int, tol: float = 0.0):
        """P = G Q (PowerSGD: M = G + err first).  Iteration 0 re-activates every layer; later
        ones first stop a layer whose last Q changed by less than ``tol`` (rank-dAD dad_tol)."""
        self._stage(0, it, tol)

    def orth_gtp(self, it: int):
        """Pn = P R^{-1} (Cholesky of the fp64 Gram P^T P) -> Psend,
        Q = G^T Pn -> Qsend (one launch, all layers)."""
        self._stage(1, it)

    def recon_ef(self):
        """PowerSGD: G <- Psend Qsend^T, err <- M - G (M = G + err left by :meth:`gq`)."""
        if self.n:
            _lib.call("dn_lr_recon_ef", self.table.data_ptr(), self.host_table(), self.n,
                      _lib.stream())
