"""Python face of the hand-written gfx950 GEMM (``csrc/kernels/gemm.hip``).

``mm(a, b)`` computes ``op(a) @ op(b)`` with bf16 MFMA and fp32 accumulation for fp32 or bf16
operands of any 2-D stride pattern that is contiguous along one axis (both transposes are free:
the kernel stages either layout).  Fused epilogue: ``alpha``, ``bias``, ``relu``, ``beta``
accumulate, output row remap, fp32 or bf16 store.  Long-K / few-tile problems split K over
workgroups with a deterministic fp32 slab reduction.

On CPU tensors the same call runs ``torch.matmul`` in fp32 (oracle / plumbing path).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib

Tensor = torch.Tensor

_lib.register("dn_gemm", [_lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_long, _lib.c_void_p,
                          _lib.c_int, _lib.c_int, _lib.c_long, _lib.c_void_p, _lib.c_int,
                          _lib.c_long, _lib.c_int, _lib.c_int, _lib.c_int, _lib.c_float,
                          _lib.c_float, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_int,
                          _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_void_p,
                          _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_int,
                          _lib.c_void_p])

_lib.register("dn_gemm_set_dma", [_lib.c_int])
_lib.register("dn_gemm_dma_on", [])
_lib.register("dn_gemm_arm_bump", [_lib.c_void_p, _lib.c_void_p])
_lib.register("dn_gemm_bump_armed", [])
_lib.register("dn_gemm_grouped", [_lib.c_int] + [_lib.c_void_p] * 19 + [_lib.c_int] * 8
              + [_lib.c_void_p, _lib.c_void_p] + [_lib.c_void_p] * 4 + [_lib.c_void_p])

# Operands read in place from a dataset resident in HBM (csrc/kernels/gemm.hip RowGather): a
# registered tensor (the device-fed step's static batch buffer, 2-D [B*S, F]) stands for rows
# X[subj[r // S] * S + r % S] of the dataset X [N*S, F] -- the GEMMs that consume the batch read
# it through the step's subject indices, so the step needs no batch copy.
_ROWS = {}


class rows_from:
    """``with rows_from(buf2d, X2d, subj, S):`` GEMMs that take ``buf2d`` as a k-contiguous A or a
    k-major B read dataset rows instead (the LDS-DMA kernels; ``S >= 64``)."""

    def __init__(self, buf2d: Tensor, X2d: Tensor, subj: Tensor, S: int):
        self.key = (buf2d.data_ptr(), tuple(buf2d.shape))
        self.val = (X2d, subj, int(S))

    def __enter__(self):
        _ROWS[self.key] = self.val
        return self

    def __exit__(self, *a):
        _ROWS.pop(self.key, None)
        return False


def _gather_of(t: Tensor):
    """(X, subj, S) when ``t`` (an operand as passed: rows = its first axis, row-contiguous) is
    a registered batch buffer, else None."""
    if not _ROWS or t.dim() != 2 or t.dtype != torch.bfloat16 or not t.is_contiguous():
        return None
    return _ROWS.get((t.data_ptr(), tuple(t.shape)))


def _gather_args(a: Tensor, b: Tensor, trans_a: bool, trans_b: bool):
    """(gx, subj, S, op) for the kernel: A's rows when ``a`` is a registered buffer used
    untransposed (k-contiguous A), B's k rows when ``b`` is one used untransposed (k-major B)."""
    ga, gb = _gather_of(a), _gather_of(b)
    if (ga is not None and trans_a) or (gb is not None and trans_b) or (
            ga is not None and gb is not None):
        raise ValueError("rows_from: a gathered batch buffer is read as a k-contiguous A or a "
                         "k-major B only (one per GEMM)")
    if ga is not None:
        return ga[0].data_ptr(), ga[1].data_ptr(), ga[2], 1
    if gb is not None:
        return gb[0].data_ptr(), gb[1].data_ptr(), gb[2], 2
    return None, None, 0, 0

# DINUNET_SPLITK_INLAUNCH=1: split-K partials are combined inside the GEMM launch by each
# tile's last-arriving workgroup (csrc/kernels/gemm.hip splitk_epilogue) instead of by the
# separate reduce kernel.  Measured on the B = 32 ICA step (grouped weight gradients, 284 tiles x
# 3 splits): 34.8 us in-launch vs 18.9 + 6.9 us for GEMM + reduce kernel -- the combiners'
# 4-byte write-through slab traffic and serial partial reads cost more than the launch they
# save -- so the reduce kernel stays the default.  The arrival tickets live in one persistent
# zeroed buffer per device (each combiner resets its ticket, so the buffer is all-zero between
# launches); launches that use it must not overlap in time (one-stream training step).
_SPLITK_INLAUNCH = __import__("os").environ.get("DINUNET_SPLITK_INLAUNCH", "0") == "1"
_TICKETS = {}


def _tickets(device, tiles: int) -> Optional[Tensor]:
    if not _SPLITK_INLAUNCH:
        return None
    t = _TICKETS.get(device)
    if t is None or t.numel() < tiles:
        if torch.cuda.is_current_stream_capturing():
            return None  # cannot allocate a zeroed buffer inside a capture: reduce kernel
        t = torch.zeros(max(tiles, 4096), dtype=torch.int32, device=device)
        _TICKETS[device] = t
    return t

_NCU = 256
GMAX = 12  # problems per grouped launch (csrc/kernels/gemm.hip)


def _layout(t: Tensor, rows_first: bool):
    """Return (tensor, transposed_flag, leading_dim) for a logical 2-D operand.

    For A (logical [M,K]) ``rows_first`` is True: k-contiguous -> flag 0.
    For B (logical [K,N]) ``rows_first`` is False: k-contiguous -> flag 1.
    """
    if t.dtype not in (torch.float32, torch.bfloat16):
        t = t.float()
    s0, s1 = t.stride()
    # axis 1 contiguous: A -> [M][lda] (k contiguous), B -> [K][ldb] (n contiguous): flag 0
    if t.shape[1] == 1 or s1 == 1:
        return t, 0, (s0 if t.shape[0] > 1 else max(t.shape[1], 1))
    # axis 0 contiguous: A -> stored [K][M], B -> stored [N][K]: flag 1
    if t.shape[0] == 1 or s0 == 1:
        return t, 1, (s1 if t.shape[1] > 1 else max(t.shape[0], 1))
    t = t.contiguous()
    return t, 0, t.stride(0)


# 256 x 256 tiles for large-M GEMMs with k-contiguous operands (csrc/kernels/gemm.hip
# gemm256_kernel); DINUNET_GEMM256=0 keeps 128 x 128 (A/B switch)
GEMM256 = __import__("os").environ.get("DINUNET_GEMM256", "1") != "0"

# tuning override of the grouped launches' split-K (0 = heuristic); tools/gpu sweeps
_GROUP_SPLITS = int(__import__("os").environ.get("DINUNET_GROUP_SPLITS", "0"))
_GROUP_TILE = int(__import__("os").environ.get("DINUNET_GROUP_TILE", "-1"))


def choose_tiling(M: int, N: int, K: int):
    """(tile, split-K).  Few-tile long-K GEMMs (the weight gradients, 64 tiles of K = 3136) cut K
    into ~384-deep chunks on separate workgroups; from ~128 tiles on, the deterministic slab
    reduce costs more than it saves (tools/bench_gemm_sweep.py on MI355X: encoder 3136x256x1000
    18.1 us unsplit vs 21.2 at 2 splits; dx 3136x256x1536 19.6 vs 21.8)."""
    t128 = ((M + 127) // 128) * ((N + 127) // 128)
    t64 = ((M + 63) // 64) * ((N + 63) // 64)
    if t128 >= 2 * _NCU:
        # >= a chip of 256 x 256 tiles: tile 2 (the kernel library takes it for k-contiguous
        # bf16 operands with a vector epilogue, 128 x 128 otherwise)
        t256 = ((M + 255) // 256) * ((N + 255) // 256)
        return (2 if (GEMM256 and t256 >= _NCU) else 1), 1
    return 0, _split_rule(t64, K)


_LONG_K = 16384


def _split_rule(t64: int, K: int, per_cu: int = 8) -> int:
    """Split-K count for ``t64`` 64x64 tiles of depth K.  A tile's K loop is latency-bound (one
    workgroup keeps ~32 KB in flight), so long-K problems cut K until ~3 workgroups share each
    CU; medium K only splits when few tiles exist (a second ~5 us reduce launch otherwise eats
    the gain).  Measured on MI355X (bench.py, merged ICA weight-gradient launch: 284 tiles of
    K = 3136): 1 split 0.4156 ms/step, 2: 0.4045, 3: 0.4010, 4: 0.4024."""
    if K >= _LONG_K:
        # very long K (large-batch weight gradients, K = B*S): ~8 workgroups per CU, each still
        # >= 2048 deep (B = 2048 ICA step, grouped dW: 3 splits 1556 us, see profiles/r2_*);
        # `t64` counts the launch's tiles of whatever size it uses
        return max(1, min(32, -(-per_cu * _NCU // max(t64, 1)), K // 2048))
    if K >= 2048:
        return max(1, min(8, round(3 * _NCU / max(t64, 1)), K // 512))
    if K >= 768 and t64 < _NCU // 2:
        return max(1, min(8, round(K / 384), (4 * _NCU) // max(t64, 1)))
    return 1


def mm(a: Tensor, b: Tensor, trans_a: bool = False, trans_b: bool = False,
       out_dtype: torch.dtype = torch.float32, out: Optional[Tensor] = None,
       bias: Optional[Tensor] = None, relu: bool = False, alpha: float = 1.0, beta: float = 0.0,
       row_map: Optional[Tensor] = None, splits: Optional[int] = None,
       tile: Optional[int] = None, mask: Optional[Tensor] = None) -> Tensor:
    """``out (+)= alpha * op(a) @ op(b) (+ bias) (ReLU)``; ``mask`` (bf16 [M, N], row-contiguous):
    outputs where ``mask <= 0`` are zeroed in the epilogue (a ReLU backward fused into the GEMM
    producing its incoming gradient)."""
    A = a.t() if trans_a else a
    B = b.t() if trans_b else b
    M, K = A.shape
    K2, N = B.shape
    if K != K2:
        raise ValueError(f"mm shape mismatch {tuple(A.shape)} x {tuple(B.shape)}")
    if not A.is_cuda:
        res = alpha * (A.float() @ B.float())
        if bias is not None:
            res = res + bias.float()
        if relu:
            res = torch.relu(res)
        if mask is not None:
            res = res * (mask.float() > 0)
        if out is None:
            out = torch.zeros(M if row_map is None else int(row_map.max()) + 1, N,
                              dtype=out_dtype) if row_map is not None else None
        if row_map is not None:
            if beta != 0:
                res = res + beta * out[row_map.long()].float()
            out[row_map.long()] = res.to(out.dtype)
            return out
        if out is not None:
            if beta != 0:
                res = res + beta * out.float()
            out.copy_(res.to(out.dtype))
            return out
        return res.to(out_dtype)
    A, ta, lda = _layout(A, True)
    B, tb, ldb = _layout(B, False)
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype, device=a.device)
        if beta != 0:
            raise ValueError("beta != 0 needs an existing `out`")
    if out.stride(1) != 1:
        raise ValueError("mm output must be row-contiguous")
    auto_tile, auto_splits = choose_tiling(M, N, K)
    tile = auto_tile if tile is None else int(tile)
    sp = auto_splits if splits is None else max(1, int(splits))
    slab = cnt = None
    if sp > 1:
        slab = torch.empty(sp * M * N, dtype=torch.float32, device=a.device)
        b_ = 128 if tile in (1, 2) else 64
        cnt = _tickets(a.device, -(-M // b_) * -(-N // b_))
    if bias is not None:
        bias = bias.float().contiguous()
    if row_map is not None:
        row_map = row_map.to(device=a.device, dtype=torch.int32).contiguous()
    if mask is not None:
        if (mask.dtype != torch.bfloat16 or tuple(mask.shape) != (M, N) or mask.stride(1) != 1):
            raise ValueError("mm mask must be a row-contiguous bf16 [M, N] tensor")
    gargs = _gather_args(a, b, trans_a, trans_b)
    tail = _tail_rows(M, N, K, tile, sp) if slab is None else None
    Mm = M if tail is None else tail
    _lib.call("dn_gemm", A.data_ptr(), int(A.dtype == torch.bfloat16), ta, lda, B.data_ptr(),
              int(B.dtype == torch.bfloat16), tb, ldb, out.data_ptr(),
              int(out.dtype == torch.bfloat16), out.stride(0), Mm, N, K, float(alpha), float(beta),
              _lib.ptr(bias), int(relu), _lib.ptr(row_map), tile, sp, _lib.ptr(slab),
              _lib.ptr(mask), mask.stride(0) if mask is not None else 0, _lib.ptr(cnt),
              *gargs, 0, _lib.stream())
    if tail is not None:
        # the rows of the launch's last, mostly idle round of 256 x 256 tiles as a row-range view
        # (operand / output / mask / row-map pointers offset, gathered rows through r0) on
        # 64 x 64 tiles: sixteen times the workgroups, so the round fills the CUs it would idle
        r0 = tail
        Mt = M - r0
        ea, eo = A.element_size(), out.element_size()
        a_ptr = A.data_ptr() + (r0 * ea if ta else r0 * lda * ea)
        if gargs[3] == 1:  # A's rows are gathered: the kernel maps view row r to r0 + r
            a_ptr = A.data_ptr()
        _lib.call("dn_gemm", a_ptr, int(A.dtype == torch.bfloat16), ta, lda, B.data_ptr(),
                  int(B.dtype == torch.bfloat16), tb, ldb, out.data_ptr() + r0 * out.stride(0) * eo,
                  int(out.dtype == torch.bfloat16), out.stride(0), Mt, N, K, float(alpha),
                  float(beta), _lib.ptr(bias), int(relu),
                  (row_map.data_ptr() + 4 * r0) if row_map is not None else None, 0, 1, None,
                  (mask.data_ptr() + r0 * mask.stride(0) * 2) if mask is not None else None,
                  mask.stride(0) if mask is not None else 0, None, *gargs, r0, _lib.stream())
    return out


# DINUNET_GEMM_TAIL=0: no row-range tail split of 256 x 256 launches (A/B switch)
GEMM_TAIL = __import__("os").environ.get("DINUNET_GEMM_TAIL", "1") == "1"


def _tail_rows(M: int, N: int, K: int, tile: int, sp: int):
    """First row ``r0`` of a tail launch when a one-split launch of 256 x 256 tiles (one
    workgroup per CU) would end in a round of at most a quarter of the CUs: rows ``r0:`` then run
    as a second launch of 64 x 64 tiles (B = 2048 ICA step: the encoder and input-gradient GEMMs
    have 784 row tiles on 256 CUs = 3 full rounds + 16 tiles, a fourth round for 2 % of the
    work; split along K instead, the tail's slab traffic and reduce cost about what the round
    did).  None: launch as is."""
    if not (GEMM_TAIL and tile == 2 and sp == 1 and K >= 512):
        return None
    tn = -(-N // 256)
    tm = -(-M // 256)
    tiles = tm * tn
    if tiles <= _NCU:
        return None
    rem = tiles % _NCU
    if rem == 0 or 4 * rem > _NCU:
        return None
    tail_m = -(-rem // tn)
    r0 = (tm - tail_m) * 256
    if r0 <= 0 or r0 >= M:
        return None
    return r0


_ONES = {}


def ones_operand(n: int, device) -> Tensor:
    """bf16 ones ``[n, 8]`` (8 columns: the 16-B operand path), cached per (n, device): the B
    operand of a column sum formed as its own GEMM problem."""
    key = (n, str(device))
    t = _ONES.get(key)
    if t is None:
        t = torch.ones(n, 8, dtype=torch.bfloat16, device=device)
        _ONES[key] = t
    return t


# DINUNET_COLSUM_FOLD=0: bias gradients always as their own ``a^T @ ones`` problems (A/B switch)
COLSUM_FOLD = __import__("os").environ.get("DINUNET_COLSUM_FOLD", "1") == "1"


def _group_tile(probs, trans_a: bool, tile: Optional[int]) -> Optional[int]:
    if tile is None and _GROUP_TILE >= 0:
        tile = _GROUP_TILE
    maxk = max((q["a"].shape[0] if trans_a else q["a"].shape[1]) for q in probs)
    if tile is None and maxk >= _LONG_K:
        # very long K (large-batch weight gradients, K = B*S): 128x128 tiles double the MFMA
        # work per staged byte.  B = 2048 ICA step on MI355X (tools/_gpu_group_ab.sh): 64x64
        # 3.88 ms/step, 128x128 3.45 ms at ~8 workgroups per CU (24 splits); 256 x 256 (tile 2,
        # one workgroup per CU) halves the staged bytes per MFMA again
        tile = 2 if GEMM256 else 1
    return tile


def _dma_vec_ok(q, trans_a: bool, trans_b: bool) -> bool:
    """The launch-wide contract of the LDS-DMA kernel (gemm.hip run_group: bf16 operands, 16-B
    aligned bases, leading dims and contiguous-axis extents % 8), checked for one problem."""
    A = q["a"].t() if trans_a else q["a"]
    B = q["b"].t() if trans_b else q["b"]
    if A.dtype != torch.bfloat16 or B.dtype != torch.bfloat16:
        return False
    (M, K), N = A.shape, B.shape[1]
    A, ta, lda = _layout(A, True)
    B, tb, ldb = _layout(B, False)

    def ok(t, kcontig, rows, ld):
        return t.data_ptr() % 16 == 0 and ld % 8 == 0 and (K if kcontig else rows) % 8 == 0
    return ok(A, not ta, M, lda) and ok(B, bool(tb), N, ldb)


def _place_colsums(probs, trans_a: bool, trans_b: bool, tile: Optional[int]):
    """Resolve the ``colsum`` requests of a grouped launch; returns ``(problems, tile)``.

    A column sum ``op(a) @ 1`` (a bias gradient: ``dpre^T @ 1``) is folded into its own problem
    when the launch runs 128x128 tiles on the LDS-DMA kernel with a k-major ``b`` of ``N % 8 ==
    0`` columns: the kernel reads a virtual ones column as ``b``'s column N and routes result
    column N to the colsum vectors.  In the ICA step's large-batch weight-gradient launch the
    LSTM ``dW_hh`` (N = 192) and encoder ``dW`` (N = 1000) tiles have spare columns in their last
    tile column, so each bias stops costing its own tiles and a third pass over ``dpre`` / the
    encoder gradient.  Otherwise (CPU, small-batch 64x64 tiles, fp32 or k-contiguous ``b``) the
    column sum becomes its own ``a^T @ ones[K, 8]`` problem of the launch (one column stored)."""
    tile = _group_tile(probs, trans_a, tile) if probs[0]["a"].is_cuda else tile
    if not any(q.get("colsum") for q in probs):
        return probs, tile
    fold_ok = (COLSUM_FOLD and tile in (1, 2) and probs[0]["a"].is_cuda and not trans_b
               and _lib.native_available() and int(_lib.lib().dn_gemm_dma_on()) == 1
               and all(_dma_vec_ok(q, trans_a, trans_b) for q in probs))
    out = []
    extra = []
    for q in probs:
        cs = q.get("colsum")
        if not cs:
            out.append(q)
            continue
        q = {k: v for k, v in q.items() if k != "colsum"}
        a, b = q["a"], q["b"]
        x1, x2 = cs[0], (cs[1] if len(cs) > 1 else None)
        K = a.shape[0] if trans_a else a.shape[1]
        if (fold_ok and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
                and b.stride(-1) == 1 and b.shape[1] % 8 == 0 and b.stride(0) % 8 == 0
                and b.data_ptr() % 16 == 0 and q["out"].dtype == torch.float32
                and q.get("bias") is None and not q.get("ncol")
                and x1.dtype == torch.float32 and x1.is_contiguous()
                and (x2 is None or (x2.dtype == torch.float32 and x2.is_contiguous()))):
            q["colsum_folded"] = (x1, x2)
            out.append(q)
        else:
            out.append(q)
            extra.append(dict(a=a, b=ones_operand(K, a.device), out=x1.view(-1, 1),
                              beta=q.get("beta", 0.0), alpha=q.get("alpha", 1.0),
                              row_map=q.get("row_map"), ncol=1,
                              out2=x2.view(-1, 1) if x2 is not None else None))
    return out + extra, tile


# DINUNET_XCD_ORDER=0: grouped launches keep the plain problem-major tile order (A/B switch)
XCD_ORDER = __import__("os").environ.get("DINUNET_XCD_ORDER", "1") == "1"
_PERMS = {}


def _xcd_order(arrs, bt: int, dev) -> Optional[Tensor]:
    """Slot -> tile permutation of a grouped launch (``GemmGroup::perm``).

    The kernel gives each XCD a contiguous range of slots, and an XCD's L2 serves every re-read
    of an operand block its own workgroups fetched.  Tiles are therefore ordered by the block of
    their LARGER operand: an A row block (keyed by A's address, so problems sharing A -- the
    LSTM's dW_ih and dW_hh of one direction, both ``dpre^T @ .`` -- interleave per row block) or
    a B column block (the encoder dW: X, 1000 columns, outweighs its 256-row gradient).  In the
    B = 2048 ICA step's weight-gradient launch this is the difference between fetching dpre
    twice, the LSTM input 4x and X 2x across XCDs, and once-ish (profiles/r4_dw_xcd_order.md).
    Cached per permutation (graph capture cannot allocate: a miss there keeps the plain order)."""
    keys = []
    t = 0
    for i in range(len(arrs["M"])):
        M, N, K = arrs["M"][i], arrs["N"][i], arrs["K"][i]
        tm, tn = -(-M // bt), -(-N // bt)
        a_big = M >= N
        for m in range(tm):
            for nn in range(tn):
                keys.append(((0, arrs["A"][i], m, i, nn) if a_big else (1, arrs["B"][i], nn, i, m), t))
                t += 1
    order = tuple(j for _, j in sorted(keys))
    if order == tuple(range(t)):
        return None
    p = _PERMS.get((dev, order))
    if p is None:
        if torch.device(dev).type == "cuda" and torch.cuda.is_current_stream_capturing():
            return None
        p = torch.tensor(order, dtype=torch.int32, device=dev)
        _PERMS[(dev, order)] = p
    return p


def _launch_class(q, trans_a: bool, trans_b: bool):
    A = q["a"].t() if trans_a else q["a"]
    B = q["b"].t() if trans_b else q["b"]
    _, ta, _ = _layout(A, True)
    _, tb, _ = _layout(B, False)
    bf = torch.bfloat16
    return (ta, tb, A.dtype == bf, B.dtype == bf, q["out"].dtype == bf)


def mm_grouped(problems, trans_a: bool = False, trans_b: bool = False,
               splits: Optional[int] = None, tile: Optional[int] = None):
    """Several independent ``out_i (+)= alpha_i * op(a_i) @ op(b_i)`` in ONE launch.

    ``problems``: sequence of dicts with keys ``a``, ``b``, ``out`` (required, fp32 or bf16 like
    every other ``out`` of the group) and optional ``alpha``, ``beta``, ``bias``, ``row_map``,
    ``ncol`` (store only the first ``ncol`` result columns into ``out``; lets a column sum ride
    along as ``a^T @ ones[K, 8]`` with the vectorised operand path), ``colsum``: a tuple of one
    or two fp32 vectors ``[M]`` that receive (``beta``-accumulate, ``row_map``-ed) the column
    sums of ``op(a)``, i.e. ``op(a) @ 1`` -- a bias gradient beside its weight gradient (see
    :func:`_place_colsums`).
    All ``a`` (and all ``b``) share dtype and memory layout.  On CPU runs :func:`mm` per problem.
    """
    import ctypes
    probs = list(problems)
    if not probs:
        return
    probs, tile = _place_colsums(probs, trans_a, trans_b, tile)
    if probs[0]["a"].is_cuda:
        # a column sum issued as its own problem has a bf16 ones operand: it joins the launch
        # of the problems sharing its operand dtypes / layouts (one launch per class)
        classes = {}
        for q in probs:
            classes.setdefault(_launch_class(q, trans_a, trans_b), []).append(q)
        if len(classes) > 1:
            for grp in classes.values():
                mm_grouped(grp, trans_a, trans_b, splits, tile)
            return
    if len(probs) > GMAX:
        for i in range(0, len(probs), GMAX):
            mm_grouped(probs[i:i + GMAX], trans_a, trans_b, splits, tile)
        return
    if not probs[0]["a"].is_cuda:
        for q in probs:
            if q.get("ncol"):
                nc = int(q["ncol"])
                q = dict(q, b=(q["b"][:nc] if trans_b else q["b"][:, :nc]))
            for out in (q["out"], q.get("out2")):
                if out is not None:
                    mm(q["a"], q["b"], trans_a=trans_a, trans_b=trans_b, out=out,
                       alpha=q.get("alpha", 1.0), beta=q.get("beta", 0.0), bias=q.get("bias"),
                       row_map=q.get("row_map"))
        return
    n = len(probs)
    arrs = {k: [] for k in ("A", "lda", "B", "ldb", "C", "ldc", "M", "N", "K", "alpha", "beta",
                            "bias", "rmap", "ncol", "C2", "xcol", "X1", "X2", "GX", "SUBJ", "GS",
                            "GOP")}
    keep = []
    ta = tb = None
    a_bf = b_bf = c_bf = None
    maxk = 0
    t64 = t128 = t256 = 0
    for q in probs:
        A = q["a"].t() if trans_a else q["a"]
        B = q["b"].t() if trans_b else q["b"]
        M, K = A.shape
        _, N = B.shape
        A, ta_i, lda = _layout(A, True)
        B, tb_i, ldb = _layout(B, False)
        if ta is None:
            ta, tb = ta_i, tb_i
            a_bf, b_bf = A.dtype == torch.bfloat16, B.dtype == torch.bfloat16
            c_bf = q["out"].dtype == torch.bfloat16
        elif (ta_i, tb_i, A.dtype == torch.bfloat16, B.dtype == torch.bfloat16,
              q["out"].dtype == torch.bfloat16) != (ta, tb, a_bf, b_bf, c_bf):
            raise ValueError("mm_grouped: problems must share layouts and dtypes")
        out = q["out"]
        if out.stride(1) != 1:
            raise ValueError("mm_grouped output must be row-contiguous")
        out2 = q.get("out2")  # a second output of a column-sum problem (same shape / strides)
        if out2 is not None and (out2.shape != out.shape or out2.stride() != out.stride()
                                 or out2.dtype != out.dtype or not q.get("ncol")):
            raise ValueError("mm_grouped out2: a column-sum problem's twin output")
        bias = q.get("bias")
        bias = bias.float().contiguous() if bias is not None else None
        rmap = q.get("row_map")
        if rmap is not None:
            rmap = rmap.to(device=out.device, dtype=torch.int32).contiguous()
        keep += [A, B, bias, rmap]
        xs = q.get("colsum_folded")  # (x1, x2): B's virtual ones column N -> result column N
        xcol = -1
        if xs is not None:
            xcol, N = N, N + 4  # N % 4 == 0: the split-K reduce keeps its 16-B slab rows
        for k, v in (("A", A.data_ptr()), ("lda", lda), ("B", B.data_ptr()), ("ldb", ldb),
                     ("C", out.data_ptr()), ("ldc", out.stride(0)), ("M", M), ("N", N), ("K", K),
                     ("alpha", float(q.get("alpha", 1.0))), ("beta", float(q.get("beta", 0.0))),
                     ("bias", _lib.ptr(bias)), ("rmap", _lib.ptr(rmap)),
                     ("ncol", int(q.get("ncol", 0) or 0)), ("C2", _lib.ptr(out2)),
                     ("xcol", xcol), ("X1", _lib.ptr(xs[0]) if xs else None),
                     ("X2", _lib.ptr(xs[1]) if xs else None)):
            arrs[k].append(v)
        for k, v in zip(("GX", "SUBJ", "GS", "GOP"),
                        _gather_args(q["a"], q["b"], trans_a, trans_b)):
            arrs[k].append(v)
        maxk = max(maxk, K)
        t64 += ((M + 63) // 64) * ((N + 63) // 64)
        t128 += ((M + 127) // 128) * ((N + 127) // 128)
        t256 += ((M + 255) // 256) * ((N + 255) // 256)
    if splits is None and _GROUP_SPLITS:
        splits = _GROUP_SPLITS
    if splits is None:
        # 128x128 tiles: ~4 workgroups per CU (B = 2048 ICA step, 64 tiles: 16 splits 2.631 /
        # 2.634 ms vs 32 splits 2.651 / 2.650, 20 splits 2.679; B = 4096 5.179 / 5.161 vs
        # 5.195 / 5.171 -- profiles/r4_group_splits_ab.jsonl)
        splits = (_split_rule(t256, maxk, per_cu=1) if tile == 2 else
                  _split_rule(t128, maxk, per_cu=4) if tile == 1 else _split_rule(t64, maxk))
    sp = max(1, int(splits))
    dev = probs[0]["out"].device
    perm = _xcd_order(arrs, 128 if tile == 1 else 64, dev) if (XCD_ORDER and tile == 1) else None
    slab = cnt = None
    if sp > 1:
        slab = torch.empty(sp * sum(m * nn for m, nn in zip(arrs["M"], arrs["N"])),
                           dtype=torch.float32, device=dev)
        b_ = 128 if tile in (1, 2) else 64
        cnt = _tickets(dev, sum(-(-m // b_) * -(-nn // b_) for m, nn in zip(arrs["M"], arrs["N"])))
    P = ctypes.c_void_p
    L = ctypes.c_long
    I = ctypes.c_int
    F = ctypes.c_float
    _lib.call("dn_gemm_grouped", n, (P * n)(*arrs["A"]), (L * n)(*arrs["lda"]),
              (P * n)(*arrs["B"]), (L * n)(*arrs["ldb"]), (P * n)(*arrs["C"]),
              (L * n)(*arrs["ldc"]), (I * n)(*arrs["M"]), (I * n)(*arrs["N"]),
              (I * n)(*arrs["K"]), (F * n)(*arrs["alpha"]), (F * n)(*arrs["beta"]),
              (P * n)(*arrs["bias"]), (P * n)(*arrs["rmap"]), (I * n)(*arrs["ncol"]),
              (P * n)(*arrs["C2"]), (I * n)(*arrs["xcol"]), (P * n)(*arrs["X1"]),
              (P * n)(*arrs["X2"]), _lib.ptr(perm), 0,
              int(a_bf), int(b_bf), ta, tb,
              int(c_bf), 0 if tile is None else int(tile), sp, _lib.ptr(slab), _lib.ptr(cnt),
              (P * n)(*arrs["GX"]), (P * n)(*arrs["SUBJ"]), (I * n)(*arrs["GS"]),
              (I * n)(*arrs["GOP"]), _lib.stream())


# Plain GEMMs (bf16 operands, no row map) run on csrc/kernels/gemm.hip's LDS-DMA kernel, which
# beats hipBLASLt at every ICA-step shape at B = 32 (tools/bench_gemm.py on MI355X, us: encoder
# 12.7 vs 19.0, projection 13.0 vs 18.7, dX 14.4 vs 19.0) and is within 1.1-1.3x of it at
# B = 2048 (profiles/r2_gemm_shapes.md).  DINUNET_PLAIN_BLAS=1 routes them to hipBLASLt through
# torch instead (A/B switch).
import os as _os

PLAIN_BLAS = _os.environ.get("DINUNET_PLAIN_BLAS", "0") == "1"


def mm_plain(a: Tensor, b: Tensor, trans_b: bool = False, out_dtype: torch.dtype = torch.float32,
             trans_a: bool = False) -> Tensor:
    """``op(a) @ op(b)`` for bf16 operands: hipBLASLt when enabled, else :func:`mm`."""
    if (PLAIN_BLAS and a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16):
        A = a.t() if trans_a else a
        B = b.t() if trans_b else b
        if out_dtype == torch.bfloat16:
            return torch.mm(A, B)
        return torch.mm(A, B, out_dtype=out_dtype)
    return mm(a, b, trans_a=trans_a, trans_b=trans_b, out_dtype=out_dtype)

