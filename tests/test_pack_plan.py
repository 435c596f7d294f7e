"""Host-side plans of round-3 fused paths, on the CPU: the persistent operand images the fused
Adam keeps current (``ops.lstm.PersistentPack``: which flat segments map to which image, in what
order), and the grouped GEMM's second output for the LSTM bias column sum (``out2``: b_ih and
b_hh receive the same ``dpre^T 1``)."""
import torch

from dinunet_implementations_amd.models import ICALstm
from dinunet_implementations_amd.ops import FlatParams
from dinunet_implementations_amd.ops.gemm import mm_grouped
from dinunet_implementations_amd.ops.lstm import PK_BIAS, PK_CAST, PK_WHH, PK_WIH, PersistentPack


def test_persistent_pack_rows_cover_lstm_and_encoder():
    torch.manual_seed(0)
    m = ICALstm(input_size=32, hidden_size=48, num_comps=5, window_size=4)
    flat = FlatParams(m.parameters())
    pp = m.persistent_pack(torch.device("cpu"))
    assert isinstance(pp, PersistentPack)
    rows = pp.rows(flat)
    offs = [r[0] for r in rows]
    assert offs == sorted(offs) and all(o % 4 == 0 for o in offs)
    for (o0, n0, *_), (o1, *_r) in zip(rows, rows[1:]):
        assert o0 + n0 <= o1  # disjoint
    kinds = [r[2] for r in rows]
    ndir = 2
    assert kinds.count(PK_WIH) == ndir and kinds.count(PK_WHH) == ndir
    # casts: the encoder's weight and bias, and the bf16 image of every classifier weight the
    # replicated head reads (ops.head._bf16_images)
    heads = [L.linear.weight for L in m.head_spec().layers]
    assert kinds.count(PK_BIAS) == 2 * ndir and kinds.count(PK_CAST) == 2 + len(heads)
    seg = {id(p): (o, n) for p, o, n in flat.segments()}
    lin = m.encoder[0]
    for p, kind in [(lin.weight, PK_CAST), (lin.bias, PK_CAST)] + [(w, PK_CAST) for w in heads]:
        o, n = seg[id(p)]
        assert (o, n, kind) in [(r[0], r[1], r[2]) for r in rows]
    assert all(pp.bf16_of(w) is not None and pp.bf16_of(w).shape == w.shape for w in heads)
    # b_hh images start ndir * 4 HD floats after the b_ih images (the kernel's bias_split)
    GP = 4 * pp.HD
    bias_rows = [r for r in rows if r[2] == PK_BIAS]
    dsts = sorted({r[4] for r in bias_rows})
    assert dsts == [pp.bias_p.data_ptr(), pp.bias_p.data_ptr() + 4 * ndir * GP]
    assert pp.bias_p.numel() == 2 * ndir * GP
    # W_hh rows carry both images (W_hh and W_hh^T layouts)
    assert all(r[5] == pp.whhT_p.data_ptr() for r in rows if r[2] == PK_WHH)
    assert pp.matches([t for c in m.lstm.lstms for t in c.params()], (lin.weight, lin.bias))


def test_grouped_column_sum_second_output():
    g = torch.Generator().manual_seed(1)
    a = torch.randn(40, 12, generator=g)
    ones = torch.ones(40, 8)
    o1 = torch.randn(12, 1, generator=g)
    o2 = torch.randn(12, 1, generator=g)
    r1, r2 = o1.clone(), o2.clone()
    mm_grouped([dict(a=a, b=ones, out=o1, out2=o2, beta=1.0, ncol=1)], trans_a=True)
    s = a.sum(0, keepdim=True).t()
    assert torch.allclose(o1, r1 + s, atol=1e-5) and torch.allclose(o2, r2 + s, atol=1e-5)


def test_grouped_colsum_request_on_cpu():
    """``colsum`` (a bias gradient requested beside its weight gradient) on the CPU path: issued as
    its own ``a^T @ ones`` problem, row-mapped, beta-accumulated, into one or two vectors; the
    weight gradient is unchanged by the request."""
    g = torch.Generator().manual_seed(2)
    K, M, N = 50, 12, 16
    a = torch.randn(K, M, generator=g)
    b = torch.randn(K, N, generator=g)
    rmap = torch.randperm(M + 3, generator=g)[:M].to(torch.int32)
    w = torch.randn(M + 3, N, generator=g)
    x1, x2 = torch.randn(M + 3, generator=g), torch.randn(M + 3, generator=g)
    rw, r1, r2 = w.clone(), x1.clone(), x2.clone()
    mm_grouped([dict(a=a, b=b, out=w, beta=1.0, row_map=rmap, colsum=(x1, x2))], trans_a=True)
    idx = rmap.long()
    rw[idx] += a.t() @ b
    r1[idx] += a.sum(0)
    r2[idx] += a.sum(0)
    assert torch.allclose(w, rw, atol=1e-4)
    assert torch.allclose(x1, r1, atol=1e-4) and torch.allclose(x2, r2, atol=1e-4)


def test_xcd_tile_order_groups_shared_operand_blocks():
    """The grouped launch's slot -> tile permutation (ops.gemm._xcd_order) at the B = 2048 ICA
    weight-gradient shapes: the two problems sharing A (dW_ih, dW_hh of one direction) interleave
    per 128-row block, 8 slots (one XCD) hold two whole row blocks, and the encoder dW (B larger
    than A) is ordered by B column block, so each XCD reads half of X instead of all of it."""
    from dinunet_implementations_amd.ops import gemm as G
    K = 200704
    A0, A1, AE = 1000, 5000, 9000  # addresses: direction 0 / 1 gradient slices, encoder gradient
    arrs = {"A": [A0, A0, A1, A1, AE], "B": [1, 2, 1, 3, 4], "M": [768, 768, 768, 768, 256],
            "N": [256, 193, 256, 193, 1000], "K": [K] * 5}
    G._PERMS.clear()
    perm = G._xcd_order(arrs, 128, "cpu")
    assert perm is not None and sorted(perm.tolist()) == list(range(64))
    order = perm.tolist()
    starts = [0, 12, 24, 36, 48]

    def tile_of(t):  # (problem, m, n) of launch tile t (12 tiles per LSTM problem: 6 m x 2 n)
        i = max(j for j, s0 in enumerate(starts) if t >= s0)
        tn = 2 if i < 4 else 8
        return i, (t - starts[i]) // tn, (t - starts[i]) % tn
    for x in range(6):  # XCDs 0-5: one direction, two row blocks, both problems
        tiles = [tile_of(t) for t in order[8 * x:8 * x + 8]]
        assert len({i // 2 for i, _, _ in tiles}) == 1
        assert len({m for _, m, _ in tiles}) == 2
        assert {i % 2 for i, _, _ in tiles} == {0, 1}
    for x in (6, 7):  # encoder dW: 4 column blocks x both row blocks per XCD
        tiles = [tile_of(t) for t in order[8 * x:8 * x + 8]]
        assert {i for i, _, _ in tiles} == {4}
        assert len({n for _, _, n in tiles}) == 4 and len({m for _, m, _ in tiles}) == 2
