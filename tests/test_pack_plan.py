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
    assert kinds.count(PK_BIAS) == 2 * ndir and kinds.count(PK_CAST) == 2
    seg = {id(p): (o, n) for p, o, n in flat.segments()}
    lin = m.encoder[0]
    for p, kind in ((lin.weight, PK_CAST), (lin.bias, PK_CAST)):
        o, n = seg[id(p)]
        assert (o, n, kind) in [(r[0], r[1], r[2]) for r in rows]
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
