"""CPU checks of the device-fed epoch's host side (runtime.feed): the batch order it trains on is
exactly the train loader's (same passes, shuffles, drop_last, resume position), and the graph
sizes it picks."""
import torch

from dinunet_implementations_amd.data.loader import DeviceLoader
from dinunet_implementations_amd.runtime.feed import default_graph_steps


def _loader(n=23, B=4, drop_last=True, shuffle=True):
    X = torch.arange(n, dtype=torch.float32).view(n, 1).repeat(1, 3)
    y = torch.arange(n) % 2
    return DeviceLoader(X, y, B, shuffle=shuffle, drop_last=drop_last, seed=9)


def _take(it, ld, k, indices):
    out = []
    for _ in range(k):
        try:
            out.append(next(it))
        except StopIteration:
            it = ld.iter_indices() if indices else iter(ld)
            out.append(next(it))
    return it, out


def test_index_stream_matches_gathered_batches_across_passes():
    # 23 samples, batch 4, drop_last: 5 batches per pass; 3 epochs of 7 steps cross passes
    a, b = _loader(), _loader()
    ia, ib = iter(a), b.iter_indices()
    for _ in range(3):
        ia, xs = _take(ia, a, 7, False)
        ib, ix = _take(ib, b, 7, True)
        for (x, y, i), j in zip(xs, ix):
            assert torch.equal(i, j)
            assert torch.equal(x[:, 0].long(), j) and torch.equal(y, j % 2)
        assert a.state() == b.state()


def test_index_stream_resume_position():
    a = _loader()
    it = a.iter_indices()
    it, first = _take(it, a, 8, True)
    st = a.state()
    it, rest = _take(it, a, 6, True)
    b = _loader()
    jt = b.resume_iter(st, indices=True)
    jt, again = _take(jt, b, 6, True)
    assert all(torch.equal(x, y) for x, y in zip(rest, again))


def test_full_batches_rule():
    assert _loader(23, 4, drop_last=True).full_batches
    assert not _loader(23, 4, drop_last=False).full_batches
    assert _loader(24, 4, drop_last=False).full_batches
    assert not _loader(3, 4, drop_last=False).full_batches


def test_default_graph_steps():
    assert default_graph_steps(64) == 8
    assert default_graph_steps(100) == 10
    assert default_graph_steps(97) == 10  # prime: one remainder graph
    assert default_graph_steps(5) == 5
    assert default_graph_steps(1) == 1
    assert default_graph_steps(26) == 10  # divisor 2 is too small: 10 + 10 + 6
