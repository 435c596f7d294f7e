"""Persistent-kernel hand-off health (runtime.health) and the decision of when a launch whose
workgroups wait on each other may be used (parallel.group gpu_shared): CPU checks of the logic."""
import types

import pytest
import torch

from dinunet_implementations_amd.parallel.group import SiteGroup, _gpu_shared
from dinunet_implementations_amd.runtime import health


def test_error_words_raise_and_reset(monkeypatch):
    from dinunet_implementations_amd.parallel import peer
    eng = types.SimpleNamespace(peer=True, _table=types.SimpleNamespace(
        _persist=(None, None, torch.zeros(8 * 64 + 1, dtype=torch.int32))))
    ar = types.SimpleNamespace(me=1, _chunks=[1], err=torch.zeros(1, dtype=torch.int32))
    ar.error = lambda: int(ar.err.item())
    monkeypatch.setattr(peer, "arenas", lambda: [ar])
    health.check([], eng)  # all clear
    eng._table._persist[2][-1] = 0x203
    ar.err[0] = 0x100
    with pytest.raises(health.HandoffError) as e:
        health.check([], eng, "in epoch 4")
    msg = str(e.value)
    assert "lr_persist code 0x203" in msg and "layer 3 Q barrier" in msg and "epoch 4" in msg
    assert "peer_exchange code 0x100" in msg and "reduce-scatter wait" in msg and "site 0" in msg
    health.check([], eng)  # the words were cleared


class _FakeGroup(SiteGroup):
    def __init__(self, rank, world, dev, peers):
        super().__init__(rank=rank, world=world, device=dev)
        self._peers = peers

    def all_gather_object(self, obj):
        return [obj if r == self.rank else p for r, p in enumerate(self._peers)]


def test_gpu_sharing_from_actual_devices(monkeypatch):
    import socket
    host = socket.gethostname()
    cuda = lambda k: torch.device("cuda", k)  # noqa: E731
    # one process per GPU: exclusive
    g = _FakeGroup(1, 4, cuda(1), [(host, r) for r in range(4)])
    assert _gpu_shared(g) is False
    # gloo rehearsal, every site on GPU 0: shared
    g = _FakeGroup(2, 4, cuda(0), [(host, 0)] * 4)
    assert _gpu_shared(g) is True
    # 8 ranks cycling two inputspec pins over 8 GPUs of one host, two of them on GPU 1
    g = _FakeGroup(5, 8, cuda(1), [(host, r % 8) for r in range(8)][:5] + [(host, 1)] +
                   [(host, 6), (host, 7)])
    assert _gpu_shared(g) is True
    # two nodes of 8: more ranks than local GPUs, no sharing
    g = _FakeGroup(9, 16, cuda(1), [("n0", r) for r in range(8)] + [("n1", r) for r in range(8)])
    g._peers[9] = (host, 1)
    assert _gpu_shared(g) is False
    # CPU sites and single sites never share
    assert _gpu_shared(SiteGroup(device=torch.device("cpu"))) is False
    assert _gpu_shared(SiteGroup(device=cuda(0))) is False
