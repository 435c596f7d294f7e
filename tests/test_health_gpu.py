"""Negative controls of the persistent-kernel hand-off check (runtime.health) on the GPU: with the
in-kernel poll limit forced to 0 every hand-off wait of the one-launch head and every barrier of
the one-launch rank-dAD iteration gives up at once; the check must then raise -- on the kernels
directly and through the production site loop -- and stay quiet with the default limit."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def spin_zero():
    from dinunet_implementations_amd.runtime import health
    health.set_spin_limit(0)
    yield health
    health.set_spin_limit(-1)


def _step(engine="dSGD"):
    from test_step_gpu import _trainer
    m, flat, st = _trainer(0, engine=engine, use_graph=False, hidden=128)
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(32, 12, 20, 10, device="cuda", generator=g)
    y = torch.randint(0, 2, (32,), device="cuda", generator=g)
    return m, st, x, y


def test_head_step_timeout_raises(spin_zero, monkeypatch):
    from dinunet_implementations_amd.ops import head as H
    monkeypatch.setattr(H, "_HEAD_REP", False)  # head_step.hip: the head with hand-offs
    health = spin_zero
    m, st, x, y = _step()
    st(x, y)
    torch.cuda.synchronize()
    assert m._head is not None and m._head._sync is not None, "one-launch head did not run"
    with pytest.raises(health.HandoffError, match="head_step"):
        health.check([m], st.engine)
    health.set_spin_limit(-1)
    st(x, y)
    torch.cuda.synchronize()
    health.check([m], st.engine)  # default limit: no timeout


def test_rankdad_barrier_timeout_raises(spin_zero):
    health = spin_zero
    m, st, x, y = _step("rankDAD")
    eng = st.engine
    assert eng.fast and eng._persist_ok
    st(x, y)
    torch.cuda.synchronize()
    with pytest.raises(health.HandoffError, match="lr_persist"):
        health.check([m], eng)
    health.set_spin_limit(-1)
    st(x, y)
    torch.cuda.synchronize()
    health.check([m], eng)


def test_site_loop_fails_on_timed_out_handoff(tmp_path, spin_zero, monkeypatch):
    from dinunet_implementations_amd.ops import head as H
    monkeypatch.setattr(H, "_HEAD_REP", False)  # head_step.hip: the head with hand-offs
    from test_runtime_gpu import _ica_root, _run_site
    root = _ica_root(tmp_path)
    with pytest.raises(spin_zero.HandoffError):
        _run_site(root, str(tmp_path / "out"), {"epochs": 2, "batch_size": 8})


@pytest.mark.parametrize("use_graph", [False, True])
@pytest.mark.parametrize("engine", ["rankDAD", "dSGD"])
def test_persistent_kernels_beside_busy_cus(engine, use_graph, monkeypatch):
    """the persistent launches -- rank-dAD's one-launch power iteration
    (``lr_persist_kernel``) and the hand-off head (``head_step.hip``) -- on the multi-site path
    (one-rank RCCL group: ``_persist_ok`` true, collectives issued) while 64 CUs are held by
    collective-sized workgroups on a side stream, as RCCL's channel kernels hold them during a
    transfer: no in-kernel wait may time out and training must match the undisturbed run."""
    import torch.distributed as dist
    from dinunet_implementations_amd.ops import head as H
    from dinunet_implementations_amd.runtime import health
    from test_step_gpu import _OneRankGroup, _batches, _free_port, _trainer
    import os
    monkeypatch.setattr(H, "_HEAD_REP", False)  # head_step.hip: the head with hand-offs
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        grp = _OneRankGroup(dist.group.WORLD)
        xs, ys = _batches()
        ma, fa, sa = _trainer(0, engine=engine, group=grp, use_graph=use_graph)
        mb, fb, sb = _trainer(0, engine=engine, group=grp, use_graph=use_graph)
        if engine == "rankDAD":
            assert sb.engine._persist_ok, "the persistent power iteration must be on"
        side = torch.cuda.Stream()
        for i in range(xs.shape[0]):
            sa(xs[i], ys[i])
        torch.cuda.synchronize()
        for i in range(xs.shape[0]):
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                health.occupy_cus(64, 3000)
            sb(xs[i], ys[i])
        torch.cuda.synchronize()
        assert mb._head is not None and mb._head._sync is not None, "hand-off head did not run"
        health.check([mb], sb.engine)
        assert torch.equal(fa.data, fb.data)
    finally:
        dist.destroy_process_group()
