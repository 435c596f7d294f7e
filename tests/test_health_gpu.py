"""Negative controls of the in-kernel wait check (runtime.health) on the GPU: with the poll limit
forced to 0 every barrier of the one-launch rank-dAD iteration and every peer-exchange wait that
finds its flag unset gives up at once; the check must then raise -- on the kernels directly and
through the production site loop -- and stay quiet with the default limit."""
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


def test_peer_wait_timeout_raises(spin_zero):
    """A reduce whose push never ran (no site wrote its flag) gives up at once under the zero
    limit and says so; after that a complete exchange runs clean and exact."""
    from dinunet_implementations_amd.parallel import peer
    from dinunet_implementations_amd.parallel.group import SiteGroup
    health = spin_zero
    grp = SiteGroup(device=torch.device("cuda", 0), loopback=True)
    pm = peer.mean(grp, grp.device, 5000, "fp32", ("health",))
    x = torch.randn(5000, device="cuda")
    pm.finish(x)  # no push: the reduce-scatter wait cannot be satisfied
    torch.cuda.synchronize()
    eng = type("E", (), {"peer": True})()
    with pytest.raises(health.HandoffError, match="peer_exchange.*reduce-scatter"):
        health.check([], eng)
    health.set_spin_limit(-1)
    y = torch.randn(5000, device="cuda")
    ref = y.clone()
    pm.run_(y)  # one site: the mean is the value itself
    torch.cuda.synchronize()
    health.check([], eng)
    assert torch.equal(y, ref)


def test_site_loop_fails_on_timed_out_wait(tmp_path, spin_zero):
    from test_runtime_gpu import _ica_root, _run_site
    root = _ica_root(tmp_path)
    with pytest.raises(spin_zero.HandoffError):
        _run_site(root, str(tmp_path / "out"), {"epochs": 2, "batch_size": 8,
                                                "agg_engine": "rankDAD", "dad_reduction_rank": 4})


@pytest.mark.parametrize("use_graph", [False, True])
@pytest.mark.parametrize("engine,cfg", [("rankDAD", {}), ("dSGD", {"dsgd_collective": "peer"})])
def test_waiting_kernels_beside_busy_cus(engine, cfg, use_graph, monkeypatch):
    """the launches that wait -- rank-dAD's one-launch power iteration
    (``lr_persist_kernel``) and the peer exchange -- on the multi-site path (one-rank RCCL group:
    ``_persist_ok`` true, collectives issued) while 64 CUs are held by collective-sized
    workgroups on a side stream, as RCCL's channel kernels hold them during a transfer: no
    in-kernel wait may time out and training must match the undisturbed run."""
    import torch.distributed as dist
    from dinunet_implementations_amd.runtime import health
    from test_step_gpu import _OneRankGroup, _batches, _free_port, _trainer
    import os
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        grp = _OneRankGroup(dist.group.WORLD)
        xs, ys = _batches()
        ma, fa, sa = _trainer(0, engine=engine, group=grp, use_graph=use_graph, cfg=cfg)
        mb, fb, sb = _trainer(0, engine=engine, group=grp, use_graph=use_graph, cfg=cfg)
        if engine == "rankDAD":
            assert sb.engine._persist_ok, "the persistent power iteration must be on"
        else:
            assert sb.engine.peer, "the peer exchange must be on"
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
        health.check([mb], sb.engine)
        assert torch.equal(fa.data, fb.data)
    finally:
        dist.destroy_process_group()
