"""TrainStep on the GPU: HIP-graph replay vs eager, split (two-graph) capture with the dSGD
all-reduce launched between the replays over a real RCCL communicator, and the rank-dAD
activation/delta capture of the fused kernels (``dW == Delta^T A`` for every Linear)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _model(seed, hidden=128):
    from dinunet_implementations_amd.models import ICALstm
    torch.manual_seed(seed)
    m = ICALstm(input_size=64, hidden_size=hidden, num_comps=20, window_size=10).cuda().train()
    m.classifier[0].p = 0.0  # no dropout: runs must be comparable step for step
    return m


def _trainer(seed, engine="dSGD", group=None, **kw):
    from dinunet_implementations_amd.ops import FlatParams, FusedAdam
    from dinunet_implementations_amd.parallel import make_engine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    from dinunet_implementations_amd.runtime.step import TrainStep
    m = _model(seed, kw.pop("hidden", 128))
    flat = FlatParams(m.parameters())
    opt = FusedAdam(flat, lr=1e-3)
    grp = group or SiteGroup(device=torch.device("cuda"))
    eng = make_engine(engine, m, flat, grp, {"precision_bits": "32", **kw.pop("cfg", {})})
    return m, flat, TrainStep(m, flat, opt, eng, task="ica", **kw)


def _batches(n=6, B=8, S=12):
    g = torch.Generator(device="cuda").manual_seed(7)
    xs = torch.randn(n, B, S, 20, 10, device="cuda", generator=g)
    ys = torch.randint(0, 2, (n, B), device="cuda", generator=g)
    return xs, ys


def _run(step, xs, ys):
    losses = []
    for i in range(xs.shape[0]):
        losses.append(float(step(xs[i], ys[i])))
    torch.cuda.synchronize()
    return losses


def test_graph_replay_matches_eager():
    xs, ys = _batches()
    _, fe, se = _trainer(0, use_graph=False)
    _, fg, sg = _trainer(0, use_graph=True)
    le, lg = _run(se, xs, ys), _run(sg, xs, ys)
    assert sg.graph is not None
    assert max(abs(a - b) for a, b in zip(le, lg)) < 1e-4
    assert torch.allclose(fe.data, fg.data, rtol=1e-5, atol=1e-6)


def test_deferred_pack_prologue_is_bit_identical(monkeypatch):
    """The LSTM repack taken out of the graph and fused into the step prologue's launch
    (ops.lstm.defer_pack + dn_lstm_pack_prologue) trains bit-identically to the captured pack."""
    import dinunet_implementations_amd.runtime.step as st
    xs, ys = _batches()
    monkeypatch.setattr(st, "DEFER_PACK", False)
    _, f0, s0 = _trainer(0, use_graph=True)
    _run(s0, xs, ys)
    monkeypatch.setattr(st, "DEFER_PACK", True)
    _, f1, s1 = _trainer(0, use_graph=True)
    _run(s1, xs, ys)
    assert not s0._packs and len(s1._packs) == 1 and s1._bf16_in
    assert torch.equal(f0.data, f1.data)


def test_split_capture_matches_single_graph():
    xs, ys = _batches()
    _, f1, s1 = _trainer(0, use_graph=True, split=False)
    _, f2, s2 = _trainer(0, use_graph=True, split=True)
    assert s2.split and not s1.split
    _run(s1, xs, ys)
    _run(s2, xs, ys)
    assert s2.graph_b is not None
    assert torch.equal(f1.data, f2.data)


class _OneRankGroup:
    """A 1-rank RCCL group that still takes the collective code paths (``distributed``)."""

    def __new__(cls, pg):
        from dinunet_implementations_amd.parallel.group import SiteGroup

        class G(SiteGroup):
            @property
            def distributed(self):
                return True
        return G(rank=0, world=1, local_rank=0, device=torch.device("cuda", 0), backend="nccl", pg=pg)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_split_capture_overlapped_allreduce_over_rccl():
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        grp = _OneRankGroup(dist.group.WORLD)
        xs, ys = _batches()
        _, f1, s1 = _trainer(0, use_graph=True, split=False)
        _, f2, s2 = _trainer(0, group=grp, use_graph=True)
        assert s2.split, "split capture must default on when sites are distributed"
        assert len(s2.engine.buckets) == 2
        _run(s1, xs, ys)
        _run(s2, xs, ys)
        assert s2.engine.comm_bytes == f2.numel * 4
        assert torch.equal(f1.data, f2.data)
    finally:
        dist.destroy_process_group()


@pytest.fixture
def rccl1():
    """A one-rank RCCL process group the multi-site code paths run on (``_OneRankGroup``)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        yield _OneRankGroup(dist.group.WORLD)
    finally:
        dist.destroy_process_group()


def _trainer_cfg(seed, engine, group, cfg, **kw):
    from dinunet_implementations_amd.ops import FlatParams, FusedAdam
    from dinunet_implementations_amd.parallel import make_engine
    from dinunet_implementations_amd.runtime.step import TrainStep
    m = _model(seed, kw.pop("hidden", 128))
    flat = FlatParams(m.parameters())
    opt = FusedAdam(flat, lr=1e-3)
    eng = make_engine(engine, m, flat, group, {"precision_bits": "32", **cfg})
    return m, flat, TrainStep(m, flat, opt, eng, task="ica", **kw)


def _device_fed(step, xs, ys, n, K=4):
    from dinunet_implementations_amd.runtime.feed import DeviceFeed
    B = xs.shape[1]
    X = xs.reshape(-1, *xs.shape[2:]).to(torch.bfloat16)
    Y = ys.reshape(-1)
    feed = DeviceFeed(step, X, Y, B, xs.shape[0], col=1, steps_per_graph=K)
    feed.run(3)
    feed.prepare(n - 3)
    feed.run(n - 3)
    torch.cuda.synchronize()
    return feed


@pytest.mark.parametrize("apack", [True, False])
def test_comm_graph_device_fed_matches_single_site(rccl1, apack, monkeypatch):
    """The multi-site device-fed step with its RCCL collectives captured (split backward, the
    body bucket's all-reduce on RCCL's stream between the parts, the stem bucket, the update and
    the next operands) replays in K-step graphs like one site and, over a one-rank RCCL group
    (sum over one site = identity), trains bit-identically to the single-site step."""
    from dinunet_implementations_amd.parallel.group import SiteGroup
    from dinunet_implementations_amd.runtime import step as step_mod
    monkeypatch.setattr(step_mod, "ADAM_PACK", apack)
    xs, ys = _batches(n=8)
    n = 16
    _, f1, s1 = _trainer_cfg(0, "dSGD", SiteGroup(device=torch.device("cuda")), {}, use_graph=True)
    _, f2, s2 = _trainer_cfg(0, "dSGD", rccl1, {}, use_graph=True)
    assert s2.split and s2.comm_graph and not s1.comm_graph
    _device_fed(s1, xs, ys, n)
    _device_fed(s2, xs, ys, n)
    assert set(s2._dgraphs) == {4, 1}, "K-step graphs, not the two-graph split replay"
    assert (s2._apack is not None) == apack
    assert s2.opt.step_count == s1.opt.step_count == n
    assert s2.engine.comm_bytes == f2.numel * 4
    assert torch.equal(f1.data, f2.data), (f1.data - f2.data).abs().max()
    assert abs(float(s1.last_loss) - float(s2.last_loss)) == 0.0


@pytest.mark.parametrize("engine,cfg,captured", [
    ("dSGD", {}, True),
    ("dSGD", {"precision_bits": "16"}, True),           # fp16 wire: the peer exchange (auto)
    ("dSGD", {"dsgd_collective": "peer"}, True),
    ("dSGD", {"precision_bits": "16", "dsgd_collective": "direct"}, False),  # RCCL all-to-all
    ("dSGD", {"precision_bits": "16", "dsgd_collective": "allreduce", "payload_dtype": "bf16"},
     True),
    ("rankDAD", {}, True),
    ("rankDAD", {"precision_bits": "16"}, True),
    ("rankDAD", {"dsgd_collective": "peer"}, True),
    ("powerSGD", {}, True),
    ("powerSGD", {"precision_bits": "16"}, True),
])
def test_comm_graph_matches_host_issued_collectives(rccl1, engine, cfg, captured, monkeypatch):
    """Every engine and wire: the step with its collectives captured in the K-step graph gives
    the trajectory of the uncaptured multi-site step (DINUNET_CAPTURE_COMM=0: host-issued
    collectives between / after the replays, eager update).  16-bit wires default to the peer
    exchange (kernels only: captured); only an explicit RCCL all-to-all exchange
    (``dsgd_collective=direct``) keeps host-issued collectives (Engine.capturable)."""
    from dinunet_implementations_amd.runtime import step as step_mod
    xs, ys = _batches(n=8)
    n = 12
    monkeypatch.setattr(step_mod, "CAPTURE_COMM", False)
    _, fh, sh = _trainer_cfg(0, engine, rccl1, cfg, use_graph=True)
    monkeypatch.setattr(step_mod, "CAPTURE_COMM", True)
    _, fc, sc = _trainer_cfg(0, engine, rccl1, cfg, use_graph=True)
    assert sc.comm_graph == captured and not sh.comm_graph
    if not captured:
        return
    _device_fed(sh, xs, ys, n)
    _device_fed(sc, xs, ys, n)
    assert 4 in sc._dgraphs and sc._dK == 4
    assert sc.opt.step_count == sh.opt.step_count == n
    assert torch.allclose(fh.data, fc.data, rtol=1e-5, atol=1e-6), (fh.data - fc.data).abs().max()
    eng = sc.engine
    if hasattr(eng, "_table") and getattr(eng._table, "_persist", None) is not None:
        assert eng._table.persist_error() == 0


def test_comm_graph_host_fed_matches_uncaptured(rccl1, monkeypatch):
    """Host-fed steps (``TrainStep.__call__``) across sites: one captured graph per step with
    the split backward, the bucket collectives and the fused Adam inside == the two-graph
    replay with host-issued collectives and an eager update."""
    from dinunet_implementations_amd.runtime import step as step_mod
    xs, ys = _batches()
    monkeypatch.setattr(step_mod, "CAPTURE_COMM", False)
    _, fh, sh = _trainer_cfg(0, "dSGD", rccl1, {}, use_graph=True)
    monkeypatch.setattr(step_mod, "CAPTURE_COMM", True)
    _, fc, sc = _trainer_cfg(0, "dSGD", rccl1, {}, use_graph=True)
    _run(sh, xs, ys)
    _run(sc, xs, ys)
    assert sc.graph_opt and sc.graph_b is None and sh.graph_b is not None
    assert sc.opt.step_count == sh.opt.step_count == xs.shape[0]
    assert int(sc.opt.device_step().item()) == sc.opt.step_count
    assert torch.allclose(fh.data, fc.data, rtol=1e-6, atol=1e-7), (fh.data - fc.data).abs().max()


def test_rankdad_capture_reconstructs_fused_gradients():
    """Every Linear's (A, Delta) captured from the fused encoder / LSTM / head kernels must
    rebuild that Linear's weight gradient: dW = Delta^T A."""
    from dinunet_implementations_amd.ops import FlatParams
    from dinunet_implementations_amd.ops import capture as cap
    import torch.nn as nn
    m = _model(0)
    flat = FlatParams(m.parameters())
    xs, ys = _batches(1)
    lin = [mod for mod in m.modules() if isinstance(mod, nn.Linear)]
    flat.zero_grad()
    with cap.DADCapture(modules=lin) as c:
        _, loss, _ = m.forward_loss(xs[0], ys[0])
        loss.backward()
    torch.cuda.synchronize()
    assert set(c.records) == set(lin), "every Linear must be captured"
    for mod in lin:
        recs = c.records[mod]
        A = torch.cat([a.reshape(-1, a.shape[-1]).float() for a, _ in recs])
        D = torch.cat([d.reshape(-1, d.shape[-1]).float() for _, d in recs])
        g = D.t() @ A
        ref = mod.weight.grad.float()
        err = (g - ref).norm().item() / max(ref.norm().item(), 1e-12)
        assert err < 2e-2, (mod, err)


@pytest.mark.parametrize("engine", ["rankDAD", "powerSGD"])
def test_lowrank_engines_train_on_gpu(engine):
    xs, ys = _batches()
    _, flat, step = _trainer(0, engine=engine)
    before = flat.data.clone()
    losses = _run(step, xs, ys)
    assert all(l == l for l in losses)
    assert not torch.equal(before, flat.data)


def test_in_graph_adam_tracks_host_step_count_and_lr_change():
    """Single site: the fused Adam is captured in the graph with a device step counter; the
    host count stays in sync and a learning-rate change forces a re-capture."""
    xs, ys = _batches()
    _, fe, se = _trainer(0, use_graph=False)
    _, fg, sg = _trainer(0, use_graph=True)
    _run(se, xs, ys)
    _run(sg, xs, ys)
    assert sg.graph_opt and sg.opt.step_count == se.opt.step_count == xs.shape[0]
    assert int(sg.opt._tdev.item()) == sg.opt.step_count
    assert torch.allclose(fe.data, fg.data, rtol=1e-5, atol=1e-6)
    se.opt.lr = sg.opt.lr = 5e-4
    _run(se, xs, ys)
    _run(sg, xs, ys)
    assert sg._cap_lr == 5e-4
    assert torch.allclose(fe.data, fg.data, rtol=1e-4, atol=1e-5)


def test_rankdad_gradient_space_factorisation():
    """GPU rank-dAD factorises G = Delta^T A (already in .grad) by the same power iteration:
    at world 1 every large Linear's gradient becomes a rank-r approximation close to the
    optimal truncated SVD; layers with min(in, out) <= r stay exact; the step graph captures it."""
    from dinunet_implementations_amd.ops import FlatParams
    from dinunet_implementations_amd.parallel import make_engine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    m = _model(0)
    flat = FlatParams(m.parameters())
    eng = make_engine("rankDAD", m, flat, SiteGroup(device=torch.device("cuda")),
                      {"dad_reduction_rank": 4, "dad_num_pow_iters": 8, "dad_tol": 1e-4})
    assert eng.fast and eng.fast_layers
    xs, ys = _batches(1)
    flat.zero_grad()
    _, loss, _ = m.forward_loss(xs[0], ys[0])
    loss.backward()
    torch.cuda.synchronize()
    before = flat.grad.clone()
    eng.reduce()
    torch.cuda.synchronize()
    low = {id(l[0].weight) for l in eng.fast_layers}
    for p, o, n in flat.segments():
        g0, g1 = before[o:o + n], flat.grad[o:o + n]
        if id(p) not in low:
            assert torch.equal(g0, g1)
            continue
        G = g0.view_as(p).double()
        s = torch.linalg.svdvals(G)
        best = s[4:].norm() / s.norm()
        err = (g1.view_as(p).double() - G).norm() / G.norm()
        assert err <= best * 1.15 + 1e-6, (err.item(), best.item())


def test_rankdad_step_graph_matches_eager():
    xs, ys = _batches()
    _, fe, se = _trainer(0, engine="rankDAD", use_graph=False)
    _, fg, sg = _trainer(0, engine="rankDAD", use_graph=True)
    _run(se, xs, ys)
    _run(sg, xs, ys)
    assert sg.graph is not None
    assert torch.allclose(fe.data, fg.data, rtol=1e-4, atol=1e-5)


def test_step_counter_bump_is_explicit():
    """The step prologue advances exactly the counter it is given, once per launch, and
    nothing when given none."""
    from dinunet_implementations_amd.ops import FlatParams, FusedAdam, step_prologue
    lin = torch.nn.Linear(8, 4).cuda()
    flat = FlatParams(lin.parameters())
    opt = FusedAdam(flat, lr=1e-3)
    opt.step_count = 5
    opt.sync_device_step()
    x = torch.randn(4, 8, device="cuda")
    y = torch.randint(0, 2, (4,), device="cuda")
    yd = torch.empty_like(y)
    xb = torch.empty_like(x, dtype=torch.bfloat16)
    step_prologue(x, xb, y, yd, flat.grad, opt.device_step())
    step_prologue(x, xb, y, yd, flat.grad)  # no counter: no advance
    torch.cuda.synchronize()
    assert int(opt.device_step().item()) == 6
    assert torch.equal(yd, y) and torch.equal(xb, x.to(torch.bfloat16))


def test_ragged_batch_keeps_device_step_in_sync():
    """A ragged batch after capture runs eagerly; the captured Adam's device counter must follow
    the host step count so later replays match torch.optim.Adam's bias corrections."""
    from dinunet_implementations_amd.ops import FlatParams, FusedAdam
    from dinunet_implementations_amd.parallel import make_engine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    from dinunet_implementations_amd.runtime.step import TrainStep
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 2)).cuda()
    ref = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 2)).cuda()
    ref.load_state_dict(net.state_dict())
    flat = FlatParams(net.parameters())
    opt = FusedAdam(flat, lr=1e-2)
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-2)
    grp = SiteGroup(device=torch.device("cuda"))
    eng = make_engine("dSGD", net, flat, grp, {"precision_bits": "32"})

    def fl(model, x, y):
        out = model(x)
        loss = torch.nn.functional.cross_entropy(out, y)
        return out, loss, out.argmax(1)

    step = TrainStep(net, flat, opt, eng, forward_loss=fl, use_graph=True, eager_warmup=1)
    g = torch.Generator(device="cuda").manual_seed(3)
    sizes = [8, 8, 8, 5, 8, 8]
    for n in sizes:
        x = torch.randn(n, 16, device="cuda", generator=g)
        y = torch.randint(0, 2, (n,), device="cuda", generator=g)
        step(x, y)
        ropt.zero_grad()
        torch.nn.functional.cross_entropy(ref(x), y).backward()
        ropt.step()
    torch.cuda.synchronize()
    assert step.graph is not None and step.graph_opt
    assert int(opt.device_step().item()) == opt.step_count == len(sizes)
    for p, q in zip(net.parameters(), ref.parameters()):
        assert torch.allclose(p, q, rtol=1e-4, atol=1e-5)


def test_accumulated_graph_step_matches_eager():
    """local_iterations = 2 on the HIP-graph path: the second micro-batch's replay accumulates
    into the gradient (no zeroing prologue), the update runs after it; equals the eager
    accumulation (reference (loss / li).backward())."""
    xs, ys = _batches(n=10)
    _, fe, se = _trainer(0, use_graph=False, accum=2)
    _, fg, sg = _trainer(0, use_graph=True, accum=2)
    for st in (se, sg):
        for i in range(xs.shape[0]):
            st(xs[i], ys[i], first=i % 2 == 0, last=i % 2 == 1)
    torch.cuda.synchronize()
    assert sg.graph is not None and not sg.graph_opt
    assert se.opt.step_count == sg.opt.step_count == 5
    assert torch.allclose(fe.data, fg.data, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("engine", ["powerSGD", "rankDAD"])
def test_accumulated_lowrank_graph_matches_eager(engine):
    """local_iterations = 2 with a low-rank engine on the graph path: the local factorisation
    (PowerSGD error feedback, rank-dAD warm start) runs once per step, after the second
    micro-batch, exactly as in the eager accumulation (it used to be captured and so
    replayed with every micro-batch)."""
    xs, ys = _batches(n=8)
    _, fe, se = _trainer(0, engine=engine, use_graph=False, accum=2)
    _, fg, sg = _trainer(0, engine=engine, use_graph=True, accum=2)
    for st in (se, sg):
        for i in range(xs.shape[0]):
            st(xs[i], ys[i], first=i % 2 == 0, last=i % 2 == 1)
    torch.cuda.synchronize()
    assert sg.graph is not None and sg._pre_reduce is None
    assert se.opt.step_count == sg.opt.step_count == 4
    assert torch.allclose(fe.data, fg.data, rtol=1e-4, atol=1e-5), (fe.data - fg.data).abs().max()


def test_powersgd_device_matches_reference_math():
    """Device PowerSGD (csrc/kernels/lowrank.hip: P = M Q with M = G + err, Cholesky QR,
    Q = M^T P, G = P Q^T, err = M - G) == the same algorithm in torch ops (MGS), over 3
    steps of error feedback and warm-started Q."""
    from dinunet_implementations_amd.ops import FlatParams
    from dinunet_implementations_amd.parallel import PowerSGDEngine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    grp = SiteGroup(device=torch.device("cuda"))
    m = _model(0)
    fa = FlatParams(m.parameters())
    ea = PowerSGDEngine(m, fa, grp, {"powersgd_rank": 4})
    mb = _model(0)
    fb = FlatParams(mb.parameters())
    eb = PowerSGDEngine(mb, fb, grp, {"powersgd_rank": 4, "powersgd_device": False})
    assert ea.fast and not eb.fast
    g = torch.Generator(device="cuda").manual_seed(3)
    for _ in range(3):
        gr = torch.randn(fa.grad.shape, device="cuda", generator=g)
        fa.grad.copy_(gr)
        fb.grad.copy_(gr)
        ea.reduce()
        eb.reduce()
        torch.cuda.synchronize()
        assert torch.allclose(fa.grad, fb.grad, rtol=1e-3, atol=1e-4), \
            (fa.grad - fb.grad).abs().max()
        for x, y in zip(ea.err, eb.err):
            assert torch.allclose(x, y, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("rank", [4, 8, 16])
def test_powersgd_device_many_layers_and_ranks(rank):
    """More matrices than one low-rank launch indexes (20 > LR_KMAX = 16: the host cuts the table
    into launches of 16 layers) and every rank bound of lr_gtp (4, 8, 16): the device PowerSGD
    equals the torch-op algorithm over 2 steps of error feedback."""
    import torch.nn as nn
    from dinunet_implementations_amd.ops import FlatParams
    from dinunet_implementations_amd.parallel import PowerSGDEngine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    grp = SiteGroup(device=torch.device("cuda"))

    def model():
        torch.manual_seed(5)
        dims = [96, 80, 64, 72, 96] * 4 + [96]
        return nn.Sequential(*[nn.Linear(dims[i], dims[i + 1]) for i in range(20)]).cuda()
    ma, mb = model(), model()
    fa, fb = FlatParams(ma.parameters()), FlatParams(mb.parameters())
    ea = PowerSGDEngine(ma, fa, grp, {"powersgd_rank": rank})
    eb = PowerSGDEngine(mb, fb, grp, {"powersgd_rank": rank, "powersgd_device": False})
    assert ea.fast and not eb.fast and len(ea.mats) == 20
    g = torch.Generator(device="cuda").manual_seed(9)
    for _ in range(2):
        gr = torch.randn(fa.grad.shape, device="cuda", generator=g)
        fa.grad.copy_(gr)
        fb.grad.copy_(gr)
        ea.reduce()
        eb.reduce()
        torch.cuda.synchronize()
        assert torch.allclose(fa.grad, fb.grad, rtol=1e-3, atol=1e-4), \
            (fa.grad - fb.grad).abs().max()
        for x, y in zip(ea.err, eb.err):
            assert torch.allclose(x, y, rtol=1e-3, atol=1e-4)


def test_powersgd_step_graph_matches_eager():
    xs, ys = _batches()
    _, fe, se = _trainer(0, engine="powerSGD", use_graph=False)
    _, fg, sg = _trainer(0, engine="powerSGD", use_graph=True)
    _run(se, xs, ys)
    _run(sg, xs, ys)
    assert sg.graph is not None and sg.graph_opt
    assert torch.allclose(fe.data, fg.data, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("shuffle,apack", [(False, False), (True, False), (False, True),
                                           (True, True)])
def test_device_fed_multistep_graph_matches_host_fed(shuffle, apack, monkeypatch):
    """Batches resident in HBM (bf16) gathered on the device at a cursor, 4 whole steps per HIP
    graph: the same trajectory as feeding the same batches from the host loop one step per
    replay.  apack: the fused Adam also rewrites the packed LSTM / encoder operand images, zeroes
    the gradient and gathers the next batch (no pack launch in the replayed steps)."""
    from dinunet_implementations_amd.ops import DeviceSource
    from dinunet_implementations_amd.runtime import step as step_mod
    monkeypatch.setattr(step_mod, "ADAM_PACK", apack)
    xs, ys = _batches(n=8)
    B = xs.shape[1]
    X = xs.reshape(-1, *xs.shape[2:]).to(torch.bfloat16)
    Y = ys.reshape(-1)
    order = torch.randperm(X.shape[0], device="cuda") if shuffle else None
    _, fh, sh = _trainer(0, use_graph=True)
    _, fd, sd = _trainer(0, use_graph=True)
    src = DeviceSource(X, Y, B, order=order)
    sd.bind(src, steps_per_graph=4)
    assert (sd._apack is not None) == apack
    n = 16
    for c in range(n):
        xb, yb = src.batch(c)
        sh(xb.float(), yb)
    sd.run(3)
    sd.prepare(n - 3)
    assert set(sd._dgraphs) == {4, 1}
    sd.run(n - 3)
    torch.cuda.synchronize()
    assert int(src.cursor.item()) == n and sd.opt.step_count == sh.opt.step_count == n
    assert torch.equal(sd.last_labels, src.batch(n - 1)[1])
    assert torch.allclose(fh.data, fd.data, rtol=1e-6, atol=1e-7), (fh.data - fd.data).abs().max()
    assert abs(float(sh.last_loss) - float(sd.last_loss)) < 1e-5


@pytest.mark.parametrize("hidden", [128, 348, 384, 600])
def test_adam_pack_images_match_pack_kernel(hidden):
    """The persistent images the fused Adam writes (update=False: from the current parameters)
    equal dn_lstm_pack's layouts: W_ih / W_hh / W_hh^T bf16 images and the encoder copies
    bit for bit, the split bias images summing to the fused bias."""
    from dinunet_implementations_amd.ops.lstm import pack_params
    model, flat, step = _trainer(0, use_graph=True, hidden=hidden)
    opt = step.opt
    pp = model.persistent_pack(flat.data.device)
    opt.attach_pack(pp)
    flat.grad.fill_(1.0)
    opt.step_pack(update=False, gofs=0)
    torch.cuda.synchronize()
    assert float(flat.grad.abs().max()) == 0.0  # zeroed as consumed
    lin = model.encoder[0]
    casts = []
    params = [t for cell in model.lstm.lstms for t in cell.params()]
    wih_p, bias_p, whh_p, whhT_p, _ = pack_params(params, model.lstm.input_size, flat.data.device,
                                                  casts=(lin.weight, lin.bias), cast_out=casts)
    torch.cuda.synchronize()
    assert torch.equal(pp.wih_p, wih_p)
    assert torch.equal(pp.whh_p, whh_p)
    assert torch.equal(pp.whhT_p, whhT_p)
    n = bias_p.numel()
    assert torch.equal(pp.bias_p[:n] + pp.bias_p[n:], bias_p)
    for a, b in zip(pp.casts, casts):
        assert torch.equal(a, b)


@pytest.mark.parametrize("hidden,tol", [(128, 0.0), (384, 0.0), (384, 1e-3)])
def test_rankdad_persistent_launch_matches_staged(hidden, tol, monkeypatch):
    """All power iterations of every layer in ONE launch (lr_persist_kernel, per-layer barriers)
    give the staged two-launches-per-iteration factorisation: same warm start, same Gram /
    Cholesky math, sums in another order.  Repeated launches (the barrier counters reset by each
    launch) stay consistent, no barrier times out, and the iterations run are counted."""
    from dinunet_implementations_amd.models import ICALstm
    from dinunet_implementations_amd.ops import FlatParams
    from dinunet_implementations_amd.parallel import make_engine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    torch.manual_seed(0)
    m = ICALstm(input_size=256, hidden_size=hidden, num_comps=100, window_size=10).cuda()
    flat = FlatParams(m.parameters())
    cfg = {"dad_reduction_rank": 10, "dad_num_pow_iters": 5, "dad_tol": tol, "seed": 3}
    grp = SiteGroup(device=torch.device("cuda"))
    ep = make_engine("rankDAD", m, flat, grp, cfg)
    es = make_engine("rankDAD", m, flat, grp, cfg)
    assert ep.fast and ep.fast_layers
    g = torch.Generator(device="cuda").manual_seed(11)
    for call in range(3):
        G0 = torch.randn(flat.grad.shape, device="cuda", generator=g)
        # a low-rank-ish gradient: the power iteration then converges like on real gradients
        for p_, o, n in flat.segments():
            if p_.dim() == 2:
                u = torch.randn(p_.shape[0], 12, device="cuda", generator=g)
                v = torch.randn(12, p_.shape[1], device="cuda", generator=g)
                G0[o:o + n] += (u @ v).reshape(-1) * 0.5
        flat.grad.copy_(G0)
        monkeypatch.setenv("DINUNET_LR_PERSIST", "1")
        it0 = ep.power_iterations()
        ep.reduce()
        torch.cuda.synchronize()
        gp = flat.grad.clone()
        assert ep._table.persist_error() == 0
        it1 = ep.power_iterations()
        flat.grad.copy_(G0)
        monkeypatch.setenv("DINUNET_LR_PERSIST", "0")
        es.reduce()
        torch.cuda.synchronize()
        gs = flat.grad.clone()
        for (mod, o, out_f, in_f, *_r) in ep.fast_layers:
            a_, b_ = gp[o:o + out_f * in_f], gs[o:o + out_f * in_f]
            rel = float((a_ - b_).norm() / b_.norm().clamp_min(1e-30))
            assert rel < 2e-3, (call, out_f, in_f, rel)
        runs = [b - a for a, b in zip(it0, it1)]
        assert all(1 <= x <= 5 for x in runs), runs
        if tol == 0.0:
            assert all(x == 5 for x in runs), runs



@pytest.mark.parametrize("apack", [False, True])
def test_device_feed_epoch_matches_host_loop(apack, monkeypatch):
    """runtime.feed.DeviceFeed (what FederatedSite trains its epochs with): one epoch of K-step
    graph replays over an explicit batch order gives the host-fed loop's trajectory, and the
    device-side train records hold every step's loss and prob[:, 1] column (the train average and
    the train AUC of the reference, comps/icalstm/__init__.py:64-68) in step order."""
    from dinunet_implementations_amd.runtime import step as step_mod
    from dinunet_implementations_amd.runtime.feed import DeviceFeed
    monkeypatch.setattr(step_mod, "ADAM_PACK", apack)
    xs, ys = _batches(n=6)
    B = xs.shape[1]
    X = xs.reshape(-1, *xs.shape[2:]).to(torch.bfloat16)
    Y = ys.reshape(-1)
    nb = 11  # > the rows: the order cycles, and 11 = 4 + 4 + 3 needs a remainder graph
    g = torch.Generator(device="cuda").manual_seed(5)
    _, fh, sh = _trainer(0, use_graph=True)
    _, fd, sd = _trainer(0, use_graph=True)
    feed = DeviceFeed(sd, X, Y, B, nb, col=1, steps_per_graph=4)
    assert (sd._apack is not None) == apack
    host_loss, host_score = [], []
    for epoch in range(2):
        order = torch.randint(0, X.shape[0], (nb * B,), device="cuda", generator=g)
        for c in range(nb):
            rows = order[c * B:(c + 1) * B]
            loss = sh(X[rows].float(), Y[rows])
            host_loss.append(float(loss))
            host_score.append(sh.last_out[:, 1].clone())
        losses, scores, labels = feed.run_epoch(order)
        torch.cuda.synchronize()
        assert torch.equal(labels, Y[order])
        hl = torch.tensor(host_loss[-nb:], device="cuda")
        assert torch.allclose(losses, hl, rtol=1e-5, atol=1e-6), (losses, hl)
        hs = torch.cat(host_score[-nb:])
        assert torch.allclose(scores, hs, rtol=1e-4, atol=1e-6), (scores - hs).abs().max()
    assert sd.opt.step_count == sh.opt.step_count == 2 * nb
    assert torch.allclose(fh.data, fd.data, rtol=1e-6, atol=1e-7), (fh.data - fd.data).abs().max()


def _feed_vs_host(sh, sd, X, Y, B, nb, accum, col, epochs=2, seed=5):
    """One DeviceFeed epoch per loop over a random batch order vs the host-fed TrainStep on the
    same batches (``accum`` micro-batches per step); returns the two flat parameter sets."""
    from dinunet_implementations_amd.runtime.feed import DeviceFeed
    feed = DeviceFeed(sd, X, Y, B, nb, col=col, steps_per_graph=4)
    g = torch.Generator(device="cuda").manual_seed(seed)
    nbb = nb * accum
    host_loss, host_score = [], []
    for _ in range(epochs):
        order = torch.randint(0, X.shape[0], (nbb * B,), device="cuda", generator=g)
        for c in range(nbb):
            rows = order[c * B:(c + 1) * B]
            loss = sh(X[rows].float(), Y[rows], first=c % accum == 0, last=c % accum == accum - 1)
            host_loss.append(float(loss))
            host_score.append((sh.last_pred.float() if col < 0 else sh.last_out[:, col]).clone())
        losses, scores, labels = feed.run_epoch(order)
        torch.cuda.synchronize()
        assert torch.equal(labels, Y[order])
        hl = torch.tensor(host_loss[-nbb:], device="cuda")
        assert torch.allclose(losses, hl, rtol=1e-5, atol=1e-6), (losses, hl)
        hs = torch.cat(host_score[-nbb:])
        assert torch.allclose(scores, hs, rtol=1e-4, atol=1e-6), (scores - hs).abs().max()
    assert sd.opt.step_count == sh.opt.step_count == epochs * nb
    return feed


@pytest.mark.parametrize("engine,sites", [("dSGD", 1), ("dSGD", "rccl1"), ("rankDAD", 1),
                                          ("powerSGD", "rccl1")])
def test_device_feed_accumulation_matches_host_loop(engine, sites, request):
    """local_iterations > 1 on the device-fed epoch -- every replay holds
    whole accumulated steps (2 micro-batches each gathered at the cursor, d(loss)/2 into one
    gradient, one reduction and one update), giving the host-fed accumulation's trajectory and
    per-micro-batch train records; across sites the collectives are captured with the update."""
    grp = request.getfixturevalue("rccl1") if sites == "rccl1" else None
    xs, ys = _batches(n=6)
    B = xs.shape[1]
    X = xs.reshape(-1, *xs.shape[2:]).to(torch.bfloat16)
    Y = ys.reshape(-1)
    mk = (lambda: _trainer_cfg(0, engine, grp, {"dad_reduction_rank": 4}, use_graph=True,
                               accum=2)) if grp is not None else (
        lambda: _trainer(0, engine=engine, use_graph=True, accum=2))
    _, fh, sh = mk()
    _, fd, sd = mk()
    feed = _feed_vs_host(sh, sd, X, Y, B, nb=5, accum=2, col=1)
    assert sd._dK == 4 and sd._apack is None and feed.nbb == 10
    assert all(v[2] for v in sd._dgraphs.values()), "the update must be inside the replays"
    tol = dict(rtol=1e-6, atol=1e-7) if engine == "dSGD" else dict(rtol=1e-4, atol=1e-5)
    assert torch.allclose(fh.data, fd.data, **tol), (fh.data - fd.data).abs().max()


@pytest.mark.parametrize("accum", [1, 2])
def test_fs_device_feed_matches_host_loop(accum):
    """the FS task on the device-fed epoch -- 66 fp32 features resident in
    HBM (padded to 72 columns once, gathered exactly into an fp32 static input the head reads
    through its row stride) and hard-label train scores recorded from the predicted class
    (comps/fs/__init__.py:57-59)."""
    from dinunet_implementations_amd.models import MSANNet
    from dinunet_implementations_amd.ops import FlatParams, FusedAdam
    from dinunet_implementations_amd.parallel import make_engine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    from dinunet_implementations_amd.runtime.step import TrainStep

    def mk():
        torch.manual_seed(0)
        m = MSANNet(66, [64, 32], 2).cuda().train()
        flat = FlatParams(m.parameters())
        opt = FusedAdam(flat, lr=1e-3)
        eng = make_engine("dSGD", m, flat, SiteGroup(device=torch.device("cuda")), {})
        return flat, TrainStep(m, flat, opt, eng, task="fs", use_graph=True, accum=accum)

    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.randn(96, 66, device="cuda", generator=g)
    Y = torch.randint(0, 2, (96,), device="cuda", generator=g)
    fh, sh = mk()
    fd, sd = mk()
    feed = _feed_vs_host(sh, sd, X, Y, 16, nb=5, accum=accum, col=-1)
    assert feed.src.width == 66 and sd._dsx.shape == (16, 72) and sd._dsx.dtype == torch.float32
    assert torch.allclose(fh.data, fd.data, rtol=1e-6, atol=1e-7), (fh.data - fd.data).abs().max()


@pytest.mark.parametrize("engine,sites", [("dSGD", 1), ("dSGD", "rccl1")])
def test_device_fed_rows_in_place_matches_batch_copy(engine, sites, monkeypatch, request):
    """DINUNET_ROWS_FEED: the Adam-emitted pack writes the next batch's subject indices instead
    of copying the batch, and the encoder forward / weight-gradient GEMMs read the rows in place
    from the HBM-resident dataset -- the same trajectory, bit for bit, as the batch copy, on one
    site and on the captured multi-site step."""
    from dinunet_implementations_amd.runtime import step as step_mod
    from dinunet_implementations_amd.runtime.feed import DeviceFeed
    grp = request.getfixturevalue("rccl1") if sites == "rccl1" else None
    xs, ys = _batches(n=6, B=8, S=70)
    B = xs.shape[1]
    X = xs.reshape(-1, *xs.shape[2:]).to(torch.bfloat16)
    Y = ys.reshape(-1)
    mk = (lambda: _trainer_cfg(0, engine, grp, {}, use_graph=True)) if grp is not None else (
        lambda: _trainer(0, engine=engine, use_graph=True))
    runs = []
    for mode in ("0", "1"):
        monkeypatch.setattr(step_mod, "ROWS_FEED", mode)
        _, f, st = mk()
        feed = DeviceFeed(st, X, Y, B, 7, col=1, steps_per_graph=4)
        assert (st._rows is not None) == (mode == "1") and st._apack is not None
        g = torch.Generator(device="cuda").manual_seed(2)
        for _ in range(2):
            order = torch.randint(0, X.shape[0], (7 * B,), device="cuda", generator=g)
            losses, scores, _ = feed.run_epoch(order)
        torch.cuda.synchronize()
        runs.append((f.data.clone(), losses.clone(), scores.clone()))
    (f0, l0, s0), (f1, l1, s1) = runs
    assert torch.equal(f0, f1) and torch.equal(l0, l1) and torch.equal(s0, s1)
