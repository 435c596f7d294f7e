"""Aggregation engines across 2-3 gloo processes (CPU): exactness and replica identity.

Model: SURVEY.md §4 (b)/(c): dSGD mean == pooled-batch gradient for equal site sizes; rank-dAD at
full rank == dSGD; PowerSGD at full rank == dSGD; replicas stay bit-identical; the COINSTAC
file-transport arithmetic (payload/aggregate/apply) equals the collective path.
"""
import torch
import torch.nn as nn

from mp_util import run_world


def _model():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(12, 8), nn.ReLU(), nn.Linear(8, 6), nn.ReLU(), nn.Linear(6, 3))


def _data(rank, n=10):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(n, 12, generator=g), torch.randint(0, 3, (n,), generator=g)


# ---- spawned workers (module level: picklable) -------------------------------------------------
def w_grads(grp, engine_name, cfg, overlap=True):
    from dinunet_implementations_amd.ops import FlatParams
    from dinunet_implementations_amd.parallel import DSGDEngine, make_engine
    m = _model()
    flat = FlatParams(m.parameters())
    if engine_name == "dSGD":
        eng = DSGDEngine(m, flat, grp, cfg, overlap=overlap)
    else:
        eng = make_engine(engine_name, m, flat, grp, cfg)
    x, y = _data(grp.rank)
    flat.zero_grad()
    with eng.step_context():
        nn.functional.cross_entropy(m(x), y).backward()
    scale = eng.reduce()
    return (flat.grad * scale).clone()


def w_powersgd_ef(grp):
    from dinunet_implementations_amd.ops import FlatParams
    from dinunet_implementations_amd.parallel import PowerSGDEngine
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(40, 30), nn.ReLU(), nn.Linear(30, 3))
    flat = FlatParams(m.parameters())
    eng = PowerSGDEngine(m, flat, grp, {"powersgd_rank": 2})
    g = torch.Generator().manual_seed(grp.rank)
    x, y = torch.randn(16, 40, generator=g), torch.randint(0, 3, (16,), generator=g)
    flat.zero_grad()
    nn.functional.cross_entropy(m(x), y).backward()
    M = m[0].weight.grad.clone()
    eng.reduce()
    return M, m[0].weight.grad.clone(), eng.err[0].clone(), len(eng.mats)


def w_adam_steps(grp, name):
    from dinunet_implementations_amd.ops import FlatParams, FusedAdam
    from dinunet_implementations_amd.parallel import make_engine
    m = _model()
    flat = FlatParams(m.parameters())
    opt = FusedAdam(flat, lr=1e-2)
    eng = make_engine(name, m, flat, grp, {"dad_reduction_rank": 3, "powersgd_rank": 2})
    for s in range(4):
        x, y = _data(grp.rank * 10 + s)
        flat.zero_grad()
        with eng.step_context():
            nn.functional.cross_entropy(m(x), y).backward()
        opt.step(grad_scale=eng.reduce())
    return flat.data.clone()


def _pooled(world):
    m = _model()
    xs, ys = zip(*[_data(r) for r in range(world)])
    nn.functional.cross_entropy(m(torch.cat(xs)), torch.cat(ys)).backward()
    return torch.cat([p.grad.reshape(-1) for p in m.parameters()])


def _unflat(g):
    from dinunet_implementations_amd.ops import FlatParams
    fp = FlatParams(_model().parameters())
    return torch.cat([g[o:o + n] for _, o, n in fp.segments()])


# ---- tests --------------------------------------------------------------------------------------
def test_dsgd_equals_pooled_gradient():
    world = 3
    gs = run_world(w_grads, world, "dSGD", {})
    for g in gs[1:]:
        assert torch.equal(g, gs[0])  # identical on every site
    assert torch.allclose(_unflat(gs[0]), _pooled(world), atol=1e-6)


def test_dsgd_overlap_matches_blocking_and_bf16_payload():
    a = run_world(w_grads, 2, "dSGD", {}, True)
    b = run_world(w_grads, 2, "dSGD", {}, False)
    assert torch.allclose(a[0], b[0], atol=1e-7)
    h = run_world(w_grads, 2, "dSGD", {"precision_bits": "16"})
    assert torch.allclose(h[0], a[0], atol=1e-2, rtol=2e-2)


def test_rankdad_full_rank_is_exact():
    ref = run_world(w_grads, 2, "dSGD", {})[0]
    gs = run_world(w_grads, 2, "rankDAD", {"dad_reduction_rank": 16, "dad_num_pow_iters": 3,
                                           "dad_tol": 0.0})
    assert torch.equal(gs[0], gs[1])
    assert torch.allclose(gs[0], ref, atol=1e-5)


def test_rankdad_low_rank_power_iteration_converges():
    ref = run_world(w_grads, 2, "dSGD", {})[0]
    g4 = run_world(w_grads, 2, "rankDAD", {"dad_reduction_rank": 4, "dad_num_pow_iters": 10,
                                           "dad_tol": 1e-6})[0]
    g1 = run_world(w_grads, 2, "rankDAD", {"dad_reduction_rank": 1, "dad_num_pow_iters": 10,
                                           "dad_tol": 1e-6})[0]
    e4 = (g4 - ref).norm() / ref.norm()
    e1 = (g1 - ref).norm() / ref.norm()
    assert e4 < e1 < 1.0


def test_powersgd_full_rank_matches_dsgd_and_error_feedback():
    ref = run_world(w_grads, 2, "dSGD", {})[0]
    gs = run_world(w_grads, 2, "powerSGD", {"powersgd_rank": 8})
    assert torch.equal(gs[0], gs[1])
    assert torch.allclose(gs[0], ref, atol=1e-5)
    outs = run_world(w_powersgd_ef, 2)
    M0, Mh, e, nm = outs[0]
    assert nm == 2  # both weight matrices are worth compressing at rank 2
    assert torch.equal(outs[0][1], outs[1][1])
    assert torch.allclose(e, M0 - Mh, atol=1e-6)  # error feedback keeps the residual


def test_replicas_identical_after_adam_steps_all_engines():
    for name in ("dSGD", "rankDAD", "powerSGD"):
        outs = run_world(w_adam_steps, 2, name)
        assert torch.equal(outs[0], outs[1]), name


def test_file_transport_matches_collectives():
    """COINSTAC path: sites' payloads -> remote aggregate -> apply == collective reduce."""
    ref = run_world(w_grads, 2, "dSGD", {})[0]
    from dinunet_implementations_amd.ops import FlatParams
    from dinunet_implementations_amd.parallel import DSGDEngine, RankDADEngine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    for cls, cfg in ((DSGDEngine, {}), (RankDADEngine, {"dad_reduction_rank": 16, "dad_tol": 0.0})):
        sites = []
        for r in range(2):
            m = _model()
            fp = FlatParams(m.parameters())
            eng = cls(m, fp, SiteGroup(), cfg)
            x, y = _data(r)
            with eng.step_context():
                nn.functional.cross_entropy(m(x), y).backward()
            sites.append((m, fp, eng, eng.payload()))
        agg = cls.aggregate([s[3] for s in sites], cfg)
        for m, fp, eng, _ in sites:
            eng.apply(agg)
        assert torch.allclose(sites[0][1].grad, ref, atol=1e-5), cls.__name__
        assert torch.allclose(sites[1][1].grad, ref, atol=1e-5), cls.__name__


def test_dsgd_split_buckets_partition_flat_buffer():
    """Split capture: non-stem gradients form the first bucket(s), the stem the last one."""
    from dinunet_implementations_amd.models import ICALstm
    from dinunet_implementations_amd.ops import FlatParams
    from dinunet_implementations_amd.parallel import make_engine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    m = ICALstm(input_size=16, hidden_size=16, num_comps=4, window_size=3)
    flat = FlatParams(m.parameters())
    eng = make_engine("dSGD", m, flat, SiteGroup(), {})
    first = eng.split_buckets(list(m.stem_parameters()))
    covered = sorted(eng.buckets)
    assert covered[0][0] == 0 and covered[-1][1] == flat.numel
    assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))
    stem_ids = {id(p) for p in m.stem_parameters()}
    for p, o, n in flat.segments():
        b = eng._param_bucket[id(p)]
        assert (b not in first) == (id(p) in stem_ids)


class _DeferredLinear(torch.autograd.Function):
    """Mimics the fused ops: returns no gradient for the weight to autograd and writes it into
    .grad only at the end of the backward pass (ops._grad.defer/flush), then notifies."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w.t()

    @staticmethod
    def backward(ctx, g):
        from dinunet_implementations_amd.ops import _grad
        x, w = ctx.saved_tensors

        def flush():
            w.grad.add_(g.t() @ x)
            _grad.notify([w])
        torch.autograd.Variable._execution_engine.queue_callback(flush)
        return g @ w, None


class _RecordingGroup:
    """A 2-site group whose all-reduce records what it was handed at launch time."""
    distributed, world, rank, backend = True, 2, 0, "gloo"

    def __init__(self):
        self.launched = []

    def all_reduce(self, t, op=None, async_op=False):
        self.launched.append(t.detach().clone())

        class _Done:
            def wait(self_inner):
                return None
        return _Done()


def test_dsgd_waits_for_deferred_fused_gradients():
    """A parameter whose producer hands autograd no gradient (fused op writing .grad at the end
    of the backward) must not be reported ready by autograd's post-accumulate hook, which
    fires anyway: its bucket would be all-reduced before the gradient exists.  Every bucket
    must be launched with its final local gradient."""
    from dinunet_implementations_amd.ops import FlatParams
    from dinunet_implementations_amd.parallel import DSGDEngine
    torch.manual_seed(0)
    lin1, lin2 = torch.nn.Linear(6, 5), torch.nn.Linear(5, 3)
    m = torch.nn.Sequential(lin1, lin2)
    flat = FlatParams(m.parameters())
    grp = _RecordingGroup()
    eng = DSGDEngine(m, flat, grp, {}, bucket_mb=1e-5)  # a bucket per parameter
    x = torch.randn(4, 6)
    flat.zero_grad()
    with eng.step_context():
        h = _DeferredLinear.apply(x, lin1.weight) + lin1.bias
        lin2(h).pow(2).sum().backward()
    final = flat.grad.clone()
    eng.reduce()
    assert len(grp.launched) == len(eng.buckets)
    for (s0, e0), sent in zip(eng.buckets, grp.launched):
        assert torch.equal(sent, final[s0:e0]), (s0, e0)
