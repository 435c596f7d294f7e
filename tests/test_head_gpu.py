"""Fused MLP head + loss against the plain module path in fp32: csrc/kernels/mlp_head.hip for
batches <= 64, csrc/kernels/head_big.hip (row-block tiling, cross-workgroup BatchNorm statistics)
above."""
import copy

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.float(), b.float()
    return (a - b).norm().item() / max(b.norm().item(), 1e-12)


def _ica_head(p=0.25, hidden=384, ncls=2):
    return nn.Sequential(nn.Dropout(p), nn.Linear(hidden, 256), nn.BatchNorm1d(256), nn.ReLU(),
                         nn.Linear(256, 64), nn.ReLU(), nn.Linear(64, ncls))


def _fs_head(in_size=66, hidden=(256, 128, 64, 32), ncls=2, dropout_in=()):
    from dinunet_implementations_amd.models import MSANNet
    return MSANNet(in_size, list(hidden), ncls, dropout_in=list(dropout_in))


class _RoundFwd(torch.autograd.Function):
    """bf16 rounding of a forward value (an MFMA operand); gradient passes through."""
    @staticmethod
    def forward(ctx, t):
        return t.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, d):
        return d


class _RoundBwd(torch.autograd.Function):
    """Identity forward; rounds the incoming gradient to bf16 (the kernel's dZ operand)."""
    @staticmethod
    def forward(ctx, t):
        return t.view_as(t)

    @staticmethod
    def backward(ctx, d):
        return d.to(torch.bfloat16).float()


def _emulated(mods, x):
    """The module chain with the fused kernel's rounding points (bf16 MFMA operands, fp32
    bias / BatchNorm / accumulation), no dropout."""
    from dinunet_implementations_amd.ops.head import HeadSpec
    spec = HeadSpec(mods)
    a = x
    for L in spec.layers:
        lin = L.linear
        z = _RoundBwd.apply(_RoundFwd.apply(a) @ _RoundFwd.apply(lin.weight).t())
        if lin.bias is not None:
            z = z + lin.bias
        if L.bn is not None:
            z = L.bn(z)
        if L.relu:
            z = torch.relu(z)
        a = z
    return a


def _compare(mods_fused, mods_ref, fused_fn, x, y, log_out, train=True, emulate=True):
    from dinunet_implementations_amd.ops import reference as ref
    from dinunet_implementations_amd.ops.head import HeadSpec, head_loss
    spec = HeadSpec(mods_fused)
    assert spec.ok and spec.supported(x)
    xf = x.clone().requires_grad_()
    xr = x.clone().requires_grad_()
    out, loss, pred = head_loss(xf, spec, y, log_out=log_out)
    if emulate:
        z = _emulated(mods_ref, xr)
    else:
        z = xr
        for m in mods_ref:
            z = m(z)
    ro, rl, rp = (ref.log_softmax_nll if log_out else ref.softmax_ce)(z, y)
    assert abs(loss.item() - rl.item()) < 2e-2 * max(1.0, abs(rl.item()))
    assert rel(out, ro) < 2e-2
    agree = (pred == rp).float().mean().item()
    assert agree > 0.9
    if train:
        loss.backward()
        rl.backward()
        assert rel(xf.grad, xr.grad) < 2e-2
    return xf, xr


@pytest.mark.parametrize("B", [32, 7, 50, 65, 300, 2048, 5000])
def test_ica_head_train_matches_modules(B):
    torch.manual_seed(0)
    head = _ica_head(p=0.0).to(DEV).train()
    ref_head = copy.deepcopy(head)
    x = torch.randn(B, 384, device=DEV)
    y = torch.randint(0, 2, (B,), device=DEV)
    _compare(list(head), list(ref_head), None, x, y, log_out=False)
    for (n, p), (_, q) in zip(head.named_parameters(), ref_head.named_parameters()):
        if n == "1.bias":  # feeds a batch-statistics BatchNorm: true gradient is ~0
            assert p.grad.abs().max() < 1e-5
            continue
        assert rel(p.grad, q.grad) < 2e-2, n
    bn, rbn = head[2], ref_head[2]
    assert torch.allclose(bn.running_mean, rbn.running_mean, atol=2e-3, rtol=2e-2)
    assert torch.allclose(bn.running_var, rbn.running_var, atol=2e-3, rtol=2e-2)
    assert int(bn.num_batches_tracked) == int(rbn.num_batches_tracked) == 1


@pytest.mark.parametrize("B", [20, 500])
def test_ica_head_eval_uses_running_stats(B):
    torch.manual_seed(1)
    head = _ica_head().to(DEV)
    head[2].running_mean.uniform_(-0.5, 0.5)
    head[2].running_var.uniform_(0.5, 2.0)
    head.eval()
    ref_head = copy.deepcopy(head)
    x = torch.randn(B, 384, device=DEV)
    y = torch.randint(0, 2, (B,), device=DEV)
    with torch.no_grad():
        _compare(list(head), list(ref_head), None, x, y, log_out=False, train=False, emulate=False)


@pytest.mark.parametrize("B", [32, 256])
def test_ica_head_dropout_statistics_and_fresh_masks(B):
    from dinunet_implementations_amd.ops.head import HeadSpec, head_loss
    torch.manual_seed(2)
    head = _ica_head(p=0.25).to(DEV).train()
    spec = HeadSpec(list(head))
    x = torch.randn(B, 384, device=DEV).abs() + 0.1
    y = torch.randint(0, 2, (B,), device=DEV)
    masks = []
    for _ in range(2):
        xf = x.clone().requires_grad_()
        _, loss, _ = head_loss(xf, spec, y, log_out=False)
        loss.backward()
        masks.append(xf.grad != 0)
    for m in masks:
        frac = 1.0 - m.float().mean().item()
        assert 0.2 < frac < 0.3, frac
    assert not torch.equal(masks[0], masks[1])


@pytest.mark.parametrize("B,dropout_in", [(16, ()), (45, ()), (16, (1,)), (130, ()), (1000, ()),
                                         (130, (1,))])
def test_fs_network_fused_matches_modules(B, dropout_in):
    torch.manual_seed(3)
    net = _fs_head(dropout_in=dropout_in).to(DEV).train()
    ref_net = copy.deepcopy(net)
    x = torch.rand(B, 66, device=DEV)
    y = torch.randint(0, 2, (B,), device=DEV)
    out, loss, pred = net.forward_loss(x, y)
    from dinunet_implementations_amd.ops import reference as ref
    ro, rl, rp = ref.log_softmax_nll(_emulated([m for blk in ref_net.layers for m in blk]
                                               + [ref_net.fc_out], x), y)
    if dropout_in:
        assert torch.isfinite(loss) and out.shape == ro.shape
        loss.backward()
        assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in net.parameters())
        return
    assert abs(loss.item() - rl.item()) < 2e-2 * max(1.0, abs(rl.item()))
    assert rel(out, ro) < 2e-2
    loss.backward()
    rl.backward()
    # The kernel reproduces the emulated rounding exactly in most draws; a 1-ulp bf16 activation
    # difference (fp32 summation order) is amplified by the 4 batch-statistics BatchNorm
    # backwards by a few percent in some draws (see test_fs_backward_exact_given_forward_state).
    errs = sorted(rel(p.grad, q.grad) for p, q in zip(net.parameters(), ref_net.parameters()))
    assert errs[len(errs) // 2] < 6e-2 and errs[-1] < 0.1, errs


@pytest.mark.parametrize("B", [32, 300])
def test_head_grads_accumulate_and_scale(B):
    """Gradients add into existing .grad and scale with d loss (loss * 3)."""
    from dinunet_implementations_amd.ops.head import HeadSpec, head_loss
    torch.manual_seed(4)
    head = _ica_head(p=0.0).to(DEV).train()
    spec = HeadSpec(list(head))
    x = torch.randn(B, 384, device=DEV)
    y = torch.randint(0, 2, (B,), device=DEV)
    _, loss, _ = head_loss(x, spec, y, log_out=False)
    loss.backward()
    g1 = [p.grad.clone() for p in head.parameters()]
    _, loss, _ = head_loss(x, spec, y, log_out=False)
    (3.0 * loss).backward()
    for (n, p), g in zip(head.named_parameters(), g1):
        if n != "1.bias":
            assert rel(p.grad, 4.0 * g) < 1e-2, n  # 3*dZ rounds to bf16 differently


def test_ica_model_forward_loss_fused_vs_cpu():
    from dinunet_implementations_amd.models import ICALstm
    torch.manual_seed(5)
    m = ICALstm(input_size=64, hidden_size=96, num_comps=20, window_size=5, num_cls=2)
    mc = copy.deepcopy(m)
    m = m.to(DEV).eval()
    mc.eval()
    x = torch.randn(24, 11, 20, 5)
    y = torch.randint(0, 2, (24,))
    with torch.no_grad():
        out, loss, pred = m.forward_loss(x.to(DEV), y.to(DEV))
        ro, rl, rp = mc.forward_loss(x, y)
    assert rel(out.cpu(), ro) < 3e-2
    assert abs(loss.item() - rl.item()) < 3e-2


@pytest.mark.parametrize("B", [16, 45, 200])
def test_fs_backward_exact_given_forward_state(B):
    """Each backward layer (dA = dZ W, ReLU mask, batch-statistics BatchNorm backward) reproduces
    the fp32 math applied to the kernel's own saved forward state."""
    from dinunet_implementations_amd.ops import _lib
    from dinunet_implementations_amd.ops.head import HeadSpec
    torch.manual_seed(3)
    net = _fs_head().to(DEV).train()
    spec = HeadSpec([m for blk in net.layers for m in blk] + [net.fc_out])
    x = torch.rand(B, 66, device=DEV)
    y = torch.randint(0, 2, (B,), device=DEV)
    lay = spec.layout(B)
    ws = torch.zeros(lay[0], dtype=torch.uint8, device=DEV)
    out = torch.empty(B, 2, device=DEV)
    loss = torch.empty((), device=DEV)
    pred = torch.empty(B, dtype=torch.long, device=DEV)
    _lib.call("dn_head_fwd", spec.nl, spec._dims, spec._flags, spec._drops, spec._bnp,
              spec.ptrs(False), x.data_ptr(), x.stride(0), B, y.data_ptr(), out.data_ptr(),
              loss.data_ptr(), pred.data_ptr(), spec.rng(x.device).data_ptr(), ws.data_ptr(), 1, 1,
              _lib.stream())
    one = torch.ones((), device=DEV)
    dx = torch.empty_like(x)
    _lib.call("dn_head_bwd", spec.nl, spec._dims, spec._flags, spec._drops, spec._bnp,
              spec.ptrs(True), B, ws.data_ptr(), one.data_ptr(), dx.data_ptr(), 66, _lib.stream())
    Mp = 32 if B <= 32 else (64 if B <= 64 else B)  # image rows (big batches: exactly B)

    def img(off, S, n):
        return ws[off: off + 2 * Mp * S].view(torch.bfloat16).view(Mp, S)[:B, :n].float()

    for l in range(spec.nl - 1, 0, -1):
        L, P = spec.layers[l], spec.layers[l - 1]
        a_off, S_a, dz_off, S_z = lay[1 + 4 * l: 5 + 4 * l]
        pa_off, pS_a, pdz_off, pS_z = lay[1 + 4 * (l - 1): 5 + 4 * (l - 1)]
        d = img(dz_off, S_z, L.linear.out_features) @ L.linear.weight.detach().to(torch.bfloat16).float()
        d = d * (img(a_off, S_a, L.linear.in_features) > 0).float()
        z = img(pa_off, pS_a, P.linear.in_features) @ P.linear.weight.detach().to(torch.bfloat16).float().t()
        mu, var = z.mean(0), z.var(0, unbiased=False)
        rstd = (var + P.bn.eps).rsqrt()
        xh = (z - mu) * rstd
        dz = P.bn.weight.detach() * rstd * (d - d.mean(0) - xh * (d * xh).mean(0))
        kd = img(pdz_off, pS_z, P.linear.out_features)
        assert rel(kd, dz.to(torch.bfloat16).float()) < 1e-3, l


@pytest.mark.parametrize("one_launch", [True, False])
def test_fused_forward_backward_chain_matches_two_phase(one_launch, monkeypatch):
    """With a d(loss) hint the forward runs the backward too: either the WHOLE head step in one
    launch (csrc/kernels/head_rep.hip on the head's own bf16 weight images, cast right before:
    no Adam-emitted pack here) or the output-gradient chain with dW / dX left to the backward
    launch.  Both are bitwise the unfused three-phase result (same reduction orders, same bf16
    rounding points)."""
    from dinunet_implementations_amd.ops import head as H
    monkeypatch.setattr(H, "_HEAD_STEP", one_launch)
    torch.manual_seed(0)
    mods = _ica_head(p=0.0).to(DEV).train()
    ref_mods = copy.deepcopy(mods)
    x = torch.randn(32, 384, device=DEV)
    y = torch.randint(0, 2, (32,), device=DEV)
    one = torch.ones((), device=DEV)
    res = []
    for fused, m in ((True, mods), (False, ref_mods)):
        xi = x.clone().requires_grad_()
        spec = H.HeadSpec(list(m))
        with H.loss_grad_hint(one if fused else None):
            out, loss, _ = H.head_loss(xi, spec, y, log_out=False)
        torch.autograd.backward(loss, one)
        torch.cuda.synchronize()
        res.append((out.clone(), xi.grad.clone(), [p.grad.clone() for p in m.parameters()],
                    [b.clone() for b in m.buffers()]))
    (o1, dx1, g1, b1), (o2, dx2, g2, b2) = res
    assert torch.equal(o1, o2) and torch.equal(dx1, dx2)
    for a, b in zip(g1, g2):
        assert torch.equal(a, b)
    for a, b in zip(b1, b2):
        assert torch.equal(a, b)


def test_hinted_backward_with_other_dloss():
    """The two-phase fused path stays exact for a backward with another d loss tensor; the
    one-launch step (which already accumulated the gradients) refuses it loudly."""
    from dinunet_implementations_amd.ops import head as H
    torch.manual_seed(0)
    mods = _ica_head(p=0.0).to(DEV).train()
    x = torch.randn(32, 384, device=DEV, requires_grad=True)
    y = torch.randint(0, 2, (32,), device=DEV)
    one = torch.ones((), device=DEV)
    spec = H.HeadSpec(list(mods))
    with H.loss_grad_hint(one):
        _, loss, _ = H.head_loss(x, spec, y, log_out=False)
    with pytest.raises(RuntimeError, match="loss_grad_hint"):
        torch.autograd.backward(loss, torch.full((), 2.5, device=DEV))


class _Imgs:
    """bf16 weight images of a head's Linear layers in the role of the fused Adam's persistent
    operand pack (ops.lstm.PersistentPack.bf16_of), for the replicated head kernel."""

    def __init__(self, mods):
        self.m = {id(mm.weight): mm.weight.detach().to(torch.bfloat16).contiguous()
                  for mm in mods if isinstance(mm, nn.Linear)}
        self.used = False

    def bf16_of(self, t):
        return self.m.get(id(t))


def _step_vs_classic(mods, x, y, log_out, reps=1, rep=False):
    """Run the head with the one-launch step (head_rep.hip; ``rep``: on weight images handed in
    like the fused Adam's persistent pack, else on the head's own images cast right before the
    launch) and the three-launch path from identical state; return both results (outputs, dx,
    grads, buffers)."""
    from dinunet_implementations_amd.ops import head as H
    ref_mods = [copy.deepcopy(m) for m in mods]
    one = torch.ones((), device=DEV)
    res = []
    seed0 = None
    for flag, ms in ((True, mods), (False, ref_mods)):
        old = H._HEAD_STEP
        H._HEAD_STEP = flag
        try:
            spec = H.HeadSpec(ms)
            r = spec.rng(x.device)  # both paths draw the same dropout masks
            if seed0 is None:
                seed0 = r.clone()
            else:
                r.copy_(seed0)
            from dinunet_implementations_amd.ops.lstm import use_persistent
            imgs = _Imgs(ms) if (rep and flag) else None
            for _ in range(reps):
                xi = x.clone().requires_grad_()
                with H.loss_grad_hint(one), use_persistent(imgs):
                    out, loss, pred = H.head_loss(xi, spec, y, log_out=log_out)
                torch.autograd.backward(loss, one)
            torch.cuda.synchronize()
            params = [p for m in ms for p in m.parameters()]
            bufs = [b for m in ms for b in m.buffers()]
            res.append((out.clone(), loss.clone(), pred.clone(), xi.grad.clone(),
                        [p.grad.clone() for p in params], [b.clone() for b in bufs], spec))
        finally:
            H._HEAD_STEP = old
    return res


@pytest.mark.parametrize("B,p", [(32, 0.0), (17, 0.0), (32, 0.25), (2, 0.0)])
def test_head_one_launch_own_images_ica_bitwise(B, p):
    """Steps without the Adam-emitted pack (host-fed, eager): the replicated head on its own
    bf16 images (one cast launch of the fp32 weights right before) equals the three-launch path
    bitwise -- the form round 5's hand-off head (head_step.hip, deleted) served."""
    from dinunet_implementations_amd.ops import head as H
    torch.manual_seed(11)
    mods = list(_ica_head(p=p).to(DEV).train())
    x = torch.randn(B, 384, device=DEV)
    y = torch.randint(0, 2, (B,), device=DEV)
    n0 = H.REP_LAUNCHES
    a, b = _step_vs_classic(mods, x, y, log_out=False, reps=3)
    assert H.REP_LAUNCHES == n0 + 3, "the replicated head did not run"
    for u, v in zip(a[:4], b[:4]):
        assert torch.equal(u, v)
    for u, v in zip(a[4], b[4]):
        assert torch.equal(u, v)
    for u, v in zip(a[5], b[5]):  # running stats: FMA contraction may differ by an ulp
        assert torch.allclose(u.double(), v.double(), rtol=1e-6, atol=0)


@pytest.mark.parametrize("B,dropout_in", [(16, ()), (32, ()), (9, (1,))])
def test_head_one_launch_fs_outside_envelope_bitwise(B, dropout_in):
    """The FS MSANNet (66 input features: not a multiple of the replicated head's 16-B rows) is
    outside the one-launch envelope: asking for it runs the three-launch path, bitwise the same."""
    from dinunet_implementations_amd.ops import head as H
    torch.manual_seed(12)
    net = _fs_head(dropout_in=dropout_in).to(DEV).train()
    mods = [m for blk in net.layers for m in blk] + [net.fc_out]
    x = torch.rand(B, 66, device=DEV)
    y = torch.randint(0, 2, (B,), device=DEV)
    n0 = H.REP_LAUNCHES
    a, b = _step_vs_classic(mods, x, y, log_out=True, reps=2)
    assert H.REP_LAUNCHES == n0
    for u, v in zip(a[:4], b[:4]):
        assert torch.equal(u, v)
    for u, v in zip(a[4], b[4]):
        assert torch.equal(u, v)


@pytest.mark.parametrize("B,p", [(32, 0.0), (17, 0.0), (32, 0.25), (2, 0.0), (32, 0.5)])
def test_head_rep_one_launch_ica_bitwise(B, p):
    """The replicated-forward head (head_rep.hip: every workgroup runs the whole forward and
    output-gradient chain, no hand-off) on pack-provided images equals the three-launch path
    bitwise: outputs, loss, argmax, d input, every parameter gradient; running statistics to an
    ulp."""
    from dinunet_implementations_amd.ops import head as H
    torch.manual_seed(11)
    mods = list(_ica_head(p=p).to(DEV).train())
    spec = H.HeadSpec(mods)
    assert int(_lib_call_rep_supported(spec, B)) == 1
    x = torch.randn(B, 384, device=DEV)
    y = torch.randint(0, 2, (B,), device=DEV)
    n0 = H.REP_LAUNCHES
    a, b = _step_vs_classic(mods, x, y, log_out=False, reps=3, rep=True)
    assert H.REP_LAUNCHES == n0 + 3, "the replicated head did not run"
    for u, v in zip(a[:4], b[:4]):
        assert torch.equal(u, v)
    for u, v in zip(a[4], b[4]):
        assert torch.equal(u, v)
    for u, v in zip(a[5], b[5]):
        assert torch.allclose(u.double(), v.double(), rtol=1e-6, atol=0)


def _lib_call_rep_supported(spec, B):
    from dinunet_implementations_amd.ops import _lib
    return _lib.lib().dn_head_rep_supported(spec.nl, spec._dims, spec._flags, B)


def test_head_rep_graph_replay_fresh_masks():
    """The replicated head captured in a HIP graph: every replay draws a fresh dropout seed (the
    last workgroup advances it once per launch, after all read it) and a replay equals the eager
    launch from the same state."""
    from dinunet_implementations_amd.ops import head as H
    torch.manual_seed(14)
    mods = list(_ica_head(p=0.25).to(DEV).train())
    spec = H.HeadSpec(mods)
    x = torch.randn(32, 384, device=DEV, requires_grad=True)
    y = torch.randint(0, 2, (32,), device=DEV)
    one = torch.ones((), device=DEV)

    from dinunet_implementations_amd.ops.lstm import use_persistent
    imgs = _Imgs(mods)

    def run():
        with H.loss_grad_hint(one), use_persistent(imgs):
            _, loss, _ = H.head_loss(x, spec, y, log_out=False)
        torch.autograd.backward(loss, one)
        return loss

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    n0 = H.REP_LAUNCHES
    with torch.cuda.stream(s):
        for _ in range(3):
            run()
    torch.cuda.current_stream().wait_stream(s)
    assert H.REP_LAUNCHES == n0 + 3
    seed0 = int(spec.rng(x.device).item())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        sl = run()
    losses = []
    for i in range(50):
        g.replay()
        losses.append(float(sl))
    torch.cuda.synchronize()
    assert int(spec.rng(x.device).item()) == seed0 + 50
    assert int(spec.sync(x.device)[192].item()) == 0  # the done counter resets every launch
    assert len(set(losses)) > 10  # fresh masks: the loss moves with every draw
    assert torch.isfinite(x.grad).all()


def test_head_own_images_graph_replay_and_epochs():
    """Own-image head captured in a HIP graph (the weight cast and the replicated head both in
    the graph) and replayed 200 times with eager launches in between: the done counter resets
    every launch, the dropout seed advances once per launch, and the weights each replay reads
    are the CURRENT ones (a changed weight changes the replayed loss)."""
    from dinunet_implementations_amd.ops import head as H
    torch.manual_seed(13)
    mods = list(_ica_head(p=0.0).to(DEV).train())
    spec = H.HeadSpec(mods)
    x = torch.randn(32, 384, device=DEV, requires_grad=True)
    y = torch.randint(0, 2, (32,), device=DEV)
    one = torch.ones((), device=DEV)

    def run():
        with H.loss_grad_hint(one):
            _, loss, _ = H.head_loss(x, spec, y, log_out=False)
        torch.autograd.backward(loss, one)
        return loss

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    n0 = H.REP_LAUNCHES
    with torch.cuda.stream(s):
        for _ in range(3):
            run()
    torch.cuda.current_stream().wait_stream(s)
    assert H.REP_LAUNCHES == n0 + 3
    seed0 = int(spec.rng(x.device).item())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        sl = run()
    for i in range(200):
        g.replay()
        if i % 50 == 0:
            run()
    torch.cuda.synchronize()
    assert int(spec.rng(x.device).item()) == seed0 + 200 + 4
    assert int(spec.sync(x.device)[192].item()) == 0
    assert torch.isfinite(sl).all() and torch.isfinite(x.grad).all()
    before = float(sl)
    with torch.no_grad():
        spec.layers[-1].linear.weight.mul_(3.0)
    g.replay()
    torch.cuda.synchronize()
    assert float(sl) != before, "the replay read stale weight images"
