"""Fused LayerNorm kernels (csrc/kernels/layernorm.hip) against torch's fp32 layer_norm."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    return (a - b).norm().item() / max(b.norm().item(), 1e-12)


@pytest.mark.parametrize("R,D", [(32, 256), (1000, 384), (7, 2048), (5, 12), (3000, 64)])
@pytest.mark.parametrize("affine", [True, False])
def test_layernorm_matches_torch(R, D, affine):
    from dinunet_implementations_amd.ops import layernorm as L
    torch.manual_seed(R + D)
    x = (torch.randn(R, D, device="cuda") * 3 + 1).requires_grad_()
    w = (torch.randn(D, device="cuda")).requires_grad_() if affine else None
    b = (torch.randn(D, device="cuda")).requires_grad_() if affine else None
    y = L.layer_norm(x, w, b, 1e-5)
    assert L.fused_ok(x, D)
    xr = x.detach().clone().requires_grad_()
    wr = w.detach().clone().requires_grad_() if affine else None
    br = b.detach().clone().requires_grad_() if affine else None
    yr = torch.nn.functional.layer_norm(xr, (D,), wr, br, 1e-5)
    assert rel(y, yr) < 1e-5
    g = torch.randn_like(yr)
    (y * g).sum().backward()
    (yr * g).sum().backward()
    assert rel(x.grad, xr.grad) < 1e-4
    if affine:
        assert rel(w.grad, wr.grad) < 1e-4 and rel(b.grad, br.grad) < 1e-4


def test_layernorm_backward_deterministic():
    from dinunet_implementations_amd.ops import LayerNorm
    m = LayerNorm(256).cuda()
    x = torch.randn(5000, 256, device="cuda")
    grads = []
    for _ in range(2):
        m.zero_grad()
        m(x).square().sum().backward()
        grads.append((m.weight.grad.clone(), m.bias.grad.clone()))
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])


def test_ica_model_with_layernorm_trains_on_gpu():
    """norm_layer="layer": the head runs module by module (the fused head kernels fuse BatchNorm)
    with the LayerNorm kernels; a few Adam steps lower the loss on a fixed batch."""
    from dinunet_implementations_amd.models import ICALstm
    torch.manual_seed(0)
    m = ICALstm(input_size=64, hidden_size=384, num_comps=20, window_size=10,
                norm_layer="layer").cuda().train()
    x = torch.randn(32, 12, 20, 10, device="cuda")
    y = torch.randint(0, 2, (32,), device="cuda")
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    losses = []
    for _ in range(6):
        opt.zero_grad()
        _, loss, _ = m.forward_loss(x, y)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0], losses
