"""The optional LayerNorm classifier norm (config ``norm_layer``): CPU behaviour and wiring.
The fused gfx950 kernels are checked against torch on the GPU (tests/test_layernorm_gpu.py)."""
import pytest
import torch
import torch.nn as nn


def test_layernorm_module_is_nn_layernorm_on_cpu():
    from dinunet_implementations_amd.ops import LayerNorm
    torch.manual_seed(0)
    ours, ref = LayerNorm(24), nn.LayerNorm(24)
    ref.load_state_dict(ours.state_dict())
    with torch.no_grad():
        ours.weight.normal_()
        ours.bias.normal_()
    ref.load_state_dict(ours.state_dict())
    x = torch.randn(7, 24, requires_grad=True)
    xr = x.detach().clone().requires_grad_()
    ours(x).pow(2).sum().backward()
    ref(xr).pow(2).sum().backward()
    assert torch.allclose(x.grad, xr.grad)
    assert torch.allclose(ours.weight.grad, ref.weight.grad)
    assert set(ours.state_dict()) == {"weight", "bias"}


@pytest.mark.parametrize("task", ["ica", "fs"])
def test_models_take_norm_layer(task):
    from dinunet_implementations_amd.models import ICALstm, MSANNet
    from dinunet_implementations_amd.ops import LayerNorm
    torch.manual_seed(0)
    if task == "ica":
        m = ICALstm(input_size=16, hidden_size=32, num_comps=4, window_size=5, norm_layer="layer")
        x, y = torch.randn(6, 5, 4, 5), torch.randint(0, 2, (6,))
        assert isinstance(m.classifier[2], LayerNorm)
    else:
        m = MSANNet(10, [16, 8], 2, norm_layer="layer")
        x, y = torch.randn(6, 10), torch.randint(0, 2, (6,))
        assert isinstance(m.layers[0][1], LayerNorm)
    _, loss, _ = m.forward_loss(x, y)
    loss.backward()
    assert all(p.grad is not None for p in m.parameters() if p.requires_grad)
    with pytest.raises(ValueError):
        (ICALstm if task == "ica" else lambda **k: MSANNet(10, [4], 2, **k))(norm_layer="group")


def test_config_default_is_the_reference_batchnorm():
    from dinunet_implementations_amd.config import build_config
    assert build_config()["norm_layer"] == "batch"
