"""Model parity with the reference (keys, sizes, math oracle) and mergeable metrics (CPU)."""
import numpy as np
import torch

from dinunet_implementations_amd.models import ICALstm, MSANNet
from dinunet_implementations_amd.ops import FlatParams, FusedAdam, reference as ref
from dinunet_implementations_amd.utils.metrics import Averages, Metrics, merge_states, roc_auc


def test_fs_state_dict_and_params():
    m = MSANNet(66, [256, 128, 64, 32], 2)
    assert sum(p.numel() for p in m.parameters()) == 60930
    keys = set(m.state_dict())
    assert {"layers.0.0.weight", "layers.0.1.weight", "layers.0.1.bias", "fc_out.weight",
            "fc_out.bias"} <= keys
    assert not any("running" in k for k in keys)  # track_running_stats=False (A5)
    assert m.layers[0][0].bias is None  # bias=False (A7)


def test_ica_state_dict_and_params():
    m = ICALstm(input_size=256, hidden_size=384, num_comps=100, window_size=10)
    assert sum(p.numel() for p in m.parameters()) == 1063106
    m2 = ICALstm(input_size=256, hidden_size=348, num_comps=100, window_size=10)
    assert sum(p.numel() for p in m2.parameters()) == 964034
    keys = set(m.state_dict())
    assert {"encoder.0.weight", "lstm.lstms.0.i2h.weight", "lstm.lstms.1.h2h.bias",
            "classifier.2.running_mean", "classifier.2.num_batches_tracked",
            "classifier.6.weight"} <= keys


def _manual_cell(x, w_ih, b_ih, w_hh, b_hh):
    """Independent step-by-step restatement of comps/icalstm/models.py:30-41."""
    B, S, _ = x.shape
    H = w_hh.shape[1]
    h = torch.zeros(B, H, dtype=x.dtype)
    c = torch.zeros(B, H, dtype=x.dtype)
    outs = []
    for t in range(S):
        pre = x[:, t] @ w_ih.t() + b_ih + h @ w_hh.t() + b_hh
        sg = torch.sigmoid(pre[:, :3 * H])
        i, f, o = torch.sigmoid(sg[:, :H]), torch.sigmoid(sg[:, H:2 * H]), torch.sigmoid(sg[:, -H:])
        g = torch.tanh(pre[:, 3 * H:])
        c = f * c + i * g
        h = o * torch.tanh(c)
        outs.append(h)
    return torch.stack(outs, 1), h, c


def test_lstm_oracle_double_sigmoid_and_reverse_order():
    torch.manual_seed(0)
    m = ICALstm(input_size=8, hidden_size=12, num_comps=3, window_size=2)
    x = torch.randn(3, 5, 8, dtype=torch.float64)
    lstm = m.lstm.double()
    hs, (h, c) = lstm(x)
    p0 = lstm.lstms[0].params()
    p1 = lstm.lstms[1].params()
    f_hs, fh, fc = _manual_cell(x, *p0)
    r_hs, rh, rc = _manual_cell(torch.flip(x, (1,)), *p1)
    assert torch.allclose(hs, torch.cat([f_hs, r_hs], 2))  # reverse stays in processing order
    assert torch.allclose(h, torch.cat([fh, rh], 1)) and torch.allclose(c, torch.cat([fc, rc], 1))
    mean, _ = lstm(x, reduce="mean")
    assert torch.allclose(mean, hs.mean(1))


def test_ica_forward_matches_per_sample_encoder_loop():
    torch.manual_seed(1)
    m = ICALstm(input_size=16, hidden_size=8, num_comps=4, window_size=3).eval()
    x = torch.randn(5, 6, 4, 3)
    out, _ = m(x)
    enc = torch.stack([m.encoder(b.view(b.shape[0], -1)) for b in x])  # models.py:107
    o, _ = m.lstm(enc)
    assert torch.allclose(out, m.classifier(o.mean(1)), atol=1e-6)


def test_flat_params_and_adam_cpu_match_torch():
    torch.manual_seed(2)
    a = MSANNet(66, [32, 16], 2)
    b = MSANNet(66, [32, 16], 2)
    b.load_state_dict(a.state_dict())
    flat = FlatParams(a.parameters())
    opt = FusedAdam(flat, lr=1e-2)
    ropt = torch.optim.Adam(b.parameters(), lr=1e-2)
    for _ in range(4):
        x = torch.randn(16, 66)
        y = torch.randint(0, 2, (16,))
        opt.zero_grad()
        ref.log_softmax_nll(a(x), y)[1].backward()
        opt.step()
        ropt.zero_grad()
        ref.log_softmax_nll(b(x), y)[1].backward()
        ropt.step()
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.allclose(p, q, atol=1e-6)
    # params are views into the flat buffer
    assert all(p.data.data_ptr() >= flat.data.data_ptr() for p in a.parameters())


def test_auc_matches_sklearn_and_merges():
    from sklearn.metrics import roc_auc_score
    rng = np.random.default_rng(0)
    s = rng.random(300)
    y = (rng.random(300) < 0.4).astype(int)
    s[::7] = 0.5  # ties
    assert abs(roc_auc(s, y) - roc_auc_score(y, s)) < 1e-12
    m1 = Metrics().add(torch.tensor(s[:100]), torch.tensor(y[:100]))
    m2 = Metrics().add(torch.tensor(s[100:]), torch.tensor(y[100:]))
    merged = merge_states([m1.to_state(), m2.to_state()])
    assert abs(merged.auc - roc_auc_score(y, s)) < 1e-9


def test_hard_label_metrics():
    pred = torch.tensor([1, 0, 1, 1, 0, 0])
    lab = torch.tensor([1, 0, 0, 1, 1, 0])
    sc = Metrics().add(pred, lab).scores()
    assert abs(sc["accuracy"] - 4 / 6) < 1e-9
    assert abs(sc["f1"] - 2 * (2 / 3) * (2 / 3) / (4 / 3)) < 1e-9


def test_averages():
    a = Averages().add(1.0, 2).add(torch.tensor(4.0), 2)
    assert a.average == 2.5 and a.count == 4
    b = Averages.from_state(a.to_state())
    assert b.average == 2.5
