"""Direct site-mean exchange (parallel/collective.py) across gloo processes on CPU.

``precision_bits=16`` ships IEEE half like the reference (compspec.json:161-176) and accumulates
in fp32: the mean of W sites is exactly the fp32 mean of their fp16-rounded values, rounded once.
The negative control shows what the 16-bit all-reduce it replaces does with the same input.
"""
import torch
import torch.nn as nn

from mp_util import run_world
from test_engines import _model, _data, w_grads


def _vals(rank, n):
    g = torch.Generator().manual_seed(7 + rank)
    return torch.randn(n, generator=g) * (1 + rank)


def w_direct(grp, payload, n, big):
    from dinunet_implementations_amd.parallel.collective import DirectMean
    x = torch.full((n,), 40000.0) if big else _vals(grp.rank, n)
    dm = DirectMean(grp, n, payload, "cpu")
    y = x.clone()
    sent = dm.run_(y)
    return x, y, sent, dm.chunk


def w_allreduce16(grp, n):
    x = torch.full((n,), 40000.0, dtype=torch.float16)
    grp.all_reduce(x)
    return x


def _q(x, dt, e):
    return (x * 2.0 ** e).to(dt).float() * 2.0 ** -e


def _expect(xs, payload):
    """fp32 mean of the sites' payload-rounded values, rounded once; fp16 values are scaled by
    the site's power of two (max|x| * 2^e < 2^15), the mean by the smallest site exponent."""
    import math
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}[payload]
    es = [15 - math.frexp(float(x.abs().max()))[1] if payload == "fp16" else 0 for x in xs]
    acc = torch.zeros_like(xs[0], dtype=torch.float32)
    for x, e in zip(xs, es):
        acc += _q(x, dt, e)
    return _q(acc * (1.0 / len(xs)), dt, min(es))  # the kernels scale by fp32(1/W)


def test_direct_mean_fp32_accumulation_all_payloads():
    for payload in ("fp16", "bf16", "fp32"):
        for world, n in ((2, 64), (3, 37)):   # 37: padded chunk, scalar tail
            outs = run_world(w_direct, world, payload, n, False)
            xs = [o[0] for o in outs]
            want = _expect(xs, payload)
            for _, y, sent, chunk in outs:
                assert torch.equal(y, want), (payload, world, n)
                assert sent == n * {"fp16": 2, "bf16": 2, "fp32": 4}[payload]
                assert chunk % 8 == 0 and chunk * world >= n


def w_tiny(grp):
    from dinunet_implementations_amd.parallel.collective import DirectMean
    x = _vals(grp.rank, 64) * 1e-7  # fp16 subnormal / zero territory without a block scale
    y = x.clone()
    DirectMean(grp, 64, "fp16", "cpu").run_(y)
    return x, y


def test_fp16_block_scale_keeps_tiny_gradients():
    outs = run_world(w_tiny, 2)
    a, b = outs[0][0], outs[1][0]
    mean, mag = (a + b) / 2, (a.abs() + b.abs()) / 2  # error relative to the summands
    err = ((outs[0][1] - mean).abs() / mag).max()
    assert err < 2 ** -10, err
    naive = ((a.half().float() + b.half().float()) / 2 - mean).abs() / mag
    assert naive.max() > 1e-2  # what unscaled fp16 does to them


def test_direct_mean_no_16bit_overflow_negative_control():
    """3 sites x 40000: the fp16 SUM (120000) overflows half, the mean (40000) does not."""
    outs = run_world(w_direct, 3, "fp16", 16, True)
    for _, y, _, _ in outs:
        assert torch.equal(y, torch.full((16,), 40000.0))
    ctrl = run_world(w_allreduce16, 3, 16)
    assert torch.isinf(ctrl[0].float()).all()  # a 16-bit all-reduce overflows


def test_dsgd_precision16_is_fp16_direct_mean():
    ref = run_world(w_grads, 3, "dSGD", {})[0]
    h = run_world(w_grads, 3, "dSGD", {"precision_bits": "16"})
    assert torch.equal(h[0], h[1]) and torch.equal(h[0], h[2])
    # fp16: 11 significant bits, two roundings
    assert torch.allclose(h[0], ref, atol=1e-5, rtol=2e-3)
    b = run_world(w_grads, 3, "dSGD", {"precision_bits": "16", "payload_dtype": "bf16"})[0]
    eb, eh = (b - ref).abs().max(), (h[0] - ref).abs().max()
    assert eh < eb  # fp16 carries 3 more mantissa bits than bf16 on gradients of this range
    d = run_world(w_grads, 2, "dSGD", {"dsgd_collective": "direct"})[0]
    a = run_world(w_grads, 2, "dSGD", {"dsgd_collective": "allreduce"})[0]
    assert torch.allclose(d, a, atol=1e-7)


def test_rankdad_and_powersgd_honour_precision_bits():
    for name, cfg in (("rankDAD", {"dad_reduction_rank": 4, "dad_num_pow_iters": 10, "dad_tol": 0.0}),
                      ("powerSGD", {"powersgd_rank": 2})):
        full = run_world(w_grads, 2, name, cfg)[0]
        half = run_world(w_grads, 2, name, {**cfg, "precision_bits": "16"})
        assert torch.equal(half[0], half[1]), name
        assert torch.allclose(half[0], full, atol=1e-4, rtol=1e-2), name
        assert not torch.equal(half[0], full), name  # the 16-bit wire was really used


def test_payload_config_validation():
    import pytest
    from dinunet_implementations_amd.parallel.collective import payload_name
    assert payload_name({}) == "fp32"
    assert payload_name({"precision_bits": "16"}) == "fp16"
    assert payload_name({"precision_bits": 16, "payload_dtype": "BF16"}) == "bf16"
    with pytest.raises(ValueError):
        payload_name({"payload_dtype": "fp8"})


def w_engine_wire(grp, cfg):
    import warnings
    import torch.nn as nn
    from dinunet_implementations_amd.ops import FlatParams
    from dinunet_implementations_amd.parallel import make_engine
    m = nn.Linear(4, 4)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        e = make_engine("dSGD", m, FlatParams(m.parameters()), grp, cfg)
    return e.wire, e.direct, [str(x.message) for x in w]


def test_fp16_wire_never_summed_by_a_16bit_allreduce():
    """RCCL sums an all-reduce buffer in its own type, so the fp16 wire (whose block
    scale is per site) cannot ride a 16-bit all-reduce: that combination ships bf16 and warns;
    the direct exchange keeps fp16 (fp32 sum)."""
    wire, direct, warns = run_world(w_engine_wire, 2, {"precision_bits": "16",
                                                       "dsgd_collective": "allreduce"})[0]
    assert wire == "bf16" and not direct and any("bf16" in m for m in warns)
    wire, direct, warns = run_world(w_engine_wire, 2, {"precision_bits": "16"})[0]
    assert wire == "fp16" and direct and not warns


def w_calibrate(grp, cfg):
    import torch.nn as nn
    from dinunet_implementations_amd.ops import FlatParams
    from dinunet_implementations_amd.parallel import make_engine
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(64, 64), nn.Linear(64, 8))
    flat = FlatParams(m.parameters())
    e = make_engine("dSGD", m, flat, grp, cfg)
    # the chosen form still computes the site mean
    flat.grad.fill_(float(grp.rank + 1))
    e.reduce()
    return e.calibration, e.direct, flat.grad.clone() * e.last_scale


def test_dsgd_collective_calibrate_agrees_across_sites():
    """dsgd_collective='calibrate': the candidate forms timed as the step runs them, timings
    max-reduced so every site takes the same choice; the record says which and why; the mean is
    right.  On CPU sites the peer exchange (GPU memory) is not a candidate: the host-issued
    all-reduce is the only form timed."""
    outs = run_world(w_calibrate, 2, {"dsgd_collective": "calibrate", "dsgd_calibrate_reps": 3})
    (c0, d0, g0), (c1, d1, g1) = outs
    assert c0 == c1 and d0 == d1
    assert c0["choice"] == "allreduce" and not d0
    assert c0["allreduce_us"] > 0 and c0["allreduce_form"] == "host-issued"
    assert c0["peer_us"] is None and c0["peer_form"] == "unavailable"
    assert torch.allclose(g0, torch.full_like(g0, 1.5)) and torch.equal(g0, g1)
    # a 16-bit wire has one admissible form (the fp32-sum exchange: direct off the GPU)
    c16, d16, g16 = run_world(w_calibrate, 2, {"dsgd_collective": "calibrate",
                                               "precision_bits": "16"})[0]
    assert c16["choice"] == "direct" and d16 and "16-bit" in c16["reason"]
    assert torch.allclose(g16, torch.full_like(g16, 1.5))
