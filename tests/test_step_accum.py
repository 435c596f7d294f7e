"""Gradient accumulation through TrainStep (``local_iterations``) equals the
reference's loop: zero, ``(loss / li).backward()`` per micro-batch, one optimizer step (CPU)."""
import torch


def test_trainstep_accumulation_equals_reference_loop():
    from dinunet_implementations_amd.models import MSANNet
    from dinunet_implementations_amd.ops import FlatParams, FusedAdam
    from dinunet_implementations_amd.parallel import make_engine
    from dinunet_implementations_amd.parallel.group import SiteGroup
    from dinunet_implementations_amd.runtime.step import TrainStep

    def make():
        torch.manual_seed(0)
        m = MSANNet(66, [32, 16], 2).train()
        flat = FlatParams(m.parameters())
        return m, flat, FusedAdam(flat, lr=1e-2)

    g = torch.Generator().manual_seed(1)
    xs = torch.rand(6, 8, 66, generator=g)
    ys = torch.randint(0, 2, (6, 8), generator=g)
    ma, fa, oa = make()
    eng = make_engine("dSGD", ma, fa, SiteGroup(), {})
    st = TrainStep(ma, fa, oa, eng, task="fs", use_graph=False, accum=3,
                   forward_loss=lambda m, x, y: m.forward_loss(x, y))
    for i in range(6):
        st(xs[i], ys[i], first=i % 3 == 0, last=i % 3 == 2)
    mb, fb, ob = make()
    for k in range(2):
        fb.zero_grad()
        for i in range(3 * k, 3 * k + 3):
            _, loss, _ = mb.forward_loss(xs[i], ys[i])
            (loss / 3).backward()
        ob.step()
    assert oa.step_count == ob.step_count == 2
    assert torch.allclose(fa.data, fb.data, rtol=1e-6, atol=1e-7)
