"""Diagnostic: in-launch split-K combine vs the reduce kernel, error pattern by row / column."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from dinunet_implementations_amd.ops import gemm as G  # noqa: E402

torch.manual_seed(0)
for M, N, K, sp, dt in [(64, 64, 256, 2, torch.float32), (64, 64, 256, 2, torch.bfloat16),
                        (128, 64, 512, 4, torch.float32), (1536, 256, 3136, 6, torch.float32)]:
    a = torch.randn(M, K, device="cuda").to(dt)
    b = torch.randn(N, K, device="cuda").to(dt)
    ref = a.float().to(torch.bfloat16).float() @ b.float().to(torch.bfloat16).float().t()
    for inl in (True, False):
        G._SPLITK_INLAUNCH = inl
        out = G.mm(a, b, trans_b=True, splits=sp)
        torch.cuda.synchronize()
        bad = (out - ref).abs() > 1e-2 * ref.abs().max()
        rows = bad.any(1).nonzero().flatten().tolist()
        cols = bad.any(0).nonzero().flatten().tolist()
        t = G._TICKETS.get(a.device)
        print(f"M{M} N{N} K{K} sp{sp} {str(dt)[6:]} inlaunch={inl}: bad {int(bad.sum())} rows {rows[:12]} cols {cols[:12]} "
              f"tickets {None if t is None else int(t.abs().sum())}", flush=True)
        if inl and bad.any():
            r0 = rows[0]
            print("   out", out[r0, :6].tolist(), "\n   ref", ref[r0, :6].tolist())
