"""Diagnostic: does a 1-rank RCCL process group survive destroy, with/without HIP-graph capture?"""
import os, sys, torch, torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29533")
mode = sys.argv[1]
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
t = torch.ones(1000, device="cuda")
dist.all_reduce(t)
torch.cuda.synchronize()
print("allreduce ok", float(t[0]), flush=True)
if mode in ("graph", "graph_async"):
    x = torch.randn(64, 64, device="cuda")
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        y = x @ x
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = x @ x
    g.replay()
    if mode == "graph_async":
        h = dist.all_reduce(t, async_op=True); g.replay(); h.wait()
    torch.cuda.synchronize()
    print("graph ok", flush=True)
dist.destroy_process_group()
print("destroy ok", flush=True)
