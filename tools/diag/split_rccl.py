"""Diagnostic: TrainStep (graph / split graph) with a 1-rank RCCL group taking collective paths."""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29534")
split = sys.argv[1] == "split"
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
import test_step_gpu as T
grp = T._OneRankGroup(dist.group.WORLD)
xs, ys = T._batches()
_, f2, s2 = T._trainer(0, group=grp, use_graph=True, split=split)
for i in range(xs.shape[0]):
    l = s2(xs[i], ys[i]); torch.cuda.synchronize(); print("step", i, float(l), "graph", s2.graph is not None, flush=True)
print("comm_bytes", s2.engine.comm_bytes, f2.numel * 4, flush=True)
dist.destroy_process_group()
print("destroy ok", flush=True)
