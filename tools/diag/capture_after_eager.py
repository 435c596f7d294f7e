#!/usr/bin/env python3
"""Capture RCCL collectives right after eager ones, many times: the
process-group watchdog must never see an event last recorded in a capturing stream
(hipErrorCapturedEvent aborts the process).  One-rank loopback RCCL group; each round issues eager
collectives, quiesces (``runtime.step._quiesce_collectives``: device sync + the watchdog's list
drained), captures a graph holding collectives, replays it and issues eager ones again at once.
Prints one JSON line; a regression shows as a core dump (run it in a subprocess)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import torch.distributed as dist
    from dinunet_implementations_amd.parallel import init_sites, shutdown
    from dinunet_implementations_amd.runtime.step import _quiesce_collectives
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    grp = init_sites(loopback=True)
    dev = grp.device
    a = torch.ones(1 << 16, device=dev)
    b = torch.ones(1 << 16, device=dev)
    t0 = time.perf_counter()
    waits = []
    for i in range(rounds):
        hs = [dist.all_reduce(a, group=grp.pg, async_op=True) for _ in range(3)]
        for h in hs:
            h.wait()
        dist.all_reduce(b, group=grp.pg)
        q0 = time.perf_counter()
        _quiesce_collectives(grp)
        waits.append(time.perf_counter() - q0)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            dist.all_reduce(b, group=grp.pg)
            b.mul_(1.0)
            dist.all_reduce(a, group=grp.pg, async_op=True).wait()
        g.replay()
        dist.all_reduce(a, group=grp.pg)  # eager again right after the replay
    torch.cuda.synchronize()
    time.sleep(0.5)  # give the watchdog a last pass over everything issued
    print(json.dumps({"ok": True, "rounds": rounds, "wall_s": round(time.perf_counter() - t0, 2),
                      "quiesce_ms_max": round(1e3 * max(waits), 1),
                      "quiesce_ms_mean": round(1e3 * sum(waits) / len(waits), 1),
                      "event_cache": os.environ.get("TORCH_NCCL_CUDA_EVENT_CACHE")}), flush=True)
    shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
