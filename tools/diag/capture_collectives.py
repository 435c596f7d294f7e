#!/usr/bin/env python3
"""Which RCCL collectives survive HIP-graph capture on a one-rank group (diagnostic).

usage: python tools/diag/capture_collectives.py MODE
MODE: allreduce | allreduce_async | allgather | a2a | a2a_side | direct | direct_side
Captures the collective once, replays it 3 times, prints "MODE ok" (a crash ends the process:
run every mode in its own process)."""
import os
import socket
import sys

import torch
import torch.distributed as dist


def main():
    mode = sys.argv[1]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    s.close()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    x = torch.ones(1 << 16, device=dev)
    y = torch.empty_like(x)
    h = torch.ones(1 << 16, device=dev, dtype=torch.float16)
    hr = torch.empty_like(h)
    side = torch.cuda.Stream(device=dev)

    def body():
        if mode == "allreduce":
            dist.all_reduce(x)
        elif mode == "allreduce_async":
            dist.all_reduce(x, async_op=True).wait()
        elif mode == "allgather":
            dist.all_gather_into_tensor(y, x)
        elif mode == "a2a":
            dist.all_to_all_single(hr, h)
        elif mode in ("a2a_side", "direct_side"):
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                dist.all_to_all_single(hr, h)
                if mode == "direct_side":
                    dist.all_gather_into_tensor(h, hr)
                ev = torch.cuda.Event()
                ev.record(side)
            torch.cuda.current_stream().wait_event(ev)
        elif mode == "direct":
            dist.all_to_all_single(hr, h)
            dist.all_gather_into_tensor(h, hr)
        else:
            raise SystemExit(f"unknown mode {mode}")

    body()  # eager first (communicator + connections)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        body()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print(f"{mode} ok", flush=True)
    if os.environ.get("DESTROY", "1") == "1":
        dist.destroy_process_group()
        print(f"{mode} destroyed", flush=True)


if __name__ == "__main__":
    main()
