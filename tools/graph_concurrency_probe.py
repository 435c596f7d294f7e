#!/usr/bin/env python3
"""Do two kernels on forked capture streams run concurrently when a HIP graph replays?  Each
branch holds 16 CUs for 40 us (dn_busy); serial replay ~80 us, concurrent ~40 us.  Also the
eager two-stream case for comparison.

    python tools/graph_concurrency_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dinunet_implementations_amd.ops import _lib  # noqa: E402
from dinunet_implementations_amd.runtime.health import occupy_cus  # noqa: E402


def timed(fn, reps=20):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        ev[0].record()
        fn()
        ev[1].record()
        ev[1].synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    us = 40
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def two_streams():
        side.wait_stream(main_s)
        occupy_cus(16, us)
        with torch.cuda.stream(side):
            occupy_cus(16, us)
        main_s.wait_stream(side)

    def one_stream():
        occupy_cus(16, us)
        occupy_cus(16, us)

    print(f"eager one stream   {timed(one_stream):7.1f} us")
    print(f"eager two streams  {timed(two_streams):7.1f} us")
    for name, fn in (("graph one stream", one_stream), ("graph two streams", two_streams)):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(main_s)
        with torch.cuda.stream(s):
            fn()  # warm
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            fn()
        print(f"{name:18s} {timed(g.replay):7.1f} us")


if __name__ == "__main__":
    main()
