#!/usr/bin/env python3
"""One training step's kernel timeline from a rocprofv3 --kernel-trace CSV (steps delimited by
the fused Adam launch): start / end (us, relative to the previous Adam's end), duration, queue.

usage: python tools/timeline.py gpurun_out/prof/run_kernel_trace.csv [step_from_end=2]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"]]
    a, b = idx[-back - 1], idx[-back]
    t0 = int(rows[a]["End_Timestamp"])
    busy_end = t0
    for r in rows[a + 1:b + 1]:
        s = int(r["Start_Timestamp"]) - t0
        e = int(r["End_Timestamp"]) - t0
        gap = (int(r["Start_Timestamp"]) - busy_end) / 1000
        busy_end = max(busy_end, int(r["End_Timestamp"]))
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:64]
        print(f"{s / 1000:8.1f} {e / 1000:8.1f} {(e - s) / 1000:7.1f} gap {gap:6.1f} q{r.get('Queue_Id', '?')} {name}")
    print(f"step: {(int(rows[b]['End_Timestamp']) - t0) / 1000:.1f} us")


if __name__ == "__main__":
    main()
