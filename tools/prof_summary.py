#!/usr/bin/env python3
"""Markdown summary of a rocprofv3 ``--kernel-trace --stats`` run (per-step kernel times).

usage: python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv STEPS "title" > profiles/x.md
"""
import csv
import re
import subprocess
import sys


def short(name: str) -> str:
    if name.startswith("_Z"):
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = name.split("(")[0] if not name.startswith("void") else name.split("(")[0][5:]
    return name[:80]


def main():
    path, steps, title = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    print(f"Kernel time per step (sum over {steps} profiled steps / {steps}): **{tot / steps / 1e3:.1f} us**\n")
    print("| kernel | calls/step | us/step | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    for r in rows:
        t = float(r["TotalDurationNs"])
        print(f"| `{short(r['Name'])}` | {int(r['Calls']) / steps:.1f} | {t / steps / 1e3:.1f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {100 * t / tot:.1f} |")


if __name__ == "__main__":
    main()
