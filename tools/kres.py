#!/usr/bin/env python3
"""Print per-kernel VGPR/AGPR/spill/LDS/occupancy for a .hip file (hipcc resource remarks).

usage: python tools/kres.py path/to/file.hip [extra hipcc flags]
"""
import re
import subprocess
import sys


def main():
    src = sys.argv[1]
    cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o",
           "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
    out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode:
        print(out.stderr)
        sys.exit(out.returncode)
    rows, cur = [], None
    for line in out.stderr.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        kv = m.group(1).strip()
        if kv.startswith("Function Name:"):
            cur = {"name": kv.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in kv:
            k, v = kv.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        name = r["name"]
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        name = re.sub(r"\(anonymous namespace\)::", "", name)[:70]
        print(f"{name:70s} vgpr={r.get('VGPRs','?'):>4} agpr={r.get('AGPRs','?'):>3} "
              f"spill={r.get('VGPRs Spill','?'):>3} lds={r.get('LDS Size [bytes/block]','?'):>6} "
              f"occ={r.get('Occupancy [waves/SIMD]','?')}")


if __name__ == "__main__":
    main()
