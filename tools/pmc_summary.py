#!/usr/bin/env python3
"""Per-kernel mean of rocprofv3 ``--pmc`` counters over dispatches (CSV counter collections of one
or more passes), for the kernels whose name matches a pattern.

usage: python tools/pmc_summary.py PATTERN dir1/g_counter_collection.csv [dir2/...csv ...]
"""
import collections
import csv
import re
import sys


def main():
    pat = re.compile(sys.argv[1])
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for path in sys.argv[2:]:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            if not pat.search(name):
                continue
            key = name[:90]
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[key] = (r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"], r["VGPR_Count"],
                         r["Accum_VGPR_Count"], r["Scratch_Size"])
    for key, cs in vals.items():
        g, w, lds, v, av, scr = meta[key]
        print(f"## {key}\ngrid {g} wg {w} lds {lds} vgpr {v}+{av} scratch {scr}")
        for c, xs in sorted(cs.items()):
            print(f"  {c:28s} {sum(xs) / len(xs):16.1f}  (n={len(xs)})")
        m = {c: sum(xs) / len(xs) for c, xs in cs.items()}
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            wc = m["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in m:
                    print(f"  share {c:22s} {m[c] / wc:6.3f}")
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            print(f"  L2 hit rate {m['TCC_HIT_sum'] / max(1.0, m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.3f}")
        if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            pass
        if "FETCH_SIZE" in m:
            print(f"  fetch (x2 gfx950 correction) {2 * m['FETCH_SIZE'] / 1e6:.1f} GB-ish (KB units -> GB)")
        if "WRITE_SIZE" in m:
            print(f"  write {m['WRITE_SIZE'] / 1e6:.2f} GB (KB units)")


if __name__ == "__main__":
    main()
