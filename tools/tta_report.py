#!/usr/bin/env python3
"""Markdown table of time-to-AUC JSON lines (tools/bench_time_to_auc.py output):

    python tools/tta_report.py profiles/r2_time_to_auc_fidelity.jsonl [more.jsonl ...]
"""
import json
import statistics
import sys


def first(curve, t):
    return next((s for s, a in curve if a >= t), None)


def main():
    rows = []
    for p in sys.argv[1:]:
        with open(p) as f:
            rows += [json.loads(l) for l in f if l.strip().startswith("{")]
    print("| engine | sites | path | seed | reached | steps to target | wall s to target | "
          "final AUC | best AUC | AUC @500 | AUC @1000 | AUC @2000 |")
    print("|---|---:|---|---:|---|---:|---:|---:|---:|---:|---:|---:|")
    for r in rows:
        cv = dict((s, a) for s, a in r.get("curve", []))

        def at(s):
            return f"{cv[s]:.3f}" if s in cv else "-"
        print(f"| {r.get('engine', 'dSGD')} | {r['n_sites']} | {r.get('compute_path', 'fused')} "
              f"({r['dtype']}) | {r.get('seed', 0)} | {r['reached']} | "
              f"{r['steps'] if r['reached'] else '>' + str(r['steps'])} | "
              f"{r['value'] if r['reached'] else '-'} | {r['final_auc']:.3f} | "
              f"{r['best_auc']:.3f} | {at(500)} | {at(1000)} | {at(2000)} |")
    groups = {}
    for r in rows:
        groups.setdefault((r.get("engine", "dSGD"), r["n_sites"], r.get("compute_path")), []).append(r)
    print()
    print("| engine | sites | path | runs | steps to AUC 0.70 | to 0.75 | to 0.80 | mean final AUC | "
          "mean best AUC |")
    print("|---|---:|---|---:|---|---|---|---:|---:|")
    for (e, n, cp), rs in groups.items():
        def steps(t):
            v = [first(r.get("curve", []), t) for r in rs]
            return ", ".join(str(x) if x is not None else "-" for x in v)
        print(f"| {e} | {n} | {cp} | {len(rs)} | {steps(0.70)} | {steps(0.75)} | {steps(0.80)} | "
              f"{statistics.fmean(r['final_auc'] for r in rs):.3f} | "
              f"{statistics.fmean(r['best_auc'] for r in rs):.3f} |")


if __name__ == "__main__":
    main()
