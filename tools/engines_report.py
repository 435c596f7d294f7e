#!/usr/bin/env python3
"""Markdown report of ``tools/_gpu_engines_8site.sh`` (8 sites on one GPU over gloo, hard
synthetic ICA cohort, dSGD / rank-dAD / PowerSGD at the same seeds): per run the final / best
global validation AUC and the steps to AUC targets; per engine the means.

    python tools/engines_report.py gpurun_out/engines_8site.jsonl [--out profiles/r5_engines_8site.md]
"""
import argparse
import json
import statistics


def steps_to(curve, target):
    for st, v in curve or []:
        if v is not None and v >= target:
            return st
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--out", default=None)
    ap.add_argument("--every", type=int, default=50)
    a = ap.parse_args()
    runs = [json.loads(x) for x in open(a.path) if x.strip()]
    targets = (0.65, 0.70, 0.75)
    md = ["# 8 sites, dSGD vs rank-dAD vs PowerSGD (BASELINE config 4 accuracy, one GPU)", "",
          "8 ranks share one MI355X over gloo (`tools/_gpu_engines_8site.sh`): every site holds a "
          "private hard synthetic ICA cohort, batch 32 per site, the engines' default settings "
          "(rank-dAD rank 10, 5 power iterations, tol 1e-3; PowerSGD rank 4), global validation AUC "
          f"every {a.every} steps.  Accuracy evidence, not a throughput number.", "",
          "| engine | seed | final AUC | best AUC | steps to " + " / ".join(f"{t:.2f}" for t in targets)
          + " | wall s |", "|---|---:|---:|---:|---|---:|"]
    by = {}
    for r in runs:
        run = r["run"]
        cur = run.get("curve") or []
        st = " / ".join(str(steps_to(cur, t) or "-") for t in targets)
        md.append(f"| {r['engine']} | {r['seed']} | {run.get('final_auc')} | {run.get('best_auc')} | "
                  f"{st} | {run.get('value')} |")
        by.setdefault(r["engine"], []).append(run)
    md += ["", "| engine | runs | final AUC mean | best AUC mean |", "|---|---:|---:|---:|"]
    for e, rs in by.items():
        fa = [x.get("final_auc") for x in rs if x.get("final_auc") is not None]
        ba = [x.get("best_auc") for x in rs if x.get("best_auc") is not None]
        md.append(f"| {e} | {len(rs)} | {statistics.mean(fa):.4f} | {statistics.mean(ba):.4f} |")
    text = "\n".join(md) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    print(text)


if __name__ == "__main__":
    main()
