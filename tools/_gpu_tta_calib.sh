#!/bin/bash
# hard-cohort calibration: validation-AUC curves for a few signal strengths (1 site, fused path)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
: > gpurun_out/tta_calib.jsonl
for S in ${SIGNALS:-0.5 0.35 0.25}; do
  timeout -k 10 300 python tools/bench_time_to_auc.py --cohort hard --signal $S --target ${TARGET:-0.8} --max-steps ${STEPS:-3000} --eval-every 50 --full ${EXTRA} > gpurun_out/tta_s$S.log 2>&1 || { tail -20 gpurun_out/tta_s$S.log; exit 3; }
  grep '"metric"' gpurun_out/tta_s$S.log >> gpurun_out/tta_calib.jsonl
  python -c "import json,sys; d=json.loads(open('gpurun_out/tta_s$S.log').read().strip().splitlines()[-1]); print('$S', d['reached'], d['steps'], d['best_auc'], d['curve'][::6])"
done
