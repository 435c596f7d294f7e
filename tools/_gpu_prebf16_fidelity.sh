#!/bin/bash
# training fidelity of bf16 stored gate pre-activations at a large batch: the hard ICA cohort,
# B = 512, same seeds with DINUNET_LSTM_PRE_BF16=0 (fp32 store) and =auto (bf16 from B >= 512)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
out=gpurun_out/pre_bf16_fidelity.jsonl; rm -f $out
for s in ${SEEDS:-0 1 2}; do
  for m in 0 auto; do
    DINUNET_LSTM_PRE_BF16=$m timeout -k 10 240 python tools/bench_time_to_auc.py --cohort hard --signal 0.35 \
      --batch 512 --subjects ${SUBJ:-4096} --val 1024 --target 0.99 --lr ${LR:-1e-3} --full \
      --max-steps ${MAXSTEPS:-300} --eval-every 25 --seed $s > gpurun_out/fid_case.log 2>&1 || { tail -20 gpurun_out/fid_case.log; exit 3; }
    echo "{\"pre_bf16\": \"$m\", \"seed\": $s, \"run\": $(grep '^{' gpurun_out/fid_case.log | tail -1)}" >> $out
    python - "$out" <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().splitlines()[-1])
print(r["pre_bf16"], r["seed"], "final", r["run"].get("final_auc"), "best", r["run"].get("best_auc"))
PY
  done
done
exit 0
