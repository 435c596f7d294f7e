#!/bin/bash
# BASELINE config 4 on one GPU: 8 sites (8 ranks sharing the GPU over gloo) training the hard
# synthetic ICA cohort with dSGD / rank-dAD / PowerSGD, same seeds; global validation AUC curve
# per run -> gpurun_out/engines_8site.jsonl (accuracy evidence, not a throughput number)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
out=gpurun_out/engines_8site.jsonl; : > $out
port=29611
for s in ${SEEDS:-0 1}; do
  for e in dSGD rankDAD powerSGD; do
    port=$((port + 1))
    DINUNET_BACKEND=gloo timeout -k 10 ${RUNLIMIT:-280} python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
      --master-addr 127.0.0.1 --master-port $port tools/bench_time_to_auc.py --engine $e --cohort hard \
      --effect 0.35 --subjects ${SUBJ:-384} --val 128 --batch 32 --max-steps ${STEPS:-600} --eval-every 50 \
      --target 0.99 --full --seed $s > gpurun_out/e8_${e}_$s.log 2>&1 || { tail -30 gpurun_out/e8_${e}_$s.log; exit 3; }
    echo "{\"engine\": \"$e\", \"seed\": $s, \"sites\": 8, \"run\": $(grep '^{' gpurun_out/e8_${e}_$s.log | tail -1)}" >> $out
    python - "$out" <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().splitlines()[-1])
print(r["engine"], r["seed"], "final", r["run"].get("final_auc"), "best", r["run"].get("best_auc"), "wall", r["run"].get("value"))
PY
  done
done
