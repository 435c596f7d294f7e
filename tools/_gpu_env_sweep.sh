#!/bin/bash
# bench.py under each environment assignment of $SWEEP (space separated, e.g. "A=0 A=1")
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
i=0
for kv in $SWEEP; do
  i=$((i+1))
  env $kv timeout -k 10 200 python bench.py --steps 200 --warmup 30 > gpurun_out/sweep_$i.log 2>&1 || { tail -5 gpurun_out/sweep_$i.log; exit 5; }
  echo "$kv $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep_$i.log)"
done
