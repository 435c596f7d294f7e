#!/bin/bash
# bench.py under several environment settings (A/B of runtime switches), one process each:
#   CASES="label:ENV=1,ENV2=x label2:..." BATCH=32
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for c in $CASES; do
  label=${c%%:*}; envs=${c#*:}
  [ "$envs" = "-" ] && envs=""
  env $(echo $envs | tr ',' ' ') timeout -k 10 240 python bench.py --steps ${STEPS:-100} --warmup 20 --batch ${BATCH:-32} ${BENCH_ARGS} > gpurun_out/ab_$label.log 2>&1 || { echo "$label FAILED"; tail -5 gpurun_out/ab_$label.log; exit 3; }
  echo "$label $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$label.log)"
done
