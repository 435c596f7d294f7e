#!/bin/bash
# end of round: every GPU test, then the headline bench three times and the loopback forms
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
bash tools/_gpu_tests_all.sh || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 > gpurun_out/r6f_bench_$i.log 2>&1 || { tail -20 gpurun_out/r6f_bench_$i.log; exit 2; }
  grep '^{' gpurun_out/r6f_bench_$i.log | tail -1 >> gpurun_out/r6_final_bench.jsonl
done
for args in "--loopback-rccl" "--loopback-rccl --precision-bits 16" "--engine rankDAD" "--engine powerSGD" "--batch 2048 --pool 8 --site-loop 0 --steps 50" "--batch 4096 --pool 4 --site-loop 0 --steps 30"; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 $args > gpurun_out/r6f_x.log 2>&1 || { tail -20 gpurun_out/r6f_x.log; exit 3; }
  echo "{\"args\": \"$args\", \"line\": $(grep '^{' gpurun_out/r6f_x.log | tail -1)}" >> gpurun_out/r6_final_bench.jsonl
done
python -c "
import json
for l in open('gpurun_out/r6_final_bench.jsonl'):
    d=json.loads(l); x=d.get('line',d); print(d.get('args','headline'), x['ms_per_step'], x['value'], x.get('collective'))
"
