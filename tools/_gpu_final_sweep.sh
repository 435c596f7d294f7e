#!/bin/bash
# end-of-round evidence: batch sweep (dSGD, one process per batch size) and the three engines at
# B = 32, one box -> gpurun_out/final_sweep.jsonl
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
: > gpurun_out/final_sweep.jsonl
for B in ${BATCHES:-32 512 2048 4096 8192}; do
  timeout -k 10 240 python bench.py --steps ${BSTEPS:-30} --warmup 10 --batch $B --pool 8 --site-loop 0 > gpurun_out/fs_b$B.log 2>&1 || { tail -20 gpurun_out/fs_b$B.log; exit 3; }
  grep '"metric"' gpurun_out/fs_b$B.log >> gpurun_out/final_sweep.jsonl
  echo "B=$B $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fs_b$B.log) $(grep -o '"value": [0-9.]*' gpurun_out/fs_b$B.log)"
done
for e in rankDAD powerSGD; do
  timeout -k 10 240 python bench.py --steps 100 --warmup 20 --engine $e > gpurun_out/fs_$e.log 2>&1 || { tail -20 gpurun_out/fs_$e.log; exit 4; }
  grep '"metric"' gpurun_out/fs_$e.log >> gpurun_out/final_sweep.jsonl
  echo "$e $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fs_$e.log)"
done
