#!/bin/bash
# Large-batch throughput sweep (B = 32 .. 2048, dSGD, HIP graph) + a rocprofv3 kernel summary at
# B = 2048; one bench process per batch size, each under its own time limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
: > gpurun_out/batch_sweep.jsonl
for B in ${BATCHES:-32 128 512 2048}; do
  timeout -k 10 ${BLIMIT:-240} python bench.py --steps ${BSTEPS:-30} --warmup 10 --batch $B --pool ${POOL:-8} > gpurun_out/bench_b$B.log 2>&1 || { tail -20 gpurun_out/bench_b$B.log; exit 3; }
  grep '"metric"' gpurun_out/bench_b$B.log >> gpurun_out/batch_sweep.jsonl
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_b$B.log
done
if [ -n "$PROF_B" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b$PROF_B -o run -- python3 bench.py --steps 20 --warmup 5 --batch $PROF_B > gpurun_out/prof_b$PROF_B.log 2>&1 || { tail -20 gpurun_out/prof_b$PROF_B.log; exit 4; }
  find gpurun_out/prof_b$PROF_B -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof_b${PROF_B}_kernel_stats.csv
fi
