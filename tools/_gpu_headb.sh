#!/bin/bash
# batched-head iteration: its GPU tests, B=2048 / 4096 bench, B=2048 step timeline (-> gpurun_out/)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_head_gpu.py > gpurun_out/headb_tests.log 2>&1 || { tail -30 gpurun_out/headb_tests.log; exit 3; }
tail -2 gpurun_out/headb_tests.log
: > gpurun_out/headb_bench.jsonl
for B in 2048 4096 2048; do
  timeout -k 10 240 python bench.py --steps 30 --warmup 10 --batch $B --pool 8 --site-loop 0 > gpurun_out/headb_b$B.log 2>&1 || { tail -20 gpurun_out/headb_b$B.log; exit 4; }
  echo "B=$B $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/headb_b$B.log) $(grep -o '"value": [0-9.]*' gpurun_out/headb_b$B.log)"
  grep '"metric"' gpurun_out/headb_b$B.log >> gpurun_out/headb_bench.jsonl
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/hprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 5 --batch 2048 --pool 8 --site-loop 0 > $GRAFT_REPO_ROOT/gpurun_out/hprof.log 2>&1 || exit 5
cd $GRAFT_REPO_ROOT && python tools/timeline.py gpurun_out/hprof/run_kernel_trace.csv 2 > gpurun_out/hprof_timeline.txt; cat gpurun_out/hprof_timeline.txt
