#!/bin/bash
# low-rank engine iteration: GPU tests of the PowerSGD / rank-dAD paths, bench of both engines,
# kernel stats of the PowerSGD step (-> gpurun_out/)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_step_gpu.py tests/test_multirank_gpu.py tests/test_runtime_gpu.py tests/test_engines.py > gpurun_out/lr_tests.log 2>&1 || { tail -30 gpurun_out/lr_tests.log; exit 3; }
tail -3 gpurun_out/lr_tests.log
: > gpurun_out/bench_lr.jsonl
for e in powerSGD rankDAD; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 20 --engine $e > gpurun_out/bench_$e.log 2>&1 || { tail -20 gpurun_out/bench_$e.log; exit 4; }
  grep '^{' gpurun_out/bench_$e.log >> gpurun_out/bench_lr.jsonl
done
cat gpurun_out/bench_lr.jsonl
ENGINE=${PROF_ENGINE:-powerSGD}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/eprof_${ENGINE} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --engine ${ENGINE} > $GRAFT_REPO_ROOT/gpurun_out/eprof_${ENGINE}.log 2>&1 || exit 5
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/eprof_${ENGINE}/run_kernel_stats.csv 2>/dev/null | head -30
