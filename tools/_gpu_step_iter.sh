#!/bin/bash
# headline-step iteration: GEMM / step GPU tests (TESTS, default the kernel + step suites), two
# bench.py runs, a kernel-trace profile of the graph step (-> gpurun_out/)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
T=${TESTS:-tests/test_kernels_gpu.py tests/test_step_gpu.py}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $T > gpurun_out/step_tests.log 2>&1 || { tail -30 gpurun_out/step_tests.log; exit 3; }
tail -2 gpurun_out/step_tests.log
: > gpurun_out/bench_step.jsonl
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 30 $BENCH_ARGS > gpurun_out/bench_step_$i.log 2>&1 || { tail -20 gpurun_out/bench_step_$i.log; exit 4; }
  grep '^{' gpurun_out/bench_step_$i.log >> gpurun_out/bench_step.jsonl
done
python - <<'PY'
import json
for l in open("gpurun_out/bench_step.jsonl"):
    d = json.loads(l); print(d["config"].get("engine"), d["ms_per_step"], d["value"])
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 20 --site-loop 0 $BENCH_ARGS > $GRAFT_REPO_ROOT/gpurun_out/sprof.log 2>&1 || exit 5
cd $GRAFT_REPO_ROOT && python tools/timeline.py gpurun_out/sprof/run_kernel_trace.csv 2
