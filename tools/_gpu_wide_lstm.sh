#!/bin/bash
# streamed-weight LSTM variants (per-direction hidden > 192): numerics tests, then step times
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread -k "lstm or wide" > gpurun_out/pytest_wide.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_wide.log | tail -20; tail -2 gpurun_out/pytest_wide.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_wide.log | head -30; exit $rc; }
for h in 512 768 1024; do
timeout -k 10 120 python bench.py --hidden $h --steps 20 --warmup 5 > gpurun_out/bench_h$h.log 2>&1 || { tail -5 gpurun_out/bench_h$h.log; exit 3; }
echo "hidden $h: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_h$h.log)"
done
