#!/bin/bash
# every GPU test (one pytest process), then bench; stops at the first failure
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/} -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -12; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|error" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --steps 100 --warmup 20 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 3; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench.log
