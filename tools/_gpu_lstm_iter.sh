#!/bin/bash
# LSTM iteration on the GPU: kernel numerics tests -> bench -> stamped per-phase cycles.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_kernels_gpu.py tests/test_step_gpu.py} -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --steps 100 --warmup 20 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 3; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench.log
timeout -k 10 300 python tools/lstm_stamps.py > gpurun_out/stamps.log 2>&1 || { tail -20 gpurun_out/stamps.log; exit 4; }
cat gpurun_out/stamps.log
