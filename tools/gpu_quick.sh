#!/bin/bash
# quick GPU iteration: numerics tests, op micro-bench, bench.py (no profiler)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest ${TESTS:-tests/test_kernels_gpu.py} -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
timeout -k 10 300 python tools/bench_ops.py > gpurun_out/bench_ops.log 2>&1; rc=$?
cat gpurun_out/bench_ops.log | head -40
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps ${STEPS:-50} --warmup 10 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?
cat gpurun_out/bench.log
exit $rc
