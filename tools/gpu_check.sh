#!/bin/bash
# One GPU session: numerics tests -> bench -> rocprofv3 kernel stats. Stops at the first
# crash/timeout (exit codes other than 0/1 from pytest).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-30}
python -c "import torch;print(torch.cuda.get_device_name(0), torch.__version__)" > gpurun_out/env.log 2>&1
timeout -k 10 900 python -m pytest ${TESTS:-tests/test_kernels_gpu.py} -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --steps $STEPS --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 3; }
timeout -k 10 300 python bench.py --steps $STEPS --warmup 5 --graph 0 ${BENCH_ARGS} >> gpurun_out/bench.log 2>&1 || { echo "bench eager failed"; tail -30 gpurun_out/bench.log; exit 3; }
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --graph 0 ${BENCH_ARGS} > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 4; }
fi
cat "$GRAFT_REPO_ROOT/gpurun_out/pytest_gpu.log" | tail -15
cat "$GRAFT_REPO_ROOT/gpurun_out/bench.log"
