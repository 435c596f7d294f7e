#!/bin/bash
# deferred-pack check: TrainStep GPU tests, bench (on/off), one kernel trace of the replayed step
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/step_gpu.log 2>&1 || { tail -30 gpurun_out/step_gpu.log; exit 3; }
tail -3 gpurun_out/step_gpu.log
timeout -k 10 240 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_on.log 2>&1 || { tail -5 gpurun_out/bench_on.log; exit 4; }
DINUNET_DEFER_PACK=0 timeout -k 10 240 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_off.log 2>&1 || { tail -5 gpurun_out/bench_off.log; exit 5; }
timeout -k 10 240 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_on2.log 2>&1 || { tail -5 gpurun_out/bench_on2.log; exit 6; }
grep -h metric gpurun_out/bench_on.log gpurun_out/bench_off.log gpurun_out/bench_on2.log | cut -c1-200
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/dprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/dprof.log 2>&1 || exit 7
echo prof-ok
