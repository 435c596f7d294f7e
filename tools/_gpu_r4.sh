#!/bin/bash
# round-4 iteration: selected GPU tests, bench (device feed + site loop), optional rocprof timeline
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
if [ -n "${TESTS}" ]; then
  timeout -k 10 ${TTIME:-600} python -u -m pytest ${TESTS} -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -40
  [ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
fi
if [ "${BENCH:-1}" = "1" ]; then
  for a in ${BENCH_AB:-"DINUNET_ADAM_PACK=1"}; do
    env $a timeout -k 10 400 python bench.py --steps ${STEPS:-200} --warmup 20 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 3; }
    echo "$a $(tail -1 gpurun_out/bench.log)"
  done
fi
if [ "${PROF:-0}" = "1" ]; then
  R=$PWD; rm -rf gpurun_out/prof
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 30 --warmup 20 --site-loop 0 ${BENCH_ARGS} > $R/gpurun_out/prof.log 2>&1) || { tail -20 gpurun_out/prof.log; exit 4; }
  f=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
  python tools/timeline.py $f > gpurun_out/timeline.txt 2>&1; cat gpurun_out/timeline.txt
fi
