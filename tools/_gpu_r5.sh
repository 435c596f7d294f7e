#!/bin/bash
# round-5 iteration: selected GPU tests, bench runs (N=1 and the loopback-RCCL N>1 path, A/B env
# settings), optional rocprof timeline of one bench configuration
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
if [ -n "${TESTS}" ]; then
  timeout -k 10 ${TTIME:-600} python -u -m pytest ${TESTS} -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -60
  [ $rc -eq 0 ] || { tail -80 gpurun_out/pytest_gpu.log; exit $rc; }
fi
# RUNS: ';'-separated list of "ENV=.. ENV2=..|bench args"
if [ -n "${RUNS}" ]; then
  IFS=';' read -ra RR <<< "${RUNS}"
  for r in "${RR[@]}"; do
    e="${r%%|*}"; a="${r#*|}"
    env $e timeout -k 10 300 python bench.py --steps ${STEPS:-200} --warmup 20 --site-loop 0 $a > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 3; }
    echo "[$e | $a] $(tail -1 gpurun_out/bench.log)" | tee -a gpurun_out/bench_runs.jsonl
  done
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 400 python bench.py --steps ${STEPS:-200} --warmup 20 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 3; }
  tail -1 gpurun_out/bench.log
fi
if [ "${PROF:-0}" = "1" ]; then
  R=$PWD; rm -rf gpurun_out/prof
  (cd /tmp && env ${PROF_ENV} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 30 --warmup 20 --site-loop 0 ${PROF_ARGS} > $R/gpurun_out/prof.log 2>&1) || { tail -20 gpurun_out/prof.log; exit 4; }
  f=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
  python tools/timeline.py $f > gpurun_out/timeline.txt 2>&1; cat gpurun_out/timeline.txt
  s=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
  [ -n "$s" ] && python tools/prof_summary.py $s 30 "${PROF_ARGS}" > gpurun_out/kernel_stats.md 2>&1
fi
exit 0
