#!/bin/bash
# end-of-session check, as the driver runs it: every GPU test, smoke(), bench.py default, engines,
# rocprofv3 kernel timeline of the default bench; each GPU step under its own limit, stop on failure
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 5; }
echo smoke-ok
: > gpurun_out/bench_final.jsonl
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 3; }
grep metric gpurun_out/bench_default.log >> gpurun_out/bench_final.jsonl
for e in rankDAD powerSGD; do
  timeout -k 10 300 python bench.py --engine $e > gpurun_out/bench_$e.log 2>&1 || { tail -20 gpurun_out/bench_$e.log; exit 3; }
  grep metric gpurun_out/bench_$e.log >> gpurun_out/bench_final.jsonl
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_final.jsonl
R=$PWD; rm -rf gpurun_out/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 30 --warmup 20 > $R/gpurun_out/prof.log 2>&1) || { tail -20 gpurun_out/prof.log; exit 4; }
f=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
python tools/timeline.py $f > gpurun_out/timeline.txt 2>&1; cat gpurun_out/timeline.txt
s=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1); cp $s gpurun_out/kernel_stats.csv
