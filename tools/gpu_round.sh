#!/bin/bash
# Full GPU check, mirroring the driver's round end: gpu tests -> smoke -> bench -> rocprofv3 stats.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 5; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 3; }
grep metric gpurun_out/bench.log
if [ "${PROF:-1}" = "1" ]; then
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --graph 0 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || exit 4
echo prof-ok
fi
