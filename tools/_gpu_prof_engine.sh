#!/bin/bash
# kernel stats of bench.py for one engine (ENGINE=...), graph replay, 20 steps
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/eprof_${ENGINE} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --engine ${ENGINE} > $GRAFT_REPO_ROOT/gpurun_out/eprof_${ENGINE}.log 2>&1 || exit 4
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/eprof_${ENGINE}/run_kernel_stats.csv 2>/dev/null | head -30 || head -30 gpurun_out/eprof_${ENGINE}/run_kernel_stats.csv
