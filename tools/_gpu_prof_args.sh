#!/bin/bash
# rocprofv3 kernel stats of bench.py with arbitrary arguments: TAG=name ARGS="--batch 2048 ..."
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 ${ARGS} > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log 2>&1 || exit 4
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_${TAG}/run_kernel_stats.csv 25 "${TAG}" > gpurun_out/prof_${TAG}_summary.md && head -40 gpurun_out/prof_${TAG}_summary.md
