#!/bin/bash
# phase stamps of the replicated head and the rank-dAD power iteration; rank-dAD step timeline
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 120 python tools/head_rep_stamps.py 32 0.25 > gpurun_out/r6_head_stamps.txt 2>&1 || { tail -20 gpurun_out/r6_head_stamps.txt; exit 1; }
cat gpurun_out/r6_head_stamps.txt
timeout -k 10 120 python tools/lowrank_persist_stamps.py > gpurun_out/r6_lr_stamps.txt 2>&1 || { tail -20 gpurun_out/r6_lr_stamps.txt; exit 2; }
cat gpurun_out/r6_lr_stamps.txt
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r6_rd -o run -- python3 $GRAFT_REPO_ROOT/bench.py --engine rankDAD --steps 20 --warmup 5 --site-loop 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_r6_rd.log 2>&1 || exit 5
cd $GRAFT_REPO_ROOT && python tools/timeline.py gpurun_out/prof_r6_rd/run_kernel_trace.csv > gpurun_out/r6_rd_timeline.txt && cat gpurun_out/r6_rd_timeline.txt
