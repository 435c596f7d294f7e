#!/bin/bash
# rank-dAD after the split MFMAs + argument warm-up + reconstruction rewrite: stamps, tests, bench,
# step timeline
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 120 python tools/lowrank_persist_stamps.py > gpurun_out/r6_lr_stamps_v2.txt 2>&1 || { tail gpurun_out/r6_lr_stamps_v2.txt; exit 1; }
grep -E "median|span" gpurun_out/r6_lr_stamps_v2.txt
timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py tests/test_multirank_gpu.py tests/test_health_gpu.py -x -q -k "rankdad or rankDAD" --timeout 120 --timeout-method thread > gpurun_out/r6_lr_tests2.log 2>&1 || { tail -30 gpurun_out/r6_lr_tests2.log; exit 3; }
tail -1 gpurun_out/r6_lr_tests2.log
timeout -k 10 200 python bench.py --engine rankDAD --steps 300 --warmup 30 --site-loop 0 > gpurun_out/r6_lr_bench2.log 2>&1 || { tail -20 gpurun_out/r6_lr_bench2.log; exit 4; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_lr_bench2.log
timeout -k 10 200 python bench.py --steps 300 --warmup 30 --site-loop 0 > gpurun_out/r6_lr_bench2_dsgd.log 2>&1 || { tail -20 gpurun_out/r6_lr_bench2_dsgd.log; exit 4; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_lr_bench2_dsgd.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r6_rd2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --engine rankDAD --steps 20 --warmup 5 --site-loop 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_r6_rd2.log 2>&1 || exit 5
cd $GRAFT_REPO_ROOT && python tools/timeline.py gpurun_out/prof_r6_rd2/run_kernel_trace.csv > gpurun_out/r6_rd2_timeline.txt && tail -6 gpurun_out/r6_rd2_timeline.txt
