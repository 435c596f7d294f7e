#!/bin/bash
# round 6: the folded head (head_rep on own images), health negative controls, step tests
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_head_gpu.py tests/test_health_gpu.py tests/test_capture_quiesce_gpu.py tests/test_step_gpu.py tests/test_runtime_gpu.py > gpurun_out/r6_head.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r6_head.log | grep -v PASSED | head; tail -2 gpurun_out/r6_head.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r6_head.log | head -20; exit $rc; }
timeout -k 10 200 python bench.py --steps 300 --warmup 30 --site-loop 0 > gpurun_out/r6_bench_head.log 2>&1 && grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_bench_head.log
