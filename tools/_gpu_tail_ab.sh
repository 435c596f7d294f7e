#!/bin/bash
# A/B of the 256-tile tail split (DINUNET_GEMM_TAIL) at large batch, same box, + its GPU test
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "tail or gemm256 or gathered" > gpurun_out/tail_tests.log 2>&1 || { tail -30 gpurun_out/tail_tests.log; exit 3; }
tail -2 gpurun_out/tail_tests.log
: > gpurun_out/tail_ab.jsonl
for B in ${BATCHES:-2048 4096}; do
  for T in 0 1 0 1; do
    DINUNET_GEMM_TAIL=$T timeout -k 10 240 python bench.py --steps 30 --warmup 10 --batch $B --pool 8 --site-loop 0 > gpurun_out/tail_b${B}_t$T.log 2>&1 || { tail -20 gpurun_out/tail_b${B}_t$T.log; exit 4; }
    echo "B=$B tail=$T $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tail_b${B}_t$T.log) $(grep -o '"value": [0-9.]*' gpurun_out/tail_b${B}_t$T.log)" | tee -a gpurun_out/tail_ab.txt
    grep '"metric"' gpurun_out/tail_b${B}_t$T.log | sed "s/^{/{\"gemm_tail\": $T, /" >> gpurun_out/tail_ab.jsonl
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 5 --batch 2048 --pool 8 --site-loop 0 > $GRAFT_REPO_ROOT/gpurun_out/tprof.log 2>&1 || exit 5
cd $GRAFT_REPO_ROOT && python tools/timeline.py gpurun_out/tprof/run_kernel_trace.csv 2
