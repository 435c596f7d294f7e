#!/bin/bash
# LDS-DMA issue with per-chunk sources resolved at init (default lib) vs the previous issue code
# (variant lib): GEMM tests, then B=32 / 2048 / 4096 step A/B on one box
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 200 --timeout-method thread > gpurun_out/r6_issue_tests.log 2>&1 || { tail -30 gpurun_out/r6_issue_tests.log; exit 1; }
tail -1 gpurun_out/r6_issue_tests.log
V=dinunet_implementations_amd/_native/ab/oldissue.so
: > gpurun_out/r6_issue_ab.txt
for args in "--batch 2048 --pool 8 --site-loop 0 --steps 60" "--batch 4096 --pool 4 --site-loop 0 --steps 40" "--steps 300"; do
  for lib in new old new old; do
    if [ $lib = old ]; then export DINUNET_KERNEL_LIB=$V DINUNET_ALLOW_STALE=1; else unset DINUNET_KERNEL_LIB DINUNET_ALLOW_STALE; fi
    timeout -k 10 300 python bench.py --warmup 10 $args > gpurun_out/r6_issue_b.log 2>&1 || { tail -20 gpurun_out/r6_issue_b.log; exit 2; }
    echo "$args $lib $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_issue_b.log) $(grep -o '"final_loss": [0-9.e-]*' gpurun_out/r6_issue_b.log)" | tee -a gpurun_out/r6_issue_ab.txt
  done
done
