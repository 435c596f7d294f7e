#!/bin/bash
# rank-dAD power iteration: split-bf16 MFMAs (default) vs fp32 MFMAs (variant lib): stamps,
# persistent-vs-staged numerics, bench; then the several-GPUs-per-site runtime test
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
V=dinunet_implementations_amd/_native/ab/f32mfma.so
timeout -k 10 120 python tools/lowrank_persist_stamps.py > gpurun_out/r6_lr_stamps_x3.txt 2>&1 || { tail gpurun_out/r6_lr_stamps_x3.txt; exit 1; }
DINUNET_KERNEL_LIB=$V DINUNET_ALLOW_STALE=1 timeout -k 10 120 python tools/lowrank_persist_stamps.py > gpurun_out/r6_lr_stamps_f32.txt 2>&1 || { tail gpurun_out/r6_lr_stamps_f32.txt; exit 2; }
grep -E "median|span" gpurun_out/r6_lr_stamps_x3.txt gpurun_out/r6_lr_stamps_f32.txt
timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py -x -q -k "rankdad_persistent or rankdad" --timeout 120 --timeout-method thread > gpurun_out/r6_lr_tests.log 2>&1 || { tail -30 gpurun_out/r6_lr_tests.log; exit 3; }
tail -1 gpurun_out/r6_lr_tests.log
for lib in base f32; do
  if [ $lib = f32 ]; then export DINUNET_KERNEL_LIB=$V DINUNET_ALLOW_STALE=1; fi
  timeout -k 10 200 python bench.py --engine rankDAD --steps 300 --warmup 30 --site-loop 0 > gpurun_out/r6_lr_bench_$lib.log 2>&1 || { tail -20 gpurun_out/r6_lr_bench_$lib.log; exit 4; }
  echo "$lib $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_lr_bench_$lib.log) $(grep -o '"final_loss": [0-9.e-]*' gpurun_out/r6_lr_bench_$lib.log)"
done | tee gpurun_out/r6_lr_bench.txt
unset DINUNET_KERNEL_LIB DINUNET_ALLOW_STALE
timeout -k 10 300 python -u -m pytest tests/test_runtime_gpu.py -x -v -k "two_gpus_each" --timeout 150 --timeout-method thread > gpurun_out/r6_replica_gpu.log 2>&1 || { tail -30 gpurun_out/r6_replica_gpu.log; exit 5; }
tail -4 gpurun_out/r6_replica_gpu.log
