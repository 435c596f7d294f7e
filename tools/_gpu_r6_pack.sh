#!/bin/bash
# vectorised weight-image packing in the fused Adam: tests, kernel time, step A/B vs the previous
# packing (variant lib)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_step_gpu.py tests/test_kernels_gpu.py -x -q -k "pack or apack or device_feed or device_fed" --timeout 150 --timeout-method thread > gpurun_out/r6_pack_tests.log 2>&1 || { tail -30 gpurun_out/r6_pack_tests.log; exit 1; }
tail -1 gpurun_out/r6_pack_tests.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_pack -o run -- python3 $R/bench.py --steps 100 --warmup 10 --site-loop 0 > $R/gpurun_out/prof_pack.log 2>&1 || exit 5
cd $R && python -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_pack/run_kernel_stats.csv')):
    if 'adam' in r['Name']: print('new', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1000,2))
"
: > gpurun_out/r6_pack_ab.txt
for lib in new old new old; do
  if [ $lib = old ]; then export DINUNET_KERNEL_LIB=$R/dinunet_implementations_amd/_native/ab/oldpack.so DINUNET_ALLOW_STALE=1; else unset DINUNET_KERNEL_LIB DINUNET_ALLOW_STALE; fi
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 > gpurun_out/r6_pack_b.log 2>&1 || { tail -20 gpurun_out/r6_pack_b.log; exit 2; }
  echo "$lib $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_pack_b.log) $(grep -o '"final_loss": [0-9.e-]*' gpurun_out/r6_pack_b.log)" | tee -a gpurun_out/r6_pack_ab.txt
done
