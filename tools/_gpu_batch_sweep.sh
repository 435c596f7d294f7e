#!/bin/bash
# bench.py at larger per-site batches (BASELINE config 5: large-batch sizing for 288 GB HBM)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for b in ${BATCHES:-32 128 512 2048}; do
  timeout -k 10 240 python bench.py --batch $b --steps 30 --warmup 5 > gpurun_out/batch_$b.log 2>&1 || { tail -5 gpurun_out/batch_$b.log; exit 5; }
  echo "B=$b $(grep -o '"value": [0-9.]*, "unit"' gpurun_out/batch_$b.log | cut -d' ' -f2) samples/s $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/batch_$b.log)"
done
