#!/bin/bash
# bench.py under each grouped split-K override (DINUNET_GROUP_SPLITS), graph mode
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for sp in 0 2 3 4; do
  DINUNET_GROUP_SPLITS=$sp timeout -k 10 200 python bench.py --steps 200 --warmup 30 > gpurun_out/split_$sp.log 2>&1 || exit 5
  echo "splits=$sp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/split_$sp.log)"
done
