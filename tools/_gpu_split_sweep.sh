#!/bin/bash
# bench.py under grouped-GEMM overrides: "tile:splits" pairs (DINUNET_GROUP_TILE/_SPLITS)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for ts in ${SWEEP:-"-1:0 -1:2 -1:3 -1:4"}; do
  t=${ts%%:*}; sp=${ts##*:}
  DINUNET_GROUP_TILE=$t DINUNET_GROUP_SPLITS=$sp timeout -k 10 200 python bench.py --steps 200 --warmup 30 > gpurun_out/split_${t}_$sp.log 2>&1 || exit 5
  echo "tile=$t splits=$sp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/split_${t}_$sp.log)"
done
