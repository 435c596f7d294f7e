#!/bin/bash
# grouped weight-gradient GEMM tiling A/B at a large batch (bench.py, env knobs of ops/gemm.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
B=${B:-2048}
for cfg in "" "DINUNET_GROUP_TILE=1" "DINUNET_GROUP_TILE=1 DINUNET_GROUP_SPLITS=24" "DINUNET_GROUP_TILE=1 DINUNET_GROUP_SPLITS=48" "DINUNET_GROUP_SPLITS=16"; do
  env $cfg timeout -k 10 120 python bench.py --steps 20 --warmup 5 --batch $B > gpurun_out/gab.log 2>&1 || { tail -5 gpurun_out/gab.log; exit 3; }
  echo "[$cfg] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gab.log)"
done
