#!/bin/bash
# Rehearsal of the N>1 bench path on a 1-GPU box: 2 ranks share the GPU over gloo (split capture,
# bucketed all-reduce between the graph replays, eager Adam).  Not a throughput number.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
DINUNET_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 \
  > gpurun_out/rehearse2.log 2>&1 || { tail -40 gpurun_out/rehearse2.log; exit 6; }
grep metric gpurun_out/rehearse2.log
