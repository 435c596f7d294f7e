#!/bin/bash
# Rehearsal of the N=8 bench path on a 1-GPU box: 8 ranks share the GPU over gloo (split capture,
# host-issued bucket collectives); checks the one-JSON-line contract at 8 ranks.  Not a throughput
# number (8 processes time-share one GPU and a CPU all-reduce).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for e in dSGD rankDAD powerSGD; do
  DINUNET_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port $((29700 + ${#e})) bench.py --gpus 8 --steps 10 --warmup 3 --engine $e \
    > gpurun_out/rehearse8_$e.log 2>&1 || { tail -40 gpurun_out/rehearse8_$e.log; exit 6; }
  grep -c '"metric"' gpurun_out/rehearse8_$e.log
  grep '"metric"' gpurun_out/rehearse8_$e.log | python -c "
import json,sys
d=json.loads(sys.stdin.read().splitlines()[0]); print(d['config']['engine'], d['n_gpus'], d['config']['parallelism'], d['ms_per_step'], d['value'])"
done
