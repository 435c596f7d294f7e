#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for r in 1 2; do
DINUNET_PEER_FUSED=1 DINUNET_PEER_TIMEOUT_MS=5000 DINUNET_BACKEND=gloo timeout -k 10 100 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2978$r tools/multirank_check.py --engine dSGD --precision 16 --ragged > gpurun_out/r6_rd.out 2> gpurun_out/r6_rd$r.err
echo "rc=$?"; grep "^# site" gpurun_out/r6_rd$r.err; grep -o '"peer_errors": .*' gpurun_out/r6_rd.out
done
