#!/bin/bash
# device-fed multi-site diagnosis: multirank_check --feed device --oracle under both update forms
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for ap in 0 1; do
  for w in 1 2; do
    sp=""; [ $w = 1 ] && sp="--split 1"
    DINUNET_ADAM_PACK=$ap DINUNET_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node $w --master-addr 127.0.0.1 --master-port $((29600 + w + 10 * ap)) tools/multirank_check.py --engine dSGD --precision 32 --feed device --oracle $sp ${EXTRA} > gpurun_out/mr_feed_${ap}_$w.log 2>&1
    echo "apack=$ap world=$w rc=$? $(grep -o '"split.*' gpurun_out/mr_feed_${ap}_$w.log | cut -c1-400)"
  done
done
