#!/bin/bash
# round 6: bench.py as the driver launches it for N > 1 (torch.distributed.run, default
# --collective calibrate), rehearsed with N site processes sharing the one GPU over gloo
# (the IPC peer exchange competes against gloo's host-issued all-reduce)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=gpurun_out/r6_bench_gloo.jsonl; : > $OUT
for n in 2 4; do for prec in 32 16; do
  DINUNET_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2980$n bench.py --gpus $n --steps 40 --warmup 10 --precision-bits $prec > gpurun_out/r6_bg.out 2> gpurun_out/r6_bg.err || { grep -v "^frame" gpurun_out/r6_bg.err | tail -8; exit 4; }
  grep "^{" gpurun_out/r6_bg.out | python -c "
import json,sys
r=json.loads(sys.stdin.read().splitlines()[-1])
print(json.dumps({'n':r['n_gpus'],'prec':r['config']['precision_bits'],'ms':r['ms_per_step'],'value':r['value'],'comm_graph':r['comm_graph'],'collective':r['collective']}))" >> $OUT
  tail -1 $OUT
done; done
