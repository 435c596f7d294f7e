#!/bin/bash
# Hard-cohort time-to-AUC study (signal 0.35, target 0.75): (a) bf16 fused kernels vs the fp32
# reference math, 1 site, several seeds; (b) the three engines at 2 sites (gloo ranks sharing
# the GPU: step counts comparable, wall-clock not).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=gpurun_out/tta_study.jsonl
COMMON="--cohort hard --effect 0.35 --target 0.75 --eval-every 50 --full"
if [ -z "$SKIP_FID" ]; then
for seed in ${SEEDS:-0 1 2}; do
  for cp in fused reference; do
    timeout -k 10 ${FID_LIMIT:-400} python tools/bench_time_to_auc.py $COMMON --max-steps ${FID_STEPS:-2000} --seed $seed --compute-path $cp > gpurun_out/tta_${cp}_$seed.log 2>&1 || { tail -20 gpurun_out/tta_${cp}_$seed.log; exit 3; }
    grep '"metric"' gpurun_out/tta_${cp}_$seed.log >> $OUT
    tail -1 gpurun_out/tta_${cp}_$seed.log | cut -c1-400
  done
done
fi
if [ -z "$SKIP_ENG" ]; then
for eng in dSGD rankDAD powerSGD; do
  DINUNET_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 tools/bench_time_to_auc.py $COMMON --max-steps ${ENG_STEPS:-3000} --engine $eng > gpurun_out/tta_eng_$eng.log 2>&1 || { tail -20 gpurun_out/tta_eng_$eng.log; exit 4; }
  grep '"metric"' gpurun_out/tta_eng_$eng.log >> $OUT
  grep '"metric"' gpurun_out/tta_eng_$eng.log | cut -c1-400
done
fi
