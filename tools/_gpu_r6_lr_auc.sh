#!/bin/bash
# rank-dAD validation AUC, split-bf16 (default lib) vs fp32 MFMAs (variant lib), seeds 0-2
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for seed in ${SEEDS:-0 1 2}; do
  for lib in split f32; do
    if [ $lib = f32 ]; then export DINUNET_KERNEL_LIB=dinunet_implementations_amd/_native/ab/f32mfma.so DINUNET_ALLOW_STALE=1; else unset DINUNET_KERNEL_LIB DINUNET_ALLOW_STALE; fi
    timeout -k 10 120 python tools/rankdad_error.py --modes rankdad --svd-every 200 --seed $seed > gpurun_out/r6_lr_auc_${lib}_$seed.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/r6_lr_auc_${lib}_$seed.json'))['rankdad']; print('$lib seed $seed', d['final_auc'], d['best_auc'], d['err_engine']['encoder.0']['mean'])"
  done
done | tee -a gpurun_out/r6_lr_auc.txt
