#!/bin/bash
# config-5 study tuning: scratch-only federated runs at a few learning rates, to find a regime whose
# best-validation epoch falls in the tens
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out/pt_profiles
for lr in ${LRS:-1e-4 3e-5}; do
  timeout -k 10 ${LIMIT:-420} python -u tools/ica_pretrain_study.py --sites ${SITES:-8} --big ${BIG:-1024} --small ${SMALL:-128} --signal ${SIGNAL:-0.35} --epochs ${EPOCHS:-60} --patience ${PATIENCE:-15} --modes ${MODES:-scratch} --lr $lr --seeds ${SEEDS:-11} --work /tmp/ica_pt_$lr --profiles gpurun_out/pt_profiles --tag pt_tune_lr$lr --logdir gpurun_out/pt_logs_$lr ${EXTRA} > gpurun_out/pt_tune_$lr.log 2>&1; rc=$?
  echo "lr $lr rc=$rc"; grep -E "^seed|^\| (scratch|pretrain)" gpurun_out/pt_tune_$lr.log | tail -6
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
  rm -rf /tmp/ica_pt_$lr
done
exit 0
