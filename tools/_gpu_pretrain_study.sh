#!/bin/bash
# BASELINE config 5 on one GPU: 8 site processes (gloo, sharing cuda:0), pretrain vs scratch
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out/pt_profiles
timeout -k 10 ${LIMIT:-1080} python -u tools/ica_pretrain_study.py --sites ${SITES:-8} --big ${BIG:-4096} --small ${SMALL:-256} --epochs ${EPOCHS:-40} --patience ${PATIENCE:-12} --pretrain-batch ${PBATCH:-512} --work /tmp/ica_pretrain --profiles gpurun_out/pt_profiles --logdir gpurun_out/pt_logs ${EXTRA} > gpurun_out/pretrain_study.log 2>&1; rc=$?
tail -12 gpurun_out/pretrain_study.log
for m in scratch pretrain; do [ -f /tmp/ica_pretrain/$m.log ] && tail -5 /tmp/ica_pretrain/$m.log > gpurun_out/pretrain_$m.tail; done
exit $rc
