#!/bin/bash
# round-5 ICA pretrain study: every site >= 1,024 validation subjects
# (split 0.1 / 0.8 / 0.1: site 0 10,240 subjects -> 1,024 train, sites 1..7 1,280 -> 128 train),
# 8 site processes sharing cuda:0 over gloo, SEEDS per call; per-run JSON under gpurun_out/pt5
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out/pt5
timeout -k 10 ${LIMIT:-1080} python -u tools/ica_pretrain_study.py --sites 8 --big 10240 --small 1280 \
  --split 0.1,0.8,0.1 --epochs 60 --patience 15 --lr 1e-4 --pretrain-lr 1e-3 --pretrain-batch 128 \
  --pretrain-epochs 40 --pretrain-patience 10 --seeds ${SEEDS:-11} --tag r5_ica_pretrain \
  --work /tmp/ica_pretrain5 --profiles gpurun_out/pt5 --logdir gpurun_out/pt5_logs \
  > gpurun_out/pretrain5.log 2>&1; rc=$?
tail -8 gpurun_out/pretrain5.log
exit $rc
