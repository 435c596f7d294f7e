#!/bin/bash
# LSTM numerics tests, then bench.py A/B over an env switch (AB_VAR, default DINUNET_LSTM_BWD_KS)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
V=${AB_VAR:-DINUNET_LSTM_BWD_KS}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_step_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "${TK:-lstm or step}" > gpurun_out/pt_ab.log 2>&1; rc=$?
tail -2 gpurun_out/pt_ab.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pt_ab.log | head -30; exit $rc; }
for rep in 1 2; do for val in 0 1; do
env $V=$val timeout -k 10 120 python bench.py --steps 200 --warmup 20 > gpurun_out/ab_$val.log 2>&1 || { tail -5 gpurun_out/ab_$val.log; exit 3; }
echo "$V=$val: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$val.log)"
done; done
