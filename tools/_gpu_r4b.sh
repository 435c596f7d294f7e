#!/bin/bash
# round-4 session 2: big-tile GEMM tests + shape sweep at B=2048, comm model, multirank oracle tests
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "${KSEL:-pre_activations or lstm_fwd_bwd or vector_epilogue or grouped_matches}" -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/bigtile_tests.log 2>&1 || { tail -30 gpurun_out/bigtile_tests.log; exit 1; }
tail -2 gpurun_out/bigtile_tests.log
if [ -n "${PROBES}" ]; then
  bash tools/_gpu_probe.sh || exit 5
fi
if [ "${SWEEP:-0}" = "1" ]; then
  timeout -k 10 400 python -u tools/bench_gemm.py --rows 200704 --tiles 1 2 3 --splits ${SPL:-1 8 16} --out-bf16 > gpurun_out/gemm_b2048.log 2>&1 || { tail -20 gpurun_out/gemm_b2048.log; exit 2; }
  cat gpurun_out/gemm_b2048.log
fi
if [ "${COMM:-1}" = "1" ]; then
  timeout -k 10 200 python tools/comm_model.py --out gpurun_out/r4_comm_model.md > gpurun_out/comm_model.log 2>&1 || { tail -20 gpurun_out/comm_model.log; exit 3; }
  head -30 gpurun_out/r4_comm_model.md
fi
if [ "${RUNPY:-0}" = "1" ]; then
  timeout -k 10 400 python -u tools/runpy_rate.py --out gpurun_out/r4_runpy_rate.json > gpurun_out/runpy.log 2>&1 || { tail -20 gpurun_out/runpy.log; exit 4; }
  tail -1 gpurun_out/runpy.log
fi
if [ "${MR:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/mr.log 2>&1; rc=$?
  grep -E "PASS|FAIL|passed|failed" gpurun_out/mr.log | tail -30
  exit $rc
fi
