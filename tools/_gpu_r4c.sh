#!/bin/bash
# round-4 large-batch iteration: GEMM tests, B=2048 A/B probes, GEMM shapes vs hipBLASLt, B=32 bench
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
if [ -n "${TESTS}" ]; then
  timeout -k 10 ${TTIME:-500} python -u -m pytest ${TESTS} -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  grep -E "passed|failed|FAIL|ERROR" gpurun_out/pytest_gpu.log | tail -15
  [ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
fi
if [ -n "${PROBES}" ]; then
  BENCH_ARGS="${PBENCH_ARGS}" STEPS=${PSTEPS:-30} bash tools/_gpu_probe.sh || exit 5
fi
if [ "${SHAPES:-0}" = "1" ]; then
  timeout -k 10 300 python -u tools/bench_gemm.py --rows 200704 --tiles 1 --splits 1 --out-bf16 > gpurun_out/gemm_shapes.log 2>&1 || { tail -20 gpurun_out/gemm_shapes.log; exit 6; }
  cat gpurun_out/gemm_shapes.log
fi
if [ "${GEMMONE:-0}" = "1" ]; then
  for f in 1 0; do
    DINUNET_COLSUM_FOLD=$f timeout -k 10 120 python tools/gemm_one.py dwstep 20 200704 || exit 7
  done
  for w in enc xp dx; do timeout -k 10 120 python tools/gemm_one.py $w 20 200704 || exit 7; done
fi
if [ "${PMC:-0}" = "1" ]; then
  R=$PWD; mkdir -p gpurun_out/pmcg; cd /tmp
  for w in ${PMC_SHAPES:-dwstep xp}; do
    timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $R/gpurun_out/pmcg/${w}_a -o g -- python3 $R/tools/gemm_one.py $w 5 200704 > $R/gpurun_out/pmcg/${w}_a.log 2>&1 || { tail -5 $R/gpurun_out/pmcg/${w}_a.log; exit 8; }
    timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcg/${w}_b -o g -- python3 $R/tools/gemm_one.py $w 5 200704 > $R/gpurun_out/pmcg/${w}_b.log 2>&1 || { tail -5 $R/gpurun_out/pmcg/${w}_b.log; exit 8; }
    timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/pmcg/${w}_c -o g -- python3 $R/tools/gemm_one.py $w 5 200704 > $R/gpurun_out/pmcg/${w}_c.log 2>&1 || { tail -5 $R/gpurun_out/pmcg/${w}_c.log; exit 8; }
  done
  cd $R; echo pmc-ok
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py --steps ${STEPS:-200} --warmup 20 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 3; }
  tail -1 gpurun_out/bench.log
fi
exit 0
