#!/bin/bash
# counters of the B=2048 step kernels (eager step, no graph: one dispatch per kernel per step) and
# the engine benches at the headline config
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out/pmc2048
R=$PWD
for e in rankDAD powerSGD; do
  timeout -k 10 300 python bench.py --engine $e --steps 200 --warmup 20 --site-loop 0 > gpurun_out/bench_$e.log 2>&1 || { tail -20 gpurun_out/bench_$e.log; exit 3; }
  tail -1 gpurun_out/bench_$e.log | cut -c1-400
done
cd /tmp
A="--batch 2048 --steps 3 --warmup 2 --site-loop 0 --graph 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $R/gpurun_out/pmc2048/a -o g -- python3 $R/bench.py $A > $R/gpurun_out/pmc2048/a.log 2>&1 || { tail -5 $R/gpurun_out/pmc2048/a.log; exit 4; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc2048/b -o g -- python3 $R/bench.py $A > $R/gpurun_out/pmc2048/b.log 2>&1 || { tail -5 $R/gpurun_out/pmc2048/b.log; exit 5; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/pmc2048/c -o g -- python3 $R/bench.py $A > $R/gpurun_out/pmc2048/c.log 2>&1 || { tail -5 $R/gpurun_out/pmc2048/c.log; exit 6; }
cd $R
python tools/pmc_summary.py "lstm_fwd|lstm_bwd|gemm_dma|adam_pack|headb_fwd" gpurun_out/pmc2048/a/g_counter_collection.csv gpurun_out/pmc2048/b/g_counter_collection.csv gpurun_out/pmc2048/c/g_counter_collection.csv > gpurun_out/pmc2048/summary.txt
echo pmc-ok
