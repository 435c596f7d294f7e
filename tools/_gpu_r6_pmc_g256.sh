#!/bin/bash
# counters of the 256 x 256 GEMMs in the B=2048 step (eager step: one dispatch per kernel)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out/pmc256
R=$PWD
cd /tmp
A="--batch 2048 --steps 3 --warmup 2 --site-loop 0 --graph 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $R/gpurun_out/pmc256/a -o g -- python3 $R/bench.py $A > $R/gpurun_out/pmc256/a.log 2>&1 || { tail -5 $R/gpurun_out/pmc256/a.log; exit 4; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pmc256/b -o g -- python3 $R/bench.py $A > $R/gpurun_out/pmc256/b.log 2>&1 || { tail -5 $R/gpurun_out/pmc256/b.log; exit 5; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/pmc256/c -o g -- python3 $R/bench.py $A > $R/gpurun_out/pmc256/c.log 2>&1 || { tail -5 $R/gpurun_out/pmc256/c.log; exit 6; }
cd $R
python tools/pmc_summary.py "gemm256|gemm_dma" gpurun_out/pmc256/a/g_counter_collection.csv gpurun_out/pmc256/b/g_counter_collection.csv gpurun_out/pmc256/c/g_counter_collection.csv > gpurun_out/pmc256/summary.txt
cat gpurun_out/pmc256/summary.txt | head -120
