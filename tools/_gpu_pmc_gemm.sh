#!/bin/bash
# counters of the grouped weight-gradient GEMM (inside tools/lstm_one.py's backward)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmcg
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcg/a -o g -- python3 $GRAFT_REPO_ROOT/tools/lstm_one.py 5 > $GRAFT_REPO_ROOT/gpurun_out/pmcg/a.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmcg/a.log; exit 4; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcg/b -o g -- python3 $GRAFT_REPO_ROOT/tools/lstm_one.py 5 > $GRAFT_REPO_ROOT/gpurun_out/pmcg/b.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmcg/b.log; exit 5; }
echo pmc-ok
