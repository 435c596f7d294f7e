#!/bin/bash
# LDS / MFMA / VALU activity of the fused head kernels (two counter passes, each its own run)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmch
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmch/a -o l -- python3 $GRAFT_REPO_ROOT/tools/head_one.py 5 > $GRAFT_REPO_ROOT/gpurun_out/pmch/a.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmch/a.log; exit 4; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_MISC SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmch/b -o l -- python3 $GRAFT_REPO_ROOT/tools/head_one.py 5 > $GRAFT_REPO_ROOT/gpurun_out/pmch/b.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmch/b.log; exit 5; }
echo pmc-ok
