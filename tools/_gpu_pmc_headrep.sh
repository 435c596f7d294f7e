#!/bin/bash
# instruction mix / issue of the replicated head (head_rep.hip): counter passes, each
# its own run (tools/head_rep_stamps.py drives 35 launches)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmcr
R=$GRAFT_REPO_ROOT
cd /tmp
for k in ${KERNELS:-rep}; do
  T=$R/tools/head_rep_stamps.py
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmcr/${k}_a -o p -- python3 $T > $R/gpurun_out/pmcr/${k}_a.log 2>&1 || { tail -5 $R/gpurun_out/pmcr/${k}_a.log; exit 4; }
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC --output-format csv -d $R/gpurun_out/pmcr/${k}_b -o p -- python3 $T > $R/gpurun_out/pmcr/${k}_b.log 2>&1 || { tail -5 $R/gpurun_out/pmcr/${k}_b.log; exit 5; }
done
cd $R
for k in ${KERNELS:-rep}; do
  python3 tools/pmc_summary.py "head_rep_kernel" $(find gpurun_out/pmcr/${k}_a gpurun_out/pmcr/${k}_b -name "*counter_collection.csv") > gpurun_out/pmcr/${k}.txt
  cat gpurun_out/pmcr/${k}.txt
done
