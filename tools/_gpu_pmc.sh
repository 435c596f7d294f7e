cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmc
W=${W:-xp}
cd /tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VMEM_RD --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc/a -o $W -- python3 $GRAFT_REPO_ROOT/tools/gemm_one.py $W 20 > $GRAFT_REPO_ROOT/gpurun_out/pmc/a_$W.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc/a_$W.log; exit 4; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE TCP_TCC_READ_REQ_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc/b -o $W -- python3 $GRAFT_REPO_ROOT/tools/gemm_one.py $W 20 > $GRAFT_REPO_ROOT/gpurun_out/pmc/b_$W.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc/b_$W.log; exit 5; }
echo pmc-ok
