cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sprof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_gemm_sweep.py > $GRAFT_REPO_ROOT/gpurun_out/sprof.log 2>&1 || exit 4
echo ok
