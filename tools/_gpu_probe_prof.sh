cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/probe -o run -- python3 $GRAFT_REPO_ROOT/tools/gemm_probe.py > $GRAFT_REPO_ROOT/gpurun_out/probe.log 2>&1 || exit 4
echo ok
