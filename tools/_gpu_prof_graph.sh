cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/gprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/gprof.log 2>&1 || exit 4
grep metric $GRAFT_REPO_ROOT/gpurun_out/gprof.log
