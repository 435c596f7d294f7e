cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_head_gpu.py -q -m gpu > gpurun_out/pytest_head.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_head.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/bench_head.py > gpurun_out/bench_head.log 2>&1; rc=$?; cat gpurun_out/bench_head.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench.log 2>&1 || exit 3
grep metric gpurun_out/bench.log
