cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_head_gpu.py -q -m gpu > gpurun_out/pytest_head.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_head.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TESTS="tests/test_kernels_gpu.py" bash tools/gpu_quick.sh
