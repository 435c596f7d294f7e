cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k gemm > gpurun_out/pytest_gemm.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gemm.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python tools/bench_gemm.py > gpurun_out/gemm.log 2>&1 || exit 5
cat gpurun_out/gemm.log
bash tools/gpu_quick.sh
