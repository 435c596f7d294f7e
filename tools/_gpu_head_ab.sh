cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_head_gpu.py tests/test_step_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/head_tests.log 2>&1 && \
timeout -k 10 200 python tools/bench_head.py > gpurun_out/head2.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 200 --warmup 30 > gpurun_out/bench2.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 200 --warmup 30 >> gpurun_out/bench2.log 2>&1
