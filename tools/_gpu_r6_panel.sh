#!/bin/bash
# row-panel projection kernel + deep rings of the 256 x 256 GEMM: GPU tests, projection timing,
# B=2048 / 4096 step A/B, rocprof timeline of the B=2048 step
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "panel or gemm256" --timeout 200 --timeout-method thread > gpurun_out/r6_panel_test.log 2>&1 || { tail -40 gpurun_out/r6_panel_test.log; exit 1; }
tail -2 gpurun_out/r6_panel_test.log
timeout -k 10 200 python tools/panel_time.py 32,512,2048,4096 > gpurun_out/r6_panel_time.jsonl 2>&1 || { tail -20 gpurun_out/r6_panel_time.jsonl; exit 2; }
cat gpurun_out/r6_panel_time.jsonl
run() {  # B PANEL RING
  DINUNET_PANEL=$2 DINUNET_G256_RING=$3 timeout -k 10 300 python bench.py --batch $1 --pool 8 --site-loop 0 --steps 20 --warmup 5 > gpurun_out/r6_pb_$1_$2_$3.log 2>&1 || { tail -20 gpurun_out/r6_pb_$1_$2_$3.log; return 3; }
  echo "B=$1 panel=$2 ring=$3 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_pb_$1_$2_$3.log) $(grep -o '"value": [0-9.]*' gpurun_out/r6_pb_$1_$2_$3.log)" | tee -a gpurun_out/r6_panel_ab.txt
}
rm -f gpurun_out/r6_panel_ab.txt
run 2048 0 2x64 && run 2048 1 2x64 && run 2048 1 4x32 && run 2048 1 5x32 && run 4096 0 2x64 && run 4096 1 4x32 && run 4096 1 5x32 && run 32 0 2x64 && run 32 1 2x64 || exit 3
cd /tmp && DINUNET_G256_RING=4x32 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r6_b2048p -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 2048 --pool 8 --site-loop 0 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_r6_b2048p.log 2>&1 || exit 5
cd $GRAFT_REPO_ROOT && python tools/timeline.py gpurun_out/prof_r6_b2048p/run_kernel_trace.csv > gpurun_out/r6_b2048p_timeline.txt && cat gpurun_out/r6_b2048p_timeline.txt
