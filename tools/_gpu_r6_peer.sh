#!/bin/bash
# Round 6: the peer exchange inside the captured N>1 step on one GPU (loopback group) -- the
# comm_graph GPU tests, bench variants (N=1 vs loopback: RCCL all-reduce / peer fp32 / peer fp16 /
# calibrate) and a kernel-trace timeline of the loopback fp16 step.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
set -o pipefail
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_step_gpu.py -k "comm_graph" > gpurun_out/r6_step_comm.log 2>&1 || { tail -30 gpurun_out/r6_step_comm.log; exit 3; }
tail -3 gpurun_out/r6_step_comm.log
fi
OUT=gpurun_out/r6_loopback_bench.jsonl
: > $OUT
for args in "" "--loopback-rccl" "--loopback-rccl --collective peer" "--loopback-rccl --precision-bits 16" "--loopback-rccl --collective calibrate" ""; do
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 --site-loop 0 $args > gpurun_out/r6_lb.out 2> gpurun_out/r6_lb.err || { tail -20 gpurun_out/r6_lb.err; exit 4; }
  python - "$args" >> $OUT <<'EOF'
import json, sys
rec = json.loads([l for l in open("gpurun_out/r6_lb.out") if l.startswith("{")][-1])
print(json.dumps({"args": sys.argv[1], "ms_per_step": rec["ms_per_step"], "value": rec["value"],
                  "comm_graph": rec["comm_graph"], "collective": rec["collective"],
                  "split": rec["split_backward"], "parallelism": rec["config"]["parallelism"]}))
EOF
  tail -1 $OUT
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r6_lb16 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --site-loop 0 --loopback-rccl --precision-bits 16 > $GRAFT_REPO_ROOT/gpurun_out/prof_r6_lb16.log 2>&1 || exit 5
cd $GRAFT_REPO_ROOT && python tools/timeline.py gpurun_out/prof_r6_lb16/run_kernel_trace.csv > gpurun_out/r6_lb16_timeline.txt && cat gpurun_out/r6_lb16_timeline.txt
