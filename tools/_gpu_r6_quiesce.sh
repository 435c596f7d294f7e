#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 100 python tools/diag/capture_after_eager.py 30 > gpurun_out/r6_cae.out 2> gpurun_out/r6_cae.err; echo "capture_after_eager rc=$?"; cat gpurun_out/r6_cae.out
OUT=gpurun_out/r6_loopback_bench2.jsonl; : > $OUT
for args in "--loopback-rccl --collective calibrate" "--loopback-rccl --collective calibrate --precision-bits 16" "--loopback-rccl"; do
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 --site-loop 0 $args > gpurun_out/r6_lb.out 2> gpurun_out/r6_lb.err || { grep -v "^frame" gpurun_out/r6_lb.err | tail -5; exit 4; }
  python - "$args" >> $OUT <<'PY'
import json, sys
rec = json.loads([l for l in open("gpurun_out/r6_lb.out") if l.startswith("{")][-1])
print(json.dumps({"args": sys.argv[1], "ms_per_step": rec["ms_per_step"], "comm_graph": rec["comm_graph"], "collective": rec["collective"]}))
PY
  tail -1 $OUT
done
