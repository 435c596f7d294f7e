#!/bin/bash
# round 6: the peer exchange as one unsplit exchange -- correctness suites, then loopback A/B
# against the split form (DINUNET_SPLIT_GRAPH=1)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
export DINUNET_ERR_LOG=gpurun_out/r6_unsplit_errlog.jsonl; : > $DINUNET_ERR_LOG
timeout -k 10 700 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_multirank_gpu.py -k "peer or 16" > gpurun_out/r6_us_mr.log 2>&1 || { tail -30 gpurun_out/r6_us_mr.log; exit 3; }
tail -1 gpurun_out/r6_us_mr.log
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_step_gpu.py -k "comm_graph" tests/test_health_gpu.py > gpurun_out/r6_us_step.log 2>&1 || { tail -30 gpurun_out/r6_us_step.log; exit 3; }
tail -1 gpurun_out/r6_us_step.log
OUT=gpurun_out/r6_peer_unsplit_ab.jsonl; : > $OUT
for v in "0 --loopback-rccl --precision-bits 16" "1 --loopback-rccl --precision-bits 16" "0 --loopback-rccl --collective peer" "1 --loopback-rccl --collective peer" "0 " "0 --loopback-rccl --precision-bits 16" "1 --loopback-rccl --precision-bits 16"; do
  set -- $v; sp=$1; shift
  if [ $sp = 1 ]; then export DINUNET_SPLIT_GRAPH=1; else unset DINUNET_SPLIT_GRAPH; fi
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 --site-loop 0 "$@" > gpurun_out/r6_lb.out 2> gpurun_out/r6_lb.err || { tail -5 gpurun_out/r6_lb.err; exit 4; }
  python - "$sp" "$*" >> $OUT <<'PY'
import json, sys
r = json.loads([l for l in open("gpurun_out/r6_lb.out") if l.startswith("{")][-1])
print(json.dumps({"split_env": sys.argv[1], "args": sys.argv[2], "ms_per_step": r["ms_per_step"], "split": r["split_backward"], "comm_graph": r["comm_graph"], "collective": r["collective"] if isinstance(r["collective"], str) else r["collective"].get("choice")}))
PY
  tail -1 $OUT
done
unset DINUNET_SPLIT_GRAPH
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r6_lb16b -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --site-loop 0 --loopback-rccl --precision-bits 16 > $GRAFT_REPO_ROOT/gpurun_out/prof_r6_lb16b.log 2>&1 || exit 5
cd $GRAFT_REPO_ROOT && python tools/timeline.py gpurun_out/prof_r6_lb16b/run_kernel_trace.csv > gpurun_out/r6_lb16b_timeline.txt && cat gpurun_out/r6_lb16b_timeline.txt
