#!/bin/bash
# round 6: the peer exchange with fence mode 3 (release = store drain only, system-scope payload
# loads) through the multi-process correctness suite, then the loopback step times
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
export DINUNET_PEER_MODE=3 DINUNET_ERR_LOG=gpurun_out/r6_mode3_errlog.jsonl; : > $DINUNET_ERR_LOG
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_peer_gpu.py > gpurun_out/r6_m3_peer.log 2>&1 || { tail -30 gpurun_out/r6_m3_peer.log; exit 3; }
timeout -k 10 700 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_multirank_gpu.py -k "peer or 16" > gpurun_out/r6_m3_mr.log 2>&1 || { tail -30 gpurun_out/r6_m3_mr.log; exit 3; }
tail -1 gpurun_out/r6_m3_mr.log
OUT=gpurun_out/r6_mode3_bench.jsonl; : > $OUT
for m in 2 3 2 3; do
  DINUNET_PEER_MODE=$m timeout -k 10 120 python bench.py --steps 300 --warmup 30 --site-loop 0 --loopback-rccl --precision-bits 16 > gpurun_out/r6_lb.out 2> gpurun_out/r6_lb.err || { tail -5 gpurun_out/r6_lb.err; exit 4; }
  python -c "import json;r=json.loads([l for l in open('gpurun_out/r6_lb.out') if l.startswith('{')][-1]);print(json.dumps({'mode':$m,'ms':r['ms_per_step']}))" >> $OUT
done
cat $OUT
