#!/bin/bash
# Round 6: peer exchange with the fused reduce + unpack launch -- correctness (peer_check, the
# multi-rank oracle cases through the exchange, the captured-step tests) and loopback timings
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
export DINUNET_ERR_LOG=gpurun_out/r6_errlog2.jsonl; : > $DINUNET_ERR_LOG
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_peer_gpu.py > gpurun_out/r6_peer3.log 2>&1 || { tail -30 gpurun_out/r6_peer3.log; exit 3; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_multirank_gpu.py -k "peer or 16" > gpurun_out/r6_mr2.log 2>&1 || { tail -40 gpurun_out/r6_mr2.log; exit 3; }
tail -2 gpurun_out/r6_mr2.log
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_step_gpu.py -k "comm_graph" > gpurun_out/r6_step_comm2.log 2>&1 || { tail -30 gpurun_out/r6_step_comm2.log; exit 3; }
tail -2 gpurun_out/r6_step_comm2.log
SKIP_TESTS=1 bash tools/_gpu_r6_peer.sh
