#!/bin/bash
# observe the multi-site oracle errors of every engine / wire (tolerances set from these)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
out=gpurun_out/oracle_obs.jsonl; rm -f $out
port=29600
while read -r w args; do
  port=$((port+1))
  DINUNET_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 150 python -m torch.distributed.run --nnodes 1 --nproc-per-node $w --master-addr 127.0.0.1 --master-port $port tools/multirank_check.py $args --oracle --oracle-tol 1e9 --grad-tol 1e9 > gpurun_out/oracle_case.log 2>&1
  rc=$?
  line=$(grep '^{' gpurun_out/oracle_case.log | tail -1)
  echo "{\"w\": $w, \"args\": \"$args\", \"rc\": $rc, \"res\": ${line:-null}}" >> $out
  echo "w$w $args rc=$rc $(echo "$line" | grep -o '"grad_rel_err": [0-9.e-]*\|"update_rel_err": [0-9.e-]*' | tr '\n' ' ')"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && { tail -20 gpurun_out/oracle_case.log; exit 1; }
done <<'CASES'
2 --engine dSGD --precision 32
2 --engine dSGD --precision 16
3 --engine dSGD --precision 16 --ragged
2 --engine dSGD --precision 16 --payload bf16
2 --engine dSGD --precision 16 --collective allreduce
2 --engine rankDAD --precision 32 --dad-tol 0
3 --engine rankDAD --precision 32 --dad-tol 0
2 --engine rankDAD --precision 16 --dad-tol 0
2 --engine powerSGD --precision 32
3 --engine powerSGD --precision 32
2 --engine powerSGD --precision 16
2 --engine powerSGD --precision 32 --accum 2
CASES
exit 0
