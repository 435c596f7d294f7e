#!/bin/bash
# A/B probe of step-time knobs: one bench.py run per line of PROBES (env assignments), printing
# ms_per_step for each (bench: device feed, HIP graphs, no site loop)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
out=gpurun_out/probe.jsonl; rm -f $out
while read -r line; do
  [ -z "$line" ] && continue
  env $line timeout -k 10 200 python bench.py --steps ${STEPS:-100} --warmup 20 --site-loop 0 ${BENCH_ARGS} > gpurun_out/probe_case.log 2>&1
  rc=$?
  ms=$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/probe_case.log | tail -1)
  echo "{\"env\": \"$line\", \"rc\": $rc, ${ms:-\"ms_per_step\": null}}" | tee -a $out
  [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && { tail -20 gpurun_out/probe_case.log; exit 1; }
done <<< "${PROBES}"
exit 0
