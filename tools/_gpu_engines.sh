#!/bin/bash
# bench.py for every engine (1 GPU), one JSON line each -> gpurun_out/bench_engines.jsonl
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
: > gpurun_out/bench_engines.jsonl
for e in dSGD rankDAD powerSGD; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 20 --engine $e > gpurun_out/bench_$e.log 2>&1 || { tail -20 gpurun_out/bench_$e.log; exit 3; }
  grep '^{' gpurun_out/bench_$e.log >> gpurun_out/bench_engines.jsonl
done
python - <<'PY'
import json
for l in open("gpurun_out/bench_engines.jsonl"):
    d = json.loads(l); print(d["config"]["engine"], d["ms_per_step"], d["value"])
PY
