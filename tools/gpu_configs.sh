#!/bin/bash
# BASELINE.json configs measurable on one MI355X: bench.py per engine (config 2 / the 1-site
# point of configs 3-4), wall-clock to target AUC, and pretrain->finetune on a site runtime.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out/configs
O=gpurun_out/configs
for e in dSGD rankDAD powerSGD; do
  timeout -k 10 300 python bench.py --engine $e --steps 50 --warmup 10 > $O/bench_$e.log 2>&1 || { tail -20 $O/bench_$e.log; exit 3; }
  grep metric $O/bench_$e.log | cut -c1-400
done
timeout -k 10 300 python tools/bench_time_to_auc.py > $O/tta_dsgd.log 2>&1 || { tail -20 $O/tta_dsgd.log; exit 4; }
tail -1 $O/tta_dsgd.log | cut -c1-600
timeout -k 10 300 python tools/bench_time_to_auc.py --engine rankDAD > $O/tta_rankdad.log 2>&1 || { tail -20 $O/tta_rankdad.log; exit 5; }
tail -1 $O/tta_rankdad.log | cut -c1-600
