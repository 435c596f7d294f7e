#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/rankdad_error.py --steps ${STEPS:-600} --svd-every 50 --seed ${SEED:-0} > gpurun_out/r6_rankdad_err.json 2> gpurun_out/r6_rankdad_err.log; echo "rc=$?"
tail -3 gpurun_out/r6_rankdad_err.log
python -c "
import json
d=json.loads(open('gpurun_out/r6_rankdad_err.json').read())
for m in ('dsgd','rankdad','rankdad_tol0','svd'):
    r=d.get(m)
    if not r: continue
    print(m, 'final', r['final_auc'], 'best', r['best_auc'], 'wall', r['wall_s'])
    for k,v in r['err_engine'].items(): print('  eng', k, v, 'svd', r['err_svd_opt'].get(k), 'tail', r['energy_beyond_rank'].get(k))
"
