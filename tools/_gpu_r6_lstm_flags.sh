#!/bin/bash
# round 6: the LDS-flag step hand-off re-measured now that the h reads are
# batched -- barrier (in-tree) vs flags (one read per k-step) vs flags with per-group read rounds
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
L=dinunet_implementations_amd/_native
timeout -k 10 200 python tools/lstm_time.py $L/libdinunet_kernels.so $L/ab/flags1.so $L/ab/flags2.so > gpurun_out/r6_lstm_flags.txt 2>&1; cat gpurun_out/r6_lstm_flags.txt | grep -v amdgpu.ids
for v in base flags2 base flags2; do
  if [ $v = base ]; then unset DINUNET_KERNEL_LIB; else export DINUNET_KERNEL_LIB=$L/ab/$v.so DINUNET_ALLOW_STALE=1; fi
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 --site-loop 0 > gpurun_out/r6_lb.out 2> gpurun_out/r6_lb.err || { tail -5 gpurun_out/r6_lb.err; exit 4; }
  python -c "import json;r=json.loads([l for l in open('gpurun_out/r6_lb.out') if l.startswith('{')][-1]);print('$v', r['ms_per_step'], r['final_loss'])"
done
