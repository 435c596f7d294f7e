cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
OUT=gpurun_out/r6_peer_mode_ab.jsonl; : > $OUT
for m in 0 3; do
  DINUNET_PEER_MODE=$m timeout -k 10 100 python -m torch.distributed.run --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 2957$m tools/peer_check.py --wire all > gpurun_out/r6_pc.out 2> gpurun_out/r6_pc.err; echo "peer_check mode $m rc=$?"; grep "^{" gpurun_out/r6_pc.out | sed "s/^{/{\"mode\": $m, /" >> $OUT
done
for m in 0 1 2 3 0; do
  DINUNET_PEER_MODE=$m timeout -k 10 100 python bench.py --steps 300 --warmup 30 --site-loop 0 --loopback-rccl --precision-bits 16 > gpurun_out/r6_lb.out 2> gpurun_out/r6_lb.err || { tail -5 gpurun_out/r6_lb.err; exit 4; }
  python -c "import json;r=json.loads([l for l in open('gpurun_out/r6_lb.out') if l.startswith('{')][-1]);print(json.dumps({'mode':$m,'ms':r['ms_per_step']}))" >> $OUT
done
cat $OUT
