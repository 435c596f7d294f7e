cd $GRAFT_REPO_ROOT
for args in "--graph 0 --overlap 0" "--graph 0 --overlap 1 --diag" "--graph 1 --split 0 --overlap 0" "--graph 0 --overlap 0 --batch 8 --seq 6"; do
  DINUNET_BACKEND=gloo timeout -k 10 100 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29$((RANDOM%900+100)) tools/multirank_check.py $args 2>/dev/null | grep "^{" || echo "FAIL $args"
done
