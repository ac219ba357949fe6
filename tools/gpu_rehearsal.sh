# Multi-rank bench rehearsal: 4 ranks sharing the one GPU over gloo (GPU box).
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/rehearsal; mkdir -p $O
for W in project sum group topk; do
  P=$((29600 + RANDOM % 300))
  WARPDB_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port $P bench.py --gpus 4 --rows 2.5e8 --steps 5 --warmup 2 --workload $W \
    > $O/bench_4rank_$W.log 2>&1
done
echo ok
