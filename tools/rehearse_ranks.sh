#!/usr/bin/env bash
# GPU box: the multi-rank bench path with N ranks sharing the one GPU over
# gloo (rank-ordered slots / records of N shards, max-over-ranks timing, each
# line's own check).  usage: bash tools/rehearse_ranks.sh TAG N
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-rehearsal}; N=${2:-4}
O=$R/gpurun_out/$TAG; mkdir -p "$O"
P=29611
for w in "project:--rows 2e7 --c4-rows 80000001 --c3-rows 40000001" "sum:--total-rows 80000001" "group:--rows 1e7" \
         "group_keys:--workload group --rows 4e6 --keys 100000" "topk:--rows 1e7"; do
  name=${w%%:*}; args=${w#*:}
  case $name in group_keys) wl="";; *) wl="--workload $name";; esac
  P=$((P + 1))
  t0=$(date +%s.%N)
  WARPDB_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
    --master-addr 127.0.0.1 --master-port $P bench.py --gpus "$N" $wl --steps 3 --warmup 1 $args \
    > "$O/${name}_${N}rank.json" 2> "$O/${name}_${N}rank.err" || { echo "$name failed"; exit 1; }
  t1=$(date +%s.%N)
  # wall time of the whole launch (torchrun start, N imports, data, warm-up, timed steps, checks)
  echo "$name ${N} ranks: $(awk "BEGIN{printf \"%.1f\", $t1 - $t0}") s wall" | tee -a "$O/wall_${N}rank.txt"
done
