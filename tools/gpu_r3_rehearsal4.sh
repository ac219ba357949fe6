#!/usr/bin/env bash
# Round 3, session 2: the default bench (all secondary lines and checks) with
# 4 gloo ranks sharing the one GPU, reduced sizes; then 4-rank many-key GROUP BY.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/rehearsal4
mkdir -p "$O"
WARPDB_BENCH_VERBOSE=1 WARPDB_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 4 --rows 1e8 --c4-rows 8e8 \
  --c3-rows 1e8 --steps 5 --warmup 2 > "$O/default_4rank.json" 2> "$O/default_4rank.err"
WARPDB_BENCH_VERBOSE=1 WARPDB_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --workload group --keys 200000 \
  --rows 3e7 --steps 3 --warmup 1 --no-cpu-baseline > "$O/group_200k_4rank.json" 2> "$O/group_200k_4rank.err"
echo done
