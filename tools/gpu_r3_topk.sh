#!/usr/bin/env bash
# C5 top-K scan: row quads per batch (WX_UNROLL) and workgroups per CU, bench lines, alternating.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/topk
mkdir -p "$O"
for r in 1 2; do
  for v in "8 2" "16 2" "12 2" "8 3" "16 3" "8 4"; do
    set -- $v
    WARPDB_EXTRA_DEFINES=WX_UNROLL=$1 WARPDB_GRID_PER_CU=$2 timeout -k 10 200 python3 bench.py --workload topk \
      --steps 50 --warmup 10 --no-cpu-baseline > "$O/topk_u$1_g$2_r$r.json" 2> "$O/topk_u$1_g$2_r$r.err"
  done
done
echo done
