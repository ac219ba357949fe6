#!/usr/bin/env bash
# C2 (1e8 rows): compaction tile size (row quads per thread x data waves) A/B,
# alternating, each a full bench line.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/c2tile
mkdir -p "$O"
for r in 1 2; do
  for v in "4 12" "2 12" "3 12" "4 8" "2 8"; do
    set -- $v
    WARPDB_COMPACT_GROUPS=$1 WARPDB_COMPACT_DWAVES=$2 timeout -k 10 200 python3 bench.py --rows 1e8 --steps 100 \
      --warmup 20 --no-cpu-baseline --no-secondary > "$O/c2_g$1_w$2_r$r.json" 2> "$O/c2_g$1_w$2_r$r.err"
  done
done
echo done
