#!/usr/bin/env bash
# Radix key + payload geometry / variant sweep (GPU box): one process each.
# usage: sweep_sort_pairs.sh "BLOCK ITEMS EXTRA_DEFINES" ...
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
for g in "$@"; do
  set -- $g
  echo "== block $1 items $2 ${3:-}" >> "$O/sweep_pairs.txt"
  WARPDB_RS_BLOCK=$1 WARPDB_RS_ITEMS=$2 WARPDB_EXTRA_DEFINES=${3:-} timeout -k 10 120 python3 -u "$R/tools/bench_sort.py" 1e9 0 2>&1 | grep pairs >> "$O/sweep_pairs.txt"
done
