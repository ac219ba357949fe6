#!/usr/bin/env bash
# Radix key passes: tile counts {A} published before the ranking (WX_RS_EARLY_A), A/B.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/s12
mkdir -p "$O"
AB_ROUNDS=3 timeout -k 10 600 python3 tools/ab_sort_rank.py 1e9 keys 0 \
  ";WX_RS_EARLY_A=1;WX_RS_EARLY_A=1,WARPDB_RS_LBW=2" > "$O/abl_sort_early_a.txt" 2>&1
echo done
