#!/usr/bin/env bash
# Round 3: on top of the atomic ranking -- the permutation's slot base folded
# into the per-wave counts (WX_RS_FOLD_LD), and smaller tiles at three
# workgroups per CU (the LDS budget allows it at 16 keys per lane).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3rk
mkdir -p "$O"
timeout -k 10 400 python3 tools/ab_sort_rank.py 1e9 keys 0 ";WX_RS_FOLD_LD=1;WX_RS_FOLD_LD=1,WARPDB_RS_ITEMS=16,WX_RS_MINW=6;WX_RS_FOLD_LD=1,WARPDB_RS_ITEMS=24" > "$O/abl_fold_keys.txt" 2>&1
timeout -k 10 300 python3 tools/ab_sort_rank.py 1e9 pairs 0 ";WX_RS_FOLD_LD=1" > "$O/abl_fold_pairs.txt" 2>&1
echo done
