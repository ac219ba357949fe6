#!/usr/bin/env bash
# Round 3: atomic ranking x folded slot base, 2 x 2, rotating order, 8 rounds.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3rk
mkdir -p "$O"
AB_ROUNDS=8 timeout -k 10 500 python3 tools/ab_sort_rank.py 1e9 keys 0 ";WX_RS_FOLD_LD=0;WX_RS_RANK_ATOMIC=0;WX_RS_RANK_ATOMIC=0,WX_RS_FOLD_LD=0" > "$O/abl_2x2_keys.txt" 2>&1
echo done
