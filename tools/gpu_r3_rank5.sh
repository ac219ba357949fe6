#!/usr/bin/env bash
# Round 3: atomic ranking x folded slot base, 2 x 2 with every variant
# explicit, rotating order, 6 rounds; pairs; then the sort GPU tests on the
# new defaults.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3rk
mkdir -p "$O"
AB_ROUNDS=6 timeout -k 10 500 python3 tools/ab_sort_rank.py 1e9 keys 0 "WX_RS_RANK_ATOMIC=1,WX_RS_FOLD_LD=1;WX_RS_RANK_ATOMIC=1,WX_RS_FOLD_LD=0;WX_RS_RANK_ATOMIC=0,WX_RS_FOLD_LD=1;WX_RS_RANK_ATOMIC=0,WX_RS_FOLD_LD=0" > "$O/abl_2x2b_keys.txt" 2>&1
AB_ROUNDS=4 timeout -k 10 400 python3 tools/ab_sort_rank.py 1e9 pairs 0 "WX_RS_RANK_ATOMIC=1,WX_RS_FOLD_LD=1;WX_RS_RANK_ATOMIC=0,WX_RS_FOLD_LD=0" > "$O/abl_2x2b_pairs.txt" 2>&1
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "sort or order or topk or limit" > "$O/pytest_sort_b.log" 2>&1
echo done
