#!/usr/bin/env bash
# Round 3: the new radix defaults (atomic ranking + folded slot base) against
# the round-2 ranking on one box, keys and pairs, plus the sort GPU tests.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3rk
mkdir -p "$O"
timeout -k 10 300 python3 tools/ab_sort_rank.py 1e9 keys 0 ";WX_RS_RANK_ATOMIC=0,WX_RS_FOLD_LD=0;WX_RS_FOLD_LD=0" > "$O/abl_new_keys.txt" 2>&1
timeout -k 10 300 python3 tools/ab_sort_rank.py 1e9 pairs 0 ";WX_RS_RANK_ATOMIC=0,WX_RS_FOLD_LD=0" > "$O/abl_new_pairs.txt" 2>&1
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "sort or order or topk or limit" > "$O/pytest_sort.log" 2>&1
echo done
