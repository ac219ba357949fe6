#!/usr/bin/env bash
# Round 3: atomic ranking (WX_RS_RANK_ATOMIC) for key + payload pairs, with
# stability checks, over full-range, narrow and nearly constant keys.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3rk
mkdir -p "$O"
V=";WX_RS_RANK_ATOMIC=1"
timeout -k 10 300 python3 tools/ab_sort_rank.py 1e9 pairs 0 "$V" > "$O/abl_pairs_full.txt" 2>&1
timeout -k 10 200 python3 tools/ab_sort_rank.py 2e8 pairs 65536 "$V" > "$O/abl_pairs_64k.txt" 2>&1
timeout -k 10 200 python3 tools/ab_sort_rank.py 2e8 pairs 4 "$V" > "$O/abl_pairs_4.txt" 2>&1
echo done
