#!/usr/bin/env bash
# Round 3: radix ranking by one returning LDS add per key (WX_RS_RANK_ATOMIC)
# against the peer-mask ranking, 1e9 float keys, alternating, with the order check.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3rk
mkdir -p "$O"
timeout -k 10 400 python3 tools/ab_sort_pair.py 1e9 ";WX_RS_RANK_ATOMIC=1" > "$O/abl_sort_rank_atomic.txt" 2>&1
echo done
