#!/usr/bin/env bash
# Round 3: C3 GROUP BY grid density / unroll A/B at 1.25e8 and 1e9 rows.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3grp
mkdir -p "$O"
timeout -k 10 500 python3 tools/ab_group_grid.py 1.25e8,1e9 "2:2:512,2:1:512,3:2:512,2:3:512,4:4:256,3:1:512" > "$O/ab_group_grid4.txt" 2>&1
echo done
