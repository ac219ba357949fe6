#!/usr/bin/env bash
# Round 3, session 2: persistent radix key tiles with the next ticket taken
# after the look-back (A/B against one tile per workgroup), sort tests.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/s6
mkdir -p "$O"
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests -m gpu -k "sort or order or limit" > "$O/pytest_sort.log" 2>&1
AB_ROUNDS=4 timeout -k 10 500 python3 tools/ab_sort_rank.py 1e9 keys 0 "WARPDB_RS_PERSIST=1;WARPDB_RS_PERSIST=0" \
  > "$O/abl_sort_persist_late.txt" 2>&1
echo done
