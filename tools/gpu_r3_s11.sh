#!/usr/bin/env bash
# Radix key passes at the new look-back window: keys per lane and window
# width around the defaults, alternating, 1e9 float keys; sort tests.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/s11
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  -k "sort or order or limit" > "$O/pytest_sort.log" 2>&1
AB_ROUNDS=3 timeout -k 10 600 python3 tools/ab_sort_rank.py 1e9 keys 0 \
  ";WARPDB_RS_ITEMS=30;WARPDB_RS_ITEMS=28;WARPDB_RS_LBW=4" > "$O/abl_sort_items_lbw.txt" 2>&1
echo done
