#!/usr/bin/env bash
# Radix key passes: look-back poll spacing (s_sleep 0 / 1 / 2) and window
# (2 / 3 words per round), alternating, 1e9 float keys.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/s9
mkdir -p "$O"
AB_ROUNDS=4 timeout -k 10 600 python3 tools/ab_sort_rank.py 1e9 keys 0 \
  "WX_RS_SLEEP=1;WX_RS_SLEEP=0;WX_RS_SLEEP=2;WARPDB_RS_LBW=3" > "$O/abl_sort_sleep_lbw.txt" 2>&1
echo done
