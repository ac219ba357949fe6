#!/usr/bin/env bash
# Session-2 last GPU call: pair-sort look-back window A/B, then the whole GPU
# suite and smoke on the final tree.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/last
mkdir -p "$O"
AB_ROUNDS=3 timeout -k 10 500 python3 tools/ab_sort_rank.py 1e9 pairs 0 \
  "WARPDB_RS_LBW=4;WARPDB_RS_LBW=3;WARPDB_RS_LBW=5" > "$O/abl_sort_pairs_lbw.txt" 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
echo done
