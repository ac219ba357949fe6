#!/usr/bin/env bash
# Round 3: where a radix key pass spends its time -- the full sort, without
# the key stores, without stores + look-back (loads, ranking, LDS
# permutation), and without ranking too (diagnostic builds, wrong results).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3sd
mkdir -p "$O"
timeout -k 10 500 python3 tools/ab_sort_pair.py 1e9 ";WX_RS_DIAG_NO_STORE=1;WX_RS_DIAG_NO_STORE=1,WX_RS_DIAG_NO_LOOKBACK=1;WX_RS_DIAG_NO_STORE=1,WX_RS_DIAG_NO_LOOKBACK=1,WX_RS_DIAG_NO_RANK=1" > "$O/abl_sort_diag3.txt" 2>&1
echo done
