#!/usr/bin/env bash
# Radix key passes: speculative first loads of tile blockIdx.x beside the ticket (WX_RS_SPEC), A/B; sort tests on it.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/spec
mkdir -p "$O"
AB_ROUNDS=3 timeout -k 10 600 python3 tools/ab_sort_rank.py 1e9 keys 0 \
  ";WX_RS_SPEC=1;WX_RS_SPEC=1,WARPDB_RS_LBW=2" > "$O/abl_sort_spec.txt" 2>&1
WARPDB_EXTRA_DEFINES=WX_RS_SPEC=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests -m gpu -k "sort or order or limit" > "$O/pytest_sort_spec.log" 2>&1
echo done
