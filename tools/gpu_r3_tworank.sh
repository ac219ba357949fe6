#!/usr/bin/env bash
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/tworank
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_warpdb_api.py \
  -k "two_ranks" > "$O/pytest_two_ranks.log" 2>&1
echo done
