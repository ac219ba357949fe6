#!/usr/bin/env bash
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/facade
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_exchange.py \
  -k "warpdb_multi" > "$O/pytest_facade.log" 2>&1
echo done
