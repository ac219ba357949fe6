#!/usr/bin/env bash
# Ranking-mode agreement test and the radix sort tests.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/lead
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "ranking_modes or sort" > "$O/pytest_sort.log" 2>&1
echo done
