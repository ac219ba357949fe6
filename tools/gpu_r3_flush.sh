#!/usr/bin/env bash
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3fl
mkdir -p "$O"
timeout -k 10 300 python3 tools/ab_group_flush.py > "$O/ab_group_flush.txt" 2>&1
echo done
