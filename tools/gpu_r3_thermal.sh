#!/usr/bin/env bash
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3th
mkdir -p "$O"
timeout -k 10 300 python3 tools/thermal_group.py > "$O/thermal_group2.txt" 2>&1
echo done
