#!/usr/bin/env bash
# Round 3: the exchange kernels' own cost on one GPU (C3 / C5 shard of an
# 8-GPU strong-scaled run), events and rocprofv3.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3xk
mkdir -p "$O"
timeout -k 10 200 python3 tools/exchange_kernels.py > "$O/exchange_kernels.txt" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
  python3 "$R/tools/exchange_kernels.py" > "$O/prof.log" 2>&1
echo done
