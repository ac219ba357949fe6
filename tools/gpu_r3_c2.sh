#!/usr/bin/env bash
# Round 3: where C2's fixed cost goes (compaction timeline at 1e8 / 1e9 rows).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3c2
mkdir -p "$O"
timeout -k 10 300 python3 tools/timeline_compact.py 1e8 1e9 > "$O/timeline.txt" 2>&1
echo done
