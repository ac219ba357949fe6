#!/usr/bin/env bash
# Round 3: C2's fixed cost -- kernel durations (rocprofv3) of the deep
# compaction at 1 tile per workgroup (3.1e6 rows), 1e8 and 1e9 rows, beside
# the workgroup timelines of the same sizes.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3c2b
mkdir -p "$O"
timeout -k 10 300 python3 tools/timeline_compact.py 3145728 1e8 > "$O/timeline.txt" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
  python3 "$R/tools/timeline_compact.py" 3145728 1e8 > "$O/prof.log" 2>&1
echo done
