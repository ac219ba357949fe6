#!/usr/bin/env bash
# Round-3 closing GPU call on the committed tree: smoke, the default bench
# line (the driver's own command), and the whole GPU suite.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/end
mkdir -p "$O"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
timeout -k 10 300 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
echo done
