#!/usr/bin/env bash
# Round 3: the default bench with the secondary lines' time-based warm-up,
# then the headline alone with 3 and 30 warm-up steps (clock ramp check).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3w
mkdir -p "$O"
timeout -k 10 300 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err"
timeout -k 10 200 python3 bench.py --no-secondary --no-cpu-baseline --warmup 3 > "$O/bench_w3.json" 2> "$O/bench_w3.err"
timeout -k 10 200 python3 bench.py --no-secondary --no-cpu-baseline --warmup 30 > "$O/bench_w30.json" 2> "$O/bench_w30.err"
timeout -k 10 200 python3 bench.py --no-secondary --no-cpu-baseline --warmup 3 > "$O/bench_w3b.json" 2> "$O/bench_w3b.err"
echo done
