#!/usr/bin/env bash
# Which code objects the default bench and the sort / many-key lines compile
# on a fresh box (cache misses of the in-tree .kernel_cache), and their wall time.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/s8
mkdir -p "$O"
export WARPDB_DEBUG=1 WARPDB_BENCH_VERBOSE=1
s=$(date +%s)
timeout -k 10 300 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err"
e=$(date +%s)
echo "bench.py wall seconds: $((e - s))" > "$O/bench_wall.txt"
s=$(date +%s)
timeout -k 10 300 python3 bench.py > "$O/bench_default2.json" 2> "$O/bench_default2.err"
e=$(date +%s)
echo "bench.py second run wall seconds: $((e - s))" >> "$O/bench_wall.txt"
timeout -k 10 200 python3 bench.py --workload sort --steps 10 --no-cpu-baseline > "$O/bench_sort.json" 2> "$O/bench_sort.err"
echo done
