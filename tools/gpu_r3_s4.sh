#!/usr/bin/env bash
# Round 3, session 2: persistent key tiles (next ticket + next keys in flight
# during the tile) -- sort GPU tests, A/B against one tile per workgroup,
# the sort bench line.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/s4
mkdir -p "$O"
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests -m gpu -k "sort or order or limit" > "$O/pytest_sort.log" 2>&1
AB_ROUNDS=4 timeout -k 10 500 python3 tools/ab_sort_rank.py 1e9 keys 0 "WARPDB_RS_PERSIST=1;WARPDB_RS_PERSIST=0" \
  > "$O/abl_sort_persist.txt" 2>&1
AB_ROUNDS=2 timeout -k 10 300 python3 tools/ab_sort_rank.py 1e8 keys 0 "WARPDB_RS_PERSIST=1;WARPDB_RS_PERSIST=0" \
  > "$O/abl_sort_persist_1e8.txt" 2>&1
timeout -k 10 200 python3 bench.py --workload sort --steps 10 --no-cpu-baseline > "$O/bench_sort.json" 2> "$O/bench_sort.err"
echo done
