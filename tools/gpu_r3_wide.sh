#!/usr/bin/env bash
# Round 3: GROUP BY with many distinct keys -- the partitioned path's GPU
# tests, then the bench at 1e8 / 1e9 rows x 1e6 keys, the hash path beside
# it (WARPDB_GROUP_PARTITION=0, 1e8 rows), and C3 (1K keys) unchanged.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3w
mkdir -p "$O"
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_group_wide.py > "$O/pytest_wide.log" 2>&1
B="python3 bench.py --workload group --no-cpu-baseline"
timeout -k 10 200 $B --rows 1e8 --keys 1000000 > "$O/bench_group_1e6k_1e8.json" 2> "$O/b1.err"
timeout -k 10 300 $B --rows 1e9 --keys 1000000 > "$O/bench_group_1e6k_1e9.json" 2> "$O/b2.err"
WARPDB_GROUP_PARTITION=0 timeout -k 10 200 $B --rows 1e8 --keys 1000000 --steps 3 > "$O/bench_group_1e6k_1e8_hash.json" 2> "$O/b3.err"
timeout -k 10 200 $B > "$O/bench_group_c3.json" 2> "$O/b4.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_wide" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload group --rows 1e9 --keys 1000000 --no-cpu-baseline --steps 5 > "$O/prof_wide.log" 2>&1
echo done
