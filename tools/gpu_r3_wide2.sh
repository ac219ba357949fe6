#!/usr/bin/env bash
# Round 3: the staged scatter of the partitioned GROUP BY -- tests, then
# 1e9 rows x 1e6 keys with the staged and the direct scatter, kernel stats.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3w2
mkdir -p "$O"
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_group_wide.py > "$O/pytest_wide.log" 2>&1
timeout -k 10 400 $PYT tests/test_gpu_multi.py -k "virtual_shards or resident_shards or topk" > "$O/pytest_multi_topk.log" 2>&1
B="python3 bench.py --workload group --no-cpu-baseline --no-check"
timeout -k 10 200 $B --rows 1e9 --keys 1000000 > "$O/bench_group_1e6k_1e9.json" 2> "$O/b1.err"
WARPDB_GP_STAGE=0 timeout -k 10 200 $B --rows 1e9 --keys 1000000 > "$O/bench_group_1e6k_1e9_direct.json" 2> "$O/b2.err"
timeout -k 10 200 $B --rows 1e9 --keys 100000 > "$O/bench_group_1e5k_1e9.json" 2> "$O/b3.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_wide" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload group --rows 1e9 --keys 1000000 --no-cpu-baseline --no-check --steps 5 > "$O/prof_wide.log" 2>&1
echo done
