#!/usr/bin/env bash
# Round 3: the one-collective GROUP BY exchange and the top-K merge kernel on
# the GPU box -- their GPU tests, the multi-rank bench rehearsal (2 ranks on
# one GPU over gloo), the C++ virtual-shard path, and the high-cardinality
# GROUP BY baseline (1e6 keys).  Each GPU step has its own limit; the first
# failure ends the script.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3x
mkdir -p "$O"
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_exchange.py > "$O/pytest_exchange.log" 2>&1
timeout -k 10 500 $PYT tests/test_gpu_multi.py > "$O/pytest_multi.log" 2>&1
timeout -k 10 600 $PYT tests/test_warpdb_api.py -k "two_ranks" > "$O/pytest_two_ranks.log" 2>&1
timeout -k 10 300 python3 bench.py --workload group --rows 1e8 --keys 1000000 --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_group_1e6keys_1e8.json" 2> "$O/bench_group_1e6keys_1e8.err"
echo done
