#!/usr/bin/env bash
# Round 3: RCCL on a one-GPU box -- the multi-rank bench step, ResidentShards
# and WarpDB::query_multi_gpu_* with a one-rank communicator
# (WARPDB_EXCHANGE_ONE_RANK=1), plus the thermal check of the secondary
# GROUP BY line.  Each GPU step has its own limit; the first failure ends it.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3r
mkdir -p "$O"
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_gpu_exchange.py -k "one_rank or one_device" > "$O/pytest_rccl_one_rank.log" 2>&1
timeout -k 10 300 python3 tools/thermal_group.py > "$O/thermal_group.txt" 2>&1
echo done
