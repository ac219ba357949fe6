#!/usr/bin/env bash
# Final bench lines with bench.py's device kernel arguments: default, sort,
# C3 strong per-rank size (one-rank RCCL), and the multi-rank bench tests.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/final2
mkdir -p "$O"
s=$(date +%s)
timeout -k 10 300 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err"
e=$(date +%s)
echo "bench.py wall seconds: $((e - s))" > "$O/bench_wall.txt"
timeout -k 10 200 python3 bench.py --workload sort --steps 10 --no-cpu-baseline > "$O/bench_sort.json" 2> "$O/bench_sort.err"
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29631 WARPDB_EXCHANGE_ONE_RANK=1 \
  timeout -k 10 200 python3 bench.py --workload group --total-rows 1.25e8 --steps 200 --warmup 50 --no-cpu-baseline \
  > "$O/bench_c3s_125e8_rccl1.json" 2> "$O/bench_c3s_125e8_rccl1.err"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_exchange.py \
  tests/test_warpdb_api.py -k "bench" > "$O/pytest_bench.log" 2>&1
echo done
