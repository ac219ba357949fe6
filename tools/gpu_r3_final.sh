#!/usr/bin/env bash
# Round 3, session 2, final checkpoint: smoke, the whole GPU suite, the
# default bench line (wall time), sort, C3 strong at 1.25e8 per rank and the
# many-key GROUP BY on a one-rank RCCL communicator, rocprofv3 kernel stats.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/final
mkdir -p "$O"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
s=$(date +%s)
timeout -k 10 300 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err"
e=$(date +%s)
echo "bench.py wall seconds: $((e - s))" > "$O/bench_wall.txt"
timeout -k 10 200 python3 bench.py --workload sort --steps 10 --no-cpu-baseline > "$O/bench_sort.json" 2> "$O/bench_sort.err"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
(
  export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29591 WARPDB_EXCHANGE_ONE_RANK=1
  timeout -k 10 200 python3 bench.py --workload group --total-rows 1.25e8 --steps 200 --warmup 50 --no-cpu-baseline \
    > "$O/bench_c3s_125e8_rccl1.json" 2> "$O/bench_c3s_125e8_rccl1.err"
  MASTER_PORT=29592 timeout -k 10 300 python3 bench.py --workload group --keys 1000000 --steps 10 --warmup 3 \
    --no-cpu-baseline > "$O/bench_group_1e6k_rccl1.json" 2> "$O/bench_group_1e6k_rccl1.err"
)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_default" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline > "$O/prof_default.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_sort" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload sort --steps 10 --no-cpu-baseline > "$O/prof_sort.log" 2>&1
echo done
