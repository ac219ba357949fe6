#!/usr/bin/env bash
# Round 3, session 2: state check after the container rebuild -- smoke, the
# whole GPU suite, the default bench line, the sort bench, and the C3 strong
# line at the per-GPU size an 8-GPU run gives it (1.25e8 rows, one-rank RCCL).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/s2
mkdir -p "$O"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
timeout -k 10 200 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err"
timeout -k 10 200 python3 bench.py --workload sort --steps 10 --no-cpu-baseline > "$O/bench_sort.json" 2> "$O/bench_sort.err"
WARPDB_EXCHANGE_ONE_RANK=1 timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --workload group --total-rows 1.25e8 --steps 50 --warmup 20 \
  --no-cpu-baseline > "$O/bench_group_125e6_rccl1.json" 2> "$O/bench_group_125e6_rccl1.err"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
echo done
