#!/usr/bin/env bash
# Kernel trace of the many-key multi-rank GROUP BY step (one-rank RCCL):
# which kernels a timed step launches.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/trace_lists
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29651 WARPDB_EXCHANGE_ONE_RANK=1 \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload group --keys 1000000 --rows 1e8 --steps 20 --warmup 3 --no-cpu-baseline \
  > "$O/bench.json" 2> "$O/bench.err"
echo done
