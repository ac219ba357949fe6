#!/usr/bin/env bash
# Kernel-argument placement (HIP_FORCE_DEV_KERNARG) vs the gaps between the
# dependent kernels of a step: C3 strong at 1.25e8 rows (one-rank RCCL) and
# the headline line, alternating.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/kernarg
mkdir -p "$O"
for r in 1 2; do
  for k in 0 1; do
    HIP_FORCE_DEV_KERNARG=$k RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=296$k$r \
      WARPDB_EXCHANGE_ONE_RANK=1 timeout -k 10 200 python3 bench.py --workload group --total-rows 1.25e8 --steps 200 \
      --warmup 50 --no-cpu-baseline > "$O/c3s_k${k}_r$r.json" 2> "$O/c3s_k${k}_r$r.err"
    HIP_FORCE_DEV_KERNARG=$k timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 \
      > "$O/default_k${k}_r$r.json" 2> "$O/default_k${k}_r$r.err"
  done
done
echo done
