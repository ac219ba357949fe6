#!/usr/bin/env bash
# Round 3, session 2: persistent radix key tiles (A/B, sort tests) and the
# GROUP BY finalize fused into the last workgroup (group tests, A/B, the
# C3 strong-scaled step at its 8-GPU per-rank size on a one-rank RCCL
# communicator, kernel trace).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/s5
mkdir -p "$O"
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests -m gpu -k "sort or order or limit" > "$O/pytest_sort.log" 2>&1
timeout -k 10 900 $PYT tests -m gpu -k "group or exchange or slots or workload or fuzz or multi or sql" > "$O/pytest_group.log" 2>&1
AB_ROUNDS=4 timeout -k 10 500 python3 tools/ab_sort_rank.py 1e9 keys 0 "WARPDB_RS_PERSIST=1;WARPDB_RS_PERSIST=0" \
  > "$O/abl_sort_persist.txt" 2>&1
timeout -k 10 200 python3 bench.py --workload sort --steps 10 --no-cpu-baseline > "$O/bench_sort.json" 2> "$O/bench_sort.err"
for F in 1 0; do
  WARPDB_GROUP_FUSED_FIN=$F timeout -k 10 200 python3 bench.py --workload group --steps 50 --warmup 20 --no-cpu-baseline \
    --no-secondary > "$O/bench_group_fused$F.json" 2> "$O/bench_group_fused$F.err"
done
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29571 WARPDB_EXCHANGE_ONE_RANK=1
for F in 1 0; do
  WARPDB_GROUP_FUSED_FIN=$F MASTER_PORT=2957$F timeout -k 10 200 python3 bench.py --workload group --total-rows 1.25e8 \
    --steps 200 --warmup 50 --no-cpu-baseline > "$O/bench_c3s_fused$F.json" 2> "$O/bench_c3s_fused$F.err"
done
cd /tmp && export TMPDIR=/tmp
MASTER_PORT=29579 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c3s" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload group --total-rows 1.25e8 --steps 200 --warmup 20 --no-cpu-baseline \
  > "$O/prof_c3s.log" 2>&1
echo done
