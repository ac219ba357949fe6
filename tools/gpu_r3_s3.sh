#!/usr/bin/env bash
# Round 3, session 2: the many-key list merge (wx_group_merge_lists) -- its
# GPU tests, the exchange / multi-shard tests around it, the many-key
# multi-rank bench on a one-rank RCCL communicator, a kernel trace of the
# strong-scaled C3 step at its 8-GPU per-rank size (1.25e8 rows); the radix
# sort's plain order flip (sort tests, A/B) and its per-tile phase times.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/s3
mkdir -p "$O"
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests/test_gpu_exchange.py tests/test_gpu_multi.py \
  -k "merge_lists or slots or one_rank or one_device or virtual or resident" > "$O/pytest.log" 2>&1
timeout -k 10 600 $PYT tests -m gpu -k "sort or order or limit" > "$O/pytest_sort.log" 2>&1
AB_ROUNDS=4 timeout -k 10 500 python3 tools/ab_sort_rank.py 1e9 keys 0 \
  "WARPDB_RS_PLAIN=1,WARPDB_RS_LEAD=auto;WARPDB_RS_PLAIN=0,WARPDB_RS_LEAD=auto;WARPDB_RS_PLAIN=1,WARPDB_RS_LEAD=1;WARPDB_RS_PLAIN=0,WARPDB_RS_LEAD=1" \
  > "$O/abl_sort_plain_lead.txt" 2>&1
AB_ROUNDS=3 timeout -k 10 400 python3 tools/ab_sort_rank.py 1e9 pairs 0 "WARPDB_RS_LEAD=auto;WARPDB_RS_LEAD=1" \
  > "$O/abl_sort_lead_pairs.txt" 2>&1
AB_ROUNDS=1 timeout -k 10 300 python3 tools/ab_sort_rank.py 1e9 keys 0 \
  "WX_RS_DIAG_PHASES=1;WX_RS_DIAG_PHASES=1,WARPDB_RS_PLAIN=0,WARPDB_RS_LEAD=1" > "$O/sort_phases.txt" 2>&1
timeout -k 10 200 python3 bench.py --workload sort --steps 10 --no-cpu-baseline > "$O/bench_sort.json" 2> "$O/bench_sort.err"
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 WARPDB_EXCHANGE_ONE_RANK=1
timeout -k 10 300 python3 bench.py --workload group --keys 1000000 --steps 10 --warmup 3 --no-cpu-baseline \
  > "$O/bench_group_1e6k_lists_rccl1.json" 2> "$O/bench_group_1e6k_lists_rccl1.err"
cd /tmp && export TMPDIR=/tmp
MASTER_PORT=29562 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c3s" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload group --total-rows 1.25e8 --steps 200 --warmup 20 --no-cpu-baseline \
  > "$O/prof_c3s.log" 2>&1
echo done
