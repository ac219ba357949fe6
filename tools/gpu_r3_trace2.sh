#!/usr/bin/env bash
# Round 3: kernel trace of a 2-rank rehearsal step (two ranks sharing the
# GPU over gloo; rank 0 under rocprofv3, rank 1 plain, each started by this
# shell) for GROUP BY and top-K -- the timed steps must show only wx_*
# kernels (the exchange itself is gloo's host copy here, RCCL on a node).
# Then the many-key reference fixture tests.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3t
mkdir -p "$O"
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_workload_golden.py > "$O/pytest_workload.log" 2>&1 || exit 1
export MASTER_ADDR=127.0.0.1 WORLD_SIZE=2 WARPDB_DIST_BACKEND=gloo
port=29611
for wl in group topk; do
  port=$((port + 1))
  export MASTER_PORT=$port
  RANK=1 LOCAL_RANK=1 timeout -k 10 240 python3 "$R/bench.py" --gpus 2 --workload $wl --rows 2e7 --steps 10 --warmup 2 \
     --no-cpu-baseline > "$O/rank1_$wl.log" 2>&1 &
  p1=$!
  (cd /tmp && TMPDIR=/tmp RANK=0 LOCAL_RANK=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/trace2_$wl" -o run \
     --output-format csv -- python3 "$R/bench.py" --gpus 2 --workload $wl --rows 2e7 --steps 10 --warmup 2 \
     --no-cpu-baseline > "$O/rank0_$wl.json" 2> "$O/rank0_$wl.err")
  r0=$?
  wait $p1
  r1=$?
  echo "$wl rank0=$r0 rank1=$r1" >> "$O/status.txt"
  [ $r0 -eq 0 ] && [ $r1 -eq 0 ] || exit 1
done
echo done
