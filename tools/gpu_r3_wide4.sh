#!/usr/bin/env bash
# Round 3: pipelined staged scatter (partitioned GROUP BY) -- tests, A/B of
# tile depth and partition width at 1e9 rows x 1e6 keys, kernel stats.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3w4
mkdir -p "$O"
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_group_wide.py > "$O/pytest_wide.log" 2>&1
B="python3 bench.py --workload group --no-cpu-baseline --no-check --steps 10 --rows 1e9 --keys 1000000"
for cfg in "4 13" "2 13" "4 12" "3 13" "4 13"; do
  set -- $cfg
  WARPDB_GP_SUNROLL=$1 WARPDB_GP_SHIFT=$2 timeout -k 10 200 $B > "$O/ab_u$1_s$2.json" 2>> "$O/ab.err"
  echo "u=$1 shift=$2 $(python3 -c "import json,sys; d=json.load(open('$O/ab_u$1_s$2.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'])")" >> "$O/ab.txt"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_wide" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload group --rows 1e9 --keys 1000000 --no-cpu-baseline --no-check --steps 5 > "$O/prof_wide.log" 2>&1
echo done
