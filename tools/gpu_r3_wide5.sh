#!/usr/bin/env bash
# Round 3: partitioned GROUP BY with the sampled-range first pass -- tests,
# then 1e9 rows x 1e6 / 1e5 keys with and without the guess, kernel stats.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3w5
mkdir -p "$O"
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_group_wide.py > "$O/pytest_wide.log" 2>&1
B="python3 bench.py --workload group --no-cpu-baseline --steps 10 --rows 1e9"
for g in 1 0 1; do
  WARPDB_GP_GUESS=$g timeout -k 10 200 $B --keys 1000000 --no-check > "$O/ab_g$g.json" 2>> "$O/ab.err"
  echo "guess=$g $(python3 -c "import json,sys; d=json.load(open('$O/ab_g$g.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'])")" >> "$O/ab.txt"
done
timeout -k 10 200 $B --keys 1000000 > "$O/bench_group_1e6k_1e9.json" 2> "$O/b1.err"
timeout -k 10 200 $B --keys 100000 > "$O/bench_group_1e5k_1e9.json" 2> "$O/b2.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_wide" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload group --rows 1e9 --keys 1000000 --no-cpu-baseline --no-check --steps 5 > "$O/prof_wide.log" 2>&1
echo done
