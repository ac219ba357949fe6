#!/usr/bin/env bash
# Round-3 baseline on the round-2 code (GPU box): smoke, the default bench
# line with its wall time, C2 at its own 1e8 rows, GROUP BY at 1e9, and
# rocprofv3 kernel stats of the default command.  Every GPU step has its own
# limit; the first failure ends the script.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3base
mkdir -p "$O"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
s=$(date +%s)
timeout -k 10 300 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err"
e=$(date +%s)
echo "bench.py wall seconds: $((e - s))" > "$O/bench_wall.txt"
timeout -k 10 200 python3 bench.py --rows 1e8 --no-secondary --no-c4 --no-cpu-baseline > "$O/bench_project_1e8.json" 2> "$O/bench_project_1e8.err"
timeout -k 10 200 python3 bench.py --workload group --no-cpu-baseline > "$O/bench_group.json" 2> "$O/bench_group.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_default" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline > "$O/prof_default.log" 2>&1
echo done
