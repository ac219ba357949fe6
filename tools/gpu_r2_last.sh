#!/usr/bin/env bash
# Round-2 last pass on the final code (GPU box): smoke, the full GPU suite,
# the default bench line (wall time recorded) and rocprofv3 kernel stats of
# the same default command.  Every GPU step has its own limit; the first
# failure ends the script.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r2last
mkdir -p "$O"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
s=$(date +%s)
timeout -k 10 300 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err"
e=$(date +%s)
echo "bench.py wall seconds: $((e - s))" > "$O/bench_wall.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_default" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline > "$O/prof_default.log" 2>&1
echo done
