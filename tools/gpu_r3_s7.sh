#!/usr/bin/env bash
# Round 3, session 2 checkpoint: smoke, the whole GPU suite, the default
# bench line (wall time), the sort bench, and rocprofv3 kernel stats of both.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/s7
mkdir -p "$O"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
s=$(date +%s)
timeout -k 10 300 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err"
e=$(date +%s)
echo "bench.py wall seconds: $((e - s))" > "$O/bench_wall.txt"
timeout -k 10 200 python3 bench.py --workload sort --steps 10 --no-cpu-baseline > "$O/bench_sort.json" 2> "$O/bench_sort.err"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_default" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline > "$O/prof_default.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_sort" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload sort --steps 10 --no-cpu-baseline > "$O/prof_sort.log" 2>&1
echo done
