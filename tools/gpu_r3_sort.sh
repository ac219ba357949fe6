#!/usr/bin/env bash
# Round 3: the radix sort's paired look-back -- sort tests, in-process A/B,
# the bench's sort workload and its kernel stats.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3s
mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_warpdb_api.py -x -q -k "sort or order" \
  --timeout 200 --timeout-method thread > "$O/pytest_sort.log" 2>&1
timeout -k 10 300 python3 tools/ab_sort_pair.py 1e9 > "$O/ab_sort_pair.txt" 2>&1
timeout -k 10 200 python3 bench.py --workload sort --no-cpu-baseline > "$O/bench_sort.json" 2> "$O/bench_sort.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_sort" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload sort --no-cpu-baseline --no-check --steps 10 > "$O/prof_sort.log" 2>&1
echo done
