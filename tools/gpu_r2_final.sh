#!/usr/bin/env bash
# Round-2 refresh (GPU box): smoke(), one bench line per workload (C2 at 1e8
# and the metric's 1e9, C3, C4's g = 1 leg at 8e9, C5, dense, sort) and
# rocprofv3 kernel stats for the headline and C2.  Every step has its own
# time limit; the first failure ends the script.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r2f
mkdir -p "$O"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
B="timeout -k 10 300 python3 $R/bench.py"
$B > "$O/bench_project_1e9.json"
$B --rows 1e8 --steps 100 --no-cpu-baseline > "$O/bench_project_1e8.json"
$B --workload dense --no-cpu-baseline > "$O/bench_dense.json"
$B --workload group > "$O/bench_group.json"
$B --workload sum --total-rows 8e9 --steps 10 > "$O/bench_c4_g1.json"
$B --workload topk > "$O/bench_topk.json"
$B --workload sort --steps 10 > "$O/bench_sort.json"
echo benches done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_project_1e9" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-check > "$O/prof_project_1e9.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_project_1e8" -o run --output-format csv -- \
  python3 "$R/bench.py" --rows 1e8 --steps 50 --no-cpu-baseline --no-check > "$O/prof_project_1e8.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_sort" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload sort --steps 5 --no-cpu-baseline --no-check > "$O/prof_sort.log" 2>&1
echo done
