#!/usr/bin/env bash
# Round-2 measurement pass (GPU box): bench lines for every workload, C2 at
# its own 1e8 rows, C4's g=1 leg (8e9 rows, product path and the C++ --api
# path), and rocprofv3 kernel stats for C2 @ 1e8 and C4 @ 8e9.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r2m
mkdir -p "$O"
B="timeout -k 10 300 python3 $R/bench.py"
$B > "$O/project_1e9.json"
$B --rows 1e8 --steps 100 --no-cpu-baseline > "$O/project_1e8.json"
$B --workload sum --total-rows 8e9 --steps 10 > "$O/c4_g1.json"
$B --workload sum --total-rows 8e9 --steps 10 --api --no-cpu-baseline > "$O/c4_g1_api.json"
$B --workload group --no-cpu-baseline > "$O/group.json"
$B --workload group --api --no-cpu-baseline > "$O/group_api.json"
$B --workload topk --no-cpu-baseline > "$O/topk.json"
$B --workload dense --no-cpu-baseline > "$O/dense.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c2_1e8" -o run --output-format csv -- \
  python3 "$R/bench.py" --rows 1e8 --steps 50 --no-cpu-baseline > "$O/prof_c2_1e8.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c4_8e9" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload sum --total-rows 8e9 --steps 10 --no-cpu-baseline > "$O/prof_c4_8e9.log" 2>&1
echo done
