#!/usr/bin/env bash
# Box comparison: the sort line, the headline project line and the LBW A/B
# in one call, with the device's name and clocks.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/s10
mkdir -p "$O"
(rocm-smi --showproductname --showclocks --showmeminfo vram 2>&1 || true) > "$O/smi.txt"
timeout -k 10 200 python3 bench.py --workload sort --steps 10 --no-cpu-baseline > "$O/bench_sort.json" 2> "$O/bench_sort.err"
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-secondary > "$O/bench_project.json" 2> "$O/bench_project.err"
AB_ROUNDS=3 timeout -k 10 400 python3 tools/ab_sort_rank.py 1e9 keys 0 "WARPDB_RS_LBW=2;WARPDB_RS_LBW=3" \
  > "$O/abl_sort_lbw.txt" 2>&1
echo done
