#!/usr/bin/env bash
# PMC traffic of the sort on the round-3 kernels (FETCH_SIZE / WRITE_SIZE passes).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
timeout -k 10 400 bash tools/pmc_run.sh sort 1e9 "" sort_r3 > gpurun_out/pmc_sort_r3.log 2>&1
echo done
