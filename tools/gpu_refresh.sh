#!/usr/bin/env bash
# One GPU-box pass: GPU test suite, bench per workload, kernel-trace stats
# and PMC traffic per workload.  Every GPU step has its own time limit and
# the script stops at the first failure.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/refresh
mkdir -p "$O"
WL=${WL:-"project dense sum group topk sort"}
cd "$R"
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > "$O/pytest_gpu.log" 2>&1
fi
for W in $WL; do
  timeout -k 10 300 python3 bench.py --workload "$W" > "$O/bench_$W.log" 2>&1
done
cd /tmp && export TMPDIR=/tmp
for W in $WL; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$W" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload "$W" --steps 10 --warmup 2 --no-cpu-baseline > "$O/prof_$W.log" 2>&1
done
if [ -n "${PMC:-}" ]; then
  for W in $WL; do
    [ "$W" = sort ] && continue  # several kernels per step: no per-launch traffic
    timeout -k 10 700 bash "$R/tools/pmc_run.sh" "$W" > "$O/pmc_$W.log" 2>&1
  done
fi
echo done
