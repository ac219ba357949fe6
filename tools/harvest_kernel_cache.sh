#!/usr/bin/env bash
# GPU box: run the GPU suite, smoke() and the default / API / sort / wide
# GROUP BY benches against an EMPTY code-object cache, then pack the objects
# they compiled into gpurun_out/<tag>/kernel_cache.tgz.  Unpacked into
# warpdb_amd/.kernel_cache/ (tools/harvest_unpack.sh), the tree then carries
# exactly the code objects its own GPU runs need, so the round-end suite and
# bench pay no hiprtc compile.  usage: bash tools/harvest_kernel_cache.sh TAG
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-harvest}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
KC=/tmp/wx_kernel_cache_$$
rm -rf "$KC" && mkdir -p "$KC"
export WARPDB_KERNEL_CACHE=$KC
step() { echo "[$(date +%T)] $1" >> "$O/steps.log"; }
step suite
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread --durations=25 \
  > "$O/pytest_gpu.log" 2>&1 || { step "suite FAILED"; exit 1; }
step smoke
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { step "smoke FAILED"; exit 1; }
for b in "default:" "sort:--workload sort --no-cpu-baseline" "api_sum:--api --workload sum --no-cpu-baseline" \
         "api_group:--api --workload group --no-cpu-baseline" "api_topk:--api --workload topk --no-cpu-baseline" \
         "group_wide:--workload group --keys 1000000 --no-cpu-baseline" "dense:--workload dense --no-cpu-baseline"; do
  name=${b%%:*}; args=${b#*:}
  step "bench $name"
  timeout -k 10 300 python3 -u bench.py $args > "$O/bench_$name.json" 2> "$O/bench_$name.err" || { step "bench $name FAILED"; exit 1; }
done
step pack
tar czf "$O/kernel_cache.tgz" -C "$KC" . && ls "$KC" | wc -l > "$O/kernel_cache_count.txt"
rm -rf "$KC"
step done
