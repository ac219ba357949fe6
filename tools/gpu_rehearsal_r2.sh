#!/usr/bin/env bash
# Multi-rank bench rehearsal on the 1-GPU box (gloo, ranks sharing the GPU),
# progress marks on stderr; each run under its own time limit.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/rehearsal; mkdir -p "$O"
run() {
  local name=$1 np=$2; shift 2
  WARPDB_BENCH_VERBOSE=1 WARPDB_DIST_BACKEND=gloo timeout -k 10 100 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $np \
    --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) "$R/bench.py" --gpus $np "$@" > "$O/$name.json" 2> "$O/$name.err"
  echo "$name rc=$?" >> "$O/rc.txt"
}
for spec in "$@"; do
  set -- $spec
  run "$@"
done
