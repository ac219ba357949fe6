#!/usr/bin/env bash
# PMC traffic passes for one bench workload (GPU box).  FETCH_SIZE and
# WRITE_SIZE go in separate rocprofv3 passes (TCC slots), kernel trace only.
set -euo pipefail
W=${1:-project}
ROWS=${2:-1e9}
EXTRA=${3:-}   # more bench.py arguments (e.g. "--keys 1000000")
TAG=${4:-$W}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d "$OUT/$C" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload "$W" --rows "$ROWS" --steps 3 --warmup 1 --no-cpu-baseline --no-check \
    --no-secondary $EXTRA > "$OUT/$C.log" 2>&1
done
python3 "$R/tools/pmc_summary.py" $(find "$OUT" -name "*counter_collection.csv") > "$OUT/summary.json"
cat "$OUT/summary.json"
# the tracked record bench.py reads (collection date + kernel-source sha)
PW=$W
[[ "$W" == group && "$EXTRA" == *--keys* ]] && PW=group_wide
python3 "$R/tools/pmc_record.py" "$PW" "$ROWS" "$OUT/summary.json" "$TAG"
cp "$R/profiles/pmc_$PW.json" "$OUT/"
