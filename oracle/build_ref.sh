#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY.  Builds oracle/_ref/ref_harness from the
# reference's own sources where they lie under /root/reference (read-only).
# Only the CUDA-free parts of three files are compiled (the snapshot as a
# whole does not build: SURVEY.md section 0); nothing is copied into the
# repository -- the slices are extracted into oracle/_ref/ (git-ignored).
set -euo pipefail
REF=${WARPDB_REFERENCE:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
if [ ! -d "$REF/src" ]; then
  echo "reference not present at $REF; skipping oracle/_ref" >&2
  exit 0
fi
mkdir -p "$OUT"
# tokenize / parse_expression / parse_logical_{and,or}  (parse_query follows
# and is the part with the unbalanced brace, src/expression.cpp:515-531)
sed -n '1,268p' "$REF/src/expression.cpp" > "$OUT/slice_expression.inc"
# get_value / eval_node / eval_condition (anonymous namespace)
sed -n '109,157p' "$REF/src/warpdb.cpp" > "$OUT/slice_eval.inc"
# load_csv_to_host (the CUDA upload helpers that follow are excluded)
sed -n '49,124p' "$REF/src/csv_loader.cpp" > "$OUT/slice_csv.inc"
g++ -std=c++17 -O2 -ffp-contract=off -I"$REF/include" -I"$OUT" \
    "$HERE/ref_harness.cpp" -o "$OUT/ref_harness"
echo "built $OUT/ref_harness"
