#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY.  Compiles the reference's own CUDA-free C++ tests
# UNCHANGED, straight from /root/reference/tests (read-only, nothing copied
# into the repository), against this repository's drop-in headers
# (include/warpdb/*.hpp, found under the reference's own include names) and
# libwarpdb -- the direct check that a caller of the reference's API compiles
# and behaves the same.  NDEBUG stays undefined, so every assert runs.
# Outputs: oracle/_ref/reftests/<test> (git-ignored; they travel to the GPU
# box with the tree, which has no /root/reference).
#   expression.hpp only (CPU suite): test_expression precedence_tests
#     tokenizer_tests expression_tests parsing_error_tests tokenize_error_test
#     parse_query_error_test query_parser_test identifier_validation_test
#   warpdb.hpp (GPU suite): extended_types_test having_distinct_test
# Excluded: sql_features_test.cpp reads h.price / h.quantity, members the
# reference's own HostTable does not have (include/csv_loader.hpp:39-51), so
# it does not compile against the reference either;
# jit_arch_test / jit_error_test include <cuda_runtime.h>.
set -euo pipefail
REF=${WARPDB_REFERENCE:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/.." && pwd)
OUT="$HERE/_ref/reftests"
if [ ! -d "$REF/tests" ]; then
  echo "reference not present at $REF; skipping oracle/_ref/reftests" >&2
  exit 0
fi
mkdir -p "$OUT"
TESTS="test_expression precedence_tests tokenizer_tests expression_tests parsing_error_tests tokenize_error_test
parse_query_error_test query_parser_test identifier_validation_test extended_types_test having_distinct_test"
for t in $TESTS; do
  g++ -std=c++17 -O1 -I"$ROOT/include/warpdb" -I"$ROOT/include" "$REF/tests/$t.cpp" -o "$OUT/$t" \
      -L"$ROOT/warpdb_amd" -lwarpdb -lwarpexec -Wl,-rpath,'$ORIGIN/../../../warpdb_amd' &
done
wait
for t in $TESTS; do [ -x "$OUT/$t" ] || { echo "failed to build $t" >&2; exit 1; }; done
echo "built $OUT ($(echo $TESTS | wc -w) reference tests)"
