/*
 * warpdb_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference WarpDB query path, used as the parity
 * checker for the HIP engine.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product path
 * (warpdb_amd/, libwarpexec.so) never links or calls it.
 *
 * Parity pinning: the restatement is checked against the golden vectors the
 * reference's own tests and data hold (tests/golden/)
 * and, in this container, against oracle/_ref (the reference's own
 * tokenizer/parser/evaluator compiled from /root/reference; see
 * oracle/build_ref.sh).
 */
#ifndef WARPDB_ORACLE_H
#define WARPDB_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same numbering as DataType in the reference (include/csv_loader.hpp:13). */
enum { ORA_INT32 = 0, ORA_INT64 = 1, ORA_FLOAT32 = 2, ORA_FLOAT64 = 3, ORA_STRING = 4 };

typedef struct {
  const char *name;
  int32_t dtype;
  const void *data; /* host pointer, n_rows elements */
} ora_col;

typedef struct {
  int64_t n_rows;
  int32_t n_cols;
  const ora_col *cols;
} ora_table;

/* Evaluation semantics.
 *  ORA_SEM_CPU  -- src/warpdb.cpp:111-155: every column value is cast to float
 *                  first, all arithmetic in float, condition = value != 0.0f.
 *  ORA_SEM_JIT  -- the C semantics of the JIT kernel the reference builds
 *                  (src/jit.cpp:55-83): columns keep their C type (int, long
 *                  long, float, double), float literals, usual arithmetic
 *                  conversions, result converted to float.
 * Both extend the reference CPU evaluator with &&, || (C truthiness) and the
 * custom.cu function discount(p, r) = p * r (custom.cu:1-3); the reference
 * CPU evaluator returns 0.0f for those nodes (src/warpdb.cpp:150). */
enum { ORA_SEM_CPU = 0, ORA_SEM_JIT = 1 };

/* Lower an expression to the reference's CUDA-C string
 * (include/expression.hpp:32-78).  Returns 0 on success. */
int ora_lower(const char *expr, char *out, size_t outlen, char *err, size_t errlen);

/* Split "expr WHERE cond" at the first case-insensitive "WHERE"
 * (src/warpdb.cpp:204-213). */
void ora_split_where(const char *query, char *expr, size_t elen, char *cond, size_t clen);

/* Project + filter.  Evaluates `expr` on every row where `cond` holds
 * (cond may be NULL/empty = all rows).  Writes the compacted values and the
 * ascending row indices of passing rows.  out_* may be NULL to only count.
 * dense_out (nullable, n_rows floats) receives expr at passing rows; it is
 * left untouched elsewhere, as the reference kernel does. */
int ora_project_filter(const ora_table *t, const char *expr, const char *cond, int sem,
                       float *out_vals, int64_t *out_idx, int64_t *out_count,
                       float *dense_out, char *err, size_t errlen);

/* SUM(expr) WHERE cond in double, row order; also returns the row count. */
int ora_sum(const ora_table *t, const char *expr, const char *cond, int sem,
            double *out_sum, int64_t *out_count, char *err, size_t errlen);

/* SUM(val) GROUP BY key WHERE cond.  key = (int)eval(key_expr), val =
 * (float)eval(val_expr), accumulated in double; groups in ascending key
 * order (tests/sql_features_test.cpp:14-19).  Capacity = max groups. */
/* SUM / COUNT / MIN / MAX of (float)expr WHERE cond; MIN / MAX skip NaN,
 * fold -0.0 to +0.0 and read NaN when empty (AggData, src/warpdb.cpp:375-385). */
int ora_stats(const ora_table *t, const char *expr, const char *cond, int sem, double *out_sum,
              int64_t *out_count, float *out_min, float *out_max, char *err, size_t errlen);
/* ora_group_sum plus per-group MIN / MAX (nullable outputs). */
int ora_group_agg(const ora_table *t, const char *val_expr, const char *key_expr, const char *cond,
                  int sem, int64_t capacity, int32_t *out_keys, double *out_sums,
                  int64_t *out_counts, float *out_mins, float *out_maxs, int64_t *out_groups, char *err,
                  size_t errlen);
int ora_group_sum(const ora_table *t, const char *val_expr, const char *key_expr,
                  const char *cond, int sem, int64_t capacity, int32_t *out_keys,
                  double *out_sums, int64_t *out_counts, int64_t *out_groups, char *err,
                  size_t errlen);

/* ORDER BY order_expr [DESC] LIMIT k over rows passing cond; ties broken by
 * ascending row index (a stable sort).  Outputs key, row index and the value
 * of select_expr (NULL = the order key) for up to k rows. */
int ora_topk(const ora_table *t, const char *order_expr, const char *cond,
             const char *select_expr, int64_t k, int descending, int sem, float *out_keys,
             int64_t *out_idx, float *out_vals, int64_t *out_count, char *err, size_t errlen);

/* Single-threaded reference-style per-row interpreter timing loop used by
 * bench.py's cpu_baseline: evaluates "expr WHERE cond" over n rows,
 * compacting into out arrays.  Returns the passing count. */
int64_t ora_scan_baseline(const ora_table *t, const char *query, float *out_vals,
                          int64_t *out_idx);

#ifdef __cplusplus
}
#endif
#endif
