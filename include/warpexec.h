/*
 * warpexec.h -- C ABI of the MI355X (gfx950) query execution layer.
 *
 * This is the drop-in boundary for WarpDB's execution path.  Every entry
 * point takes plain pointers and sizes, returns a wx_status and reports
 * failures through an (err, errlen) buffer; no C++ exception and no torch
 * type crosses it.  Device buffers are caller-owned (hipMalloc / torch);
 * warpexec owns only its compiled kernel cache and a per-(device, stream)
 * workspace.
 *
 * Reference interfaces replaced (paths relative to the WarpDB snapshot):
 *   wx_project_filter   jit_compile_and_launch   include/jit.hpp:7-10, src/jit.cpp:48-174
 *                       + the launch/D2H part of WarpDB::query src/warpdb.cpp:243-256
 *   wx_group_sum        jit_group_sum            include/jit.hpp:15-18, src/jit.cpp:179-246
 *   wx_sort_pairs       jit_sort_pairs           include/jit.hpp:22-23, src/jit.cpp:248-281
 *   wx_sort_float       jit_sort_float           include/jit.hpp:26-27, src/jit.cpp:283-307
 *   wx_sort_float_from  projection + jit_sort_float of ORDER BY <column>  src/warpdb.cpp:450-455
 *   wx_sort_by_key      ORDER BY <expr> keyed sort  src/warpdb.cpp:470-476
 *   wx_topk             jit_sort_float + LIMIT   src/warpdb.cpp:453-455,483-495
 *   wx_reduce_sum       per-shard SUM of query_multi_gpu (new; the reference
 *                       gathers dense results on the host, src/multi_gpu_utils.cpp:5-63)
 *   wx_reduce_stats     ungrouped SUM / COUNT / AVG / MIN / MAX of query_sql
 *                       (src/warpdb.cpp:297-498, AggData :383-384) and the column
 *                       statistics of the optimizer (include/csv_loader.hpp:22-37,
 *                       src/optimizer.cpp:13-17)
 *   wx_group_agg        jit_group_sum + the per-group MIN / MAX of query_sql's
 *                       AggData (src/warpdb.cpp:375-385)
 *   wx_group_partials,  GROUP BY over row shards: per-shard
 *   wx_group_combine    partials in an all-reduce layout and the final merge;
 *                       the reference's multi-GPU path gathers dense results
 *                       on the host instead (src/multi_gpu_utils.cpp:5-63)
 *   wx_group_partials_slots,  the same in ONE collective: window + per-shard
 *   wx_group_combine_slots    slots of out-of-window groups (src/multi_gpu_utils.cpp:23-60)
 *   wx_group_merge_lists  GROUP BY over row shards with many groups: the
 *                       device merge of the shards' gathered group lists (the
 *                       reference gathers on the host, src/multi_gpu_utils.cpp:23-60)
 *   wx_topk_merge       ORDER BY .. LIMIT over row shards: the merge of the
 *                       shards' candidate records (src/warpdb.cpp:453-455,
 *                       483-495 sort the gathered dense results instead)
 *   wx_cast             device-side type conversion (jit_group_sum's float
 *                       outputs, include/jit.hpp:15-18)
 *
 * Expression inputs are the reference's lowered C expressions over
 * identifiers `<column>[idx]` (include/expression.hpp:32-78), e.g.
 * "(price[idx] * quantity[idx])".  An empty / NULL condition means no filter
 * (src/jit.cpp:56).  The text of custom.cu (or custom_src) is prepended to
 * every generated kernel exactly as src/jit.cpp:65-73 does.
 *
 * All work is enqueued on `stream` (a hipStream_t; NULL = the null stream)
 * and is asynchronous unless WX_F_SYNC is set or a host output pointer is
 * passed, in which case the call returns with results complete.
 */
#ifndef WARPEXEC_H
#define WARPEXEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WX_ABI_VERSION 1

typedef enum wx_status {
  WX_OK = 0,
  WX_ERR_INVALID = 1,     /* bad argument / unknown column type / overflow */
  WX_ERR_COMPILE = 2,     /* hiprtc failed; err holds the compiler log */
  WX_ERR_DEVICE = 3,      /* a HIP runtime call failed */
  WX_ERR_CAPACITY = 4,    /* an output or group table was too small */
  WX_ERR_UNSUPPORTED = 5, /* request outside what the engine implements */
  WX_ERR_INTERNAL = 6     /* a device-side check failed (e.g. look-back timeout) */
} wx_status;

/* Same numbering as WarpDB's DataType (include/csv_loader.hpp:13). */
typedef enum wx_dtype {
  WX_INT32 = 0,
  WX_INT64 = 1,
  WX_FLOAT32 = 2,
  WX_FLOAT64 = 3,
  WX_STRING = 4 /* accepted in a table, cannot be referenced by an expression */
} wx_dtype;

/* One device column: mirrors ColumnDesc (include/csv_loader.hpp:15-20);
 * the length is the table's n_rows. */
typedef struct wx_col {
  const char *name;
  int32_t dtype;
  const void *d_ptr;
} wx_col;

/* Mirrors Table (include/csv_loader.hpp:39-51) with 64-bit row counts. */
typedef struct wx_table {
  int64_t n_rows;
  int32_t n_cols;
  const wx_col *cols;
} wx_table;

/* Where and how to run. */
typedef struct wx_launch {
  int32_t device;         /* HIP device ordinal */
  void *stream;           /* hipStream_t (NULL = null stream) */
  const char *custom_src; /* NULL: read $WARPDB_CUSTOM_PATH or ./custom.cu per call */
  uint32_t flags;         /* WX_F_* */
} wx_launch;

#define WX_F_SYNC 1u      /* synchronise the stream and check device errors before returning */
#define WX_F_NO_CUSTOM 2u /* do not prepend custom.cu */
#define WX_F_TIME 4u      /* record HIP events around the main kernel (wx_timing_read) */
#define WX_F_F64_COUNTS 8u /* wx_reduce_sum: d_out's count is written as a double (exact below
                            * 2^53), so ONE all-reduce of two doubles combines shards */
#define WX_F_ROW_ORDER 16u /* wx_group_sum / wx_group_agg: each group's sum folded in ascending row
                            * order, one double add per row -- the reference's std::map fold
                            * (src/warpdb.cpp:373-385) to the bit, the same on every run.
                            * Synchronous; two ordered compactions, a stable pair sort and a
                            * per-group fold whose time grows with the largest group's rows */

/* wx_project_filter modes */
#define WX_MODE_DENSE 0      /* out_vals[row] = expr where cond holds, other rows untouched (src/jit.cpp:55-61) */
#define WX_MODE_DENSE_FILL 1 /* as DENSE, other rows set to 0.0f */
#define WX_MODE_COMPACT 2    /* ordered stream compaction: k-th passing row -> out_vals[k], out_idx[k] */

/* Project + filter.  DENSE modes write n_rows floats to d_out_vals.
 * COMPACT writes the passing rows in ascending row order: d_out_vals[k] (nullable)
 * and d_out_idx[k] = row_base + row (nullable; idx_bytes 4 -> int32, 8 -> int64);
 * both must hold n_rows entries.  d_count (device int64, nullable) receives the
 * passing count; h_count (host, nullable) too, which synchronises. */
wx_status wx_project_filter(const wx_table *table, const char *expr, const char *cond,
                            const wx_launch *launch, int32_t mode, float *d_out_vals,
                            void *d_out_idx, int32_t idx_bytes, int64_t row_base,
                            int64_t *d_count, int64_t *h_count, char *err, size_t errlen);

/* SUM((float)expr) over rows where cond holds, accumulated in double.
 * d_out (device, nullable) receives {sum as double, count as int64 bits};
 * h_sum / h_count (host, nullable) synchronise. */
wx_status wx_reduce_sum(const wx_table *table, const char *expr, const char *cond,
                        const wx_launch *launch, void *d_out, double *h_sum, int64_t *h_count,
                        char *err, size_t errlen);

/* SUM / COUNT / MIN / MAX of (float)expr over rows where cond holds.  MIN and
 * MAX skip NaN values and read NaN when no value qualifies (SQL NULL); -0.0
 * and +0.0 compare equal and come back as +0.0. */
typedef struct wx_stats {
  double sum;
  int64_t count;
  float min;
  float max;
} wx_stats;

/* d_out (device, nullable): a wx_stats; h_out (host, nullable) synchronises. */
wx_status wx_reduce_stats(const wx_table *table, const char *expr, const char *cond,
                          const wx_launch *launch, void *d_out, wx_stats *h_out, char *err,
                          size_t errlen);

/* SUM((float)val_expr) GROUP BY (int)key_expr WHERE cond.  Sums in double,
 * counts in int64, groups in ascending key order.  capacity = entries of the
 * device outputs (and the distinct-key bound of the general-key table).
 * Keys in [key_window_lo, key_window_lo + 2048) take the LDS fast path; at
 * most 4096 distinct keys may fall outside it unless capacity is larger.
 * With capacity > 4096 on >= 2^20 rows (a caller expecting many groups) the
 * call first takes a key-range guess: the previous call's over the same
 * expressions, columns and row count (no host read), else a 65 536-row sample
 * (one host synchronisation), else an exact min / max pass (one more).  A
 * range of at most 2048 keys moves the window onto it and the call stays
 * asynchronous after that; a range of up to 2^24 keys runs the
 * range-partitioned kernels, which end with one host read
 * of their range summary (the call returns with the result complete, and
 * runs again over the exact range when a row fell outside the guess); a
 * wider one the window + hash path.  Results are the same either way. */
wx_status wx_group_sum(const wx_table *table, const char *val_expr, const char *key_expr,
                       const char *cond, const wx_launch *launch, int32_t key_window_lo,
                       int64_t capacity, int32_t *d_keys, double *d_sums, int64_t *d_counts,
                       int64_t *d_n_groups, int64_t *h_n_groups, char *err, size_t errlen);

/* On WX_ERR_CAPACITY from wx_group_sum / wx_group_agg, *h_n_groups (when
 * given) holds the number of groups found, a lower bound of the capacity
 * needed (exact unless the general-key table itself overflowed). */

/* Row-sharded GROUP BY, step 1 (per shard): SUM((float)val_expr) GROUP BY
 * (int)key_expr WHERE cond in the exchange layout.  d_window (device,
 * WX_GROUP_EXCHANGE_DOUBLES doubles) receives the dense key window
 * [key_window_lo, key_window_lo + WX_GROUP_WINDOW_BINS): the sums at
 * [0, W), the counts as doubles at [W, 2W) (exact below 2^53), and at [2W]
 * the number of groups outside the window.  Summing the shards' buffers
 * element-wise -- one ncclAllReduce(SUM, ncclFloat64) -- yields the global
 * window.  Groups outside the window go to d_keys / d_sums / d_counts
 * (ascending keys, `capacity` entries) and their count to d_n_extra /
 * h_n_extra. */
#define WX_GROUP_WINDOW_BINS 2048
#define WX_GROUP_EXCHANGE_DOUBLES (2 * WX_GROUP_WINDOW_BINS + 1)
wx_status wx_group_partials(const wx_table *table, const char *val_expr, const char *key_expr,
                            const char *cond, const wx_launch *launch, int32_t key_window_lo,
                            double *d_window, int64_t capacity, int32_t *d_keys, double *d_sums,
                            int64_t *d_counts, int64_t *d_n_extra, int64_t *h_n_extra, char *err,
                            size_t errlen);

/* Row-sharded GROUP BY, step 2: the final groups in ascending key order from
 * a combined window (wx_group_partials layout) and the combined
 * out-of-window groups (n_extra entries, ascending keys, none inside the
 * window; device arrays, nullable when n_extra is 0).  Writes at most
 * `capacity` groups; the total goes to d_n_groups / h_n_groups (a host
 * request that exceeds capacity returns WX_ERR_CAPACITY). */
wx_status wx_group_combine(const double *d_window, int32_t key_window_lo, const int32_t *d_x_keys,
                           const double *d_x_sums, const int64_t *d_x_counts, int64_t n_extra,
                           const wx_launch *launch, int64_t capacity, int32_t *d_keys, double *d_sums,
                           int64_t *d_counts, int64_t *d_n_groups, int64_t *h_n_groups, char *err,
                           size_t errlen);

/* Row-sharded GROUP BY in ONE collective (replaces the
 * reference's host gather of dense shard results, src/multi_gpu_utils.cpp:23-60).
 * The exchange buffer holds WX_GROUP_SLOTS_DOUBLES(n_slots, slot_groups)
 * doubles: the dense window exactly as wx_group_partials writes it, then one
 * slot per shard of 1 + 3 * slot_groups doubles -- the shard's out-of-window
 * group count (-1: its general-key table overflowed), then up to slot_groups
 * (key, sum, count) triples in ascending key order.  wx_group_partials_slots
 * writes the window, shard `slot`'s slot and zeros in every other slot, so an
 * element-wise SUM all-reduce of the shards' buffers (one ncclAllReduce,
 * ncclFloat64) both reduces the window and gathers the slots.  It also writes
 * ALL of the shard's out-of-window groups to d_keys / d_sums / d_counts
 * (`capacity` entries) and their count to d_n_extra / h_n_extra, for the
 * fallback below.  1 <= n_slots <= WX_GROUP_EXCHANGE_MAX_SLOTS, slot_groups >= 1,
 * n_slots * slot_groups <= 4096. */
#define WX_GROUP_EXCHANGE_MAX_SLOTS 1024
#define WX_GROUP_SLOTS_DOUBLES(n_slots, slot_groups) \
  (WX_GROUP_EXCHANGE_DOUBLES + (int64_t)(n_slots) * (1 + 3 * (int64_t)(slot_groups)))
#define WX_GROUP_NEEDS_MERGE (-2)
wx_status wx_group_partials_slots(const wx_table *table, const char *val_expr, const char *key_expr,
                                  const char *cond, const wx_launch *launch, int32_t key_window_lo,
                                  double *d_exchange, int32_t n_slots, int32_t slot, int32_t slot_groups,
                                  int64_t capacity, int32_t *d_keys, double *d_sums, int64_t *d_counts,
                                  int64_t *d_n_extra, int64_t *h_n_extra, char *err, size_t errlen);

/* The final groups (ascending keys) from a combined exchange buffer
 * (wx_group_partials_slots layout, summed over the shards): the slots' groups
 * of equal key are added in slot order, then merged with the window.  The
 * group count goes to d_n_groups / h_n_groups; it is -1 when a shard's
 * general-key table overflowed and WX_GROUP_NEEDS_MERGE when some shard had
 * more than slot_groups out-of-window groups -- every rank reads the same
 * combined buffer, so every rank sees the same value and can take the
 * fallback together: a variable-size exchange of the d_keys / d_sums /
 * d_counts lists of wx_group_partials_slots, then wx_group_combine.  The
 * kernel never reads the host; a host request over capacity returns
 * WX_ERR_CAPACITY. */
wx_status wx_group_combine_slots(const double *d_exchange, int32_t n_slots, int32_t slot_groups,
                                 int32_t key_window_lo, const wx_launch *launch, int64_t capacity,
                                 int32_t *d_keys, double *d_sums, int64_t *d_counts, int64_t *d_n_groups,
                                 int64_t *h_n_groups, char *err, size_t errlen);

/* Row-sharded GROUP BY with many groups per shard, in ONE collective and no
 * host read (replaces the host-side gather and merge of shard results,
 * src/multi_gpu_utils.cpp:23-60 / src/warpdb.cpp:508-542, for results that
 * outgrow the exchange slots).  Each shard writes its groups -- keys
 * ascending and unique, e.g. straight from wx_group_sum, or the out-of-window
 * groups of wx_group_partials_slots -- into one fixed-size list record of
 * WX_GROUP_LIST_BYTES(list_capacity) bytes: int64 count at offset 0, then
 * list_capacity int32 keys, doubles sums at WX_GROUP_LIST_SUMS_OFF, int64
 * counts at WX_GROUP_LIST_COUNTS_OFF.  One all-gather of the records
 * (ncclAllGather, bytes) hands every rank the n_lists records back to back;
 * this call merges them on the device: groups of equal key summed in list
 * order (so every rank computes the same bits), then, with d_window (the
 * combined wx_group_partials window, nullable), merged with the window's
 * non-empty bins, none of whose keys may appear in a list.  Ascending keys,
 * at most `capacity` written; the count goes to d_n_groups / h_n_groups.
 * It is -1 when a list's count is negative or above list_capacity (a shard
 * whose table or list overflowed): every rank sees the same records, so
 * every rank gets the same -1.  1 <= n_lists <= 1024, 1 <= list_capacity
 * <= 2^31; the merge keeps 24 bytes of workspace per gathered list entry. */
#define WX_GROUP_LIST_SUMS_OFF(cap) (8 + 8 * (((int64_t)(cap) + 1) / 2))
#define WX_GROUP_LIST_COUNTS_OFF(cap) (WX_GROUP_LIST_SUMS_OFF(cap) + 8 * (int64_t)(cap))
#define WX_GROUP_LIST_BYTES(cap) (WX_GROUP_LIST_COUNTS_OFF(cap) + 8 * (int64_t)(cap))
wx_status wx_group_merge_lists(const void *d_lists, int32_t n_lists, int64_t list_capacity,
                               const double *d_window, int32_t key_window_lo, const wx_launch *launch,
                               int64_t capacity, int32_t *d_keys, double *d_sums, int64_t *d_counts,
                               int64_t *d_n_groups, int64_t *h_n_groups, char *err, size_t errlen);

/* dst[i] = (dst type) src[i] for i < n, types in wx_dtype numbering (not
 * WX_STRING); C conversion semantics. */
wx_status wx_cast(const void *d_src, int32_t src_dtype, void *d_dst, int32_t dst_dtype, int64_t n,
                  const wx_launch *launch, char *err, size_t errlen);

/* wx_group_sum plus per-group MIN / MAX of (float)val_expr (d_mins / d_maxs,
 * nullable, `capacity` entries; NaN skipped as in wx_reduce_stats). */
wx_status wx_group_agg(const wx_table *table, const char *val_expr, const char *key_expr,
                       const char *cond, const wx_launch *launch, int32_t key_window_lo,
                       int64_t capacity, int32_t *d_keys, double *d_sums, int64_t *d_counts,
                       float *d_mins, float *d_maxs, int64_t *d_n_groups, int64_t *h_n_groups,
                       char *err, size_t errlen);

/* ORDER BY order_expr [DESC] LIMIT k (1 <= k <= 32) over rows where cond
 * holds; ties broken by ascending row index.  Outputs (device, nullable):
 * order keys, row_base + row indices, and (float)select_expr at those rows
 * (select_expr NULL = the order key).  The count (<= k) goes to d_count / h_count. */
wx_status wx_topk(const wx_table *table, const char *order_expr, const char *cond,
                  const char *select_expr, int32_t k, int32_t descending,
                  const wx_launch *launch, int64_t row_base, float *d_keys, int64_t *d_idx,
                  float *d_vals, int64_t *d_count, int64_t *h_count, char *err, size_t errlen);

/* One shard's ORDER BY .. LIMIT candidates in the exchange layout (520 bytes):
 * wx_topk's d_keys / d_vals / d_idx / d_count pointed at keys, vals, rows and
 * count fill it, so the records of all shards are one all-gather of bytes. */
typedef struct wx_topk_record {
  float keys[32];
  float vals[32];
  int64_t rows[32]; /* global row numbers (wx_topk's row_base + row) */
  int64_t count;    /* valid candidates, <= k */
} wx_topk_record;

/* Global ORDER BY .. LIMIT k of a row-sharded query (the
 * reference gathers dense shard results on the host, src/multi_gpu_utils.cpp:
 * 23-60, then sorts them, src/warpdb.cpp:453-455,483-495) from the records
 * of every shard (device memory, n_records * k <= 4096): better key first (NaN
 * last, -0.0 == +0.0), ties by the smaller row.  Outputs as wx_topk; the
 * count (<= k) goes to d_count / h_count.  Runs on the device, no host read. */
wx_status wx_topk_merge(const wx_topk_record *d_records, int32_t n_records, int32_t k, int32_t descending,
                        const wx_launch *launch, float *d_keys, int64_t *d_idx, float *d_vals,
                        int64_t *d_count, int64_t *h_count, char *err, size_t errlen);

/* ORDER BY .. LIMIT of any length over row shards (the k > 32 form of
 * wx_topk / wx_topk_merge; single-GPU query_sql sorts the whole projection
 * with wx_sort_*_limit, src/warpdb.cpp:453-455,483-495).  A head record of
 * capacity cap holds: count (int64) | keys (float x cap) | vals (float x cap)
 * | rows (int64 x cap); WX_HEAD_RECORD_BYTES(cap) bytes, so the records of all
 * shards are one all-gather of bytes.
 *
 * wx_order_head: this shard's first min(limit, passing) rows in ORDER BY
 * order -- the rows passing cond, keyed by order_expr, stably sorted (the
 * order of wx_sort_by_key: NaN keys last, -0.0 == +0.0, ties by ascending
 * row), with select_expr's value (null: the key) and the global row
 * (row_base + row) -- written to d_record (limit <= cap).  Synchronous (the
 * sort needs the passing count).  Scratch: 16 bytes per table row.  A shard
 * holds at most 2^31 - 1 rows (WX_ERR_UNSUPPORTED beyond).
 *
 * wx_head_merge: the global head of n_records shard records (record order =
 * row order): the first min(limit, total) of their candidates in the same
 * order, keys / rows / vals to the (nullable) outputs, the count to d_count /
 * h_count.  n_records * cap < 2^32. */
#define WX_HEAD_RECORD_BYTES(cap) (8 + 16 * (int64_t)(cap))
wx_status wx_order_head(const wx_table *table, const char *order_expr, const char *cond, const char *select_expr,
                        int64_t limit, int32_t descending, const wx_launch *launch, int64_t row_base, void *d_record,
                        int64_t cap, char *err, size_t errlen);
wx_status wx_head_merge(const void *d_records, int32_t n_records, int64_t cap, int64_t limit, int32_t descending,
                        const wx_launch *launch, float *d_keys, int64_t *d_rows, float *d_vals, int64_t *d_count,
                        int64_t *h_count, char *err, size_t errlen);

/* In-place sorts used by the legacy jit_sort_* entry points.  Stable. */
wx_status wx_sort_pairs(int32_t *d_keys, float *d_vals, int64_t count, int32_t ascending,
                        const wx_launch *launch, char *err, size_t errlen);
wx_status wx_sort_float(float *d_vals, int64_t count, int32_t ascending, const wx_launch *launch,
                        char *err, size_t errlen);
/* As wx_sort_float, reading the keys from d_src (not written) and leaving
 * the sorted keys in d_dst: ORDER BY a bare float column with no WHERE sorts
 * straight out of the column instead of projecting a copy first
 * (query_sql's projection + jit_sort_float, src/warpdb.cpp:450-455,
 * src/jit.cpp:283-307).  d_src == d_dst sorts in place; partial overlap is
 * refused. */
wx_status wx_sort_float_from(const float *d_src, float *d_dst, int64_t count, int32_t ascending,
                             const wx_launch *launch, char *err, size_t errlen);
/* Stable sort of float keys carrying a 4-byte payload (the ORDER BY key of
 * each selected row and its SELECT value: the keyed sort query_sql intends,
 * src/warpdb.cpp:470-476).  Same order as wx_sort_float: NaN keys last,
 * -0.0 == +0.0, ties keep their input order. */
wx_status wx_sort_by_key(float *d_keys, float *d_vals, int64_t count, int32_t ascending,
                         const wx_launch *launch, char *err, size_t errlen);

/* ORDER BY .. LIMIT: as wx_sort_float / wx_sort_by_key, but only the first
 * min(limit, count) positions are required to hold the sorted order (the
 * rest of the buffers is left unspecified). */
wx_status wx_sort_float_limit(float *d_vals, int64_t count, int64_t limit, int32_t ascending,
                              const wx_launch *launch, char *err, size_t errlen);
wx_status wx_sort_by_key_limit(float *d_keys, float *d_vals, int64_t count, int64_t limit,
                               int32_t ascending, const wx_launch *launch, char *err, size_t errlen);

/* Seeded synthetic column generator (counter-based, so every shard can
 * generate its own rows on the device):  h = splitmix64(row + seed * 0xD1B54A32D192ED03)
 *   kind 0: uniform float  lo + ((h >> 40) * 2^-24) * (hi - lo)   (float arithmetic)
 *   kind 1: uniform int    lo + (h >> 32) % (hi - lo + 1)
 * row = row_base + i; the value is converted to `dtype`. */
wx_status wx_fill_synthetic(void *d_ptr, int32_t dtype, int64_t n, uint64_t seed,
                            int32_t kind, double lo, double hi, int64_t row_base,
                            const wx_launch *launch, char *err, size_t errlen);

/* Build (and cache) the kernels a call would use, without launching.  Works
 * without a GPU (arch taken from $WARPDB_ARCH, default gfx950).  op: 0 project
 * dense, 1 project compact, 2 sum, 3 group, 4 topk (k = LIMIT; for sum and
 * group, k = 1 selects the MIN / MAX build).  src_out (nullable)
 * receives the generated HIP source. */
wx_status wx_prepare(const wx_table *table, int32_t op, const char *expr, const char *cond,
                     const char *aux_expr, int32_t k, const wx_launch *launch, char *src_out,
                     size_t src_len, char *err, size_t errlen);

/* Synchronise `stream` and report any device-side failure flagged since the
 * last check (look-back timeout, table capacity). */
wx_status wx_check(const wx_launch *launch, char *err, size_t errlen);

/* Sum of the HIP-event durations of the main kernels launched with WX_F_TIME
 * (by any thread of the process) since the last read, and their number
 * (synchronises on the recorded events).  _device: only those launched on
 * `device`; the others stay for a later read. */
wx_status wx_timing_read(double *total_ms, int64_t *launches, char *err, size_t errlen);
wx_status wx_timing_read_device(int32_t device, double *total_ms, int64_t *launches, char *err, size_t errlen);

/* Kernel-cache statistics: compiled modules and hits since load. */
void wx_cache_stats(int64_t *compiles, int64_t *hits);

/* Release cached modules and workspaces of every device. */
void wx_shutdown(void);

int32_t wx_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* WARPEXEC_H */
