// wx_args.h -- kernel argument blocks shared by the host runtime
// (warpexec.cpp includes this file) and the device templates (warpexec
// prepends the same text to every hiprtc program), so the two layouts can
// never drift.  Plain C++ only: no host or device headers.
#ifndef WX_ARGS_H
#define WX_ARGS_H

typedef unsigned long long wx_u64;
typedef long long wx_i64;
typedef unsigned int wx_u32;

#define WX_MAX_COLS 16
#define WX_BLOCK 256
#define WX_WAVES (WX_BLOCK / 64)

// device-side error bits, OR-ed into the workspace counter word ctrs[1]
#define WX_DEVERR_LOOKBACK 1u
#define WX_DEVERR_CAPACITY 2u
#define WX_DEVERR_UNSUPPORTED 4u
#define WX_DEVERR_INTERNAL_KEY 8u  // GROUP BY consistency check: a key outside its planned range, or counts that disagree
// Look-back abort report, workspace ctrs[WX_LBD_BASE ..  + 4]: [0] claim (the
// first aborting waiter sets it and fills the rest), [1] kind | launch epoch
// << 8 | digit << 16 | pass << 32, [2] the waiting tile, [3] the tile it
// waited on, [4] that tile's status word as last seen.  Cleared by the host.
#define WX_LBD_BASE 3
#define WX_LBD_COMPACT 1u
#define WX_LBD_RADIX 2u

#define WX_OP_DENSE 0
#define WX_OP_COMPACT 1
#define WX_OP_SUM 2
#define WX_OP_GROUP 3
#define WX_OP_TOPK 4
#define WX_OP_UTIL 5

#ifndef WX_COMPACT_GROUPS
#define WX_COMPACT_GROUPS 4  // row quads per thread per tile (host passes its choice)
#endif
#ifndef WX_COMPACT_DWAVES
#define WX_COMPACT_DWAVES 15  // data waves per compaction workgroup (host passes its choice)
#endif
#define WX_GROUP_WINDOW 2048
#ifndef WX_GBLOCK
#define WX_GBLOCK 512  // wx_group_sum workgroup size (host and device agree through this header)
#endif
#define WX_GROUP_HSORT_MAX 4096
#define WX_TOPK_MAX 32
#define WX_TOPK_SLOTS 64        // top-K grid-wide bound: one slot per wave lane
#define WX_TOPK_SLOT_STRIDE 64  // u32 elements between slots (256 B)
#define WX_TOPK_SEED_SPANS 128  // top-K seed pass: workgroups, one 8 192-row span each (~1M rows)
#define WX_SORT_LDS (WX_BLOCK * 8)
// LSD radix sort (wx_radix_*): 8-bit digits, 4 passes over 32-bit keys;
// one tile = WX_RS_BLOCK threads x WX_RS_ITEMS keys, one 64-bit look-back
// status word per (tile, digit).
#ifndef WX_RS_BLOCK
#define WX_RS_BLOCK 1024  // >= 256: threads 0..255 own one digit each
#endif
#ifndef WX_RS_ITEMS
#define WX_RS_ITEMS 32
#endif
#define WX_RS_TILE (WX_RS_BLOCK * WX_RS_ITEMS)
#define WX_RS_EPOCHS 63
#define WX_CS_EPOCHS 63  // compaction status epochs (6 bits, 0 = never written)

struct WxDenseArgs {
  const void *col[WX_MAX_COLS];
  float *out;
  wx_i64 n_rows;
  int fill;
};

struct WxCompactArgs {
  const void *col[WX_MAX_COLS];
  float *out_val;     // nullable
  void *out_idx;      // nullable; int32 or int64
  wx_u64 *status;     // [n_tiles + 1] {epoch:6 | flag:2 | value:56}; [n_tiles] = abort word
  wx_u64 *ctrs;       // [0] tile ticket, [1] error bits, [2] retired workgroups (0 between launches), [3..7] WX_LBD_*
  wx_i64 *count_out;  // nullable
  wx_i64 n_rows;
  wx_i64 n_tiles;
  wx_i64 row_base;
  int idx64;
  wx_u32 epoch;  // 1..WX_CS_EPOCHS: tags this launch's status words
  wx_u64 *diag;  // nullable; WX_DIAG_PROFILE builds: [block][16] phase times (10 ns ticks)
};

struct WxSumArgs {
  const void *col[WX_MAX_COLS];
  double *part_sum;  // [gridDim.x]
  wx_i64 *part_cnt;  // [gridDim.x]
  wx_u32 *part_min;  // [gridDim.x] order-mapped (WX_MINMAX builds)
  wx_u32 *part_max;  // [gridDim.x]
  wx_i64 n_rows;
};

struct WxGroupFinArgs {
  double *win_sum;
  wx_u64 *win_cnt;
  wx_u64 *h_tag;
  double *h_sum;
  wx_u64 *h_cnt;
  wx_u32 *h_used;
  wx_u64 *ctrs;
  wx_u32 *win_min;
  wx_u32 *win_max;
  wx_u32 *h_min;
  wx_u32 *h_max;
  int *out_keys;
  double *out_sums;
  wx_i64 *out_counts;
  float *out_mins;  // nullable
  float *out_maxs;  // nullable
  wx_i64 *n_groups_out;
  wx_i64 capacity;
  int key_lo;
  const wx_u64 *sorted;  // nullable: general-key entries pre-sorted on the device (> WX_GROUP_HSORT_MAX)
  // nullable: partials mode (wx_group_partials): the window goes here densely
  // as [W sums | W counts as f64 | 1 out-of-window group count], and only the
  // out-of-window groups go to out_keys / out_sums / out_counts
  double *win_out;
  // nullable (partials mode): the one-collective exchange slots that follow
  // the window -- n_slots x (1 + 3 * slot_groups) doubles; this shard writes
  // its own slot (count, then (key, sum, count) triples) and zeros the others
  double *slots;
  int n_slots;
  int slot_rank;
  int slot_groups;
};

struct WxGroupArgs {
  const void *col[WX_MAX_COLS];
  wx_i64 n_rows;
  double *win_sum;  // [WX_GROUP_WINDOW]
  wx_u64 *win_cnt;  // [WX_GROUP_WINDOW]
  wx_u64 *h_tag;    // [hcap] 0 = empty, else (u32)key | 1<<32
  double *h_sum;    // [hcap]
  wx_u64 *h_cnt;    // [hcap]
  wx_u32 *h_used;   // [hcap] slots taken, in insertion order
  wx_u64 *ctrs;     // [0] used slots, [1] error bits
  wx_u32 *win_min;  // [WX_GROUP_WINDOW] order-mapped, ~0 = none (WX_MINMAX builds)
  wx_u32 *win_max;  // [WX_GROUP_WINDOW] order-mapped, 0 = none
  wx_u32 *h_min;    // [hcap]
  wx_u32 *h_max;    // [hcap]
  wx_u32 hmask;     // hcap - 1 (hcap a power of two)
  int key_lo;
};


// Slot layout of the one-collective GROUP BY exchange (wx_group_partials_slots)
#define WX_GROUP_EXCHANGE (2 * WX_GROUP_WINDOW + 1)
#define WX_GROUP_SLOT_MAX 4096  // n_slots * slot_groups bound (the merge sorts them in LDS)

// Final GROUP BY result from a combined one-collective exchange buffer: the
// window and every shard's slot of out-of-window groups.
struct WxGroupSlotsArgs {
  const double *exchange;  // [WX_GROUP_EXCHANGE + n_slots * (1 + 3 * slot_groups)]
  int n_slots;
  int slot_groups;
  int key_lo;
  int *out_keys;
  double *out_sums;
  wx_i64 *out_counts;
  wx_i64 capacity;
  wx_i64 *n_groups_out;  // -1: a shard's general-key table overflowed; -2: a slot overflowed (merge needed)
};

// Range-partitioned GROUP BY for many distinct keys (wx_group_part_*): the
// passing rows' keys span [key_lo, key_lo + P << shift); partition p holds
// keys [key_lo + p << shift, key_lo + (p + 1) << shift).  Each 16 384-row
// tile's passing rows are written back in place sorted by partition (f32
// value + u16 bin), a directory word per (partition, tile) locates the runs,
// each partition is aggregated in an LDS window of 1 << shift bins per work
// item, and the items' partial windows are summed into ascending-key output.
#define WX_GP_BLOCK 1024
struct WxGroupPartArgs {
  const void *col[WX_MAX_COLS];
  wx_i64 n_rows;
  wx_i64 rows_per_wg;   // minmax: contiguous rows per workgroup (a multiple of 4)
  wx_i64 n_tiles;       // tiles: ceil(n_rows / WX_GP_TILE)
  int tiles_per_wg;     // tiles of workgroup g: [g * tiles_per_wg, (g + 1) * tiles_per_wg)
  int n_wg;             // G: tile workgroups
  int n_part;           // P
  int key_lo;
  int shift;
  wx_i64 *mm;           // [gridDim.x][4] per workgroup (min key, max key, passing rows, rows outside the range)
  wx_u32 *pcount;       // [P][G] passing rows of partition p in workgroup g's tiles
  wx_u64 *ptotal;       // [P] passing rows of partition p (zero between calls: the plan clears it)
  wx_u32 *dir;          // [P][n_tiles] run of partition p in tile t: start | length << 16
  float *vals;          // [n_tiles * WX_GP_TILE] each tile's passing values, partition-sorted
  unsigned short *bins; // [n_tiles * WX_GP_TILE] their bins (key - key_lo - p << shift)
  wx_i64 *work;         // [work_cap][2]: (p << 40 | g0 << 20 | g1, 0)
  wx_i64 *n_work;
  wx_u32 *pitem;        // [P + 1] first work item of partition p
  wx_u32 *order;        // [work_cap] aggregation dispatch order (items by first workgroup)
  wx_i64 work_cap;
  wx_i64 chunk;         // at least this many rows per work item
  wx_i64 target_items;  // about this many work items over all partitions
  double *psum;         // [work_cap][1 << shift] partial window sums of each work item
  wx_u32 *pcnt;         // [work_cap][1 << shift] partial window counts
  wx_i64 *summary;      // [4] passing rows, rows outside the range, min key, max key (host-read)
  wx_u32 *pnz;          // [P] non-empty keys per partition
  int *out_keys;
  double *out_sums;
  wx_i64 *out_counts;
  wx_i64 capacity;
  wx_i64 *n_groups_out;
  wx_u64 *ctrs;  // [1]: error bits
  wx_u64 *diag;  // nullable; WX_GP_DIAG builds: [blockIdx][16] tile-phase times (10 ns ticks)
};

// Top-K exchange record of one shard (wx_topk_record in warpexec.h)
#define WX_TOPK_REC_BYTES (WX_TOPK_MAX * 16 + 8)
#define WX_TOPK_MERGE_MAX 4096  // n_records * k bound

struct WxTopkMergeArgs {
  const unsigned char *records;  // n_records x WX_TOPK_REC_BYTES
  int n_records;
  int k;
  int descending;
  float *out_keys;
  wx_i64 *out_idx;
  float *out_vals;
  wx_i64 *count_out;
};

// Final GROUP BY result from a combined exchange window (wx_group_partials
// layout) and the combined out-of-window groups (ascending keys, unique).
struct WxGroupCombineArgs {
  const double *window;  // [2 * WX_GROUP_WINDOW + 1]
  const int *x_keys;     // [n_extra], ascending, none inside the window
  const double *x_sums;
  const wx_i64 *x_counts;
  wx_i64 n_extra;
  int key_lo;
  int *out_keys;
  double *out_sums;
  wx_i64 *out_counts;
  wx_i64 capacity;
  wx_i64 *n_groups_out;
};

// Many-key row-sharded GROUP BY (wx_group_merge_lists): n_lists gathered
// list records (count, then list_cap keys / sums / counts, ascending unique
// keys) merged in (key, list) order into scratch, then the runs of equal keys
// summed in list order and merged with the (optional) combined window.
#define WX_GLIST_BLOCK 1024
#define WX_GLIST_PER 4  // merged positions per thread in the count / emit kernels
#define WX_GLIST_SPAN (WX_GLIST_BLOCK * WX_GLIST_PER)
struct WxGroupListsArgs {
  const unsigned char *lists;  // n_lists x list_bytes
  wx_i64 list_bytes;
  wx_i64 list_cap;
  wx_i64 sums_off;    // byte offsets inside one record
  wx_i64 counts_off;
  int n_lists;
  int key_lo;
  const double *window;  // nullable: [2 * WX_GROUP_WINDOW + 1] combined window
  int *m_keys;           // scratch [n_lists * list_cap], merged order
  double *m_sums;
  wx_i64 *m_cnts;
  wx_u32 *m_head;  // 1: first of its key in merged order
  wx_i64 *blk;     // [n_blk] heads per WX_GLIST_SPAN positions -> exclusive prefix
  wx_i64 n_blk;
  wx_i64 *meta;  // [0] merged elements, [1] unique keys below key_lo, [2] non-empty window bins, [3] status
  int *out_keys;
  double *out_sums;
  wx_i64 *out_counts;
  wx_i64 capacity;
  wx_i64 *n_groups_out;  // -1: a list's count was negative or above list_cap
};

// General-key entries -> (key ^ sign) << 32 | used-list position, padded
// with ~0 to npad, for the device-wide sort of a large GROUP BY.
struct WxGroupGatherArgs {
  const wx_u64 *ctrs;
  const wx_u32 *h_used;
  const wx_u64 *h_tag;
  wx_u64 *keys;
  wx_i64 npad;
};

struct WxTopkArgs {
  const void *col[WX_MAX_COLS];
  wx_u32 *cand_k;    // [gridDim.x * K]
  wx_i64 *cand_i;    // [gridDim.x * K]
  wx_u32 *g_thresh;  // [WX_TOPK_SLOTS * WX_TOPK_SLOT_STRIDE] lower bounds on the K-th best rank (0 = none), zeroed per call
  wx_i64 n_rows;
  wx_i64 q_stride;   // row quads between consecutive workgroups' first spans (the scan: one span)
  wx_i64 q_step;     // row quads a workgroup advances per batch (the scan: gridDim.x spans)
};

struct WxTopkFinArgs {
  const void *col[WX_MAX_COLS];
  const wx_u32 *cand_k;
  const wx_i64 *cand_i;
  wx_i64 n_cand;
  wx_i64 row_base;
  float *out_keys;
  wx_i64 *out_idx;
  float *out_vals;
  wx_i64 *count_out;
  wx_u32 *g_thresh;  // the scan's grid-wide bound slots: zeroed here for the next query
  int seed;          // 1: the seed pass -- raise slot 0 to the K-th best rank, keep the slots, no outputs
};

struct WxFillArgs {
  void *out;
  wx_i64 n;
  wx_u64 seed;
  double lo, hi;
  wx_i64 row_base;
  int dtype;
  int kind;
};

struct WxCastArgs {
  const void *src;
  void *dst;
  wx_i64 n;
  int src_dtype;  // wx_dtype numbering (0 int32, 1 int64, 2 float32, 3 float64)
  int dst_dtype;
};

// ORDER BY .. LIMIT heads of any length (wx_order_head / wx_head_merge).  A
// head record is count i64 | keys f32[cap] | vals f32[cap] | rows i64[cap]
// (WX_HEAD_RECORD_BYTES in warpexec.h).
struct WxHeadArgs {
  wx_i64 n;               // iota: elements
  wx_u32 *idx;            // iota output; gather / emit: sorted positions (the sort's payload)
  const float *keys;      // gather / emit: sorted keys
  const float *vals;      // gather: SELECT values by position (null: the keys themselves)
  const int *rows;        // gather: shard-local rows by position
  wx_i64 row_base;
  const wx_i64 *count;    // gather: passing rows; emit: gathered candidates (device)
  wx_i64 limit;
  unsigned char *record;  // gather: this shard's head record
  float *cat_keys;        // concat: every record's keys, record-major
  wx_u32 *cat_idx;        // concat: their record * cap + position
  wx_i64 *cat_count;      // concat: candidates
  const unsigned char *records;  // concat / emit: n_records head records
  int n_records;
  wx_i64 cap;
  float *out_keys;
  wx_i64 *out_rows;
  float *out_vals;
  wx_i64 *count_out;
};

// Row-order GROUP BY sums (WX_F_ROW_ORDER): the passing rows' values sorted
// stably by key (row order within a key), folded per group one double add at
// a time.
struct WxGroupFoldArgs {
  const int *skeys;        // [m] sorted keys
  const float *svals;      // [m] their values, row order within a key
  wx_i64 m;
  const int *gkeys;        // [n_groups] the groups, ascending
  const wx_i64 *gcounts;   // [n_groups] their row counts
  wx_i64 n_groups;
  double *out_sums;        // [n_groups]
  wx_u64 *ctrs;            // [1]: error bits (a group whose rows do not match its count)
  wx_i64 skip_above;       // > 0: groups of more rows are folded by the wx_xf_big_* kernels instead
  wx_i64 *starts;          // [n_groups] each group's first row in the sorted arrays (the counts' exclusive prefix)
  wx_i64 *chunk_sums;      // [n_chunks] the counts' sums per WX_GS_CHUNK groups, then their exclusive prefix
  wx_i64 n_chunks;
  wx_i64 small_max;        // groups of at most this many rows: one lane each (wx_group_fold_small)
  wx_i64 *big_list;        // [n_groups] the other groups, for wx_group_fold (one wave each), in any order
  wx_u32 *big_n;           // [1] their number (zeroed before wx_group_fold_small)
};
// The groups of a key-sorted array by run-length encoding (the general
// row-order path without the ordinary call): wx_rle_count / _scan / _emit /
// _counts.  Wave r of n_blk (WX_RLE_BLOCK / 64 per workgroup) takes rows
// [r * span, (r + 1) * span), span a multiple of 64.
struct WxRleArgs {
  const int *sk;           // [m] sorted keys
  wx_i64 m;
  wx_i64 span;             // rows per wave
  int n_blk;               // wave ranges
  wx_i64 *blk;             // [n_blk] runs starting in each wave's rows, then their exclusive prefix
  wx_i64 *n_out;           // [1] the runs (groups)
  wx_i64 *n_groups_out;    // the caller's group count (nullable)
  wx_i64 capacity;         // outputs beyond it are not written
  int *out_keys;           // [capacity] each run's key, ascending
  wx_i64 *out_counts;      // [capacity] its length
  wx_i64 *starts;          // [capacity] its first row
};
#define WX_RLE_BLOCK 1024
// wx_group_starts_*: WX_GS_BLOCK threads, WX_GS_PER consecutive groups each
#define WX_GS_BLOCK 256
#define WX_GS_PER 16
#define WX_GS_CHUNK (WX_GS_BLOCK * WX_GS_PER)
#define WX_FOLD_SMALL 4096

// Row-order folds of groups larger than WX_XF_BIG rows, split into chunks of
// WX_XF_CHUNK values (wx_xf_big_approx / _exact / _combine, wx_util.hip).
#define WX_XF_CHUNK (1 << 16)
#define WX_XF_BIG (4 << 20)
struct WxXfBigArgs {
  const float *svals;   // key-major values, row order within a group
  const wx_i64 *ent;    // [n_ent][4]: group index, first value, values, first chunk (ascending)
  int n_ent;
  wx_i64 n_chunks;      // chunks over all entries
  double *approx;       // [n_chunks] each chunk's sum in any order
  double *rec;          // [n_chunks][8] under a guessed binade: k, sum r (ties after the first), bound on sum |r|, ok, has a tie, cf
  double *out_sums;     // [n_groups]
};

struct WxSortPrepArgs {
  const void *src;
  wx_u64 *keys;
  wx_i64 n;
  wx_i64 npad;
  int kind;  // 0 float values, 1 int keys
  int ascending;
};

struct WxSortPassArgs {
  wx_u64 *keys;
  wx_i64 npad;
  wx_i64 k;
  wx_i64 j;  // global pass: partner distance; LDS pass: kend
};

struct WxSortApplyArgs {
  const wx_u64 *keys;
  wx_i64 n;
  const void *src_a;
  void *dst_a;
  const float *src_v;
  float *dst_v;
};

struct WxRadixHistArgs {
  const wx_u32 *src;
  wx_i64 n;
  wx_u32 *hist;  // [4][256], zeroed by the host
  int aligned;   // src is 16-byte aligned
};

struct WxRadixPassArgs {
  const wx_u32 *src_k;
  wx_u32 *dst_k;
  const wx_u32 *src_v;  // payload (pairs) or null
  wx_u32 *dst_v;
  const wx_u32 *digit_base;  // [256]: first output slot of each digit
  wx_u64 *status;            // [n_tiles][256] look-back words {epoch:6 | flag:2 | count:56}
  wx_u32 *ctl;               // [0] tile ticket, [1] abort word
  wx_u32 *err;               // sticky device error bits (workspace ctrs[1])
  wx_u64 *lbd;               // look-back abort report (workspace ctrs[WX_LBD_BASE], WX_LBD_*)
  wx_i64 n;
  int shift;
  int kind;
  int ascending;
  wx_u32 epoch;  // 1..WX_RS_EPOCHS
  int lead;      // 1: rank lane 0's digit group by one ballot (a skewed digit); 0: one LDS add per key
};

// Row-order GROUP BY over a key span of at most 2048 (wx_group_rows.hip)
#define WX_RO_TILE_ROWS 8192
#define WX_RO_THREADS 512
struct WxRoArgs {
  const void *col[WX_MAX_COLS];
  wx_i64 n_rows;
  int key_lo;
  int span;           // the passing rows' keys lie in [key_lo, key_lo + span), span <= 2048
  int ranges;         // static ranges of whole tiles, one workgroup each
  wx_u32 *cnt;        // wx_ro_count: [ranges][2048] passing rows per (range, key - key_lo)
  const wx_u32 *off;  // wx_ro_scatter: [ranges][2048] first output slot of each bin in each range
  float *out;         // wx_ro_scatter: the passing rows' values, key-major, row order within a key
  wx_u64 *ctrs;       // [1]: error bits (a key outside the span)
  wx_i64 *info;       // nullable; the direct path: [2] set when a key lies outside the span (no error bit)
};

struct WxRoScanArgs {
  const wx_u32 *cnt;   // [ranges][2048]
  wx_u32 *totals;      // [2048] or null
  const wx_u32 *base;  // [2048] (with off)
  wx_u32 *off;         // [ranges][2048] or null
  int ranges;
};

struct WxRoBaseArgs {
  const wx_u32 *totals;    // [2048]
  wx_u32 *base;            // [2048] exclusive prefix of the totals
  const int *gkeys;        // [n_groups] the ordinary call's groups
  const wx_i64 *gcounts;   // [n_groups]
  wx_i64 n_groups;
  int key_lo;
  wx_u64 *ctrs;            // [1]: error bits (counts that do not match; capacity)
  // the direct path (out_counts set): the groups come from the totals instead
  // of an ordinary call -- keys / counts of the non-empty bins in ascending
  // order (at most capacity of them), their number, and info[0] groups,
  // info[1] passing rows, info[3] / info[4] the smallest / largest key
  int *out_keys;
  wx_i64 *out_counts;
  wx_i64 capacity;
  wx_i64 *n_groups_out;
  wx_i64 *info;
};

struct WxRoFoldArgs {
  const float *svals;      // the key-major values (group g's rows after the groups before it)
  const wx_i64 *gcounts;   // [n_groups]
  wx_i64 n_groups;
  double *out_sums;        // [n_groups]
  wx_i64 skip_above;       // > 0: groups of more rows are folded by the wx_xf_big_* kernels instead
};

struct WxSumFinArgs {
  const double *part_sum;
  const wx_i64 *part_cnt;
  const wx_u32 *part_min;
  const wx_u32 *part_max;
  double *out;  // wx_stats: {sum f64, count i64, min f32, max f32} (min/max in WX_MINMAX builds)
  int n_parts;
  int count_f64;  // write the count as a double (WX_F_F64_COUNTS: all-reduce layout)
};

#endif  // WX_ARGS_H
