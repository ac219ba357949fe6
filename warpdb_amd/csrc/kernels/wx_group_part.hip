// wx_group_part.hip -- GROUP BY over many distinct keys: the range-partitioned kernels
// (one of the kernel sources warpexec concatenates after wx_common.hip, whose
// header describes the prelude they expect)

#if WX_OP == WX_OP_GROUP
// ---------------------------------------------------------------------------
// Range-partitioned GROUP BY (many distinct keys).  With 1e6 keys and 1e9
// rows every workgroup sees each key about once, so neither the LDS window nor
// a per-workgroup LDS hash can absorb anything and the global hash pays two
// memory-side atomics per row (9.1 ms per 1e8 rows, 1 % of the read
// roofline).  Instead the rows are partitioned by key range so that each
// partition fits an LDS window of 1 << shift bins.  Round 4 layout (no
// counting pass, no partial-line scatter):
//   tiles  each 16 384-row tile is counting-sorted by partition in LDS and
//          written back IN PLACE (tile t's passing rows at [t * TILE, ...)):
//          f32 values + u16 bins (6 B per passing row, full-line stores),
//          plus a directory word (run start | run length << 16) per
//          (partition, tile) and per-(workgroup, partition) totals; the
//          passing rows' exact key range and the rows outside the planned
//          range are counted on the way (mm)
//   plan   one workgroup: range summary, and per partition its aggregation
//          work items (runs of whole workgroup tile ranges, about `chunk`
//          rows each); nothing to aggregate when some row fell outside
//   agg    per work item: the partition's runs of its tiles gathered through
//          the directory into an LDS window (ds_add_f64 / ds_add_u32),
//          written as the item's partial window (plain stores, no atomics)
//   count / scan2 / emit   non-empty keys per partition (over its items'
//          partial windows), their prefix, and the outputs in ascending key
//          order (the partials summed)
#define WX_GP_UNROLL 2
#define WX_GP_SPAN ((wx_i64)WX_GP_BLOCK * WX_GP_UNROLL)
#define WX_GP_QUAD(u) (wx_base + (wx_i64)(u) * WX_GP_BLOCK + threadIdx.x)
#define WX_DECL_GP(name, T, slot) T wx_u##slot[WX_GP_UNROLL][4];
#define WX_LOAD_GP_FAST(name, T, slot) ::wx::load4_full<T>(wx_a.col[slot], wx_r0u, wx_u##slot[wx_u]);
#define WX_LOAD_GP(name, T, slot) ::wx::load4_tail<T>(wx_a.col[slot], wx_r0u, wx_rend, wx_u##slot[wx_u]);
// rows [RB, RE) of this workgroup (RB a multiple of 4), WX_GP_SPAN quads per
// step, WX_GP_BLOCK threads (the launch must use that block size)
#define WX_RANGE_LOOP_BEGIN(RB, RE)                                                                 \
  const wx_i64 wx_rend = (RE);                                                                      \
  const wx_i64 wx_qe = (wx_rend + 3) >> 2, wx_qfull = wx_rend >> 2;                                 \
  for (wx_i64 wx_base = (RB) >> 2; wx_base < wx_qe; wx_base += WX_GP_SPAN) {                        \
    WX_COLS(WX_DECL_GP)                                                                             \
    if (WX_ALIGNED16 && wx_base + WX_GP_SPAN <= wx_qfull) {                                         \
      _Pragma("unroll") for (int wx_u = 0; wx_u < WX_GP_UNROLL; ++wx_u) {                          \
        const wx_i64 wx_r0u = WX_GP_QUAD(wx_u) << 2;                                                \
        WX_COLS(WX_LOAD_GP_FAST)                                                                    \
      }                                                                                             \
    } else {                                                                                        \
      _Pragma("unroll") for (int wx_u = 0; wx_u < WX_GP_UNROLL; ++wx_u) {                          \
        const wx_i64 wx_r0u = WX_GP_QUAD(wx_u) << 2;                                                \
        WX_COLS(WX_LOAD_GP)                                                                         \
      }                                                                                             \
    }                                                                                               \
    _Pragma("unroll") for (int wx_u = 0; wx_u < WX_GP_UNROLL; ++wx_u) {                            \
      const wx_i64 wx_r0 = WX_GP_QUAD(wx_u) << 2;                                                   \
      if (WX_GP_QUAD(wx_u) < wx_qe) {                                                               \
        _Pragma("unroll") for (int wx_e = 0; wx_e < 4; ++wx_e) {                                   \
          WX_COLS(WX_BIND_U)                                                                        \
          const wx_i64 idx = wx_r0 + wx_e;
#define WX_RANGE_LOOP_END \
  }                       \
  }                       \
  }                       \
  }

// Block-wide (min key, max key, passing rows, outside rows) of per-thread
// values, written by thread 0 to mm[4 * blockIdx.x ...] (WX_GP_BLOCK threads)
template <int NT = WX_GP_BLOCK>
__device__ __forceinline__ void wx_gp_stats_out(int mn, int mx, wx_u64 c, wx_u64 o, wx_i64 *mm) {
  __shared__ int s_mn[NT / 64], s_mx[NT / 64];
  __shared__ wx_u64 s_c[NT / 64], s_o[NT / 64];
#pragma unroll
  for (int k = 32; k > 0; k >>= 1) {
    const int a = __shfl_xor(mn, k), b = __shfl_xor(mx, k);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
    c += __shfl_xor(c, k);
    o += __shfl_xor(o, k);
  }
  if ((threadIdx.x & 63) == 0) {
    const int w = threadIdx.x >> 6;
    s_mn[w] = mn; s_mx[w] = mx; s_c[w] = c; s_o[w] = o;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < NT / 64; ++w) {
      mn = s_mn[w] < mn ? s_mn[w] : mn;
      mx = s_mx[w] > mx ? s_mx[w] : mx;
      c += s_c[w];
      o += s_o[w];
    }
    mm[4 * blockIdx.x] = mn;
    mm[4 * blockIdx.x + 1] = mx;
    mm[4 * blockIdx.x + 2] = (wx_i64)c;
    mm[4 * blockIdx.x + 3] = (wx_i64)o;
  }
}

// Exact (min, max) key and passing rows of each workgroup's contiguous row
// range (the probe when no sample guess is usable); WX_GP_BLOCK threads.
extern "C" __global__ __launch_bounds__(WX_GP_BLOCK) void wx_group_part_minmax(WxGroupPartArgs wx_a) {
  int wx_mn = 0x7fffffff, wx_mx = (int)0x80000000;
  wx_u64 wx_c = 0;
  const wx_i64 wx_rb = (wx_i64)blockIdx.x * wx_a.rows_per_wg;
  const wx_i64 wx_re = wx_rb + wx_a.rows_per_wg < wx_a.n_rows ? wx_rb + wx_a.rows_per_wg : wx_a.n_rows;
  {
    WX_RANGE_LOOP_BEGIN(wx_rb, wx_re)
    if (idx < wx_rend && WX_EVAL_COND()) {
      const int wx_k = static_cast<int>(WX_KEY);
      wx_mn = wx_k < wx_mn ? wx_k : wx_mn;
      wx_mx = wx_k > wx_mx ? wx_k : wx_mx;
      ++wx_c;
    }
    WX_RANGE_LOOP_END
  }
  wx_gp_stats_out(wx_mn, wx_mx, wx_c, 0ull, wx_a.mm);
}

// A strided sample of the rows (thread i: row i * n / S): the (min, max) key
// and passing rows per workgroup, from which the host guesses the range of
// the first pass (mm[4g .. 4g+2]).
extern "C" __global__ __launch_bounds__(WX_GP_BLOCK) void wx_group_part_sample(WxGroupPartArgs wx_a) {
  int wx_mn = 0x7fffffff, wx_mx = (int)0x80000000;
  wx_u64 wx_c = 0;
  const wx_i64 wx_s = (wx_i64)gridDim.x * WX_GP_BLOCK;
  const wx_i64 wx_i = (wx_i64)blockIdx.x * WX_GP_BLOCK + threadIdx.x;
  if (wx_a.n_rows > 0) {
    const wx_i64 idx = wx_i * (wx_a.n_rows / wx_s) + (wx_i * (wx_a.n_rows % wx_s)) / wx_s;  // i * n / S
    WX_COLS(WX_BIND_ROW)
    if (WX_EVAL_COND()) {
      const int wx_k = static_cast<int>(WX_KEY);
      wx_mn = wx_k;
      wx_mx = wx_k;
      wx_c = 1;
    }
  }
  wx_gp_stats_out(wx_mn, wx_mx, wx_c, 0ull, wx_a.mm);
}

// Exclusive scan of a device array of n values (one 1024-thread block, 4
// consecutive values per thread per step); returns the total to every thread.
template <typename In, typename Out>
__device__ __forceinline__ wx_i64 wx_block_scan_excl(const In *in, Out *out, wx_i64 n, wx_i64 *s_w) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  wx_i64 carry = 0;
  for (wx_i64 base = 0; base < n; base += 4 * 1024) {
    wx_i64 v[4], loc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const wx_i64 i = base + (wx_i64)tid * 4 + j;
      v[j] = i < n ? (wx_i64)in[i] : 0;
      loc += v[j];
    }
    wx_i64 incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const wx_i64 t = __shfl_up(incl, o);
      if (lane >= o) incl += t;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    wx_i64 wb = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      const wx_i64 x = s_w[w];
      wb += w < wave ? x : 0;
      tot += x;
    }
    wx_i64 run = carry + wb + incl - loc;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const wx_i64 i = base + (wx_i64)tid * 4 + j;
      if (i < n) out[i] = (Out)run;
      run += v[j];
    }
    carry += tot;
    __syncthreads();
  }
  return carry;
}

// Exclusive scan over the block (WX_GP_BLOCK threads, one value each) of
// u32 values; s_w holds WX_GP_BLOCK / 64 words.  Returns the exclusive
// prefix, the total in *tot.
__device__ __forceinline__ wx_u32 wx_gp_block_excl(wx_u32 v, wx_u32 *s_w, wx_u32 *tot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  wx_u32 incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const wx_u32 t = __shfl_up(incl, o);
    if (lane >= o) incl += t;
  }
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  wx_u32 wb = 0, tt = 0;
#pragma unroll
  for (int w = 0; w < WX_GP_BLOCK / 64; ++w) {
    const wx_u32 x = s_w[w];
    wb += w < wave ? x : 0u;
    tt += x;
  }
  *tot = tt;
  return wb + incl - v;
}

#define WX_GP_STAGE_MAXP 2048  // two partitions per thread in the tile scan
#ifndef WX_GP_SUNROLL
#define WX_GP_SUNROLL 4  // row quads per thread per tile (the host sizes the LDS and the tiles to match)
#endif
#ifndef WX_GP_TBLOCK
// the tile kernel's workgroup: 1024 threads, one per CU, 16 384-row tiles.
// 512 threads at two per CU (8192-row tiles) ran the tile pass 2.75 vs 2.90
// ms per 1e9 rows x 10^6 keys but halved the runs the aggregation gathers
// (≈ 66 rows): 2.11 vs 1.64 ms there, 4.98 vs 4.60 ms per query
#define WX_GP_TBLOCK 1024
#endif
#define WX_GP_TILE (WX_GP_TBLOCK * 4 * WX_GP_SUNROLL)
#define WX_GP_SSPAN ((wx_i64)WX_GP_TBLOCK * WX_GP_SUNROLL)
#define WX_GT_QUAD(u) (wx_base + (wx_i64)(u) * WX_GP_TBLOCK + threadIdx.x)
static_assert(WX_GP_TILE <= 32768, "directory words hold 16-bit run starts and lengths");
#define WX_DECL_GS(name, T, slot) T wx_u##slot[WX_GP_SUNROLL][4];
#define WX_LOAD_GS(name, T, slot) ::wx::load4_tail<T>(wx_a.col[slot], wx_r0u, wx_rend, wx_u##slot[wx_u]);
// Tiles [g * tiles_per_wg, ...) of workgroup g, software-pipelined: the next
// tile's column loads are issued as soon as this tile's rows are evaluated,
// so they are in flight during the LDS phases, and the previous tile's
// write-out (LDS -> HBM) opens each iteration, so its stores drain during
// this tile's evaluation.  Per tile, three barriers: evaluate and count rows
// per partition (ds_add); barrier; wave 0 scans the counts into run starts
// (the directory words, the run cursors, the workgroup's per-partition
// totals); barrier; every row placed at its run's next LDS slot (ds_add_rtn
// on the cursor: each row keeps only its 32-bit key offset and value in
// registers, no rank -- with the next tile's loads in flight a kept rank
// spills); barrier.  LDS: the tile's staged values (f32) and bins (u16) +
// 12 B per partition.
#ifndef WX_GP_PLACE_BATCH
// row quads whose cursor adds go out together in the place phase (0: one
// add and its stores at a time).  Batches measured slower: 1 / 2 / 4 quads
// 4.40 / 4.40 / 4.33 vs 4.24 ms per 1e9 rows x 10^6 keys
// (profiles/r04/abl_group_wide_place_batch.txt) -- the phase is bound by
// same-address cursor adds, not by round trips
#define WX_GP_PLACE_BATCH 0
#endif
#ifndef WX_GP_DIAG
#define WX_GP_DIAG 0  // diagnostic: per-phase times of waves 0 and 15 (s_memrealtime) into wx_a.diag
#endif
#if WX_GP_DIAG
#define WX_GT_PT(slot)                                                    \
  do {                                                                    \
    const wx_u64 wx_now = __builtin_amdgcn_s_memrealtime();               \
    wx_pt[slot] += wx_now - wx_pt_t;                                      \
    wx_pt_t = wx_now;                                                     \
  } while (0)
#else
#define WX_GT_PT(slot) \
  do {                 \
  } while (0)
#endif
extern "C" __global__ __launch_bounds__(WX_GP_TBLOCK) void wx_group_part_tiles(WxGroupPartArgs wx_a) {
  extern __shared__ wx_u32 wx_s_dyn[];
#if WX_GP_DIAG
  wx_u64 wx_pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  wx_u64 wx_pt_t = __builtin_amdgcn_s_memrealtime();
#endif
  float *s_val = reinterpret_cast<float *>(wx_s_dyn);                       // [WX_GP_TILE]
  unsigned short *s_bin = reinterpret_cast<unsigned short *>(s_val + WX_GP_TILE);  // [WX_GP_TILE]
  wx_u32 *s_cnt = reinterpret_cast<wx_u32 *>(s_bin + WX_GP_TILE);           // [P] this tile's rows of p
  wx_u32 *s_cur = s_cnt + wx_a.n_part;                                       // [P] next LDS slot of p's run
  wx_u32 *s_tot = s_cur + wx_a.n_part;                                       // [P] this workgroup's rows of p
  __shared__ wx_u32 s_tile_tot;
  const int P = wx_a.n_part;
  const int tid = threadIdx.x, lane = tid & 63;
  for (int p = tid; p < P; p += WX_GP_TBLOCK) { s_cnt[p] = 0u; s_tot[p] = 0u; }
  int wx_mn = 0x7fffffff, wx_mx = (int)0x80000000;
  wx_u64 wx_c = 0, wx_o = 0;
  const wx_i64 t_begin = (wx_i64)blockIdx.x * wx_a.tiles_per_wg;
  wx_i64 t_end = t_begin + wx_a.tiles_per_wg;
  t_end = t_end < wx_a.n_tiles ? t_end : wx_a.n_tiles;
  const wx_i64 wx_rb = t_begin * WX_GP_TILE;
  const wx_i64 wx_re = t_end * WX_GP_TILE < wx_a.n_rows ? t_end * WX_GP_TILE : wx_a.n_rows;
  const wx_u32 wx_bmask = (1u << wx_a.shift) - 1u;
  const wx_u32 wx_span = (wx_u32)P << wx_a.shift;
  const int ppl = (P + 63) / 64;  // wave 0's partitions per lane in the scan
  const wx_i64 wx_rend = wx_re;
  const wx_i64 wx_qe = (wx_rend + 3) >> 2, wx_qfull = wx_rend >> 2;
  WX_COLS(WX_DECL_GS)
  wx_i64 wx_base = wx_rb >> 2;
  // one tile's loads into the column registers (unguarded when whole)
#define WX_GS_LOAD_TILE()                                                        \
  if (WX_ALIGNED16 && wx_base + WX_GP_SSPAN <= wx_qfull) {                       \
    _Pragma("unroll") for (int wx_u = 0; wx_u < WX_GP_SUNROLL; ++wx_u) {        \
      const wx_i64 wx_r0u = WX_GT_QUAD(wx_u) << 2;                               \
      WX_COLS(WX_LOAD_GP_FAST)                                                   \
    }                                                                            \
  } else if (wx_base < wx_qe) {                                                  \
    _Pragma("unroll") for (int wx_u = 0; wx_u < WX_GP_SUNROLL; ++wx_u) {        \
      const wx_i64 wx_r0u = WX_GT_QUAD(wx_u) << 2;                               \
      WX_COLS(WX_LOAD_GS)                                                        \
    }                                                                            \
  }
  // the staged tile's passing rows in partition order, written in place: four
  // per thread (16-byte value stores, 8-byte bin stores; slots past `tot`
  // hold junk no directory run reaches)
#define WX_GS_WRITE_OUT(T, TOT)                                                         \
  {                                                                                     \
    typedef float f4v __attribute__((ext_vector_type(4)));                              \
    typedef unsigned short s4v __attribute__((ext_vector_type(4)));                     \
    f4v *ov = reinterpret_cast<f4v *>(wx_a.vals + (T) * WX_GP_TILE);                  \
    s4v *ob = reinterpret_cast<s4v *>(wx_a.bins + (T) * WX_GP_TILE);                  \
    const f4v *sv = reinterpret_cast<const f4v *>(s_val);                               \
    const s4v *sb = reinterpret_cast<const s4v *>(s_bin);                               \
    for (wx_u32 q = tid; 4 * q < (TOT); q += WX_GP_TBLOCK) {                             \
      __builtin_nontemporal_store(sv[q], ov + q);                                       \
      __builtin_nontemporal_store(sb[q], ob + q);                                       \
    }                                                                                   \
  }
  WX_GS_LOAD_TILE()
  __syncthreads();
  wx_u32 tot_prev = 0u;
  for (wx_i64 t = t_begin; t < t_end; ++t, wx_base += WX_GP_SSPAN) {
    if (t > t_begin) WX_GS_WRITE_OUT(t - 1, tot_prev)
    WX_GT_PT(0);
    wx_u32 wx_d[WX_GP_SUNROLL][4];  // key - key_lo, or >= P << shift: not staged (failed WHERE / outside)
    wx_u32 wx_v[WX_GP_SUNROLL][4];
#pragma unroll
    for (int wx_u = 0; wx_u < WX_GP_SUNROLL; ++wx_u) {
      const wx_i64 wx_r0 = WX_GT_QUAD(wx_u) << 2;
#pragma unroll
      for (int wx_e = 0; wx_e < 4; ++wx_e) {
        WX_COLS(WX_BIND_U)
        const wx_i64 idx = wx_r0 + wx_e;
        wx_d[wx_u][wx_e] = 0xffffffffu;
        wx_v[wx_u][wx_e] = 0u;
        if (idx < wx_rend && WX_EVAL_COND()) {
          const int wx_k = static_cast<int>(WX_KEY);
          const wx_u32 wx_dd = (wx_u32)wx_k - (wx_u32)wx_a.key_lo;
          wx_mn = wx_k < wx_mn ? wx_k : wx_mn;
          wx_mx = wx_k > wx_mx ? wx_k : wx_mx;
          ++wx_c;
          // keys below key_lo wrap to huge offsets: outside like keys above the range
          if (wx_dd < wx_span) {
            wx_d[wx_u][wx_e] = wx_dd;
            wx_v[wx_u][wx_e] = __float_as_uint(static_cast<float>(WX_EXPR));
            atomicAdd(&s_cnt[wx_dd >> wx_a.shift], 1u);
          } else {
            ++wx_o;
          }
        }
      }
    }
    // keep the next tile's loads below this tile's evaluation (hoisted above
    // it, both register sets are live at once and the kernel spills)
    __builtin_amdgcn_sched_barrier(0);
    WX_GT_PT(1);
    {  // the next tile's loads, in flight during this tile's LDS phases
      const wx_i64 wx_cur = wx_base;
      wx_base += WX_GP_SSPAN;
      WX_GS_LOAD_TILE()
      wx_base = wx_cur;
    }
    WX_GT_PT(2);
    __syncthreads();  // counts complete; the previous tile's write-out has read the stage
    WX_GT_PT(3);
    if (tid < 64) {
      // wave 0: exclusive scan of the counts (lane l: partitions [l ppl, (l + 1) ppl)),
      // the directory words and run cursors, the totals; the counts cleared.
      // The lane's partition range comes from a lane id computed here
      // (mbcnt, which the compiler rematerialises): derived from a value kept
      // across the tile loop it was spilled, and each scratch reload waited
      // (vmcnt) behind this wave's next-tile loads -- 1.9 us of every ~12-us
      // tile with the other 15 waves at the barrier (WX_GP_DIAG profile)
      const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
      const int pb = ln * ppl, pe = pb + ppl < P ? pb + ppl : P;
      wx_u32 loc = 0u;
      for (int p = pb; p < pe; ++p) loc += s_cnt[p];
      wx_u32 incl = loc;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const wx_u32 x = __shfl_up(incl, o);
        if (lane >= o) incl += x;
      }
      wx_u32 run = incl - loc;
      for (int p = pb; p < pe; ++p) {
        const wx_u32 c = s_cnt[p];
        s_cur[p] = run;
        s_cnt[p] = 0u;
        s_tot[p] += c;
        wx_a.dir[(wx_i64)p * wx_a.n_tiles + t] = run | (c << 16);
        run += c;
      }
      if (lane == 63) s_tile_tot = incl;
    }
    WX_GT_PT(4);
    __syncthreads();
    WX_GT_PT(5);
    tot_prev = s_tile_tot;
#if WX_GP_PLACE_BATCH
    // WX_GP_PLACE_BATCH row quads' cursor adds go out together
    // (unconditional: a row that is not staged adds 0 to partition 0's
    // cursor), then their stores -- one LDS round trip per batch instead of
    // one per row
#pragma unroll
    for (int wx_ub = 0; wx_ub < WX_GP_SUNROLL; wx_ub += WX_GP_PLACE_BATCH) {
      wx_u32 j[WX_GP_PLACE_BATCH][4];
#pragma unroll
      for (int wx_u = 0; wx_u < WX_GP_PLACE_BATCH; ++wx_u)
#pragma unroll
        for (int wx_e = 0; wx_e < 4; ++wx_e) {
          const wx_u32 dd = wx_d[wx_ub + wx_u][wx_e];
          const bool st = dd < wx_span;
          j[wx_u][wx_e] = atomicAdd(&s_cur[st ? dd >> wx_a.shift : 0u], st ? 1u : 0u);
        }
#pragma unroll
      for (int wx_u = 0; wx_u < WX_GP_PLACE_BATCH; ++wx_u)
#pragma unroll
        for (int wx_e = 0; wx_e < 4; ++wx_e)
          if (wx_d[wx_ub + wx_u][wx_e] < wx_span) {
            s_val[j[wx_u][wx_e]] = __uint_as_float(wx_v[wx_ub + wx_u][wx_e]);
            s_bin[j[wx_u][wx_e]] = (unsigned short)(wx_d[wx_ub + wx_u][wx_e] & wx_bmask);
          }
    }
#else
#pragma unroll
    for (int wx_u = 0; wx_u < WX_GP_SUNROLL; ++wx_u)
#pragma unroll
      for (int wx_e = 0; wx_e < 4; ++wx_e)
        if (wx_d[wx_u][wx_e] < wx_span) {
          const wx_u32 j = atomicAdd(&s_cur[wx_d[wx_u][wx_e] >> wx_a.shift], 1u);
          s_val[j] = __uint_as_float(wx_v[wx_u][wx_e]);
          s_bin[j] = (unsigned short)(wx_d[wx_u][wx_e] & wx_bmask);
        }
#endif
    WX_GT_PT(6);
    __syncthreads();
    WX_GT_PT(7);
  }
#if WX_GP_DIAG
  if ((threadIdx.x & 63) == 0 && (threadIdx.x == 0 || threadIdx.x == WX_GP_TBLOCK - 64) && wx_a.diag) {
    wx_u64 *d = wx_a.diag + (wx_u64)blockIdx.x * 16 + (threadIdx.x ? 8 : 0);
    for (int i = 0; i < 8; ++i) d[i] = wx_pt[i];
  }
#endif
#undef WX_GT_PT
  if (t_end > t_begin) WX_GS_WRITE_OUT(t_end - 1, tot_prev)
#undef WX_GS_LOAD_TILE
#undef WX_GS_WRITE_OUT
  for (int p = tid; p < P; p += WX_GP_TBLOCK) {
    const wx_u32 c = s_tot[p];
    wx_a.pcount[(wx_i64)p * wx_a.n_wg + blockIdx.x] = c;
    if (c) atomicAdd(&wx_a.ptotal[p], (wx_u64)c);
  }
  wx_gp_stats_out<WX_GP_TBLOCK>(wx_mn, wx_mx, wx_c, wx_o, wx_a.mm);
}

// One 1024-thread workgroup: the range summary (passing rows, rows outside
// the planned range, min key, max key -> summary[0..3]) and the aggregation
// work items.  Per partition (one wave each): its workgroups' rows
// pcount[p][g], their exclusive prefix e_g, and K = ceil(rows / chunk)
// items, item k taking the workgroups with e_g in [k chunk, (k + 1) chunk)
// -- [b_k, b_(k+1)) with b_k = #{g : e_g < k chunk} (possibly empty).  Item
// words are (p << 40 | g0 << 20 | g1, rows).  When some row fell outside the
// range there is nothing to aggregate (the host re-plans from the exact one).
#define WX_GP_MAX_GPL 16  // workgroups per lane in the plan's wave scans (G <= 1024)
#define WX_GP_MAX_ITEMS 4096  // work items (P + 4 x CUs + 2 <= 2048 + 1024 + 2)
#ifndef WX_GP_AGG_ORDER
#define WX_GP_AGG_ORDER 1  // 0: aggregation items in partition order (A/B)
#endif
#ifndef WX_GP_AGG_XCD
// 1: the dispatch order is dealt to the 8 XCDs in blocks (workgroups b and
// b + 8 share an XCD): XCD x runs the x-th eighth of the items sorted by
// first workgroup, so the neighbouring partitions' runs of the same tiles --
// which share their boundary lines -- are read through one L2.  Measured
// slower: 4.38 vs 4.24-4.29 ms per 1e9 rows x 10^6 keys
// (profiles/r04/abl_group_wide_agg_xcd.txt) -- the chip-wide sweep over one
// tile range at a time matters more than the shared boundary lines
#define WX_GP_AGG_XCD 0
#endif
extern "C" __global__ __launch_bounds__(1024) void wx_group_part_plan(WxGroupPartArgs a) {
  __shared__ wx_u32 s_w[16];
  __shared__ wx_i64 s_r[16][4];
  __shared__ wx_u32 s_k[WX_GP_STAGE_MAXP];
  __shared__ wx_u32 s_hist[1024];                 // items per first workgroup g0, then their offsets
  __shared__ unsigned short s_ig0[WX_GP_MAX_ITEMS];  // each item's first workgroup
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, G = a.n_wg, P = a.n_part;
  s_hist[tid] = 0u;
  {  // range summary over the tile workgroups (G <= 1024: one per thread)
    wx_i64 c = 0, o = 0, mn = 0x7fffffff, mx = -0x7fffffffll - 1;
    if (tid < G && a.mm[4 * tid + 2]) {
      mn = a.mm[4 * tid];
      mx = a.mm[4 * tid + 1];
      c = a.mm[4 * tid + 2];
      o = a.mm[4 * tid + 3];
    }
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) {
      const wx_i64 x = __shfl_xor(mn, k), y = __shfl_xor(mx, k);
      mn = x < mn ? x : mn;
      mx = y > mx ? y : mx;
      c += __shfl_xor(c, k);
      o += __shfl_xor(o, k);
    }
    if (lane == 0) { s_r[wave][0] = c; s_r[wave][1] = o; s_r[wave][2] = mn; s_r[wave][3] = mx; }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < 16; ++w) {
        c += s_r[w][0];
        o += s_r[w][1];
        mn = s_r[w][2] < mn ? s_r[w][2] : mn;
        mx = s_r[w][3] > mx ? s_r[w][3] : mx;
      }
      s_r[0][0] = c; s_r[0][1] = o;
      a.summary[0] = c; a.summary[1] = o; a.summary[2] = mn; a.summary[3] = mx;
    }
    __syncthreads();
  }
  const bool abort = s_r[0][1] != 0;
  wx_i64 chunk = (s_r[0][0] + a.target_items - 1) / a.target_items;
  chunk = chunk > a.chunk ? chunk : a.chunk;
  const int gpl = (G + 63) / 64;
  // pass 1: item count per partition from its rows (ptotal, summed by the
  // tile workgroups' atomics; cleared here for the next query, aborted or not)
  for (int p = tid; p < P; p += 1024) {
    const wx_i64 t = (wx_i64)a.ptotal[p];
    a.ptotal[p] = 0ull;
    s_k[p] = abort || !t ? 0u : (wx_u32)((t - 1) / chunk + 1);
  }
  __syncthreads();
  const int p0 = 2 * tid, p1 = 2 * tid + 1;
  const wx_u32 n0 = p0 < P ? s_k[p0] : 0u, n1 = p1 < P ? s_k[p1] : 0u;
  wx_u32 tot;
  const wx_u32 ex = wx_gp_block_excl(n0 + n1, s_w, &tot);
  __syncthreads();
  if (p0 < P) s_k[p0] = ex;  // s_k now holds the first item of each partition
  if (p1 < P) s_k[p1] = ex + n0;
  const wx_u32 cap = (wx_u32)a.work_cap;
  if (p0 < P) a.pitem[p0] = ex < cap ? ex : cap;
  if (p1 < P) a.pitem[p1] = ex + n0 < cap ? ex + n0 : cap;
  if (tid == 0) {
    a.pitem[P] = tot < cap ? tot : cap;
    *a.n_work = tot < cap ? tot : cap;
    if (tot > cap) atomicOr(reinterpret_cast<unsigned int *>(&a.ctrs[1]), WX_DEVERR_INTERNAL_KEY);
  }
  __syncthreads();
  if (abort) return;
  // pass 2: the items (b_k by a wave count of e_g < k chunk)
  for (int p = wave; p < P; p += 16) {
    wx_i64 e[WX_GP_MAX_GPL], loc = 0;
    for (int i = 0; i < WX_GP_MAX_GPL; ++i) {
      const int g = lane * gpl + i;
      const wx_i64 c = (i < gpl && g < G) ? (wx_i64)a.pcount[(wx_i64)p * G + g] : 0;
      e[i] = loc;
      loc += c;
    }
    wx_i64 incl = loc;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
      const wx_i64 x = __shfl_up(incl, k);
      if (lane >= k) incl += x;
    }
    const wx_i64 lb = incl - loc;  // rows of the lanes below
    wx_i64 total = __shfl(incl, 63);
    if (!total) continue;
    const wx_i64 K = (total - 1) / chunk + 1, first = s_k[p];
    wx_i64 bprev = 0;
    for (wx_i64 k = 1; k <= K; ++k) {
      wx_i64 b = G;
      if (k < K) {
        wx_i64 n = 0;
        for (int i = 0; i < gpl; ++i) {
          const int g = lane * gpl + i;
          n += (g < G && lb + e[i] < k * chunk) ? 1 : 0;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
        b = n;
      }
      const wx_i64 item = first + k - 1;
      if (lane == 0 && item < a.work_cap) {
        a.work[2 * item] = ((wx_i64)p << 40) | (bprev << 20) | b;
        a.work[2 * item + 1] = 0;
        s_ig0[item] = (unsigned short)bprev;
        atomicAdd(&s_hist[bprev < G ? bprev : G - 1], 1u);
      }
      bprev = b;
    }
  }
  __syncthreads();
  // pass 3: the dispatch order, by first workgroup: the items of every
  // partition that start in the same tile range run side by side, so the
  // aggregation reads each tile's runs (all partitions') at about the same
  // time -- DRAM pages and L2 lines shared instead of ~1 KB random reads
  {
    wx_u32 tt;
    const wx_u32 h = tid < G ? s_hist[tid] : 0u;
    const wx_u32 ex2 = wx_gp_block_excl(h, s_w, &tt);
    __syncthreads();
    if (tid < G) s_hist[tid] = ex2;
    __syncthreads();
    const wx_i64 ni = tot < cap ? tot : cap;
    const wx_i64 xchunk = (ni + 7) / 8;  // WX_GP_AGG_XCD: items per XCD
    if (WX_GP_AGG_XCD) {  // slots no item maps to (ni not a multiple of 8) stay empty
      for (wx_i64 b = tid; b < 8 * xchunk; b += 1024) a.order[b] = 0xffffffffu;
      __syncthreads();
    }
    for (wx_i64 i = tid; i < ni; i += 1024) {
      const wx_u32 g = s_ig0[i];
      const wx_u32 pos = atomicAdd(&s_hist[g < (wx_u32)G ? g : G - 1], 1u);
      const wx_u32 slot = WX_GP_AGG_XCD ? (wx_u32)((pos % xchunk) * 8 + pos / xchunk) : pos;
      a.order[WX_GP_AGG_ORDER ? slot : (wx_u32)i] = (wx_u32)i;
    }
  }
}

// Work item blockIdx.x: its partition's runs in the tiles of workgroups
// [g0, g1), aggregated in an LDS window of 1 << shift bins and written as
// the item's partial window.  The directory words of the item's tiles are
// staged in LDS, WX_GP_DIRCH at a time; each wave takes WX_GP_AGG_R
// consecutive tiles at a time and walks their runs as one sequence,
// 64 x WX_GP_AGG_K elements per step with every lane busy: a lane finds the
// run of its element by WX_GP_AGG_R - 1 compares against the wave-uniform run
// prefix and selects that run's 32-bit offset from the group's first tile.
// Measured alternatives (1e9 rows x 1e6 keys): one 64-bit select per compare
// 2.2 ms; wave-uniform 64-row chunks (lanes idle past a run's end) 4.3 ms;
// 16-lane groups on four runs per load instruction 14.5 ms; the dispatch
// order by first workgroup (the plan's pass 3) took the agg from 2.3 to 1.64.
#ifndef WX_GP_AGG_R
#define WX_GP_AGG_R 8
#endif
#ifndef WX_GP_AGG_K
// 64-element chunks per fetch (two fetches in flight): 6 -> 4.51 ms per
// 1e9 rows x 10^6 keys, 4 -> 4.58, 8 -> 4.65 (profiles/r04/abl_group_wide_agg.txt)
#define WX_GP_AGG_K 6
#endif
#ifndef WX_GP_AGG_DIAG_NOBIN
#define WX_GP_AGG_DIAG_NOBIN 0  // diagnostic: values only, bins made up (results invalid)
#endif
#ifndef WX_GP_AGG_DIAG_NOADD
#define WX_GP_AGG_DIAG_NOADD 0  // diagnostic: loads without the LDS adds (results invalid)
#endif
#define WX_GP_DIRCH 4096  // directory words staged per round
extern "C" __global__ __launch_bounds__(WX_GP_BLOCK) void wx_group_part_agg(WxGroupPartArgs a) {
  extern __shared__ wx_u32 wx_s_dyn[];
  const int B = 1 << a.shift;
  double *s_sum = reinterpret_cast<double *>(wx_s_dyn);  // [B]
  wx_u32 *s_cnt = reinterpret_cast<wx_u32 *>(s_sum + B);  // [B]
  wx_u32 *s_dir = s_cnt + B;                              // [WX_GP_DIRCH]
  const wx_i64 nw = *a.n_work;
  if ((wx_i64)blockIdx.x >= (WX_GP_AGG_XCD && WX_GP_AGG_ORDER ? 8 * ((nw + 7) / 8) : nw)) return;
  const wx_u32 wo = a.order[blockIdx.x];  // items in first-workgroup order (the plan's pass 3)
  if (wo == 0xffffffffu) return;          // an empty XCD slot (WX_GP_AGG_XCD)
  const wx_i64 w = wo;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const wx_i64 w0 = a.work[2 * w];
  const int p = (int)(w0 >> 40);
  const wx_i64 g0 = (w0 >> 20) & 0xfffff, g1 = w0 & 0xfffff;
  const wx_i64 ta = g0 * a.tiles_per_wg;
  wx_i64 tb = g1 * a.tiles_per_wg;
  tb = tb < a.n_tiles ? tb : a.n_tiles;
  for (int b = tid; b < B; b += WX_GP_BLOCK) { s_sum[b] = 0.0; s_cnt[b] = 0u; }
#if WX_GP_AGG_DIAG_NOADD
  float wx_diag = 0.0f;
#endif
  const wx_u32 *dir = a.dir + (wx_i64)p * a.n_tiles;
  for (wx_i64 c0 = ta; c0 < tb; c0 += WX_GP_DIRCH) {
    const int nt = (int)(tb - c0 < WX_GP_DIRCH ? tb - c0 : WX_GP_DIRCH);
    for (int i = tid; i < nt; i += WX_GP_BLOCK) s_dir[i] = dir[c0 + i];
    __syncthreads();
    // Wave-uniform walk over this wave's groups of WX_GP_AGG_R tiles (r0 =
    // wave * R, + 16 R, ...): the runs' prefix pre[] and each run's start
    // relative to the group's first tile minus its prefix (element j of the
    // group's sequence in run r sits at gv + rel[r] + j).  Software-pipelined
    // by two register sets: a step's loads are issued before the previous
    // step's LDS adds, so 2 x 64 x WX_GP_AGG_K elements per wave are in
    // flight; every fetch issues its loads unconditionally (junk from the
    // array start where the walk has ended, masked out by the sentinel bin)
    // so the adds wait only for their own set.
    int r0 = wave * WX_GP_AGG_R - (WX_GP_BLOCK / 64) * WX_GP_AGG_R;
    wx_u32 pre[WX_GP_AGG_R + 1];
    int rel[WX_GP_AGG_R];
    wx_u32 total = 0u, sj = 0u;
    const float *gv = a.vals;
    const unsigned short *gb = a.bins;
#define WX_GA_NEXT_GROUP()                                                                     \
  do {                                                                                          \
    r0 += (WX_GP_BLOCK / 64) * WX_GP_AGG_R;                                                     \
    total = 0u;                                                                                 \
    sj = 0u;                                                                                    \
    if (r0 < nt) {                                                                              \
      pre[0] = 0u;                                                                              \
      _Pragma("unroll") for (int r = 0; r < WX_GP_AGG_R; ++r) {                                \
        const wx_u32 e = __builtin_amdgcn_readfirstlane(r0 + r < nt ? s_dir[r0 + r] : 0u);     \
        rel[r] = r * WX_GP_TILE + (int)(e & 0xffffu) - (int)pre[r];                             \
        pre[r + 1] = pre[r] + (e >> 16);                                                        \
      }                                                                                         \
      total = pre[WX_GP_AGG_R];                                                                 \
      gv = a.vals + (c0 + r0) * WX_GP_TILE;                                                     \
      gb = a.bins + (c0 + r0) * WX_GP_TILE;                                                     \
    }                                                                                           \
  } while (r0 < nt && total == 0u)
    // one step's loads into (V, BN), the valid lanes' bits in OK; HAS: whether
    // the walk had a step left
#define WX_GA_FETCH(V, BN, OK, HAS)                                                            \
  {                                                                                             \
    HAS = r0 < nt;                                                                              \
    const float *fv = HAS ? gv : a.vals;                                                        \
    const unsigned short *fb = HAS ? gb : a.bins;                                               \
    OK = 0u;                                                                                    \
    _Pragma("unroll") for (int k = 0; k < WX_GP_AGG_K; ++k) {                                  \
      const wx_u32 j = sj + 64 * k + lane;                                                      \
      const bool ok = HAS && j < total;                                                         \
      int o = rel[0];                                                                           \
      _Pragma("unroll") for (int r = 1; r < WX_GP_AGG_R; ++r) o = j >= pre[r] ? rel[r] : o;    \
      o = ok ? o + (int)j : 0;                                                                  \
      OK |= (ok ? 1u : 0u) << k;                                                                \
      V[k] = __builtin_nontemporal_load(fv + o);                                                \
      BN[k] = WX_GP_AGG_DIAG_NOBIN ? (unsigned short)(o & 4095) : __builtin_nontemporal_load(fb + o); \
    }                                                                                           \
    if (HAS) {                                                                                  \
      sj += 64 * WX_GP_AGG_K;                                                                   \
      if (sj >= total) WX_GA_NEXT_GROUP();                                                      \
    }                                                                                           \
  }
#if WX_GP_AGG_DIAG_NOADD
#define WX_GA_ADD(V, BN, OK)                                                                   \
  _Pragma("unroll") for (int k = 0; k < WX_GP_AGG_K; ++k) if ((OK >> k) & 1u) wx_diag += V[k] + (float)BN[k];
#else
#define WX_GA_ADD(V, BN, OK)                                                                   \
  _Pragma("unroll") for (int k = 0; k < WX_GP_AGG_K; ++k) {                                    \
    if (!((OK >> k) & 1u)) continue;                                                            \
    atomicAdd(&s_sum[BN[k]], (double)V[k]);                                                     \
    atomicAdd(&s_cnt[BN[k]], 1u);                                                               \
  }
#endif
    WX_GA_NEXT_GROUP();
    float va[WX_GP_AGG_K], vb[WX_GP_AGG_K];
    unsigned short ba[WX_GP_AGG_K], bb[WX_GP_AGG_K];
    wx_u32 oka, okb;
    bool ha, hb;
    WX_GA_FETCH(va, ba, oka, ha)
    while (ha) {
      WX_GA_FETCH(vb, bb, okb, hb)
      WX_GA_ADD(va, ba, oka)
      if (!hb) break;
      WX_GA_FETCH(va, ba, oka, ha)
      WX_GA_ADD(vb, bb, okb)
    }
#undef WX_GA_NEXT_GROUP
#undef WX_GA_FETCH
#undef WX_GA_ADD
    __syncthreads();
  }
#if WX_GP_AGG_DIAG_NOADD
  if (wx_diag == 1.2345f) s_cnt[0] = 1u;  // keeps the loads live
  __syncthreads();
#endif
  double *ps = a.psum + w * B;
  wx_u32 *pc = a.pcnt + w * B;
  for (int b = tid; b < B; b += WX_GP_BLOCK) {
    ps[b] = s_sum[b];
    pc[b] = s_cnt[b];
  }
}

// non-empty keys of partition blockIdx.x (over its items' partial windows)
extern "C" __global__ __launch_bounds__(WX_GP_BLOCK) void wx_group_part_count(WxGroupPartArgs a) {
  __shared__ wx_u32 s_n;
  if (threadIdx.x == 0) s_n = 0u;
  __syncthreads();
  const int B = 1 << a.shift;
  const wx_i64 i0 = a.pitem[blockIdx.x], i1 = a.pitem[blockIdx.x + 1];
  wx_u32 n = 0;
  for (int b = threadIdx.x; b < B; b += WX_GP_BLOCK) {
    wx_u32 nz = 0;
    for (wx_i64 i = i0; i < i1 && !nz; ++i) nz = a.pcnt[i * B + b];
    n += nz ? 1u : 0u;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(&s_n, n);
  __syncthreads();
  if (threadIdx.x == 0) a.pnz[blockIdx.x] = s_n;
}

// exclusive prefix of the partitions' key counts in place; the total is the group count
extern "C" __global__ __launch_bounds__(1024) void wx_group_part_scan2(WxGroupPartArgs a) {
  __shared__ wx_i64 s_w[16];
  const wx_i64 total = wx_block_scan_excl(a.pnz, a.pnz, (wx_i64)a.n_part, s_w);
  if (threadIdx.x == 0) {
    *a.n_groups_out = total;
    if (total > a.capacity) atomicOr(reinterpret_cast<unsigned int *>(&a.ctrs[1]), WX_DEVERR_CAPACITY);
  }
}

// partition blockIdx.x's groups at their ascending-key positions, its items'
// partial windows summed
extern "C" __global__ __launch_bounds__(WX_GP_BLOCK) void wx_group_part_emit(WxGroupPartArgs a) {
  __shared__ wx_u32 s_w[WX_GP_BLOCK / 64];
  const int B = 1 << a.shift;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const wx_i64 g0 = (wx_i64)blockIdx.x << a.shift;
  const wx_i64 i0 = a.pitem[blockIdx.x], i1 = a.pitem[blockIdx.x + 1];
  if (i0 == i1) return;  // no rows in this partition (uniform)
  wx_i64 pos = a.pnz[blockIdx.x];
  for (int b0 = 0; b0 < B; b0 += WX_GP_BLOCK) {
    const int b = b0 + tid;
    wx_u64 c = 0;
    double s = 0.0;
    if (b < B)
      for (wx_i64 i = i0; i < i1; ++i) {
        c += a.pcnt[i * B + b];
        s += a.psum[i * B + b];
      }
    const wx_u64 m = __builtin_amdgcn_ballot_w64(c != 0ull);
    if (lane == 0) s_w[wave] = (wx_u32)__builtin_popcountll(m);
    __syncthreads();
    wx_u32 wb = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < WX_GP_BLOCK / 64; ++w) {
      const wx_u32 x = s_w[w];
      wb += w < wave ? x : 0u;
      tot += x;
    }
    if (c) {
      const wx_i64 o = pos + wb + ::wx::lanes_below(m);
      if (o < a.capacity) {
        a.out_keys[o] = (int)((wx_u32)a.key_lo + (wx_u32)(g0 + b));
        a.out_sums[o] = s;
        a.out_counts[o] = (wx_i64)c;
      }
    }
    pos += tot;
    __syncthreads();
  }
}

#endif  // WX_OP == WX_OP_GROUP
