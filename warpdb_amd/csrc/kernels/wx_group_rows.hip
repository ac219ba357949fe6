// wx_group_rows.hip -- GROUP BY with every group's sum folded in ascending
// row order (WX_F_ROW_ORDER): the reference's std::map fold
// (src/warpdb.cpp:373-385, `g.sum += val` over the rows in order) to the bit.
// Part of the GROUP and util modules' sources (after wx_common.hip and their own).
//
// When the groups' keys span at most 2048 values (C3's 1K keys), the
// passing rows' values are put into key-major, row-ordered segments by one
// stable counting sort straight from the table -- no compaction, no key bits
// written, no radix passes:
//   wx_ro_count   (GROUP module)  per static range of whole tiles (two
//                                 ranges per CU), the passing rows of each
//                                 key (bin = key - key_lo), one 2048-bin LDS
//                                 histogram per range;
//   wx_ro_scan / wx_ro_base (util) per-bin totals over the ranges, the bins'
//                                 exclusive prefix (checked against the
//                                 ordinary call's group counts), and each
//                                 range's first output slot of every bin;
//   wx_ro_scatter (GROUP module)  the range's 8 192-row tiles in order (512
//                                 threads, two workgroups per CU): cond / key /
//                                 value per row, stable in-wave ranks by one
//                                 returning LDS add per row, the tile's bin
//                                 prefix, the values permuted into bin order
//                                 in LDS and written at their segment slots;
//   wx_ro_fold    (util)          one wave per group: the segment's values
//                                 widened into LDS in 64-value chunks (a ring
//                                 of loads ahead) and broadcast back, one
//                                 dependent double add per row in row order.
// Nothing waits on another workgroup.  Wider key spans keep the general path
// (two ordered compactions + the stable radix pair sort + wx_group_fold).

#define WX_RO_BLOCK 512
#define WX_RO_WAVES (WX_RO_BLOCK / 64)
#define WX_RO_ITEMS 16
#define WX_RO_TILE (WX_RO_BLOCK * WX_RO_ITEMS)  // 8 192 rows (wx_args.h WX_RO_TILE_ROWS)
#define WX_RO_BINS 2048
#define WX_RO_BPT (WX_RO_BINS / WX_RO_BLOCK)  // bins per thread in the tile scan: 4
#ifndef WX_RO_HC
#define WX_RO_HC 4  // count kernel: LDS copies of the 2048 counters (32 KB), lane % 4
#endif

// Range r of R: tiles [r * T / R, (r + 1) * T / R) of the table's rows.
__device__ __forceinline__ void wx_ro_range(wx_i64 n, int ranges, int r, wx_i64 &t0, wx_i64 &t1) {
  const wx_i64 T = (n + WX_RO_TILE - 1) / WX_RO_TILE;
  t0 = (wx_i64)r * T / ranges;
  t1 = (wx_i64)(r + 1) * T / ranges;
}

// Inclusive prefix sum over the 64 lanes of a wave by DPP row shifts and row
// broadcasts (no LDS, no address registers).
__device__ __forceinline__ wx_u32 wx_ro_wave_incl(wx_u32 v) {
  v += (wx_u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (wx_u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (wx_u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (wx_u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (wx_u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += (wx_u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

#if WX_OP == WX_OP_GROUP
// ---------------------------------------------------------------- counts
// rows [b, b + 8 * 512) of a range: whole spans load unconditionally (the
// eight rows' loads in flight together), the range's tail guarded
template <bool WHOLE>
__device__ __forceinline__ void wx_ro_count_span(const WxRoArgs &wx_a, wx_u32 *h, wx_i64 b, wx_i64 e1, int copy,
                                                 bool &bad) {
  wx_u32 bins[8];  // all eight rows evaluated first: their loads issue together (an LDS
                   // atomic between two loads would make each load wait for the one before)
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const wx_i64 idx = b + (wx_i64)u * WX_RO_BLOCK + threadIdx.x;
    bins[u] = 0xffffffffu;
    if (WHOLE || idx < e1) {
      WX_COLS(WX_BIND_ROW)
      if (WX_EVAL_COND()) {
        const wx_u32 bin = (wx_u32)(static_cast<int>(WX_KEY) - wx_a.key_lo);
        if (bin < (wx_u32)wx_a.span) bins[u] = bin;
        else bad = true;
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (bins[u] != 0xffffffffu) atomicAdd(&h[bins[u] * WX_RO_HC + copy], 1u);
}

extern "C" __global__ __launch_bounds__(WX_RO_BLOCK) void wx_ro_count(WxRoArgs wx_a) {
  __shared__ wx_u32 h[WX_RO_BINS * WX_RO_HC];
  for (int i = threadIdx.x; i < WX_RO_BINS * WX_RO_HC; i += WX_RO_BLOCK) h[i] = 0u;
  __syncthreads();
  const int r = blockIdx.x, copy = threadIdx.x % WX_RO_HC;
  wx_i64 t0, t1;
  wx_ro_range(wx_a.n_rows, wx_a.ranges, r, t0, t1);
  const wx_i64 e0 = t0 * WX_RO_TILE, e1 = t1 * WX_RO_TILE < wx_a.n_rows ? t1 * WX_RO_TILE : wx_a.n_rows;
  bool bad = false;
  constexpr wx_i64 SPAN = (wx_i64)WX_RO_BLOCK * 8;
  wx_i64 b = e0;
  for (; b + SPAN <= e1; b += SPAN) wx_ro_count_span<true>(wx_a, h, b, e1, copy, bad);
  if (b < e1) wx_ro_count_span<false>(wx_a, h, b, e1, copy, bad);
  if (bad) {
    if (wx_a.info)  // the direct path's guessed span missed a key: the host falls back
      atomicOr(reinterpret_cast<unsigned int *>(&wx_a.info[2]), 1u);
    else
      atomicOr(reinterpret_cast<unsigned int *>(&wx_a.ctrs[1]), WX_DEVERR_INTERNAL_KEY);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < WX_RO_BINS; i += WX_RO_BLOCK) {
    wx_u32 c = 0u;
#pragma unroll
    for (int j = 0; j < WX_RO_HC; ++j) c += h[i * WX_RO_HC + ((j + i) & (WX_RO_HC - 1))];  // rotated: distinct banks
    wx_a.cnt[(wx_u64)r * WX_RO_BINS + i] = c;
  }
}

// ---------------------------------------------------------------- scatter
struct WxRoShared {
  // per-wave bin counts of the tile, waves 2k / 2k + 1 in the low / high half
  // of word [k][d]; then each wave's first tile-local slot of bin d; then,
  // per slot, the output position of the value staged there
  wx_u32 wc[WX_RO_WAVES / 2][WX_RO_BINS];
  static_assert(WX_RO_WAVES / 2 * WX_RO_BINS >= WX_RO_TILE, "the counters' place holds a position per slot");
  wx_u32 gb[WX_RO_BINS];  // output slot of the tile's first row of bin d, minus its tile-local slot
  wx_u32 ws[WX_RO_WAVES];  // block scan: per-wave sums
};

// the tile's column values, wave-striped, loaded all at once (whole tiles
// unconditionally), then bound like the streamed registers
#define WX_RO_DECL(name, T, slot) T wx_n##slot[WX_RO_ITEMS];
#define WX_RO_LOAD(name, T, slot) \
  wx_n##slot[i] = (WHOLE || e < wx_a.n_rows) ? static_cast<const T *>(wx_a.col[slot])[e] : static_cast<T>(0);
#define WX_RO_BIND(name, T, slot) const ::wx::reg<T> name{wx_n##slot[i]};
#define WX_RO_PARAM(name, T, slot) , const T (&wx_n##slot)[WX_RO_ITEMS]
#define WX_RO_ARG(name, T, slot) , wx_n##slot

// Tile t of range r (run[]: the range's next output slot of this thread's
// bins BPT * tid + j).  Row i * 64 + lane of wave w's 1024 rows is row
// t * TILE + w * 1024 + i * 64 + lane, so (wave, item, lane) is row order.
// Two 512-thread workgroups per CU hide each other's loads.
// (0) tile t's rows: bin (0xffffffff = not passing) and value, from the
// column registers wx_n* (loaded by WX_RO_LOAD_TILE)
#define WX_RO_LOAD_TILE(t_, LOADX)                                                                \
  {                                                                                               \
    const wx_i64 wb_ = (t_) * WX_RO_TILE + (threadIdx.x >> 6) * 64 * WX_RO_ITEMS + (threadIdx.x & 63); \
    _Pragma("unroll") for (int i = 0; i < WX_RO_ITEMS; ++i) {                                    \
      const wx_i64 e = wb_ + (wx_i64)i * 64;                                                      \
      WX_COLS(LOADX)                                                                               \
    }                                                                                             \
  }
template <bool WHOLE>
__device__ __forceinline__ void wx_ro_eval(const WxRoArgs &wx_a, wx_i64 wb, wx_u32 (&bin)[WX_RO_ITEMS],
                                           float (&val)[WX_RO_ITEMS], bool &bad WX_COLS(WX_RO_PARAM)) {
#pragma unroll
  for (int i = 0; i < WX_RO_ITEMS; ++i) {
    const wx_i64 idx = wb + (wx_i64)i * 64;
    bin[i] = 0xffffffffu;
    val[i] = 0.0f;
    if (WHOLE || idx < wx_a.n_rows) {
      WX_COLS(WX_RO_BIND)
      if (WX_EVAL_COND()) {
        const wx_u32 b = (wx_u32)(static_cast<int>(WX_KEY) - wx_a.key_lo);
        val[i] = static_cast<float>(WX_EXPR);
        if (b < (wx_u32)wx_a.span) bin[i] = b;
        else bad = true;
      }
    }
  }
}

// Steps (1)-(4) of tile t from its rows' bins and values.
__device__ __forceinline__ void wx_ro_place(const WxRoArgs &wx_a, WxRoShared &S, float *s_v,
                                            wx_u32 (&run)[WX_RO_BPT], wx_u32 (&bin)[WX_RO_ITEMS],
                                            const float (&val)[WX_RO_ITEMS], wx_i64 t);

template <bool WHOLE>
__device__ __forceinline__ void wx_ro_tile(const WxRoArgs &wx_a, WxRoShared &S, float *s_v, wx_i64 t,
                                           wx_u32 (&run)[WX_RO_BPT], bool &bad) {
  const wx_i64 wb = t * WX_RO_TILE + (threadIdx.x >> 6) * 64 * WX_RO_ITEMS + (threadIdx.x & 63);
  // whole tiles load every row unconditionally (all loads in flight together)
  wx_u32 bin[WX_RO_ITEMS];
  float val[WX_RO_ITEMS];
  WX_COLS(WX_RO_DECL)
  WX_RO_LOAD_TILE(t, WX_RO_LOAD)
  // every load issued before any row is evaluated (the scheduler would
  // otherwise wait for each row's loads in turn to save registers)
  __builtin_amdgcn_sched_barrier(0);
  wx_ro_eval<WHOLE>(wx_a, wb, bin, val, bad WX_COLS(WX_RO_ARG));
  wx_ro_place(wx_a, S, s_v, run, bin, val, t);
}

__device__ __forceinline__ void wx_ro_place(const WxRoArgs &wx_a, WxRoShared &S, float *s_v,
                                            wx_u32 (&run)[WX_RO_BPT], wx_u32 (&bin)[WX_RO_ITEMS],
                                            const float (&val)[WX_RO_ITEMS], wx_i64 t) {
  typedef wx_u32 u4 __attribute__((ext_vector_type(4)));
  // an opaque copy of the thread index: the slot and address arithmetic is
  // formed here, not hoisted out of the tile loop into spilled registers
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wp = wave >> 1, sh = (wave & 1) * 16;
  const wx_u64 below = (1ull << lane) - 1ull;
  wx_u32 *wcf = &S.wc[0][0];
  // (1) stable in-wave ranks: one returning LDS add per passing row on the
  // wave's counter (the LDS returns same-address lanes' results in ascending
  // lane order, gfx950); lane 0's bin group adds its size once from lane 0
  // and ranks by its ballot (few keys would serialize on one counter)
  // (the adds' raw results are unpacked only after all sixteen are issued:
  // unpacked inside the branch, each add waited for its result before the
  // next was issued)
  wx_u32 rk[WX_RO_ITEMS];
  wx_u32 lead_bits = 0u, atom_bits = 0u;
#pragma unroll
  for (int i = 0; i < WX_RO_ITEMS; ++i) {
    const bool valid = bin[i] != 0xffffffffu;
    const wx_u32 d0 = __builtin_amdgcn_readfirstlane(bin[i]);  // lane 0's (0xffffffff: not passing)
    const bool lead = valid && bin[i] == d0;
    const wx_u64 lm = __builtin_amdgcn_ballot_w64(lead);
    rk[i] = (wx_u32)__builtin_popcountll(lm & below);
    const bool atom = valid && (!lead || lane == 0);
    if (atom) {
      const wx_u32 inc = (lead ? (wx_u32)__builtin_popcountll(lm) : 1u) << sh;
      rk[i] = atomicAdd(&S.wc[wp][bin[i]], inc);  // raw: this wave's half unpacked below
    }
    lead_bits |= (lead && lane != 0 ? 1u : 0u) << i;
    atom_bits |= (atom ? 1u : 0u) << i;
  }
#pragma unroll
  for (int i = 0; i < WX_RO_ITEMS; ++i)
    if ((atom_bits >> i) & 1u) rk[i] = (rk[i] >> sh) & 0xffffu;
#pragma unroll
  for (int i = 0; i < WX_RO_ITEMS; ++i) {
    const wx_u32 base0 = __builtin_amdgcn_readlane(rk[i], 0);
    if ((lead_bits >> i) & 1u) rk[i] += base0;
    asm volatile("" : "+v"(rk[i]));  // settled here, not carried as SGPR copies into the scan
  }
  __syncthreads();
  // (2) thread tid owns bins 4 tid .. 4 tid + 3: the tile's counts, their
  // tile-local base by a block scan, each wave's first slot written back in
  // place, the output base, the range's runs advanced
  wx_u32 n_pass;  // the tile's passing rows: slots [0, n_pass)
  {
    wx_u32 c[WX_RO_BPT] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < WX_RO_WAVES / 2; ++k) {
      const u4 w4 = *reinterpret_cast<const u4 *>(&S.wc[k][WX_RO_BPT * tid]);
      c[0] += (w4.x & 0xffffu) + (w4.x >> 16);
      c[1] += (w4.y & 0xffffu) + (w4.y >> 16);
      c[2] += (w4.z & 0xffffu) + (w4.z >> 16);
      c[3] += (w4.w & 0xffffu) + (w4.w >> 16);
    }
    const wx_u32 s = c[0] + c[1] + c[2] + c[3];
    const wx_u32 inc = wx_ro_wave_incl(s);
    if (lane == 63) S.ws[wave] = inc;
    __syncthreads();
    wx_u32 lb = inc - s;
    n_pass = 0u;
#pragma unroll
    for (int w = 0; w < WX_RO_WAVES; ++w) {
      const wx_u32 ww = S.ws[w];
      lb += w < wave ? ww : 0u;
      n_pass += ww;
    }
    wx_u32 l[WX_RO_BPT];  // the tile-local first slot of each bin
    l[0] = lb;
    l[1] = l[0] + c[0];
    l[2] = l[1] + c[1];
    l[3] = l[2] + c[2];
    wx_u32 q[WX_RO_BPT] = {l[0], l[1], l[2], l[3]};
#pragma unroll
    for (int k = 0; k < WX_RO_WAVES / 2; ++k) {
      u4 w4 = *reinterpret_cast<const u4 *>(&S.wc[k][WX_RO_BPT * tid]);
      u4 o;
#define WX_RO_SLOTS(f, j)                                           \
  {                                                                 \
    const wx_u32 a0 = w4.f & 0xffffu, a1 = w4.f >> 16;               \
    o.f = q[j] | ((q[j] + a0) << 16);                                \
    q[j] += a0 + a1;                                                 \
  }
      WX_RO_SLOTS(x, 0)
      WX_RO_SLOTS(y, 1)
      WX_RO_SLOTS(z, 2)
      WX_RO_SLOTS(w, 3)
#undef WX_RO_SLOTS
      *reinterpret_cast<u4 *>(&S.wc[k][WX_RO_BPT * tid]) = o;
    }
    u4 g;
    g.x = run[0] - l[0];
    g.y = run[1] - l[1];
    g.z = run[2] - l[2];
    g.w = run[3] - l[3];
    *reinterpret_cast<u4 *>(&S.gb[WX_RO_BPT * tid]) = g;
#pragma unroll
    for (int j = 0; j < WX_RO_BPT; ++j) run[j] += c[j];
  }
  __syncthreads();
  // (3) slots; then the values into bin order in LDS and, in the counters'
  // place, each slot's output position
  // (reads unconditional -- a row that does not pass reads bin 0 -- so they
  // are all issued before the first result is waited for)
  wx_u32 gbv[WX_RO_ITEMS];
#pragma unroll
  for (int i = 0; i < WX_RO_ITEMS; ++i) {
    const wx_u32 bb = bin[i] != 0xffffffffu ? bin[i] : 0u;
    rk[i] += (S.wc[wp][bb] >> sh) & 0xffffu;
    gbv[i] = S.gb[bb];
  }
  __syncthreads();  // every slot base read: the positions take the counters' place
#pragma unroll
  for (int i = 0; i < WX_RO_ITEMS; ++i) {
    if (bin[i] != 0xffffffffu) {
      s_v[rk[i]] = val[i];
      wcf[rk[i]] = gbv[i] + rk[i];
    }
  }
  __syncthreads();
  // (4) LDS -> output: consecutive threads write consecutive slots of a key's run
  // each thread clears the counter words it read (slot p's position sits in
  // counter word p), so one barrier ends the tile
  static_assert(WX_RO_WAVES / 2 * WX_RO_BINS == WX_RO_ITEMS * WX_RO_BLOCK, "slot p's word is the counter word p");
  // (every slot's position and value read first -- unconditionally, so the
  // reads are all in flight together -- then the passing slots stored)
  wx_u32 pos[WX_RO_ITEMS];
  float sv[WX_RO_ITEMS];
#pragma unroll
  for (int j = 0; j < WX_RO_ITEMS; ++j) {
    pos[j] = wcf[j * WX_RO_BLOCK + tid];
    sv[j] = s_v[j * WX_RO_BLOCK + tid];
  }
#if !defined(WX_RO_DIAG_STORE) || !WX_DIAG
// diagnostic (a WX_DIAG build only): 1 = each tile's values stored to its
// own rows' places (coalesced, wrong order), 2 = no stores
#undef WX_RO_DIAG_STORE
#define WX_RO_DIAG_STORE 0
#endif
#pragma unroll
  for (int j = 0; j < WX_RO_ITEMS; ++j)
    if ((wx_u32)(j * WX_RO_BLOCK + tid) < n_pass) {
#if WX_RO_DIAG_STORE == 1
      wx_a.out[(wx_u64)t * WX_RO_TILE + j * WX_RO_BLOCK + tid] = sv[j];
#elif WX_RO_DIAG_STORE == 2
      if (sv[j] == -1.2345f) wx_a.out[(wx_u64)pos[j]] = sv[j];
#else
      wx_a.out[(wx_u64)pos[j]] = sv[j];
#endif
    }
#pragma unroll
  for (int j = 0; j < WX_RO_ITEMS; ++j) wcf[j * WX_RO_BLOCK + tid] = 0u;
  __syncthreads();  // every position and value read, the counters zeroed
}

// (Measured and dropped, round 6, profiles/r06/group_row_order_ab.txt: tile
// t + 1's column loads in flight while tile t is ranked and stored -- 52 B of
// scratch at two workgroups per CU (18.2 ms per query), 158 VGPRs at one
// (7.61 vs 7.38 ms).)
extern "C" __global__ __launch_bounds__(WX_RO_BLOCK, 2 * WX_RO_BLOCK / 256) void wx_ro_scatter(WxRoArgs wx_a) {
  typedef wx_u32 u4 __attribute__((ext_vector_type(4)));
  __shared__ WxRoShared S;
  __shared__ float s_v[WX_RO_TILE];
  const int r = blockIdx.x;
  wx_i64 t0, t1;
  wx_ro_range(wx_a.n_rows, wx_a.ranges, r, t0, t1);
  wx_u32 *wcf = &S.wc[0][0];
#pragma unroll
  for (int i = 0; i < WX_RO_WAVES / 2 * WX_RO_BINS / WX_RO_BLOCK; ++i) wcf[i * WX_RO_BLOCK + threadIdx.x] = 0u;
  if (t0 >= t1) return;  // workgroup-uniform: an empty range
  const u4 o4 = *reinterpret_cast<const u4 *>(wx_a.off + (wx_u64)r * WX_RO_BINS + WX_RO_BPT * threadIdx.x);
  wx_u32 run[WX_RO_BPT] = {o4.x, o4.y, o4.z, o4.w};  // the range's next output slot of this thread's bins
  __syncthreads();  // counters zeroed
  bool bad = false;
  const wx_i64 n_whole = wx_a.n_rows / WX_RO_TILE;  // tiles [0, n_whole) are whole
  for (wx_i64 t = t0; t < t1; ++t) {
    if (t < n_whole)
      wx_ro_tile<true>(wx_a, S, s_v, t, run, bad);
    else
      wx_ro_tile<false>(wx_a, S, s_v, t, run, bad);
  }
  if (bad) atomicOr(reinterpret_cast<unsigned int *>(&wx_a.ctrs[1]), WX_DEVERR_INTERNAL_KEY);
}
#undef WX_RO_DECL
#undef WX_RO_LOAD
#undef WX_RO_BIND
#undef WX_RO_PARAM
#undef WX_RO_ARG
#undef WX_RO_LOAD_TILE
#endif  // WX_OP == WX_OP_GROUP

#if WX_OP == WX_OP_UTIL
// ---------------------------------------------------------------- scans
// Totals and offsets over the ranges (one 2048-bin block of counts per range).  Workgroup b: bins (b % 32) * 64 +
// lane; wave w sums the ranges [w R / 4, (w + 1) R / 4).
//   totals[d] = sum over r of cnt[r][d]                     (if totals)
//   off[r][d] = base[d] + sum over r' < r of cnt[r'][d]     (if off)
extern "C" __global__ __launch_bounds__(256) void wx_ro_scan(WxRoScanArgs a) {
  __shared__ wx_u32 part[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int bin = (blockIdx.x % 32) * 64 + lane;
  const wx_u32 *c = a.cnt + bin;
  const int r0 = w * a.ranges / 4, r1 = (w + 1) * a.ranges / 4;
  wx_u32 s = 0u;
#pragma unroll 8
  for (int r = r0; r < r1; ++r) s += c[(wx_u64)r * WX_RO_BINS];
  part[w][lane] = s;
  __syncthreads();
  wx_u32 pre = 0u, tot = 0u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const wx_u32 v = part[k][lane];
    if (k < w) pre += v;
    tot += v;
  }
  if (a.totals && w == 0) a.totals[bin] = tot;
  if (a.off) {
    wx_u32 run = a.base[bin] + pre;
    wx_u32 *o = a.off + bin;
#pragma unroll 8
    for (int r = r0; r < r1; ++r) {
      const wx_u32 v = c[(wx_u64)r * WX_RO_BINS];
      o[(wx_u64)r * WX_RO_BINS] = run;
      run += v;
    }
  }
}

// One workgroup: base[d] = the exclusive prefix of totals[d] over the bins
// (the first slot of key key_lo + d in the key-major array), and the check
// that every group of the ordinary call has exactly its count of rows here
// (a table rewritten between the two reads would not).
extern "C" __global__ __launch_bounds__(1024) void wx_ro_base(WxRoBaseArgs a) {
  __shared__ wx_u32 ws[16];
  typedef wx_u32 u2 __attribute__((ext_vector_type(2)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const u2 t2 = *reinterpret_cast<const u2 *>(a.totals + 2 * tid);
  const wx_u32 s = t2.x + t2.y;
  const wx_u32 inc = wx_ro_wave_incl(s);
  if (lane == 63) ws[wave] = inc;
  __syncthreads();
  wx_u32 lb = inc - s, all = 0u;
  for (int w = 0; w < 16; ++w) {
    lb += w < wave ? ws[w] : 0u;
    all += ws[w];
  }
  u2 b;
  b.x = lb;
  b.y = lb + t2.x;
  *reinterpret_cast<u2 *>(a.base + 2 * tid) = b;
  if (a.out_counts) {
    // the direct path: groups = the non-empty bins, in key order
    const wx_u32 nz = (t2.x ? 1u : 0u) + (t2.y ? 1u : 0u);
    const wx_u32 ginc = wx_ro_wave_incl(nz);
    __shared__ wx_u32 gs[16];
    __shared__ int s_kmin, s_kmax;
    if (lane == 63) gs[wave] = ginc;
    if (tid == 0) {
      s_kmin = 0x7fffffff;
      s_kmax = (int)0x80000000;
    }
    __syncthreads();
    wx_u32 gi = ginc - nz, ng = 0u;
    for (int w = 0; w < 16; ++w) {
      gi += w < wave ? gs[w] : 0u;
      ng += gs[w];
    }
    if (t2.x) {
      if (gi < a.capacity) {
        a.out_keys[gi] = a.key_lo + 2 * tid;
        a.out_counts[gi] = t2.x;
      }
      atomicMin(&s_kmin, a.key_lo + 2 * tid);
      atomicMax(&s_kmax, a.key_lo + 2 * tid);
      ++gi;
    }
    if (t2.y) {
      if (gi < a.capacity) {
        a.out_keys[gi] = a.key_lo + 2 * tid + 1;
        a.out_counts[gi] = t2.y;
      }
      atomicMin(&s_kmin, a.key_lo + 2 * tid + 1);
      atomicMax(&s_kmax, a.key_lo + 2 * tid + 1);
    }
    __syncthreads();
    if (tid == 0) {
      if (a.n_groups_out) *a.n_groups_out = ng;
      a.info[0] = ng;
      a.info[1] = all;
      a.info[3] = s_kmin;
      a.info[4] = s_kmax;
      if ((wx_i64)ng > a.capacity) atomicOr(reinterpret_cast<unsigned int *>(&a.ctrs[1]), WX_DEVERR_CAPACITY);
    }
    return;
  }
  bool bad = false;
  wx_i64 sum = 0;
  for (wx_i64 g = tid; g < a.n_groups; g += 1024) {
    const wx_u32 d = (wx_u32)(a.gkeys[g] - a.key_lo);
    sum += a.gcounts[g];
    if (d >= WX_RO_BINS || (wx_i64)a.totals[d] != a.gcounts[g]) bad = true;
  }
  // every passing row belongs to a group: the totals add up to the groups' rows
  __shared__ unsigned long long s_sum;
  if (tid == 0) s_sum = 0ull;
  __syncthreads();
  atomicAdd(&s_sum, (unsigned long long)sum);
  __syncthreads();
  if (tid == 0 && (wx_i64)s_sum != (wx_i64)all) bad = true;
  if (bad) atomicOr(reinterpret_cast<unsigned int *>(&a.ctrs[1]), WX_DEVERR_INTERNAL_KEY);
}

// ---------------------------------------------------------------- fold
// One wave per group g: its rows are values [start, start + count) of the
// key-major array (start = the counts of the groups before it).  (Measured
// and dropped: the chunks staged as floats, read a chunk ahead and widened
// beside each add -- 14.3 vs 12.35 ms per C3 query, the extra v_cvt per value
// sits on the chain's issue slots; profiles/r05/group_row_order_fold_ab.txt.)  The wave
// streams them (coalesced); each 64-value chunk is widened into one half of
// a two-chunk LDS ring one chunk ahead of its adds and read back by every
// lane (same address: a broadcast), so only the dependent double adds are on
// the chain: s = ((0 + v0) + v1) + ..., the reference's fold.
#ifndef WX_RO_FOLD_AHEAD
#define WX_RO_FOLD_AHEAD 8  // 64-value chunks whose global loads are in flight ahead of the adds
#endif
extern "C" __global__ __launch_bounds__(64) void wx_ro_fold(WxRoFoldArgs a) {
  constexpr int U = WX_RO_FOLD_AHEAD;
  __shared__ double s_fold[2][64];
#if WX_FOLD_EXACT
  __shared__ double s_xf[WX_XF_B];
#endif
  const int lane = threadIdx.x;
  for (wx_i64 g = blockIdx.x; g < a.n_groups; g += gridDim.x) {
    wx_i64 start = 0;
    for (wx_i64 h = lane; h < g; h += 64) start += a.gcounts[h];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) start += __shfl_xor(start, o);
    const wx_i64 c = a.gcounts[g];
    const float *v = a.svals + start;
    if (a.skip_above > 0 && c > a.skip_above) continue;  // folded by the wx_xf_big_* kernels
#if WX_FOLD_EXACT
    const double xs = wx::fold_exact(v, c, s_xf);
    if (lane == 0) a.out_sums[g] = xs;
    __builtin_amdgcn_wave_barrier();
    continue;
#endif
    const wx_i64 nch = (c + 63) >> 6;
    double s = 0.0;
    // chunk 0 staged in half 0; chunks 1 .. U in flight (xr[u] = chunk u + 1)
    s_fold[0][lane] = (double)(lane < c ? v[lane] : 0.0f);
    float xr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const wx_i64 i = (wx_i64)(u + 1) * 64 + lane;
      xr[u] = i < c ? v[i] : 0.0f;
    }
    for (wx_i64 k0 = 0; k0 < nch; k0 += U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const wx_i64 k = k0 + u;
        if (k >= nch) break;  // wave-uniform
        const int cur = u & 1;  // U is even: chunk k sits in half k & 1
        // chunk k + 1 into the other half (the previous chunk's reads out of
        // it are done: their adds consumed them), chunk k + 1 + U's load out
        s_fold[cur ^ 1][lane] = (double)xr[u];
        const wx_i64 nx = (k + 1 + U) * 64 + lane;
        xr[u] = nx < c ? v[nx] : 0.0f;
        __builtin_amdgcn_wave_barrier();
        // a chunk past the group's end is padded with +0.0: adding it leaves
        // the running sum unchanged (it starts at +0.0, so it is never -0.0)
        double d[64];
#pragma unroll
        for (int j = 0; j < 64; ++j) d[j] = s_fold[cur][j];
#pragma unroll
        for (int j = 0; j < 64; ++j) s += d[j];
      }
    }
    if (lane == 0) a.out_sums[g] = s;
    __builtin_amdgcn_wave_barrier();
  }
}
static_assert(WX_RO_FOLD_AHEAD % 2 == 0, "the fold's ring index needs an even prefetch depth");

#endif  // WX_OP == WX_OP_UTIL
