// wx_topk.hip -- ORDER BY .. LIMIT k <= 32: the per-lane top-K scan and its finalize
// (one of the kernel sources warpexec concatenates after wx_common.hip, whose
// header describes the prelude they expect)

// ===========================================================================
#if WX_OP == WX_OP_TOPK
// ORDER BY key [DESC] LIMIT K.  Each lane keeps its K best (ord, row) pairs
// sorted in registers; a row costs one compare against the lane's worst
// entry unless it enters.  Lanes merge by K rounds of a wave64 arg-max
// (butterfly shuffles), waves merge through LDS, and blocks emit K
// candidates each; wx_topk_finalize repeats the merge over all candidates and
// evaluates the SELECT expression at the winning rows (gather binding).
// Total order: better key first, then smaller row index.
#ifndef WX_TOPK_K
#define WX_TOPK_K 5
#endif
#ifndef WX_TOPK_DESC
#define WX_TOPK_DESC 1
#endif
#ifndef WX_UNROLL
#define WX_UNROLL 8
#endif
// K up to this keeps the fully unrolled insertion (C5's K = 5); larger K
// takes the rolled one (compile time, below)
#define WX_TOPK_UNROLLED_MAX 8
#define WX_IDX_NONE 0x7fffffffffffffffll

namespace wx {
// map so that "larger is better" in both directions; NaN (0) stays worst
__device__ __forceinline__ wx_u32 rank_of(float f) {
  const wx_u32 m = f2ord(f);
  if (WX_TOPK_DESC || m == 0u) return m;
  return ~m;  // ascending: smaller float = better; m != 0 so ~m != 0xffffffff unless m == 0
}
__device__ __forceinline__ float key_of(wx_u32 r) { return ord2f((WX_TOPK_DESC || r == 0u) ? r : ~r); }
__device__ __forceinline__ bool better(wx_u32 ka, wx_i64 ia, wx_u32 kb, wx_i64 ib) {
  return ka > kb || (ka == kb && ia < ib);
}

struct TopList {
  wx_u32 k[WX_TOPK_K];
  wx_i64 i[WX_TOPK_K];
  bool full;  // K real rows held
  float wf;   // the worst held key as a float (valid when full)
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < WX_TOPK_K; ++j) { k[j] = 0u; i[j] = WX_IDX_NONE; }
    full = false;
    wf = 0.0f;
  }
  // Streaming insert of a row whose index exceeds every held index (rows of a
  // thread arrive in increasing order): a tie with the worst key never
  // enters, so one float compare rejects almost every row.
  __device__ __forceinline__ void offer(float f, wx_i64 idx) {
    if (full) {
      const bool in = WX_TOPK_DESC ? (f > wf) : (f < wf);
      if (!in && !(wf != wf && f == f)) return;  // a NaN worst is beaten by any number
    }
    push(rank_of(f), idx);
    full = i[WX_TOPK_K - 1] != WX_IDX_NONE;
    wf = key_of(k[WX_TOPK_K - 1]);
  }
  __device__ __forceinline__ void push(wx_u32 key, wx_i64 idx) {
    if (!better(key, idx, k[WX_TOPK_K - 1], i[WX_TOPK_K - 1])) return;
    bool done = false;
#pragma unroll
    for (int j = WX_TOPK_K - 1; j >= 0; --j) {
      if (!done) {
        if (j == 0 || !better(key, idx, k[j - 1], i[j - 1])) {
          k[j] = key; i[j] = idx; done = true;
        } else {
          k[j] = k[j - 1]; i[j] = i[j - 1];
        }
      }
    }
  }
  __device__ __forceinline__ void pop() {
#pragma unroll
    for (int j = 0; j < WX_TOPK_K - 1; ++j) { k[j] = k[j + 1]; i[j] = i[j + 1]; }
    k[WX_TOPK_K - 1] = 0u;
    i[WX_TOPK_K - 1] = WX_IDX_NONE;
  }
};

// Merge the lanes' lists of one wave; lane 0 ends with the wave's K best in
// out_k/out_i (all lanes compute them).
__device__ __forceinline__ void wave_merge(TopList &L, wx_u32 (&out_k)[WX_TOPK_K], wx_i64 (&out_i)[WX_TOPK_K]) {
#pragma unroll 1
  for (int r = 0; r < WX_TOPK_K; ++r) {
    wx_u32 bk = L.k[0];
    wx_i64 bi = L.i[0];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const wx_u32 ok = __shfl_xor(bk, o);
      const wx_i64 oi = __shfl_xor(bi, o);
      if (better(ok, oi, bk, bi)) { bk = ok; bi = oi; }
    }
    out_k[r] = bk;
    out_i[r] = bi;
    if (L.i[0] == bi && L.k[0] == bk && bi != WX_IDX_NONE) L.pop();
  }
}

// Merge the wave lists of a block through LDS; every thread of wave 0 returns
// the block's K best (valid in lane 0).
template <int NW>
__device__ __forceinline__ void block_merge(TopList &L, wx_u32 (*s_k)[WX_TOPK_K], wx_i64 (*s_i)[WX_TOPK_K],
                                            wx_u32 (&bk)[WX_TOPK_K], wx_i64 (&bi)[WX_TOPK_K]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  wx_u32 wk[WX_TOPK_K];
  wx_i64 wi[WX_TOPK_K];
  wave_merge(L, wk, wi);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < WX_TOPK_K; ++j) { s_k[wave][j] = wk[j]; s_i[wave][j] = wi[j]; }
  }
  __syncthreads();
  if (wave == 0) {  // lane w holds wave w's sorted list: one more wave merge
    static_assert(NW <= 64, "one lane per wave");
    TopList M;
    M.init();
    if (lane < NW) {
#pragma unroll
      for (int j = 0; j < WX_TOPK_K; ++j) { M.k[j] = s_k[lane][j]; M.i[j] = s_i[lane][j]; }
    }
    wave_merge(M, bk, bi);
  }
}
}  // namespace wx

extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_topk_scan(WxTopkArgs wx_a) {
  __shared__ wx_u32 s_k[WX_WAVES][WX_TOPK_K];
  __shared__ wx_i64 s_i[WX_WAVES][WX_TOPK_K];
  wx::TopList wx_L;
  wx_L.init();
  // Batches of WX_UNROLL row quads per thread.  Once the lane's list is full
  // (and its worst key is a number), a complete batch costs one max/min of its
  // keys against the worst (rows failing the WHERE count as -inf/+inf; NaN
  // keys never enter a full list; ties never enter, later rows lose): only
  // batches that can change the list re-evaluate their rows and insert.
  // Thresholds: the K-th best key of any set of rows is a lower bound on the
  // global K-th best, so rows strictly worse can be dropped.  After a batch in
  // which a lane inserted, the wave takes the exact K-th best over all its
  // lanes' lists (K rounds of a wave arg-max; the max over lanes of each
  // lane's own K-th best is far weaker with ≈1 900 rows per lane) and raises
  // the grid-wide bound with atomicMax on the order-preserving rank.  The
  // bound lives in WX_TOPK_SLOTS slots on separate 256-B lines (a single
  // address serialised ≈50K early atomics: 2.4 ms); a wave publishes to its
  // workgroup's slot and every 8th batch reads all slots with one vector load
  // (lane l: slot l) and a wave max (relaxed: a stale value is still a bound).
  const float wx_none = WX_TOPK_DESC ? -__builtin_inff() : __builtin_inff();
  float wx_T = wx_none;   // best known bound (this wave and the grid)
  wx_u32 wx_pub = 0u;     // best rank this wave has found
  wx_u32 wx_gseen = 0u;   // best grid-wide rank this wave has seen or published
  int wx_batch = 0;
  const wx_i64 wx_nq = (wx_a.n_rows + 3) >> 2;
  const wx_i64 wx_nfull = wx_a.n_rows >> 2;
  for (wx_i64 wx_base = (wx_i64)blockIdx.x * WX_SPAN; wx_base < wx_nq; wx_base += (wx_i64)gridDim.x * WX_SPAN) {
    WX_COLS(WX_DECL_U)
    const bool wx_whole = WX_ALIGNED16 && wx_base + WX_SPAN <= wx_nfull;  // workgroup-uniform
    if (wx_whole) {
#pragma unroll
      for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {
        const wx_i64 wx_r0u = WX_QUAD(wx_u) << 2;
        WX_COLS(WX_LOAD_U_FAST)
      }
    } else {
#pragma unroll
      for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {
        const wx_i64 wx_r0u = WX_QUAD(wx_u) << 2;
        WX_COLS(WX_LOAD_U)
      }
    }
    if ((wx_batch++ & 7) == 7) {
      wx_u32 wx_g = __hip_atomic_load(wx_a.g_thresh + (threadIdx.x & 63) * WX_TOPK_SLOT_STRIDE, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const wx_u32 x = __shfl_xor(wx_g, o);
        wx_g = x > wx_g ? x : wx_g;
      }
      if (wx_g > wx_gseen) {
        wx_gseen = wx_g;
        const float gf = wx::key_of(wx_g);
        wx_T = WX_TOPK_DESC ? fmaxf(wx_T, gf) : fminf(wx_T, gf);
      }
    }
    bool wx_slow = !wx_whole;
    if (!wx_slow) {
      // Rows strictly worse than T cannot reach the top K; rows equal to T may
      // (smaller index).  A full lane also needs a row strictly better than its
      // own worst (its rows arrive in increasing index order).
      float wx_m = wx_none;
#pragma unroll
      for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {
#pragma unroll
        for (int wx_e = 0; wx_e < 4; ++wx_e) {
          WX_COLS(WX_BIND_U)
          const wx_i64 idx = (WX_QUAD(wx_u) << 2) + wx_e;
          (void)idx;
          const float wx_v = WX_EVAL_COND() ? static_cast<float>(WX_EXPR) : wx_none;
          wx_m = WX_TOPK_DESC ? fmaxf(wx_m, wx_v) : fminf(wx_m, wx_v);
        }
      }
      const bool wx_beats_T = wx_T == wx_none || (WX_TOPK_DESC ? wx_m >= wx_T : wx_m <= wx_T);
      const bool wx_beats_own =
          !wx_L.full || wx_L.wf != wx_L.wf || (WX_TOPK_DESC ? wx_m > wx_L.wf : wx_m < wx_L.wf);
      wx_slow = wx_beats_T && wx_beats_own;
    }
    if (wx_slow) {
#if WX_TOPK_K <= WX_TOPK_UNROLLED_MAX
#pragma unroll
      for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {
        if (WX_QUAD(wx_u) < wx_nq) {
#pragma unroll
          for (int wx_e = 0; wx_e < 4; ++wx_e) {
            WX_COLS(WX_BIND_U)
            const wx_i64 idx = (WX_QUAD(wx_u) << 2) + wx_e;
            if (idx < wx_a.n_rows && WX_EVAL_COND()) {
              const float wx_f = static_cast<float>(WX_EXPR);
              if (!(WX_TOPK_DESC ? wx_f < wx_T : wx_f > wx_T)) wx_L.offer(wx_f, idx);
            }
          }
        }
      }
#else
      // large K: the batch's candidate keys first (unrolled), then ONE copy of
      // the K-deep insertion in a rolled loop (uniform index: the key array
      // stays in registers) -- 32 inlined copies of a 32-deep insertion took
      // ~50 s of hiprtc per query shape
      float wx_fv[WX_UNROLL * 4];
      wx_u32 wx_pm = 0u;  // bit 4u + e: row (u, e) is a candidate
#pragma unroll
      for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {
#pragma unroll
        for (int wx_e = 0; wx_e < 4; ++wx_e) {
          WX_COLS(WX_BIND_U)
          const wx_i64 idx = (WX_QUAD(wx_u) << 2) + wx_e;
          const bool wx_in = WX_QUAD(wx_u) < wx_nq && idx < wx_a.n_rows && WX_EVAL_COND();
          const float wx_f = wx_in ? static_cast<float>(WX_EXPR) : 0.0f;
          wx_fv[wx_u * 4 + wx_e] = wx_f;
          if (wx_in && !(WX_TOPK_DESC ? wx_f < wx_T : wx_f > wx_T)) wx_pm |= 1u << (wx_u * 4 + wx_e);
        }
      }
#pragma unroll 1
      for (int wx_r = 0; wx_r < WX_UNROLL * 4; ++wx_r)
        if ((wx_pm >> wx_r) & 1u) wx_L.offer(wx_fv[wx_r], (WX_QUAD(wx_r >> 2) << 2) + (wx_r & 3));
#endif
    }
    // after any insert in the wave: the wave's exact K-th best
    if (__builtin_amdgcn_ballot_w64(wx_slow)) {
      wx::TopList wx_c = wx_L;
      wx_u32 wk[WX_TOPK_K];
      wx_i64 wi[WX_TOPK_K];
      wx::wave_merge(wx_c, wk, wi);
      const wx_u32 r = wi[WX_TOPK_K - 1] != WX_IDX_NONE ? wk[WX_TOPK_K - 1] : 0u;  // 0: fewer than K rows, or NaN
      if (r > wx_pub) {
        const float t = wx::key_of(r);
        wx_T = WX_TOPK_DESC ? fmaxf(wx_T, t) : fminf(wx_T, t);
        wx_pub = r;
        // publish only what beats the grid's bound as last seen: one address
        // taking an atomic from every wave on every improvement serialises
        if (r > wx_gseen) {
          if ((threadIdx.x & 63) == 0)
            atomicMax(wx_a.g_thresh + (blockIdx.x % WX_TOPK_SLOTS) * WX_TOPK_SLOT_STRIDE, r);
          wx_gseen = r;
        }
      }
    }
  }
  wx_u32 bk[WX_TOPK_K];
  wx_i64 bi[WX_TOPK_K];
  wx::block_merge<WX_WAVES>(wx_L, s_k, s_i, bk, bi);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < WX_TOPK_K; ++j) {
      wx_a.cand_k[(wx_i64)blockIdx.x * WX_TOPK_K + j] = bk[j];
      wx_a.cand_i[(wx_i64)blockIdx.x * WX_TOPK_K + j] = bi[j];
    }
  }
}

// One 1024-thread block; candidate loads are issued 8 per thread at a time
// (the loop is latency-bound otherwise: the candidates sit in other XCDs' L2).
#define WX_FIN_BLOCK 1024
#define WX_FIN_BATCH 8
extern "C" __global__ __launch_bounds__(WX_FIN_BLOCK) void wx_topk_finalize(WxTopkFinArgs wx_a) {
  // the scan has finished (stream order): reset its bound slots for the next
  // query here instead of a host memset per query
  if (wx_a.g_thresh && threadIdx.x < WX_TOPK_SLOTS)
    __hip_atomic_store(wx_a.g_thresh + threadIdx.x * WX_TOPK_SLOT_STRIDE, 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  __shared__ wx_u32 s_k[WX_FIN_BLOCK / 64][WX_TOPK_K];
  __shared__ wx_i64 s_i[WX_FIN_BLOCK / 64][WX_TOPK_K];
  __shared__ wx_u32 s_bk[WX_TOPK_K];
  __shared__ wx_i64 s_bi[WX_TOPK_K];
  wx::TopList L;
  L.init();
  for (wx_i64 c0 = threadIdx.x; c0 < wx_a.n_cand; c0 += (wx_i64)WX_FIN_BLOCK * WX_FIN_BATCH) {
    wx_u32 ck[WX_FIN_BATCH];
    wx_i64 ci[WX_FIN_BATCH];
#pragma unroll
    for (int b = 0; b < WX_FIN_BATCH; ++b) {
      const wx_i64 c = c0 + (wx_i64)b * WX_FIN_BLOCK;
      ck[b] = c < wx_a.n_cand ? wx_a.cand_k[c] : 0u;
      ci[b] = c < wx_a.n_cand ? wx_a.cand_i[c] : WX_IDX_NONE;
    }
#if WX_TOPK_K <= WX_TOPK_UNROLLED_MAX
#pragma unroll
#else
#pragma unroll 1
#endif
    for (int b = 0; b < WX_FIN_BATCH; ++b)
      if (ci[b] != WX_IDX_NONE) L.push(ck[b], ci[b]);
  }
  wx_u32 bk[WX_TOPK_K];
  wx_i64 bi[WX_TOPK_K];
  wx::block_merge<WX_FIN_BLOCK / 64>(L, s_k, s_i, bk, bi);
  if (threadIdx.x == 0) {
    int n = 0;
#pragma unroll
    for (int j = 0; j < WX_TOPK_K; ++j) {
      s_bk[j] = bk[j];
      s_bi[j] = bi[j];
      n += bi[j] != WX_IDX_NONE ? 1 : 0;
    }
    if (wx_a.count_out) *wx_a.count_out = n;
  }
  __syncthreads();
  const int wx_j = threadIdx.x;
  if (wx_j < WX_TOPK_K && s_bi[wx_j] != WX_IDX_NONE) {
    const wx_i64 idx = s_bi[wx_j];
    WX_COLS(WX_BIND_ROW)
    // the row's own key (not the rank's image: keeps -0.0 and NaN bits)
    const float wx_key = static_cast<float>(WX_EXPR);
    if (wx_a.out_keys) wx_a.out_keys[wx_j] = wx_key;
    if (wx_a.out_idx) wx_a.out_idx[wx_j] = wx_a.row_base + idx;
    if (wx_a.out_vals) {
#if WX_HAS_SELECT
      wx_a.out_vals[wx_j] = static_cast<float>(WX_SELECT);
#else
      wx_a.out_vals[wx_j] = wx_key;
#endif
    }
  }
}
#endif
