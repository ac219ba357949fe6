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
#ifndef WX_TOPK_UNROLLED_MAX
#define WX_TOPK_UNROLLED_MAX 8
#endif
// K from this up keeps 8-row lane lists and a spill list per wave (below):
// 1.95 vs 2.20 ms per 1e9 rows at K = 32, but 1.01 vs 0.80 at K = 9 and
// 1.17 vs 0.98 at K = 16, where the K-row lane lists' own filter still pays
// (profiles/r05/topk_by_k.txt)
#define WX_TOPK_SPILL_MIN 17
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

template <int C>
struct TopListT {
  wx_u32 k[C];
  wx_i64 i[C];
  bool full;  // C real rows held
  float wf;   // the worst held key as a float (valid when full)
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < C; ++j) { k[j] = 0u; i[j] = WX_IDX_NONE; }
    full = false;
    wf = 0.0f;
  }
  // Streaming insert of a row whose index exceeds every held index (rows of a
  // thread arrive in increasing order): a tie with the worst key never
  // enters, so one float compare rejects almost every row.  (C = K only: a
  // full list then holds K better rows, so a rejected row cannot be in the
  // top K.)
  __device__ __forceinline__ void offer(float f, wx_i64 idx) {
    if (full) {
      const bool in = WX_TOPK_DESC ? (f > wf) : (f < wf);
      if (!in && !(wf != wf && f == f)) return;  // a NaN worst is beaten by any number
    }
    push(rank_of(f), idx);
    full = i[C - 1] != WX_IDX_NONE;
    wf = key_of(k[C - 1]);
  }
  // As offer, for a lane list shorter than K: whatever leaves or never
  // enters the full list -- the evicted worst entry, or the row itself -- is
  // returned in (sk, si) for the wave's spill list (true when there is one).
  __device__ __forceinline__ bool offer_spill(float f, wx_i64 idx, wx_u32 &sk, wx_i64 &si) {
    const wx_u32 r = rank_of(f);
    if (full && !better(r, idx, k[C - 1], i[C - 1])) {
      sk = r;
      si = idx;
      return true;
    }
    const bool ev = full;
    sk = k[C - 1];
    si = i[C - 1];
    push(r, idx);
    full = i[C - 1] != WX_IDX_NONE;
    wf = key_of(k[C - 1]);
    return ev;
  }
  __device__ __forceinline__ void push(wx_u32 key, wx_i64 idx) {
    if (!better(key, idx, k[C - 1], i[C - 1])) return;
    bool done = false;
#pragma unroll
    for (int j = C - 1; j >= 0; --j) {
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
    for (int j = 0; j < C - 1; ++j) { k[j] = k[j + 1]; i[j] = i[j + 1]; }
    k[C - 1] = 0u;
    i[C - 1] = WX_IDX_NONE;
  }
};
using TopList = TopListT<WX_TOPK_K>;

// Merge the lanes' lists of one wave; lane 0 ends with the wave's K best in
// out_k/out_i (all lanes compute them).
template <int C>
__device__ __forceinline__ void wave_merge(TopListT<C> &L, wx_u32 (&out_k)[WX_TOPK_K], wx_i64 (&out_i)[WX_TOPK_K]) {
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
template <int NW, int C>
__device__ __forceinline__ void block_merge(TopListT<C> &L, wx_u32 (*s_k)[WX_TOPK_K], wx_i64 (*s_i)[WX_TOPK_K],
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

#if WX_TOPK_K >= WX_TOPK_SPILL_MIN
// Large K: each lane streams into a short list (WX_TOPK_LANE entries), and
// whatever a full lane list evicts or turns away goes to the wave's spill
// list -- K entries spread over lanes 0..K-1, best first, kept by wave-wide
// inserts.  A row is dropped only when K better rows are held (a full spill
// list) or when it is worse than the bound T, so the lanes' lists and the
// spill list together hold the wave's top K.
#define WX_TOPK_LANE 8
struct SpillList {
  wx_u32 k = 0u;              // entry `lane` (lanes >= K hold nothing)
  wx_i64 i = WX_IDX_NONE;
  // insert (nk, ni) (wave-uniform) in order; the worst entry falls off
  __device__ __forceinline__ void insert(wx_u32 nk, wx_i64 ni) {
    const int lane = threadIdx.x & 63;
    const bool ahead = lane < WX_TOPK_K && better(k, i, nk, ni);
    const int pos = __builtin_popcountll(__builtin_amdgcn_ballot_w64(ahead));  // the ahead entries are a prefix
    const wx_u32 pk = __shfl_up(k, 1);
    const wx_i64 pi = __shfl_up(i, 1);
    if (pos < WX_TOPK_K && lane < WX_TOPK_K) {
      if (lane == pos) { k = nk; i = ni; }
      else if (lane > pos) { k = pk; i = pi; }
    }
  }
  // (sk, si) would enter: the list is short, or it beats the K-th entry
  __device__ __forceinline__ bool enters(wx_u32 sk, wx_i64 si) const {
    const wx_u32 kk = (wx_u32)__builtin_amdgcn_readlane((int)k, WX_TOPK_K - 1);
    const wx_u32 lo = (wx_u32)__builtin_amdgcn_readlane((int)(wx_u32)(wx_u64)i, WX_TOPK_K - 1);
    const wx_u32 hi = (wx_u32)__builtin_amdgcn_readlane((int)(wx_u32)((wx_u64)i >> 32), WX_TOPK_K - 1);
    const wx_i64 ki = (wx_i64)(((wx_u64)hi << 32) | lo);
    return ki == WX_IDX_NONE || better(sk, si, kk, ki);
  }
  // every lane's pending spill (sp: it has one), in lane order; a spill the
  // K-th entry already beats is dropped before its turn (the serial inserts
  // are the slow batches' cost: a first batch spills ~24 rows per lane)
  __device__ __forceinline__ void take(bool sp, wx_u32 sk, wx_i64 si) {
    wx_u64 m = __builtin_amdgcn_ballot_w64(sp && enters(sk, si));
    while (m) {
      const int src = __builtin_ctzll(m);
      m &= m - 1;
      const wx_u32 nk = (wx_u32)__builtin_amdgcn_readlane((int)sk, src);
      const wx_u32 lo = (wx_u32)__builtin_amdgcn_readlane((int)(wx_u32)(wx_u64)si, src);
      const wx_u32 hi = (wx_u32)__builtin_amdgcn_readlane((int)(wx_u32)((wx_u64)si >> 32), src);
      insert(nk, (wx_i64)(((wx_u64)hi << 32) | lo));
      if (m) m &= __builtin_amdgcn_ballot_w64(enters(sk, si));
    }
  }
  // the K-th entry's rank (0: fewer than K held)
  __device__ __forceinline__ wx_u32 kth() const {
    const wx_u32 r = (wx_u32)__builtin_amdgcn_readlane((int)k, WX_TOPK_K - 1);
    const wx_u32 lo = (wx_u32)__builtin_amdgcn_readlane((int)(wx_u32)(wx_u64)i, WX_TOPK_K - 1);
    const wx_u32 hi = (wx_u32)__builtin_amdgcn_readlane((int)(wx_u32)((wx_u64)i >> 32), WX_TOPK_K - 1);
    return (((wx_u64)hi << 32) | lo) != (wx_u64)WX_IDX_NONE ? r : 0u;
  }
};
// The wave's K-th best (rank, 0 when it holds fewer than K rows): K rounds
// of a wave arg-max over the lanes' lists, popping the winner, keeping only
// the last round (no K-entry arrays).
template <int C>
__device__ __forceinline__ wx_u32 wave_kth(TopListT<C> L) {
  wx_u32 bk = 0u;
  wx_i64 bi = WX_IDX_NONE;
#pragma unroll 1
  for (int r = 0; r < WX_TOPK_K; ++r) {
    bk = L.k[0];
    bi = L.i[0];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const wx_u32 ok = __shfl_xor(bk, o);
      const wx_i64 oi = __shfl_xor(bi, o);
      if (better(ok, oi, bk, bi)) { bk = ok; bi = oi; }
    }
    if (L.i[0] == bi && L.k[0] == bk && bi != WX_IDX_NONE) L.pop();
  }
  return bi != WX_IDX_NONE ? bk : 0u;
}

// The block's K best into cand_k / cand_i[0, K): each wave writes its K best
// (K rounds of a wave arg-max) to LDS, then every entry of the NW sorted
// lists takes its place = the entries that beat it (its own list's by
// position, the others' by counting); places < K are written.  No K-entry
// register arrays.
template <int NW, int C>
__device__ __forceinline__ void block_place(TopListT<C> &L, wx_u32 (*s_k)[WX_TOPK_K], wx_i64 (*s_i)[WX_TOPK_K],
                                            wx_u32 *cand_k, wx_i64 *cand_i) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
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
    if (lane == 0) { s_k[wave][r] = bk; s_i[wave][r] = bi; }
    if (L.i[0] == bi && L.k[0] == bk && bi != WX_IDX_NONE) L.pop();
  }
  __syncthreads();
  for (int e = threadIdx.x; e < NW * WX_TOPK_K; e += NW * 64) {
    const int w = e / WX_TOPK_K, r = e % WX_TOPK_K;
    const wx_u32 k = s_k[w][r];
    const wx_i64 i = s_i[w][r];
    if (i == WX_IDX_NONE) continue;  // empty tail entries: the slots they would take stay empty below
    int place = r;
    for (int v = 0; v < NW; ++v) {
      if (v == w) continue;
      for (int q = 0; q < WX_TOPK_K; ++q) place += better(s_k[v][q], s_i[v][q], k, i) ? 1 : 0;
    }
    if (place < WX_TOPK_K) { cand_k[place] = k; cand_i[place] = i; }
  }
  // slots past the block's valid entries: empty
  int nvalid = 0;
  for (int v = 0; v < NW; ++v)
    for (int q = 0; q < WX_TOPK_K; ++q) nvalid += s_i[v][q] != WX_IDX_NONE ? 1 : 0;
  for (int j = nvalid + (int)threadIdx.x; j < WX_TOPK_K; j += NW * 64) { cand_k[j] = 0u; cand_i[j] = WX_IDX_NONE; }
}

// the lane list plus this lane's spill entry, for the wave merges
__device__ __forceinline__ TopListT<WX_TOPK_LANE + 1> with_spill(const TopListT<WX_TOPK_LANE> &L, const SpillList &W) {
  TopListT<WX_TOPK_LANE + 1> M;
#pragma unroll
  for (int j = 0; j < WX_TOPK_LANE; ++j) { M.k[j] = L.k[j]; M.i[j] = L.i[j]; }
  M.k[WX_TOPK_LANE] = 0u;
  M.i[WX_TOPK_LANE] = WX_IDX_NONE;
  M.full = false;
  M.wf = 0.0f;
  if (W.i != WX_IDX_NONE) M.push(W.k, W.i);
  return M;
}
#endif
}  // namespace wx

__device__ __forceinline__ void wx_topk_scan_body(const WxTopkArgs &wx_a) {
  __shared__ wx_u32 s_k[WX_WAVES][WX_TOPK_K];
  __shared__ wx_i64 s_i[WX_WAVES][WX_TOPK_K];
#if WX_TOPK_K > WX_TOPK_UNROLLED_MAX
  __shared__ float wx_s_fv[WX_UNROLL * 4][WX_BLOCK];  // a slow batch's candidate keys (each thread its own column)
#endif
#if WX_TOPK_K < WX_TOPK_SPILL_MIN
  wx::TopList wx_L;
#else
  wx::TopListT<WX_TOPK_LANE> wx_L;  // + the wave's spill list (large K)
  wx::SpillList wx_W;
#endif
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
  // (lane l: slot l) and a wave max (relaxed: a stale value is still a bound),
  // the first time before batch 0 (the seed pass may have raised them).
  const float wx_none = WX_TOPK_DESC ? -__builtin_inff() : __builtin_inff();
  float wx_T = wx_none;   // best known bound (this wave and the grid)
  wx_u32 wx_pub = 0u;     // best rank this wave has found
  wx_u32 wx_gseen = 0u;   // best grid-wide rank this wave has seen or published
  int wx_batch = 0;
  const wx_i64 wx_nq = (wx_a.n_rows + 3) >> 2;
  const wx_i64 wx_nfull = wx_a.n_rows >> 2;
  for (wx_i64 wx_base = (wx_i64)blockIdx.x * wx_a.q_stride; wx_base < wx_nq; wx_base += wx_a.q_step) {
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
    if ((wx_batch++ & 7) == 0) {
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
#if WX_TOPK_K < WX_TOPK_SPILL_MIN
      const bool wx_beats_own =
          !wx_L.full || wx_L.wf != wx_L.wf || (WX_TOPK_DESC ? wx_m > wx_L.wf : wx_m < wx_L.wf);
      wx_slow = wx_beats_T && wx_beats_own;
#else
      wx_slow = wx_beats_T;  // a short lane list turns nothing away: rows it cannot keep spill
#endif
    }
#if WX_TOPK_K >= WX_TOPK_SPILL_MIN
    wx_slow = __builtin_amdgcn_ballot_w64(wx_slow) != 0ull;  // the spill inserts need the whole wave
#endif
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
      // the candidate keys staged in LDS (column r, lane tid: conflict-free): a
      // register array indexed by the rolled loop below lived in scratch
      float (*wx_fv)[WX_BLOCK] = wx_s_fv;
      wx_u32 wx_pm = 0u;  // bit 4u + e: row (u, e) is a candidate
#pragma unroll
      for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {
#pragma unroll
        for (int wx_e = 0; wx_e < 4; ++wx_e) {
          WX_COLS(WX_BIND_U)
          const wx_i64 idx = (WX_QUAD(wx_u) << 2) + wx_e;
          const bool wx_in = WX_QUAD(wx_u) < wx_nq && idx < wx_a.n_rows && WX_EVAL_COND();
          const float wx_f = wx_in ? static_cast<float>(WX_EXPR) : 0.0f;
          wx_fv[wx_u * 4 + wx_e][threadIdx.x] = wx_f;
          if (wx_in && !(WX_TOPK_DESC ? wx_f < wx_T : wx_f > wx_T)) wx_pm |= 1u << (wx_u * 4 + wx_e);
        }
      }
#if WX_TOPK_K < WX_TOPK_SPILL_MIN
#pragma unroll 1
      for (int wx_r = 0; wx_r < WX_UNROLL * 4; ++wx_r)
        if ((wx_pm >> wx_r) & 1u) wx_L.offer(wx_fv[wx_r][threadIdx.x], (WX_QUAD(wx_r >> 2) << 2) + (wx_r & 3));
#else
#pragma unroll 1
      for (int wx_r = 0; wx_r < WX_UNROLL * 4; ++wx_r) {
        bool wx_sp = false;
        wx_u32 wx_sk = 0u;
        wx_i64 wx_si = WX_IDX_NONE;
        if ((wx_pm >> wx_r) & 1u) {
          wx_sp = wx_L.offer_spill(wx_fv[wx_r][threadIdx.x], (WX_QUAD(wx_r >> 2) << 2) + (wx_r & 3), wx_sk, wx_si);
          const float wx_sf = wx::key_of(wx_sk);
          if (wx_sp && (WX_TOPK_DESC ? wx_sf < wx_T : wx_sf > wx_T)) wx_sp = false;  // strictly worse than T
        }
        wx_W.take(wx_sp, wx_sk, wx_si);  // wave-uniform: every lane runs the loop
      }
#endif
#endif
    }
    // after any insert in the wave: the wave's exact K-th best
    if (__builtin_amdgcn_ballot_w64(wx_slow)) {
#if WX_TOPK_K < WX_TOPK_SPILL_MIN
      wx::TopList wx_c = wx_L;
      wx_u32 wk[WX_TOPK_K];
      wx_i64 wi[WX_TOPK_K];
      wx::wave_merge(wx_c, wk, wi);
      const wx_u32 r = wi[WX_TOPK_K - 1] != WX_IDX_NONE ? wk[WX_TOPK_K - 1] : 0u;  // 0: fewer than K rows, or NaN
#else
      // the wave's held rows: lane lists + spill list
      const wx_u32 r = wx::wave_kth(wx::with_spill(wx_L, wx_W));
#endif
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
#if WX_TOPK_K < WX_TOPK_SPILL_MIN
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
#else
  auto wx_c = wx::with_spill(wx_L, wx_W);
  wx::block_place<WX_WAVES>(wx_c, s_k, s_i, wx_a.cand_k + (wx_i64)blockIdx.x * WX_TOPK_K,
                            wx_a.cand_i + (wx_i64)blockIdx.x * WX_TOPK_K);
#endif
}

extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_topk_scan(WxTopkArgs wx_a) { wx_topk_scan_body(wx_a); }

// The seed pass (tables of 2^24 rows and more, warpexec.cpp do_topk): the
// same scan over one span per workgroup at evenly spaced offsets (about 1M
// rows), merged by wx_topk_finalize with seed = 1 into slot 0 before the scan
// starts.  Without it a wave's bound is the K-th best of the rows IT has seen
// (and the grid's the best such), which turns batches away only after ~K
// batches; the seed's K-th best of 1M rows is a bound from batch 0 on.  Exact:
// it is the key of a real row with K rows at least as good (the scan drops
// only rows strictly worse).  Its own name keeps it apart in kernel traces.
extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_topk_seed(WxTopkArgs wx_a) { wx_topk_scan_body(wx_a); }

// One 1024-thread block; candidate loads are issued 8 per thread at a time
// (the loop is latency-bound otherwise: the candidates sit in other XCDs' L2).
#define WX_FIN_BLOCK 1024
#define WX_FIN_BATCH 8
extern "C" __global__ __launch_bounds__(WX_FIN_BLOCK) void wx_topk_finalize(WxTopkFinArgs wx_a) {
  // the scan has finished (stream order): reset its bound slots for the next
  // query here instead of a host memset per query
  if (wx_a.g_thresh && !wx_a.seed && threadIdx.x < WX_TOPK_SLOTS)
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
    if (wx_a.seed && bi[WX_TOPK_K - 1] != WX_IDX_NONE)  // K rows: the K-th best rank bounds the table's
      atomicMax(wx_a.g_thresh, bk[WX_TOPK_K - 1]);
  }
  if (wx_a.seed) return;
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
