// wx_radix.hip -- the stable LSD radix sort (jit_sort_float / jit_sort_pairs, ORDER BY)
// (one of the kernel sources warpexec concatenates after wx_common.hip, whose
// header describes the prelude they expect)

#if WX_OP == WX_OP_UTIL
// ---------------------------------------------------------------------------
// LSD radix sort for the jit_sort_* entry points (src/jit.cpp:248-307): four
// stable passes of 8-bit digits over a 32-bit order key computed on the fly
// from the element itself (floats: the order map with -0.0 == +0.0 and NaN
// last; ints: sign flip; descending: the complement), so float sorts move
// only their 4-byte values and pair sorts their key + payload.
//
// wx_radix_hist: one read of the input builds the histograms of all four
// digits (one 1024-thread workgroup per CU, 32 counter copies in LDS).  The
// host scans them into per-digit output bases and skips a pass whose digit
// is the same for every key.
//
// wx_radix_tile_* (one pass, "onesweep"): a workgroup takes tile t from a
// ticket counter, loads WX_RS_ITEMS keys per lane wave-striped (key i of
// lane l of wave w at t*TILE + w*64*ITEMS + i*64 + l, so rank order is input
// order), and ranks each key inside its wave by one returning LDS add on the
// wave's digit counter (lane 0's digit group by a ballot).  Threads 0..255
// then own one digit each: prefix over the waves and digits, publish the
// tile's count {A}; the keys (and payloads) are permuted into digit order in
// LDS while the digit threads look back over the preceding tiles' words of
// their digit to an inclusive {P} and publish {P}; the tile is written out
// of LDS, consecutive lanes to consecutive addresses of a digit's run, with
// plain stores (L2 merges the runs' partial lines).  Every wait is bounded: a
// timed-out waiter raises WX_DEVERR_LOOKBACK and the abort word, and the
// launch drains.
#define WX_RS_WAVES (WX_RS_BLOCK / 64)
#ifndef WX_RS_LBW
// predecessor words per digit per look-back round: keys 3 (11.55 vs 11.71 ms
// per 1e9 keys over 2, 10.22 vs 10.35 on another box, 127 VGPRs: no spill;
// profiles/r03/abl_sort_lbw.txt, abl_sort_sleep_lbw.txt); 8 slower
#define WX_RS_LBW 3
#endif
#ifndef WX_RS_SLEEP
#define WX_RS_SLEEP 1  // look-back: s_sleep between polls of an unpublished predecessor word (0: none)
#endif
#ifndef WX_STALL_TICKS
#define WX_STALL_TICKS 200000000ull  // 2 s at 100 MHz without progress (see the compaction look-back)
#endif
#define WX_STALL_SPINS (1u << 16)  // and this many polls: a descheduled wave polls nothing
#define WX_RS_FLAG_A (1ull << 56)
#define WX_RS_FLAG_P (2ull << 56)
#define WX_RS_VAL_MASK ((1ull << 56) - 1ull)


// Order key with the direction and key kind known at compile time.
template <int KIND, bool ASC>
__device__ __forceinline__ wx_u32 wx_rs_key_t(wx_u32 x) {
  wx_u32 r;
  if constexpr (KIND == 0) {
    r = wx::f2ord(__uint_as_float(x));
    if (r == 0u) return 0xffffffffu;  // NaN last in either direction
  } else if constexpr (KIND == 2) {
    // floats with no NaN and no -0.0 (the histogram pass checked): the plain
    // order flip, equal to f2ord on every such value, in 2 VALU ops where
    // f2ord's zero and NaN fixes take 9 -- the tile kernels recompute the
    // digit three times per key
    r = x ^ ((wx_u32)((int)x >> 31) | 0x80000000u);
  } else {
    r = x ^ 0x80000000u;
  }
  return ASC ? r : ~r;
}

#ifndef WX_RS_HUNROLL
#define WX_RS_HUNROLL 4  // 16-byte loads in flight per thread (64 B): the kernel is latency-bound below that
#endif
// (Round 1's 256-thread histogram with 8 counter copies, 1.30 ms per 1e9
// keys against this kernel's 0.66, profiles/r02/abl_sort_hwide*.txt, was
// removed in round 5.)
// One 1024-thread workgroup per CU with 32 copies of every counter (128 KB):
// lane l adds to copy l % 32, so the 32 lanes of an LDS cycle always hit 32
// different banks and never one address -- no digit distribution conflicts.
#define WX_RS_HBLOCK 1024
#define WX_RS_HC 32
// returns 1 for a float key the plain order flip would misplace (NaN, -0.0)
template <int KIND, bool ASC>
__device__ __forceinline__ wx_u32 wx_rs_count_wide(wx_u32 *h, wx_u32 x, int copy) {
  const wx_u32 k = wx_rs_key_t<KIND, ASC>(x);
#pragma unroll
  for (int p = 0; p < 4; ++p) atomicAdd(&h[(p * 256 + ((k >> (8 * p)) & 255u)) * WX_RS_HC + copy], 1u);
  return KIND == 0 ? (wx_u32)((x & 0x7fffffffu) > 0x7f800000u || x == 0x80000000u) : 0u;
}
#define WX_RS_COUNT(x) (wx_sp |= wx_rs_count_wide<KIND, ASC>(h, (x), copy))

// All four digit histograms in one read: contiguous spans of 16-byte loads
// (WX_RS_HUNROLL per thread) when the array is 16-byte aligned, scalar
// loads otherwise; per-workgroup LDS counters, one global add per bin.
template <int KIND, bool ASC>
__device__ __forceinline__ void wx_radix_hist_impl(const WxRadixHistArgs &a) {
  __shared__ wx_u32 h[4 * 256 * WX_RS_HC];  // [digit][bin][copy]
  for (int i = threadIdx.x; i < 4 * 256 * WX_RS_HC; i += WX_RS_HBLOCK) h[i] = 0u;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int copy = lane % WX_RS_HC;
  (void)lane;
  wx_u32 wx_sp = 0u;  // this thread saw a NaN or -0.0 key
  if (a.aligned) {
    typedef wx_u32 u4 __attribute__((ext_vector_type(4)));
    const u4 *q = reinterpret_cast<const u4 *>(a.src);
    const wx_i64 nq = a.n >> 2;
    const wx_i64 span = (wx_i64)WX_RS_HBLOCK * WX_RS_HUNROLL;
    const wx_i64 stride = (wx_i64)gridDim.x * span;
    wx_i64 base = (wx_i64)blockIdx.x * span;
    // Whole spans, software-pipelined as wx_project_dense: the next span's
    // loads go out before this span is counted (unconditional loads; guarded
    // ones each wait for the one before and the loop ran latency-bound).
    if (base + span <= nq) {
      u4 v[WX_RS_HUNROLL], w[WX_RS_HUNROLL];
#pragma unroll
      for (int u = 0; u < WX_RS_HUNROLL; ++u) w[u] = wx::ldv(q + base + (wx_i64)u * WX_RS_HBLOCK + threadIdx.x);
      __builtin_amdgcn_s_waitcnt(0x0f70);  // the loop head inherits no pending loads
#pragma unroll
      for (int u = 0; u < WX_RS_HUNROLL; ++u) v[u] = w[u];
      while (true) {
        const wx_i64 nb = base + stride;
        const bool more = nb + span <= nq;  // workgroup-uniform
        if (more) {
#pragma unroll
          for (int u = 0; u < WX_RS_HUNROLL; ++u) w[u] = wx::ldv(q + nb + (wx_i64)u * WX_RS_HBLOCK + threadIdx.x);
        }
#pragma unroll
        for (int u = 0; u < WX_RS_HUNROLL; ++u) {
          WX_RS_COUNT(v[u].x);
          WX_RS_COUNT(v[u].y);
          WX_RS_COUNT(v[u].z);
          WX_RS_COUNT(v[u].w);
        }
        base = nb;
        if (!more) break;
#pragma unroll
        for (int u = 0; u < WX_RS_HUNROLL; ++u) v[u] = w[u];
      }
    }
    for (; base < nq; base += stride) {
      u4 v[WX_RS_HUNROLL];
      if (base + span <= nq) {  // workgroup-uniform: unconditional loads, all in flight together
#pragma unroll
        for (int u = 0; u < WX_RS_HUNROLL; ++u) v[u] = wx::ldv(q + base + (wx_i64)u * WX_RS_HBLOCK + threadIdx.x);
#pragma unroll
        for (int u = 0; u < WX_RS_HUNROLL; ++u) {
          WX_RS_COUNT(v[u].x);
          WX_RS_COUNT(v[u].y);
          WX_RS_COUNT(v[u].z);
          WX_RS_COUNT(v[u].w);
        }
        continue;
      }
#pragma unroll
      for (int u = 0; u < WX_RS_HUNROLL; ++u) {
        const wx_i64 i = base + (wx_i64)u * WX_RS_HBLOCK + threadIdx.x;
        if (i < nq) v[u] = wx::ldv(q + i);
      }
#pragma unroll
      for (int u = 0; u < WX_RS_HUNROLL; ++u) {
        if (base + (wx_i64)u * WX_RS_HBLOCK + threadIdx.x < nq) {
          WX_RS_COUNT(v[u].x);
          WX_RS_COUNT(v[u].y);
          WX_RS_COUNT(v[u].z);
          WX_RS_COUNT(v[u].w);
        }
      }
    }
    if (blockIdx.x == 0 && threadIdx.x < (a.n & 3)) WX_RS_COUNT(a.src[nq * 4 + threadIdx.x]);
  } else {
    for (wx_i64 i = (wx_i64)blockIdx.x * WX_RS_HBLOCK + threadIdx.x; i < a.n; i += (wx_i64)gridDim.x * WX_RS_HBLOCK)
      WX_RS_COUNT(wx::ldv(a.src + i));
  }
  if (__builtin_amdgcn_ballot_w64(wx_sp != 0u) != 0ull && lane == 0) atomicOr(a.hist + 2048, 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < 4 * 256; i += WX_RS_HBLOCK) {
    wx_u32 c = 0u;
    // rotated so that the 32 lanes of an LDS cycle read 32 banks
#pragma unroll
    for (int j = 0; j < WX_RS_HC; ++j) c += h[i * WX_RS_HC + ((j + i) & (WX_RS_HC - 1))];
    if (c) atomicAdd(&a.hist[i], c);
  }
}
extern "C" __global__ __launch_bounds__(WX_RS_HBLOCK) void wx_radix_hist_f_a(WxRadixHistArgs a) { wx_radix_hist_impl<0, true>(a); }
extern "C" __global__ __launch_bounds__(WX_RS_HBLOCK) void wx_radix_hist_f_d(WxRadixHistArgs a) { wx_radix_hist_impl<0, false>(a); }
extern "C" __global__ __launch_bounds__(WX_RS_HBLOCK) void wx_radix_hist_i_a(WxRadixHistArgs a) { wx_radix_hist_impl<1, true>(a); }
extern "C" __global__ __launch_bounds__(WX_RS_HBLOCK) void wx_radix_hist_i_d(WxRadixHistArgs a) { wx_radix_hist_impl<1, false>(a); }

// (Skip words -- a tile still walking back publishing the span it has summed
// so a successor jumps it in one read -- measured slower, 15.5 vs 13.9 ms per
// 1e9 keys, profiles/r02/abl_sort_skip.txt; removed in round 5.)
#ifndef WX_RS_DIAG_LBSTATS
// diagnostic: digit 0's look-back of every tile counts its rounds, sleeps and
// the predecessors it walked (ctl words 16 + 8 * pass, a 256-B control
// block); the last tile to finish prints the pass totals
#define WX_RS_DIAG_LBSTATS 0
#endif
#ifndef WX_RS_DIAG_NO_LOOKBACK
#define WX_RS_DIAG_NO_LOOKBACK 0  // diagnostic: every tile takes its offset as 0 (results invalid)
#endif
#ifndef WX_RS_RANK_LEAD
#define WX_RS_RANK_LEAD 1  // lane 0's digit group ranked by one ballot, without LDS
#endif
#ifndef WX_RS_DIAG_NO_RANK
#define WX_RS_DIAG_NO_RANK 0  // diagnostic: no in-wave ranking, keys keep their slots (results invalid)
#endif
#ifndef WX_RS_DIAG_NO_STORE
#define WX_RS_DIAG_NO_STORE 0  // diagnostic: keys are read out of LDS but not written (results invalid)
#endif
#ifndef WX_RS_RANK_BASE
#define WX_RS_RANK_BASE 1  // counts by plain LDS read + lowest-lane store (no returning atomic, no broadcast)
#endif
#ifndef WX_RS_MATCH_LDS
// Digit peers of a key by one ds_or_b64 of the lane's bit into a per-digit
// LDS mask (then read back and cleared): 3 LDS operations per key instead of
// eight ballots and ~70 VALU instructions.  0 selects the ballot form.
#define WX_RS_MATCH_LDS 1
#endif

// The peer masks live in the tile's key buffer, which is free until the
// keys are permuted into it: WX_RS_RANK_G interleaved items per round, each
// with its own [wave][digit] mask array.
#ifndef WX_RS_RANK_G
#define WX_RS_RANK_G (WX_RS_ITEMS % 2 == 0 && 2 * WX_RS_WAVES * 256 * 8 <= WX_RS_TILE * 4 ? 2 : 1)
#endif
static_assert(WX_RS_ITEMS % WX_RS_RANK_G == 0, "items per lane must be a multiple of the rank group");
// u64 words of the key buffer (tiny tuning tiles grow it to hold the masks)
#define WX_RS_SBUF (WX_RS_TILE / 2 > WX_RS_RANK_G * WX_RS_WAVES * 256 ? WX_RS_TILE / 2 : WX_RS_RANK_G * WX_RS_WAVES * 256)

struct WxRsShared {
  wx_u32 wc[WX_RS_WAVES][256];  // per-wave digit counts, then their exclusive prefix over the waves
  wx_u32 gb[256];  // output slot of digit d's first key minus its tile-local offset
  wx_u32 ld[256];  // tile-local exclusive prefix of the digit counts
  wx_u32 wsum[4];
  wx_u32 tk[2];  // tile ticket
};

template <bool PAY>
__device__ __forceinline__ void wx_rs_load(const WxRadixPassArgs &a, wx_i64 wb, bool whole, wx_u32 (&x)[WX_RS_ITEMS],
                                           wx_u32 (&v)[WX_RS_ITEMS]) {
  if (whole) {  // tile-uniform: unguarded loads
#pragma unroll
    for (int i = 0; i < WX_RS_ITEMS; ++i) {
      x[i] = wx::ldv(a.src_k + wb + (wx_i64)i * 64);
      if (PAY) v[i] = wx::ldv(a.src_v + wb + (wx_i64)i * 64);
    }
  } else {
#pragma unroll
    for (int i = 0; i < WX_RS_ITEMS; ++i) {
      const wx_i64 e = wb + (wx_i64)i * 64;
      x[i] = e < a.n ? wx::ldv(a.src_k + e) : 0u;
      if (PAY) v[i] = e < a.n ? wx::ldv(a.src_v + e) : 0u;
    }
  }
}

// The digit's tile-local base is folded into the per-wave counts once per
// tile (2 048 adds), so the permutation reads one LDS word per key, not two:
// 12.6 vs 12.8 ms per 1e9 float keys with the atomic ranking, 13.45 vs 13.75
// without (abl_sort_fold.txt).
#ifndef WX_RS_RANK_ATOMIC
// Rank by one returning LDS add per key (ds_add_rtn_u32 on the wave's digit
// counter): the LDS serialises the lanes of one instruction that hit the
// same counter in ascending lane order, so the returned counts are the
// stable in-wave ranks; the adds of item i + 1 follow item i's (one wave's
// LDS operations execute in order), so all items' adds issue back to back
// with one wait.  Lane 0's digit group (a few-valued digit -- the exponent
// byte -- sends most of a wave to one counter) adds its size once from lane
// 0 and ranks by its ballot.  0 selects the peer-mask form below.  With
// WX_RS_FOLD_LD: 12.6 vs 13.8 ms per 1e9 float keys, 17.9 vs 19.1 per 1e9
// int + payload pairs; ordered, stable, every payload on its key for
// full-range, 2^16-valued and 4-valued keys (profiles/r03/abl_sort_fold.txt,
// abl_sort_rank_atomic.txt; the sort GPU tests, pytest_sort_r3.log).
#define WX_RS_RANK_ATOMIC 1
#endif

// In-wave stable rank of each key among the wave's keys with the same digit:
// the group's lowest lane bumps the wave's count and broadcasts the old one.
template <int KIND, bool ASC, bool WHOLE>
__device__ __forceinline__ void wx_rs_rank(const WxRadixPassArgs &a, WxRsShared &S, wx_u64 *peers, wx_i64 wb,
                                           const wx_u32 (&x)[WX_RS_ITEMS], wx_u32 (&rk)[WX_RS_ITEMS]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const wx_u64 below = (1ull << lane) - 1ull;
#if WX_RS_RANK_ATOMIC
  (void)peers;
  if (!a.lead) {
    // no skewed digit in this pass (the host read the histogram): one
    // returning LDS add per key, nothing else
#pragma unroll
    for (int i = 0; i < WX_RS_ITEMS; ++i) {
      const wx_u32 d = (wx_rs_key_t<KIND, ASC>(x[i]) >> a.shift) & 255u;
      rk[i] = 0u;
      if (WHOLE || wb + (wx_i64)i * 64 < a.n) rk[i] = atomicAdd(&S.wc[wave][d], 1u);
    }
    return;
  }
  wx_u32 lead_bits = 0u;  // bit i: this lane is in lane 0's digit group of item i (and not lane 0)
#pragma unroll
  for (int i = 0; i < WX_RS_ITEMS; ++i) {
    const bool valid = WHOLE || wb + (wx_i64)i * 64 < a.n;
    const wx_u32 d = (wx_rs_key_t<KIND, ASC>(x[i]) >> a.shift) & 255u;
    const wx_u32 d0 = __builtin_amdgcn_readfirstlane(d);
    const bool lead = valid && d == d0;
    const wx_u64 lm = __builtin_amdgcn_ballot_w64(lead);
    rk[i] = (wx_u32)__builtin_popcountll(lm & below);
    if (valid && (!lead || lane == 0))
      rk[i] = atomicAdd(&S.wc[wave][d], lead ? (wx_u32)__builtin_popcountll(lm) : 1u);
    lead_bits |= (lead && lane != 0 ? 1u : 0u) << i;
  }
#pragma unroll
  for (int i = 0; i < WX_RS_ITEMS; ++i) {
    const wx_u32 base0 = __builtin_amdgcn_readlane(rk[i], 0);  // lane 0's returned count
    if ((lead_bits >> i) & 1u) rk[i] += base0;
  }
  return;
#endif
  constexpr int G = WX_RS_RANK_G;
#pragma unroll
  for (int i = 0; i < WX_RS_ITEMS; i += G) {
    if (WX_RS_DIAG_NO_RANK) {
#pragma unroll
      for (int g = 0; g < G; ++g) rk[i + g] = 0u;
      continue;
    }
    bool valid[G];
    wx_u32 d[G];
    wx_u64 m[G];
    wx_u64 *w[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      valid[g] = WHOLE || wb + (wx_i64)(i + g) * 64 < a.n;
      d[g] = (wx_rs_key_t<KIND, ASC>(x[i + g]) >> a.shift) & 255u;
      w[g] = peers + ((g * WX_RS_WAVES + wave) * 256 + d[g]);
    }
#if WX_RS_MATCH_LDS
    // the G items' ORs, then their read-backs, then their clears: one wait
    // for the group where one item at a time waited for each.  With
    // WX_RS_RANK_LEAD the lanes sharing lane 0's digit take their mask from
    // one ballot and stay off LDS: a few-valued digit (the exponent byte)
    // would otherwise send most of the wave's ORs to one word, serialized.
    bool lds[G];
    wx_u32 d0[G];  // lane 0's digit of item g (wave-uniform)
    wx_u64 lm[G];  // the lanes sharing it
#pragma unroll
    for (int g = 0; g < G; ++g) {
      lds[g] = valid[g];
      d0[g] = 0u;
      lm[g] = 0ull;
      if (WX_RS_RANK_LEAD) {
        d0[g] = __builtin_amdgcn_readfirstlane(d[g]);  // lane 0 (valid if any lane is)
        const bool lead = valid[g] && d[g] == d0[g];
        lm[g] = __builtin_amdgcn_ballot_w64(lead);
        m[g] = lm[g];
        lds[g] = valid[g] && !lead;
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (lds[g]) atomicOr(w[g], 1ull << lane);
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (lds[g]) m[g] = __hip_atomic_load(w[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      else if (!valid[g]) m[g] = 0ull;
#if WX_RS_RANK_BASE
    // Counts without a returning atomic: every key reads its digit's running
    // count (base) together with its peer mask, and the group's lowest lane
    // stores base + group size back.  One dependent LDS round trip per round
    // instead of three (mask read -> leader's atomic add -> broadcast).  Item
    // g > 0 also counts the earlier items' keys of its digit in this round:
    // their mask words are still set (cleared below), and the lanes of lane
    // 0's digit group, which stayed off LDS, are known from the ballot.
    wx_u32 base[G], before[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      base[g] = 0u;
      before[g] = 0u;
      if (valid[g]) {
        base[g] = __hip_atomic_load(&S.wc[wave][d[g]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
#pragma unroll
        for (int h = 0; h < g; ++h) {
          const wx_u64 mh = __hip_atomic_load(peers + ((h * WX_RS_WAVES + wave) * 256 + d[g]), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WAVEFRONT);
          before[g] += (wx_u32)__builtin_popcountll(mh) +
                       ((WX_RS_RANK_LEAD && d[g] == d0[h]) ? (wx_u32)__builtin_popcountll(lm[h]) : 0u);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int g = 0; g < G; ++g) {
      rk[i + g] = 0u;
      if (valid[g]) {
        const wx_u32 b = base[g] + before[g];
        rk[i + g] = b + (wx_u32)__builtin_popcountll(m[g] & below);
        if ((m[g] & below) == 0ull)  // the group's lowest lane; item g's store follows item g - 1's
          __hip_atomic_store(&S.wc[wave][d[g]], b + (wx_u32)__builtin_popcountll(m[g]), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WAVEFRONT);
      }
    }
#endif
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (lds[g]) __hip_atomic_store(w[g], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
#if WX_RS_RANK_BASE
    __builtin_amdgcn_wave_barrier();
    continue;
#endif
#else
#pragma unroll
    for (int g = 0; g < G; ++g) {
      m[g] = __builtin_amdgcn_ballot_w64(valid[g]);
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const bool bit = (d[g] >> b) & 1u;
        const wx_u64 bb = __builtin_amdgcn_ballot_w64(bit);
        m[g] &= bit ? bb : ~bb;
      }
    }
#endif
    // item i's count update is issued before item i + 1's: equal digits of
    // later keys rank after earlier ones (LDS executes a wave's operations in order)
    int leader[G];
    wx_u32 old[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      leader[g] = valid[g] ? __builtin_ctzll(m[g]) : lane;
      old[g] = 0u;
      if (valid[g] && lane == leader[g]) old[g] = atomicAdd(&S.wc[wave][d[g]], (wx_u32)__builtin_popcountll(m[g]));
    }
#pragma unroll
    for (int g = 0; g < G; ++g) rk[i + g] = __shfl(old[g], leader[g]) + (wx_u32)__builtin_popcountll(m[g] & below);
    __builtin_amdgcn_wave_barrier();
  }
}

// (Round 5: the walk spread over 2 or 4 lanes per digit -- lane q loading
// the q-th group of WX_RS_LBW words, the parts combined in order by DPP
// broadcasts -- was correct and slower, 11.77 vs 11.23 ms per 1e9 float keys
// at 1024 x 32 and 19.14 vs 18.58 per 1e9 pairs, profiles/r05/
// ab_sort_lb_lanes.txt: one lane per digit walks.)

// Exclusive prefix of digit d over the tiles before `tile`: a walk back
// from tile - 1 summing {A} / {P} words to the first {P}, WX_RS_LBW words
// per round (`first`: the first round, loaded earlier).
__device__ __forceinline__ wx_u64 wx_rs_walk(const WxRadixPassArgs &a, wx_u32 tile, int d,
                                             const wx_u64 (&first)[WX_RS_LBW]) {
  const wx_u64 E = (wx_u64)a.epoch << 58;
  wx_i64 p = (wx_i64)tile - 1;  // the nearest predecessor not yet summed
  wx_u64 excl = 0;
  wx_u32 spins = 0;
  wx_u64 t_last = 0ull;  // time of the last progress (0: not yet sampled)
  bool fresh = true;
#if WX_RS_DIAG_LBSTATS
  wx_u32 lb_rounds = 0, lb_sleeps = 0;
#endif
  while (true) {
    wx_u64 wv[WX_RS_LBW];
#pragma unroll
    for (int j = 0; j < WX_RS_LBW; ++j)
      wv[j] = fresh ? first[j] : p - j >= 0 ? wx::ld_agent(&a.status[(wx_u64)(p - j) * 256 + d]) : (E | WX_RS_FLAG_P);
    fresh = false;
    int stop = WX_RS_LBW;  // index of the first unpublished word
    bool done = false;
#pragma unroll
    for (int j = 0; j < WX_RS_LBW; ++j) {
      if (stop == WX_RS_LBW && !done) {
        const wx_u64 flag = (wv[j] >> 56) & 3ull;
        if ((wv[j] >> 58) != (wx_u64)a.epoch || flag == 0ull) {
          stop = j;
        } else {
          excl += wv[j] & WX_RS_VAL_MASK;
          done = flag == 2ull;
        }
      }
    }
#if WX_RS_DIAG_LBSTATS
    ++lb_rounds;
#endif
    if (done) break;
    if (stop == WX_RS_LBW) {
      p -= WX_RS_LBW;
      t_last = 0ull;  // progress
      spins = 0;
      continue;
    }
    if (stop > 0) t_last = 0ull, spins = 0;
    p -= stop;
#if WX_RS_DIAG_LBSTATS
    ++lb_sleeps;
#endif
    if (WX_RS_SLEEP) __builtin_amdgcn_s_sleep(WX_RS_SLEEP);
    if ((++spins & 63u) == 0u) {
      // abort only after WX_STALL_TICKS and WX_STALL_SPINS with this digit's chain not moving
      const wx_u64 now = __builtin_amdgcn_s_memrealtime();
      if (t_last == 0ull) {
        t_last = now;
      } else if (now - t_last > WX_STALL_TICKS && spins >= WX_STALL_SPINS) {
        wx_u64 seen = 0ull;  // the unpublished predecessor p's word
#pragma unroll
        for (int j = 0; j < WX_RS_LBW; ++j)
          if (j == stop) seen = wv[j];
        wx::lb_report(a.lbd, WX_LBD_RADIX | ((wx_u64)a.epoch << 8) | ((wx_u64)d << 16) | ((wx_u64)(a.shift / 8) << 32),
                      (wx_u64)tile, (wx_u64)p, seen);
        atomicOr(a.err, WX_DEVERR_LOOKBACK);
        atomicExch(&a.ctl[1], 1u);
      }
      if (__hip_atomic_load(&a.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    }
  }
#if WX_RS_DIAG_LBSTATS
  if (threadIdx.x == 0) {
    wx_u32 *st = a.ctl + 16 + 6 * (a.shift / 8);  // = control word 16 + 8 * pass
    atomicAdd(&st[0], lb_rounds);
    atomicAdd(&st[1], lb_sleeps);
    atomicAdd(&st[2], (wx_u32)((wx_i64)tile - 1 - p));
    __threadfence();
    if (atomicAdd(&st[3], 1u) == (wx_u32)((a.n + WX_RS_TILE - 1) / WX_RS_TILE) - 2u)
      printf("[lbstats] pass %d tiles %u rounds %u sleeps %u walked %u\n", a.shift / 8, atomicAdd(&st[3], 0u) + 1u,
             atomicAdd(&st[0], 0u), atomicAdd(&st[1], 0u), atomicAdd(&st[2], 0u));
  }
#endif
  return excl;
}

// The first round of digit d's walk, issued early so the loads fly across
// a barrier.
__device__ __forceinline__ void wx_rs_walk_first(const WxRadixPassArgs &a, wx_u32 tile, int d,
                                                 wx_u64 (&first)[WX_RS_LBW]) {
  const wx_u64 E = (wx_u64)a.epoch << 58;
#pragma unroll
  for (int j = 0; j < WX_RS_LBW; ++j) {
    const wx_i64 t = (wx_i64)tile - 1 - j;
    first[j] = t >= 0 ? wx::ld_agent(&a.status[(wx_u64)t * 256 + d]) : (E | WX_RS_FLAG_P);
  }
}

// The keys (and payloads) are permuted into LDS by their tile-local slots,
// which need only this tile's counts, before the look-back resolves the
// tile's global offsets: the permutation overlaps the look-back's first
// poll instead of waiting behind the whole look-back.  Key + payload tiles
// since round 2 (19.8 vs 21.8 ms per 1e9 pairs); keys since round 5, with the
// 1024 x 32 tile and plain stores: 8.67 ms per 1e9 float keys against 9.30
// with nontemporal stores, 9.81 unsplit and 10.08 unsplit with nontemporal
// stores (round 4's form), one process (profiles/r05/ab_sort_split_store.txt;
// round 2 at 512 x 32 had measured the split slower for keys, 15.4 vs 14.9).
// The unsplit form and the nontemporal stores were removed in round 5.
// Split form, part 1 (every thread; holds a barrier): threads 0..255 own
// digit tid, publish its count {A} (or {P} for tile 0), then the exclusive
// prefix over the waves (S.wc) and over the digits (S.ld).  Returns the
// tile's count of digit tid.
__device__ __forceinline__ wx_u32 wx_rs_local(const WxRadixPassArgs &a, WxRsShared &S, wx_u32 tile) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const wx_u64 E = (wx_u64)a.epoch << 58;
  const bool look = tile != 0 && !WX_RS_DIAG_NO_LOOKBACK;
  wx_u32 tot = 0u, inc = 0u;
  if (tid < 256) {
#pragma unroll
    for (int w = 0; w < WX_RS_WAVES; ++w) {
      const wx_u32 c = S.wc[w][tid];
      S.wc[w][tid] = tot;
      tot += c;
    }
    wx::st_agent(&a.status[(wx_u64)tile * 256 + tid], E | (look ? WX_RS_FLAG_A : WX_RS_FLAG_P) | tot);
    inc = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const wx_u32 t = __shfl_up(inc, o);
      if (lane >= o) inc += t;
    }
    if (lane == 63) S.wsum[wave] = inc;
  }
  __syncthreads();
  if (tid < 256) {
    wx_u32 ld = inc - tot;
    for (int w = 0; w < wave; ++w) ld += S.wsum[w];
    S.ld[tid] = ld;
#pragma unroll
    for (int w = 0; w < WX_RS_WAVES; ++w) S.wc[w][tid] += ld;
  }
  return tot;
}

// Split form, part 2 (threads 0..255): walk back for digit tid (`first`:
// the walk's first round, loaded earlier), publish {P}, set S.gb.
__device__ __forceinline__ void wx_rs_resolve(const WxRadixPassArgs &a, WxRsShared &S, wx_u32 tile, wx_u32 tot,
                                              const wx_u64 (&first)[WX_RS_LBW]) {
  const int tid = threadIdx.x;
  const wx_u64 E = (wx_u64)a.epoch << 58;
  const bool look = tile != 0 && !WX_RS_DIAG_NO_LOOKBACK;
  const wx_u64 excl = look ? wx_rs_walk(a, tile, tid, first) : 0ull;
  if (look) wx::st_agent(&a.status[(wx_u64)tile * 256 + tid], E | WX_RS_FLAG_P | (excl + tot));
  S.gb[tid] = a.digit_base[tid] + (wx_u32)excl - S.ld[tid];
}

// Keys into digit order in LDS; pos[i] keeps each key's tile-local slot
// (the payload follows through the same slots).
template <int KIND, bool ASC, bool WHOLE>
__device__ __forceinline__ void wx_rs_scatter(const WxRadixPassArgs &a, WxRsShared &S, wx_i64 wb,
                                              const wx_u32 (&x)[WX_RS_ITEMS], const wx_u32 (&rk)[WX_RS_ITEMS],
                                              wx_u32 (&pos)[WX_RS_ITEMS], wx_u32 *s_k) {
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < WX_RS_ITEMS; ++i) {
    wx_u32 p = 0u;
    if (WHOLE || wb + (wx_i64)i * 64 < a.n) {
      const wx_u32 d = (wx_rs_key_t<KIND, ASC>(x[i]) >> a.shift) & 255u;
      p = S.wc[wave][d] + rk[i];
      if (WX_RS_DIAG_NO_RANK) p = (wx_u32)(wave * 64 * WX_RS_ITEMS + i * 64 + (threadIdx.x & 63));
      s_k[p] = x[i];
    }
    pos[i] = p;
  }
}

// LDS -> output: consecutive lanes write consecutive slots of a digit's run;
// gdst[j] keeps the destination of slot j * WX_RS_BLOCK + tid for the payload.
template <int KIND, bool ASC, bool WHOLE>
__device__ __forceinline__ void wx_rs_store(const WxRadixPassArgs &a, const WxRsShared &S, int tile_n,
                                            const wx_u32 *s_k, wx_u32 (&gdst)[WX_RS_ITEMS]) {
#pragma unroll
  for (int j = 0; j < WX_RS_ITEMS; ++j) {
    const int pos = j * WX_RS_BLOCK + threadIdx.x;
    gdst[j] = 0u;
    if (WHOLE || pos < tile_n) {
      const wx_u32 xk = s_k[pos];
      const wx_u32 d = (wx_rs_key_t<KIND, ASC>(xk) >> a.shift) & 255u;
      wx_u32 g = S.gb[d] + (wx_u32)pos;
      if (WX_RS_DIAG_NO_LOOKBACK || WX_RS_DIAG_NO_RANK) g = (wx_u32)min((wx_i64)g, a.n - 1);
      if (WX_RS_DIAG_NO_STORE)
        asm volatile("" ::"v"(g), "v"(xk));  // keep the LDS read and the address math
      else
        a.dst_k[g] = xk;  // plain stores: L2 merges the digit runs' partial lines
      gdst[j] = g;
    }
  }
}

// The payload follows its key: the same LDS slots, the same destinations.
template <bool WHOLE>
__device__ __forceinline__ void wx_rs_payload(const WxRadixPassArgs &a, int tile_n, wx_i64 wb,
                                              const wx_u32 (&v)[WX_RS_ITEMS], const wx_u32 (&pos)[WX_RS_ITEMS],
                                              const wx_u32 (&gdst)[WX_RS_ITEMS], wx_u32 *s_k) {
  __syncthreads();  // every key read out of s_k
#pragma unroll
  for (int i = 0; i < WX_RS_ITEMS; ++i)
    if (WHOLE || wb + (wx_i64)i * 64 < a.n) s_k[pos[i]] = v[i];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < WX_RS_ITEMS; ++j) {
    const int p = j * WX_RS_BLOCK + threadIdx.x;
    if (WHOLE || p < tile_n) a.dst_v[gdst[j]] = s_k[p];
  }
}

// One tile per workgroup, several workgroups per CU hiding each other's
// latencies.  (A persistent variant that loaded the next tile during this
// one's look-back needed 161 VGPRs, ran one workgroup per CU and took 33 ms
// per 1e9 keys against 20.7 ms here: profiles/r01/bench_sort_variants.txt.)
#ifndef WX_RS_DIAG_PHASES
// diagnostic: thread 0 stamps s_memrealtime (10 ns) at the phase boundaries
// of every tile -- entry, ticket, keys landed (an extra vmcnt(0) wait), ranked,
// offsets resolved (look-back), permuted, stores issued, stores done (an extra
// wait) -- summed per pass over the tiles in control words 64.. (u64); the
// last tile of a pass prints the per-tile averages
#define WX_RS_DIAG_PHASES 0
#endif
#if WX_RS_DIAG_PHASES
#define WX_RS_TS_ARG , ts
#define WX_RS_TS_PARAM , wx_u64 (&ts)[8]
#define WX_RS_STAMP(i) \
  do {                   \
    if (threadIdx.x == 0) ts[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define WX_RS_VMWAIT() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#else
#define WX_RS_TS_ARG
#define WX_RS_TS_PARAM
#define WX_RS_STAMP(i) \
  do {                   \
  } while (0)
#define WX_RS_VMWAIT() \
  do {                   \
  } while (0)
#endif

template <bool PAY, int KIND, bool ASC, bool WHOLE>
__device__ __forceinline__ void wx_radix_tile_body(const WxRadixPassArgs &a, WxRsShared &S, wx_u32 *s_k,
                                                   wx_u64 *peers, wx_u32 tile, wx_i64 tb WX_RS_TS_PARAM);

template <bool PAY, int KIND, bool ASC>
__device__ __forceinline__ void wx_radix_tile_impl(const WxRadixPassArgs &a, WxRsShared &S, wx_u32 *s_k) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#if WX_RS_DIAG_PHASES
  wx_u64 ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  WX_RS_STAMP(0);
  if (tid == 0) S.tk[0] = atomicAdd(&a.ctl[0], 1u);
  wx_u64 *peers = reinterpret_cast<wx_u64 *>(s_k);
  for (int i = tid; i < WX_RS_WAVES * 256; i += WX_RS_BLOCK) (&S.wc[0][0])[i] = 0u;
  if (WX_RS_MATCH_LDS && !WX_RS_RANK_ATOMIC)
    for (int i = tid; i < WX_RS_RANK_G * WX_RS_WAVES * 256; i += WX_RS_BLOCK) peers[i] = 0ull;
  __syncthreads();
  const wx_u32 tile = S.tk[0];
  const wx_i64 tb = (wx_i64)tile * WX_RS_TILE;
  WX_RS_STAMP(1);
  // every tile but the last is whole: its copy of the body checks no bounds
  if (tb + WX_RS_TILE <= a.n)
    wx_radix_tile_body<PAY, KIND, ASC, true>(a, S, s_k, peers, tile, tb WX_RS_TS_ARG);
  else
    wx_radix_tile_body<PAY, KIND, ASC, false>(a, S, s_k, peers, tile, tb WX_RS_TS_ARG);
}

template <bool PAY, int KIND, bool ASC, bool WHOLE>
__device__ __forceinline__ void wx_radix_tile_body(const WxRadixPassArgs &a, WxRsShared &S, wx_u32 *s_k,
                                                   wx_u64 *peers, wx_u32 tile, wx_i64 tb WX_RS_TS_PARAM) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const wx_i64 wb = tb + (wx_i64)wave * 64 * WX_RS_ITEMS + lane;
  const int tile_n = WHOLE ? WX_RS_TILE : (int)(a.n - tb);
  wx_u32 x[WX_RS_ITEMS], v[WX_RS_ITEMS], rk[WX_RS_ITEMS], pos[WX_RS_ITEMS], gdst[WX_RS_ITEMS];
  wx_rs_load<PAY>(a, wb, WHOLE, x, v);
  WX_RS_VMWAIT();
  WX_RS_STAMP(2);
  wx_rs_rank<KIND, ASC, WHOLE>(a, S, peers, wb, x, rk);
  __syncthreads();
  WX_RS_STAMP(3);
  const wx_u32 tot = wx_rs_local(a, S, tile);
  __syncthreads();  // S.ld
  wx_u64 first[WX_RS_LBW];
  if (tid < 256 && tile != 0 && !WX_RS_DIAG_NO_LOOKBACK)  // in flight during the permutation
    wx_rs_walk_first(a, tile, tid, first);
  WX_RS_STAMP(4);
  wx_rs_scatter<KIND, ASC, WHOLE>(a, S, wb, x, rk, pos, s_k);
  if (tid < 256) wx_rs_resolve(a, S, tile, tot, first);
  __syncthreads();
  WX_RS_STAMP(5);
  wx_rs_store<KIND, ASC, WHOLE>(a, S, tile_n, s_k, gdst);
  if (PAY) wx_rs_payload<WHOLE>(a, tile_n, wb, v, pos, gdst, s_k);
  WX_RS_STAMP(6);
  WX_RS_VMWAIT();
  WX_RS_STAMP(7);
#if WX_RS_DIAG_PHASES
  if (tid == 0) {
    unsigned long long *st = reinterpret_cast<unsigned long long *>(a.ctl - 2 * (a.shift / 8) + 64) + 8 * (a.shift / 8);
    for (int i = 0; i < 7; ++i) atomicAdd(&st[i], (unsigned long long)(ts[i + 1] - ts[i]));
    __threadfence();
    const wx_u32 nt = (wx_u32)((a.n + WX_RS_TILE - 1) / WX_RS_TILE);
    if (atomicAdd(reinterpret_cast<unsigned int *>(&st[7]), 1u) == nt - 1u) {
      __threadfence();
      printf("[rsphase] pass %d tiles %u per-tile us: ticket %.3f load %.3f rank %.3f digits+lookback %.3f "
             "scatter %.3f store-issue %.3f store-drain %.3f\n",
             a.shift / 8, nt, atomicAdd(&st[0], 0ull) * 0.01 / nt, atomicAdd(&st[1], 0ull) * 0.01 / nt,
             atomicAdd(&st[2], 0ull) * 0.01 / nt, atomicAdd(&st[3], 0ull) * 0.01 / nt,
             atomicAdd(&st[4], 0ull) * 0.01 / nt, atomicAdd(&st[5], 0ull) * 0.01 / nt,
             atomicAdd(&st[6], 0ull) * 0.01 / nt);
    }
  }
#endif
}

#ifndef WX_RS_MINW
// minimum waves per SIMD the register allocation must allow: 2 workgroups
// per CU for the 512-thread key tiles (<= 128 VGPRs), 1 for 1024 threads
#define WX_RS_MINW (WX_RS_BLOCK <= 512 ? 2 * WX_RS_BLOCK / 256 : WX_RS_BLOCK / 256)
#endif
#define WX_RS_TILEK(NAME, PAY, KIND, ASC)                                                        \
  extern "C" __global__ __launch_bounds__(WX_RS_BLOCK, WX_RS_MINW) void NAME(WxRadixPassArgs a) { \
    __shared__ WxRsShared S;                                                            \
    __shared__ wx_u64 s_raw[WX_RS_SBUF]; /* keys / payloads; the peer masks before */ \
    wx_radix_tile_impl<PAY, KIND, ASC>(a, S, reinterpret_cast<wx_u32 *>(s_raw));        \
  }
WX_RS_TILEK(wx_radix_tile_k_f_a, false, 0, true)
WX_RS_TILEK(wx_radix_tile_k_f_d, false, 0, false)
WX_RS_TILEK(wx_radix_tile_k_i_a, false, 1, true)
WX_RS_TILEK(wx_radix_tile_k_i_d, false, 1, false)
WX_RS_TILEK(wx_radix_tile_kv_f_a, true, 0, true)
WX_RS_TILEK(wx_radix_tile_kv_f_d, true, 0, false)
WX_RS_TILEK(wx_radix_tile_kv_i_a, true, 1, true)
WX_RS_TILEK(wx_radix_tile_kv_i_d, true, 1, false)
WX_RS_TILEK(wx_radix_tile_k_fp_a, false, 2, true)
WX_RS_TILEK(wx_radix_tile_k_fp_d, false, 2, false)
WX_RS_TILEK(wx_radix_tile_kv_fp_a, true, 2, true)
WX_RS_TILEK(wx_radix_tile_kv_fp_d, true, 2, false)
#endif
