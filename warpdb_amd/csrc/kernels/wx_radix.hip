// wx_radix.hip -- the three-pass LSD radix sort behind jit_sort_float /
// jit_sort_pairs / ORDER BY (reference: a one-thread bubble sort,
// src/jit.cpp:248-307; strict compares, so stable).  Appended to the util
// module's source after wx_template.hip (it uses wx::ldv and the order maps
// wx_rs_key_t of that file).
//
// Digits: bits [0, 11), [11, 22), [22, 32) of the 32-bit order key (floats:
// the order map with -0.0 == +0.0 and NaN last; ints: sign flip; descending:
// the complement), so one sort is three stable passes, not four.
//
// Reduce-then-scan, no look-back: the keys are cut into R static ranges of
// whole 16 384-key tiles (R = the CU count), one persistent 1024-thread
// workgroup per range.  Per pass:
//   count   (wx_rx_count_*)  each range's 2048-bin histogram of the pass's
//                            digit (the first executed pass takes its counts
//                            from the histogram kernel, wx_rx_hist_*, which
//                            counts all three digits per range in one read);
//   offsets (wx_rx_scan)     off[r][d] = the digit's base + its count in the
//                            ranges before r;
//   scatter (wx_rx_pass_*)   the range's tiles in order: stable in-wave ranks
//                            by one returning LDS add per key, the tile's
//                            digit prefix, the keys permuted into digit order
//                            in LDS and written at off[r][d] + their place,
//                            while the next tile's keys are in flight.
// A workgroup writes digit d of its range as one contiguous run, tile after
// tile, so consecutive tiles complete each other's partial lines in the XCD's
// L2 (plain stores); nothing waits on another workgroup, so no spin, ticket
// or status word exists and a pass cannot stall on a workgroup that is not
// resident.  Traffic per key: 4 B (histogram) + 3 x 8 B (scatter) + 2 x 4 B
// (count) = 36 B; pairs add 8 B per scatter.
#if WX_OP == WX_OP_UTIL

#define WX_RX_BLOCK WX_RX_BLOCK_THREADS  // 1024 (wx_args.h, shared with the host)
#define WX_RX_WAVES (WX_RX_BLOCK / 64)
#define WX_RX_ITEMS (WX_RX_TILE_KEYS / WX_RX_BLOCK)  // 16
#define WX_RX_TILE WX_RX_TILE_KEYS  // 16 384 keys
#define WX_RX_BINS 2048
#ifndef WX_RX_NT_STORE
#define WX_RX_NT_STORE 0  // plain stores: consecutive tiles' runs merge in L2
#endif
#ifndef WX_RX_HC3
#define WX_RX_HC3 4  // histogram kernel: LDS copies of each of the 3 x 2048 counters (96 KB)
#endif
#ifndef WX_RX_HC1
#define WX_RX_HC1 8  // count kernel: copies of the 2048 counters (64 KB)
#endif
#ifndef WX_RX_HUNROLL
#define WX_RX_HUNROLL 4  // 16-byte loads in flight per thread in the counting kernels
#endif

__device__ __forceinline__ wx_u32 wx_rx_digit_of(wx_u32 k, int p) {
  return (k >> (11 * p)) & (p == 2 ? 1023u : 2047u);
}

// Range r of R: tiles [r * T / R, (r + 1) * T / R).
__device__ __forceinline__ void wx_rx_range(wx_i64 n, int ranges, int r, wx_i64 &t0, wx_i64 &t1) {
  const wx_i64 T = (n + WX_RX_TILE - 1) / WX_RX_TILE;
  t0 = (wx_i64)r * T / ranges;
  t1 = (wx_i64)(r + 1) * T / ranges;
}

// One key into the LDS counters h[bin][HC] of NP digits (NP = 3: all, at
// bins q * 2048 + d; NP = 1: digit `pass`).  A wave whose lanes share a
// digit adds once (a constant digit -- small int keys -- would otherwise put
// the whole wave on one address); other lanes add to copy lane % HC.
// Returns 1 for a float the plain order flip would misplace (NaN, -0.0).
template <int KIND, bool ASC, int NP, int HC>
__device__ __forceinline__ wx_u32 wx_rx_count_key(wx_u32 *h, wx_u32 x, int pass, int lane, int copy) {
  const wx_u32 k = wx_rs_key_t<KIND, ASC>(x);
  const wx_u64 act = __builtin_amdgcn_ballot_w64(true);
  const int first = __builtin_ctzll(act);
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int p = NP == 3 ? q : pass;
    const wx_u32 d = wx_rx_digit_of(k, p);
    const int hb = NP == 3 ? q * WX_RX_BINS : 0;
    const wx_u32 d0 = __builtin_amdgcn_readfirstlane(d);
    if (__builtin_amdgcn_ballot_w64(d != d0) == 0ull) {
      if (lane == first) atomicAdd(&h[(hb + d0) * HC], (wx_u32)__builtin_popcountll(act));
    } else {
      atomicAdd(&h[(hb + d) * HC + copy], 1u);
    }
  }
  return KIND == 0 ? (wx_u32)((x & 0x7fffffffu) > 0x7f800000u || x == 0x80000000u) : 0u;
}

// Per-range digit counts: cnt[(q * R + r) * 2048 + d].  One workgroup per
// range; contiguous 16-byte loads (WX_RX_HUNROLL per thread in flight,
// software-pipelined) when the keys are 16-byte aligned, dword loads
// otherwise.
template <int KIND, bool ASC, int NP>
__device__ __forceinline__ void wx_rx_count_impl(const WxRxCountArgs &a) {
  constexpr int HC = NP == 3 ? WX_RX_HC3 : WX_RX_HC1;
  constexpr int NB = NP * WX_RX_BINS;
  __shared__ wx_u32 h[NB * HC];
  for (int i = threadIdx.x; i < NB * HC; i += WX_RX_BLOCK) h[i] = 0u;
  __syncthreads();
  const int r = blockIdx.x, lane = threadIdx.x & 63, copy = lane % HC;
  wx_i64 t0, t1;
  wx_rx_range(a.n, a.ranges, r, t0, t1);
  const wx_i64 e0 = t0 * WX_RX_TILE, e1 = t1 * WX_RX_TILE < a.n ? t1 * WX_RX_TILE : a.n;
  wx_u32 sp = 0u;
#define WX_RX_CK(x) (sp |= wx_rx_count_key<KIND, ASC, NP, HC>(h, (x), a.pass, lane, copy))
  if (a.aligned) {
    typedef wx_u32 u4 __attribute__((ext_vector_type(4)));
    const u4 *q = reinterpret_cast<const u4 *>(a.src);
    const wx_i64 q0 = e0 >> 2, q1 = e1 >> 2;  // e0 is a multiple of the tile
    const wx_i64 span = (wx_i64)WX_RX_BLOCK * WX_RX_HUNROLL;
    wx_i64 base = q0;
    if (base + span <= q1) {  // whole spans, the next span's loads in flight while this one is counted
      u4 v[WX_RX_HUNROLL], w[WX_RX_HUNROLL];
#pragma unroll
      for (int u = 0; u < WX_RX_HUNROLL; ++u) w[u] = wx::ldv(q + base + (wx_i64)u * WX_RX_BLOCK + threadIdx.x);
      while (true) {
#pragma unroll
        for (int u = 0; u < WX_RX_HUNROLL; ++u) v[u] = w[u];
        const wx_i64 nb = base + span;
        const bool more = nb + span <= q1;  // workgroup-uniform
        if (more) {
#pragma unroll
          for (int u = 0; u < WX_RX_HUNROLL; ++u) w[u] = wx::ldv(q + nb + (wx_i64)u * WX_RX_BLOCK + threadIdx.x);
        }
#pragma unroll
        for (int u = 0; u < WX_RX_HUNROLL; ++u) {
          WX_RX_CK(v[u].x);
          WX_RX_CK(v[u].y);
          WX_RX_CK(v[u].z);
          WX_RX_CK(v[u].w);
        }
        base = nb;
        if (!more) break;
      }
    }
    for (wx_i64 i = base + threadIdx.x; i < q1; i += WX_RX_BLOCK) {
      const u4 v = wx::ldv(q + i);
      WX_RX_CK(v.x);
      WX_RX_CK(v.y);
      WX_RX_CK(v.z);
      WX_RX_CK(v.w);
    }
    if (threadIdx.x < (int)(e1 - (q1 << 2))) WX_RX_CK(wx::ldv(a.src + (q1 << 2) + threadIdx.x));
  } else {
    for (wx_i64 i = e0 + threadIdx.x; i < e1; i += WX_RX_BLOCK) WX_RX_CK(wx::ldv(a.src + i));
  }
#undef WX_RX_CK
  if (a.flag && __builtin_amdgcn_ballot_w64(sp != 0u) != 0ull && lane == 0) atomicOr(a.flag, 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < NB; i += WX_RX_BLOCK) {
    wx_u32 c = 0u;
#pragma unroll
    for (int j = 0; j < HC; ++j) c += h[i * HC + ((j + i) & (HC - 1))];  // rotated: the lanes read different banks
    const int q = i / WX_RX_BINS, d = i % WX_RX_BINS;
    a.cnt[((wx_u64)q * a.ranges + r) * WX_RX_BINS + d] = c;
  }
}
#define WX_RX_COUNTK(NAME, KIND, ASC, NP) \
  extern "C" __global__ __launch_bounds__(WX_RX_BLOCK) void NAME(WxRxCountArgs a) { wx_rx_count_impl<KIND, ASC, NP>(a); }
WX_RX_COUNTK(wx_rx_hist_f_a, 0, true, 3)
WX_RX_COUNTK(wx_rx_hist_f_d, 0, false, 3)
WX_RX_COUNTK(wx_rx_hist_i_a, 1, true, 3)
WX_RX_COUNTK(wx_rx_hist_i_d, 1, false, 3)
WX_RX_COUNTK(wx_rx_count_f_a, 0, true, 1)
WX_RX_COUNTK(wx_rx_count_f_d, 0, false, 1)
WX_RX_COUNTK(wx_rx_count_fp_a, 2, true, 1)
WX_RX_COUNTK(wx_rx_count_fp_d, 2, false, 1)
WX_RX_COUNTK(wx_rx_count_i_a, 1, true, 1)
WX_RX_COUNTK(wx_rx_count_i_d, 1, false, 1)

// Totals and offsets over the ranges.  Workgroup b: digit block q = b / 32,
// bins (b % 32) * 64 + lane; wave w sums the ranges [w R / 4, (w + 1) R / 4).
//   totals[q][d] = sum over r of cnt[q][r][d]                     (if totals)
//   off[q][r][d] = base[q][d] + sum over r' < r of cnt[q][r'][d]  (if off)
extern "C" __global__ __launch_bounds__(256) void wx_rx_scan(WxRxScanArgs a) {
  __shared__ wx_u32 part[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = blockIdx.x / 32, bin = (blockIdx.x % 32) * 64 + lane;
  const wx_u32 *c = a.cnt + (wx_u64)q * a.ranges * WX_RX_BINS + bin;
  const int r0 = w * a.ranges / 4, r1 = (w + 1) * a.ranges / 4;
  wx_u32 s = 0u;
#pragma unroll 8
  for (int r = r0; r < r1; ++r) s += c[(wx_u64)r * WX_RX_BINS];
  part[w][lane] = s;
  __syncthreads();
  wx_u32 pre = 0u, tot = 0u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const wx_u32 v = part[k][lane];
    if (k < w) pre += v;
    tot += v;
  }
  if (a.totals && w == 0) a.totals[q * WX_RX_BINS + bin] = tot;
  if (a.off) {
    wx_u32 run = a.base[q * WX_RX_BINS + bin] + pre;
    wx_u32 *o = a.off + (wx_u64)q * a.ranges * WX_RX_BINS + bin;
#pragma unroll 8
    for (int r = r0; r < r1; ++r) {
      const wx_u32 v = c[(wx_u64)r * WX_RX_BINS];
      o[(wx_u64)r * WX_RX_BINS] = run;
      run += v;
    }
  }
}

// Inclusive prefix sum over the 64 lanes of a wave by DPP row shifts and
// row broadcasts (no LDS, no address registers: the shuffle form's six
// hoisted bpermute addresses spilled in the pass kernel).
__device__ __forceinline__ wx_u32 wx_rx_wave_incl(wx_u32 v) {
  v += (wx_u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (wx_u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (wx_u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (wx_u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (wx_u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += (wx_u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

struct WxRxShared {
  // per-wave digit counts of the tile, waves 2k / 2k + 1 in the low / high
  // half of word [k][d]; then each wave's first tile-local slot of digit d;
  // with a payload, then the payloads in digit order
  wx_u32 wc[WX_RX_WAVES / 2][WX_RX_BINS];
  wx_u32 gb[WX_RX_BINS];  // output slot of the tile's first key of digit d, minus its tile-local slot
  wx_u32 ws[WX_RX_WAVES];  // block scan: per-wave sums
};

// 16 wave-striped dwords of `src` (keys or payloads) from element wb on
__device__ __forceinline__ void wx_rx_load(const wx_u32 *src, wx_i64 n, wx_i64 wb, bool whole,
                                           wx_u32 (&x)[WX_RX_ITEMS]) {
  if (whole) {
#pragma unroll
    for (int i = 0; i < WX_RX_ITEMS; ++i) x[i] = wx::ldv(src + wb + (wx_i64)i * 64);
  } else {
#pragma unroll
    for (int i = 0; i < WX_RX_ITEMS; ++i) {
      const wx_i64 e = wb + (wx_i64)i * 64;
      x[i] = e < n ? wx::ldv(src + e) : 0u;
    }
  }
}

// Tile t of a range.  Key i of lane l of wave w sits at t * TILE + w * 1024
// + i * 64 + l, so (wave, item, lane) is input order.  x holds this tile's
// keys; y receives the next tile's (when `nxt`, whole when `nxt_whole`).
// Payloads are loaded at the start of their own tile (a second 16-register
// prefetch spilled): their latency hides behind the ranking and the scan.
// run0 / run1: the output slot of the range's next key of digit 2 tid /
// 2 tid + 1.
template <bool PAY, int KIND, bool ASC, bool WHOLE>
__device__ __forceinline__ void wx_rx_tile(const WxRxPassArgs &a, WxRxShared &S, wx_u32 *s_k, wx_i64 t, bool nxt,
                                           bool nxt_whole, wx_u32 (&x)[WX_RX_ITEMS], wx_u32 (&y)[WX_RX_ITEMS],
                                           wx_u32 &run0, wx_u32 &run1) {
  typedef wx_u32 u2 __attribute__((ext_vector_type(2)));
  // an opaque copy of the thread index: the slot and address arithmetic is
  // formed here, not hoisted out of the tile loop into (spilled) registers
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (scalar)
  const int wp = wave >> 1, sh = (wave & 1) * 16;
  const wx_u64 below = (1ull << lane) - 1ull;
  wx_u32 *wcf = &S.wc[0][0];
  const wx_i64 tb = t * WX_RX_TILE;
  const wx_i64 wb = tb + wave * 64 * WX_RX_ITEMS + lane;
  wx_u32 v[WX_RX_ITEMS];
  if (PAY) wx_rx_load(a.src_v, a.n, wb, WHOLE, v);
  if (nxt)  // the next tile's keys fly while this one is ranked, permuted and written
    wx_rx_load(a.src_k, a.n, wb + WX_RX_TILE, nxt_whole, y);
  // (1) stable in-wave ranks: one returning LDS add per key on the wave's
  // counter (the LDS returns same-address lanes' results in ascending lane
  // order, gfx950); lane 0's digit group adds its size once from lane 0 and
  // ranks by its ballot (a skewed digit would serialize on one counter)
  wx_u32 rk[WX_RX_ITEMS];
  wx_u32 lead_bits = 0u;
#pragma unroll
  for (int i = 0; i < WX_RX_ITEMS; ++i) {
    const bool valid = WHOLE || wb + (wx_i64)i * 64 < a.n;
    const wx_u32 d = (wx_rs_key_t<KIND, ASC>(x[i]) >> a.shift) & a.mask;
    const wx_u32 d0 = __builtin_amdgcn_readfirstlane(d);
    const bool lead = valid && d == d0;
    const wx_u64 lm = __builtin_amdgcn_ballot_w64(lead);
    rk[i] = (wx_u32)__builtin_popcountll(lm & below);
    if (valid && (!lead || lane == 0)) {
      const wx_u32 inc = (lead ? (wx_u32)__builtin_popcountll(lm) : 1u) << sh;
      rk[i] = (atomicAdd(&S.wc[wp][d], inc) >> sh) & 0xffffu;
    }
    lead_bits |= (lead && lane != 0 ? 1u : 0u) << i;
  }
#pragma unroll
  for (int i = 0; i < WX_RX_ITEMS; ++i) {
    const wx_u32 base0 = __builtin_amdgcn_readlane(rk[i], 0);
    if ((lead_bits >> i) & 1u) rk[i] += base0;
    asm volatile("" : "+v"(rk[i]));  // settled here, not carried as SGPR copies into the scan
  }
  __syncthreads();
  // (2) thread tid owns digits 2 tid, 2 tid + 1: per-wave exclusive prefix,
  // the tile's count, the tile-local digit base by a block scan, the slot
  // bases written back in place, the output base, the run advanced
  {
    wx_u32 ca = 0u, cb = 0u;
#pragma unroll
    for (int k = 0; k < WX_RX_WAVES / 2; ++k) {
      const u2 c = *reinterpret_cast<const u2 *>(&S.wc[k][2 * tid]);
      ca += (c.x & 0xffffu) + (c.x >> 16);
      cb += (c.y & 0xffffu) + (c.y >> 16);
    }
    const wx_u32 s = ca + cb;
    const wx_u32 inc = wx_rx_wave_incl(s);
    if (lane == 63) S.ws[wave] = inc;
    __syncthreads();
    wx_u32 lb = inc - s;
#pragma unroll
    for (int w = 0; w < WX_RX_WAVES; ++w) lb += w < wave ? S.ws[w] : 0u;
    const wx_u32 la = lb, lbb = lb + ca;
    // the counts again (no registers held across the scan): each wave's
    // first slot of the digit, packed as the counts were
    wx_u32 ra = la, rb = lbb;
#pragma unroll
    for (int k = 0; k < WX_RX_WAVES / 2; ++k) {
      u2 c = *reinterpret_cast<const u2 *>(&S.wc[k][2 * tid]);
      const wx_u32 a0 = c.x & 0xffffu, b0 = c.y & 0xffffu;
      const wx_u32 a1 = c.x >> 16, b1 = c.y >> 16;
      c.x = ra | ((ra + a0) << 16);
      c.y = rb | ((rb + b0) << 16);
      ra += a0 + a1;
      rb += b0 + b1;
      *reinterpret_cast<u2 *>(&S.wc[k][2 * tid]) = c;
    }
    u2 g;
    g.x = run0 - la;
    g.y = run1 - lbb;
    *reinterpret_cast<u2 *>(&S.gb[2 * tid]) = g;
    run0 += ca;
    run1 += cb;
  }
  __syncthreads();
  // (3) keys (and payloads) into digit order in LDS
#pragma unroll
  for (int i = 0; i < WX_RX_ITEMS; ++i) {
    const wx_u32 d = (wx_rs_key_t<KIND, ASC>(x[i]) >> a.shift) & a.mask;
    rk[i] += (S.wc[wp][d] >> sh) & 0xffffu;
  }
  if (PAY) __syncthreads();  // every slot read: the payloads take the counters' place
#pragma unroll
  for (int i = 0; i < WX_RX_ITEMS; ++i) {
    if (WHOLE || wb + (wx_i64)i * 64 < a.n) {
      s_k[rk[i]] = x[i];
      if (PAY) wcf[rk[i]] = v[i];
    }
  }
  __syncthreads();
  // (4) LDS -> output: consecutive threads write consecutive slots of a digit's run
  const int tile_n = WHOLE ? WX_RX_TILE : (int)(a.n - tb);
#pragma unroll
  for (int j = 0; j < WX_RX_ITEMS; ++j) {
    const int p = j * WX_RX_BLOCK + tid;
    if (WHOLE || p < tile_n) {
      const wx_u32 k = s_k[p];
      const wx_u32 d = (wx_rs_key_t<KIND, ASC>(k) >> a.shift) & a.mask;
      const wx_u64 g = (wx_u64)(wx_u32)(S.gb[d] + (wx_u32)p);
      if (WX_RX_NT_STORE) {
        __builtin_nontemporal_store(k, a.dst_k + g);
        if (PAY) __builtin_nontemporal_store(wcf[p], a.dst_v + g);
      } else {
        a.dst_k[g] = k;
        if (PAY) a.dst_v[g] = wcf[p];
      }
    }
  }
  if (PAY) __syncthreads();  // every payload read out of the counters' place
#pragma unroll
  for (int i = 0; i < WX_RX_WAVES / 2 * WX_RX_BINS / WX_RX_BLOCK; ++i) wcf[i * WX_RX_BLOCK + tid] = 0u;
  __syncthreads();  // s_k free, counters zeroed
}

// One range, tile after tile; every tile but the last of the table is whole
// and runs a copy of the body without bounds checks.
template <bool PAY, int KIND, bool ASC>
__device__ __forceinline__ void wx_rx_pass_impl(const WxRxPassArgs &a, WxRxShared &S, wx_u32 *s_k) {
  typedef wx_u32 u2 __attribute__((ext_vector_type(2)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = blockIdx.x;
  wx_i64 t0, t1;
  wx_rx_range(a.n, a.ranges, r, t0, t1);
  const u2 o2 = *reinterpret_cast<const u2 *>(a.off + (wx_u64)r * WX_RX_BINS + 2 * tid);
  wx_u32 run0 = o2.x, run1 = o2.y;
  wx_u32 *wcf = &S.wc[0][0];
#pragma unroll
  for (int i = 0; i < WX_RX_WAVES / 2 * WX_RX_BINS / WX_RX_BLOCK; ++i) wcf[i * WX_RX_BLOCK + tid] = 0u;
  if (t0 >= t1) return;  // workgroup-uniform: an empty range (more ranges than tiles)
  const wx_i64 n_whole = a.n / WX_RX_TILE;  // tiles [0, n_whole) are whole
  wx_u32 x[WX_RX_ITEMS], y[WX_RX_ITEMS];
  wx_rx_load(a.src_k, a.n, t0 * WX_RX_TILE + wave * 64 * WX_RX_ITEMS + lane, t0 < n_whole, x);
  __syncthreads();  // counters zeroed
  for (wx_i64 t = t0; t < t1; ++t) {
    const bool nxt = t + 1 < t1;
    if (t < n_whole)
      wx_rx_tile<PAY, KIND, ASC, true>(a, S, s_k, t, nxt, t + 1 < n_whole, x, y, run0, run1);
    else
      wx_rx_tile<PAY, KIND, ASC, false>(a, S, s_k, t, nxt, false, x, y, run0, run1);
#pragma unroll
    for (int i = 0; i < WX_RX_ITEMS; ++i) x[i] = y[i];
  }
}

#define WX_RX_PASSK(NAME, PAY, KIND, ASC)                                                       \
  extern "C" __global__ __launch_bounds__(WX_RX_BLOCK, WX_RX_BLOCK / 256) void NAME(WxRxPassArgs a) { \
    __shared__ WxRxShared S;                                                                  \
    __shared__ wx_u32 s_k[WX_RX_TILE];                                                        \
    wx_rx_pass_impl<PAY, KIND, ASC>(a, S, s_k);                                              \
  }
WX_RX_PASSK(wx_rx_pass_k_f_a, false, 0, true)
WX_RX_PASSK(wx_rx_pass_k_f_d, false, 0, false)
WX_RX_PASSK(wx_rx_pass_k_fp_a, false, 2, true)
WX_RX_PASSK(wx_rx_pass_k_fp_d, false, 2, false)
WX_RX_PASSK(wx_rx_pass_k_i_a, false, 1, true)
WX_RX_PASSK(wx_rx_pass_k_i_d, false, 1, false)
WX_RX_PASSK(wx_rx_pass_kv_f_a, true, 0, true)
WX_RX_PASSK(wx_rx_pass_kv_f_d, true, 0, false)
WX_RX_PASSK(wx_rx_pass_kv_fp_a, true, 2, true)
WX_RX_PASSK(wx_rx_pass_kv_fp_d, true, 2, false)
WX_RX_PASSK(wx_rx_pass_kv_i_a, true, 1, true)
WX_RX_PASSK(wx_rx_pass_kv_i_d, true, 1, false)

#endif  // WX_OP == WX_OP_UTIL
