// wx_group.hip -- GROUP BY: the LDS key window + general-key hash and their finalize
// (one of the kernel sources warpexec concatenates after wx_common.hip, whose
// header describes the prelude they expect)

// ===========================================================================
#if WX_OP == WX_OP_GROUP
// GROUP BY SUM: two-stage reduction.  Stage 1 privatises a dense key window
// [key_lo, key_lo + WX_GWIN) in LDS (ds_add_f64 / ds_add_u32 per row), then
// flushes non-empty bins to global accumulators with one global_atomic_add_f64
// per bin per block.  Keys outside the window go to a global open-addressing
// table (agent-scope CAS).  wx_group_finalize emits groups in ascending key
// order and returns every accumulator it used to zero, so the next call needs
// no memset.  Sums of float values in double are exact (hence order-free)
// while every partial sum stays below 2^53 ulps of the smallest value.
#define WX_GWIN WX_GROUP_WINDOW
#ifndef WX_UNROLL
// row quads per thread per span, with WX_GBLOCK = 512 at 2 workgroups per
// CU: 1.122-1.124 ms per 1e9 rows (148.6-149.5 us per 1.25e8) against
// 1.155-1.157 (156-158 us) for 256-thread workgroups at 4 per CU with 4
// quads and 1.177-1.182 with 2 (profiles/r03/abl_group_grid.txt)
#define WX_UNROLL 2
#endif
#define WX_HSORT_MAX WX_GROUP_HSORT_MAX
#ifndef WX_GROUP_LEAD
#define WX_GROUP_LEAD 16  // lanes of a wave on one window bin from which they add once (0: off)
#endif

#ifndef WX_MINMAX
#define WX_MINMAX 0  // also per-group MIN / MAX (NaN skipped)
#endif
__device__ __forceinline__ float wx_mm_out(wx_u32 m, bool is_min) {
  return (is_min ? m == 0xffffffffu : m == 0u) ? __uint_as_float(0x7fc00000u) : wx::ord2f(m);
}

__device__ __forceinline__ void wx_hash_add(const WxGroupArgs &a, int key, double v, wx_u32 o) {
  const wx_u64 tag = (wx_u64)(wx_u32)key | (1ull << 32);
  wx_u32 h = ((wx_u32)key * 2654435761u) & a.hmask;
  for (wx_u32 probe = 0; probe <= a.hmask; ++probe) {
    wx_u64 cur = wx::ld_agent(&a.h_tag[h]);
    if (cur == 0ull) {
      const wx_u64 prev = atomicCAS(&a.h_tag[h], 0ull, tag);
      if (prev == 0ull) {
        const wx_u64 u = __hip_atomic_fetch_add(&a.ctrs[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        a.h_used[u] = h;
        cur = tag;
      } else {
        cur = prev;
      }
    }
    if (cur == tag) {
      atomicAdd(&a.h_sum[h], v);
      atomicAdd(&a.h_cnt[h], 1ull);
      if (WX_MINMAX && o != 0u) {
        atomicMin(&a.h_min[h], o);
        atomicMax(&a.h_max[h], o);
      }
      return;
    }
    h = (h + 1) & a.hmask;
  }
  atomicOr(reinterpret_cast<unsigned int *>(&a.ctrs[1]), WX_DEVERR_CAPACITY);
}

// WX_GBLOCK threads per workgroup (wx_args.h; the host launches the same):
// the window's global flush is one f64 + one u64 atomic per non-empty bin per
// workgroup, 6-10 us per query at 4 x 256-thread workgroups per CU
// (WX_DIAG_NO_FLUSH, profiles/r03/abl_group_flush.txt); fewer, larger
// workgroups flush less for the same waves per CU.
#undef WX_LBLOCK
#define WX_LBLOCK WX_GBLOCK
// (A finalize fused into the last workgroup to finish, saving the second
// launch, was measured slower and removed in round 5: 154.8 vs 148.1 us per
// 1.25e8 rows, profiles/r03/s2/bench_*fused*.json.)
extern "C" __global__ __launch_bounds__(WX_GBLOCK) void wx_group_sum(WxGroupArgs wx_a) {
  __shared__ double wx_s_sum[WX_GWIN];
  __shared__ wx_u32 wx_s_cnt[WX_GWIN];
#if WX_MINMAX
  __shared__ wx_u32 wx_s_min[WX_GWIN], wx_s_max[WX_GWIN];
#endif
  for (int i = threadIdx.x; i < WX_GWIN; i += WX_GBLOCK) {
    wx_s_sum[i] = 0.0;
    wx_s_cnt[i] = 0u;
#if WX_MINMAX
    wx_s_min[i] = 0xffffffffu;
    wx_s_max[i] = 0u;
#endif
  }
  __syncthreads();
  bool wx_lead_on = false;  // this batch's first rows had a bin shared by many lanes
  WX_STRIDE_LOOP_BEGIN
  bool wx_pass = idx < wx_a.n_rows && WX_EVAL_COND();
#if WX_GROUP_LEAD && !WX_MINMAX
  // A window bin shared by many lanes of the wave (a skewed key): their values
  // summed across the wave and added once (the LDS serialises same-address
  // adds: 90 % of the rows on one key took 7.3 ms per 1e9 rows instead of
  // 1.2).  Full waves only (the DPP total reads every lane).  Checked on the
  // first row of each batch, and on every row of a batch whose first row had
  // such a bin: the check on every row cost the uniform-key C3 query 4.5 %
  // (profiles/r06/ab_group_lead.txt).
  if ((wx_u == 0 && wx_e == 0) || wx_lead_on) {
    const wx_u32 wx_lb = wx_pass ? (wx_u32)(static_cast<int>(WX_KEY) - wx_a.key_lo) : 0xffffffffu;
    const wx_u32 wx_b0 = (wx_u32)__builtin_amdgcn_readfirstlane((int)wx_lb);
    const wx_u64 wx_m = __builtin_amdgcn_ballot_w64(wx_lb == wx_b0 && wx_b0 < (wx_u32)WX_GWIN);
    const bool wx_shared = __builtin_popcountll(wx_m) >= WX_GROUP_LEAD;
    if (wx_u == 0 && wx_e == 0) wx_lead_on = wx_shared;
    if (wx_shared && __builtin_amdgcn_read_exec() == ~0ull) {
      const bool wx_mine = wx_lb == wx_b0;
      const double wx_t = wx::wave_total_f64(wx_mine ? (double)static_cast<float>(WX_EXPR) : 0.0);
      if ((threadIdx.x & 63) == __builtin_ctzll(wx_m)) {
        atomicAdd(&wx_s_sum[wx_b0], wx_t);
        atomicAdd(&wx_s_cnt[wx_b0], (wx_u32)__builtin_popcountll(wx_m));
      }
      wx_pass = wx_pass && !wx_mine;
    }
  }
#endif
  if (wx_pass) {
    const int wx_key = static_cast<int>(WX_KEY);
    const float wx_val = static_cast<float>(WX_EXPR);
    const wx_u32 wx_bin = (wx_u32)(wx_key - wx_a.key_lo);
    const wx_u32 wx_o = WX_MINMAX ? wx::f2ord(wx_val) : 0u;  // NaN -> 0: skipped
    if (wx_bin < (wx_u32)WX_GWIN) {
      atomicAdd(&wx_s_sum[wx_bin], (double)wx_val);
      atomicAdd(&wx_s_cnt[wx_bin], 1u);
#if WX_MINMAX
      if (wx_o != 0u) {
        atomicMin(&wx_s_min[wx_bin], wx_o);
        atomicMax(&wx_s_max[wx_bin], wx_o);
      }
#endif
    } else {
      wx_hash_add(wx_a, wx_key, (double)wx_val, wx_o);
    }
  }
  WX_STRIDE_LOOP_END
  __syncthreads();
#ifndef WX_DIAG_NO_FLUSH
#define WX_DIAG_NO_FLUSH 0  // diagnostic: the window's global flush skipped (results invalid)
#endif
  for (int i = threadIdx.x; i < WX_GWIN && !WX_DIAG_NO_FLUSH; i += WX_GBLOCK) {
    const wx_u32 c = wx_s_cnt[i];
    if (c) {
      atomicAdd(&wx_a.win_sum[i], wx_s_sum[i]);
      atomicAdd(&wx_a.win_cnt[i], (wx_u64)c);
#if WX_MINMAX
      if (wx_s_max[i] != 0u) {
        atomicMin(&wx_a.win_min[i], wx_s_min[i]);
        atomicMax(&wx_a.win_max[i], wx_s_max[i]);
      }
#endif
    }
  }
}

#undef WX_LBLOCK
#define WX_LBLOCK WX_BLOCK

// One 1024-thread block: sort the general-key entries, merge with the dense
// window in ascending key order, write the outputs, zero what was used.  The
// window is two adjacent bins per thread, all loaded up front (one round trip
// to the accumulators the atomics left beyond L2), ranked by one block scan.
#define WX_GFIN_BLOCK 1024
static_assert(WX_GWIN == 2 * WX_GFIN_BLOCK, "two window bins per finalize thread");
extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_group_gather(WxGroupGatherArgs a) {
  const wx_i64 nh = (wx_i64)a.ctrs[0];
  for (wx_i64 i = (wx_i64)blockIdx.x * WX_BLOCK + threadIdx.x; i < a.npad; i += (wx_i64)gridDim.x * WX_BLOCK) {
    wx_u64 e = ~0ull;
    if (i < nh) {
      const wx_u32 key = (wx_u32)a.h_tag[a.h_used[i]];
      e = ((wx_u64)(key ^ 0x80000000u) << 32) | (wx_u32)i;
    }
    a.keys[i] = e;
  }
}

// The finalize on NT threads (the 1024-thread kernel below).  s_ent:
// WX_HSORT_MAX entries ((key ^ sign) << 32 | used-list position), s_wtot:
// NT / 64 words.
template <int NT>
__device__ __forceinline__ void wx_group_finalize_body(const WxGroupFinArgs &a, wx_u64 *s_ent, wx_u32 *s_wtot,
                                                       wx_i64 &s_nlo) {
  constexpr int BPT = WX_GWIN / NT;  // window bins per thread
  static_assert(WX_GWIN == BPT * NT, "the window divides over the threads");
  const int tid = threadIdx.x;
  const wx_i64 n_hash = (wx_i64)a.ctrs[0];
  const bool presorted = a.sorted != nullptr;
  const bool too_many = n_hash > WX_HSORT_MAX && !presorted;
  if (too_many) {
    if (tid == 0) atomicOr(reinterpret_cast<unsigned int *>(&a.ctrs[1]), WX_DEVERR_UNSUPPORTED);
  }
  const wx_i64 nh = too_many ? 0 : n_hash;
  int npad = 1;
  while (!presorted && npad < nh) npad <<= 1;
#define WX_ENT(i) (presorted ? a.sorted[(i)] : s_ent[(i)])
  // window bins of this thread, loaded before the (rare) hash-key sort
  const int b0 = tid * BPT;
  wx_u64 wc[BPT];
#pragma unroll
  for (int h = 0; h < BPT; ++h) wc[h] = a.win_cnt[b0 + h];
  for (int i = tid; !presorted && i < npad; i += NT) {
    wx_u64 e = ~0ull;
    if (i < nh) {
      const wx_u32 slot = a.h_used[i];
      const wx_u32 key = (wx_u32)a.h_tag[slot];
      e = ((wx_u64)(key ^ 0x80000000u) << 32) | (wx_u32)i;
    }
    s_ent[i] = e;
  }
  __syncthreads();
  for (int k = 2; !presorted && k <= npad; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < npad; i += NT) {
        const int p = i ^ j;
        if (p > i) {
          const wx_u64 x = s_ent[i], y = s_ent[p];
          const bool up = (i & k) == 0;
          if ((x > y) == up) { s_ent[i] = y; s_ent[p] = x; }
        }
      }
      __syncthreads();
    }
  // number of hash keys below the window (binary search in key order)
  if (tid == 0) {
    wx_i64 lo = 0, hi = nh;
    while (lo < hi) {
      const wx_i64 mid = (lo + hi) >> 1;
      if ((int)((wx_u32)(WX_ENT(mid) >> 32) ^ 0x80000000u) < a.key_lo) lo = mid + 1;
      else hi = mid;
    }
    s_nlo = lo;
  }
  __syncthreads();
  const wx_i64 nlo = s_nlo;
  // dense window compaction (ascending bins): wave scan + wave totals;
  // partials mode exports the window densely instead (f = 0: no window group
  // takes an output slot, so the out-of-window groups land at 0..nh)
  const bool part = a.win_out != nullptr;
  const int lane = tid & 63, wave = tid >> 6;
  wx_u32 f = 0u;
#pragma unroll
  for (int h = 0; h < BPT; ++h) f += (!part && wc[h]) ? 1u : 0u;
  wx_u32 incl = f;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const wx_u32 t = __shfl_up(incl, o);
    if (lane >= o) incl += t;
  }
  if (lane == 63) s_wtot[wave] = incl;
  __syncthreads();
  wx_u32 wbase = 0, wsum = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const wx_u32 v = s_wtot[w];
    wbase += (w < wave) ? v : 0u;
    wsum += v;
  }
  {
    wx_i64 pos = nlo + wbase + incl - f;
#pragma unroll
    for (int h = 0; h < BPT; ++h) {
      const int b = b0 + h;
      const wx_u64 c = wc[h];
      if (part) {
        a.win_out[b] = c ? a.win_sum[b] : 0.0;
        a.win_out[WX_GWIN + b] = (double)c;
        if (!c) continue;
        a.win_sum[b] = 0.0;
        a.win_cnt[b] = 0ull;
        continue;
      }
      if (!c) continue;
      if (pos < a.capacity) {
        a.out_keys[pos] = a.key_lo + b;
        a.out_sums[pos] = a.win_sum[b];
        a.out_counts[pos] = (wx_i64)c;
#if WX_MINMAX
        if (a.out_mins) a.out_mins[pos] = wx_mm_out(a.win_min[b], true);
        if (a.out_maxs) a.out_maxs[pos] = wx_mm_out(a.win_max[b], false);
#endif
      }
      a.win_sum[b] = 0.0;
      a.win_cnt[b] = 0ull;
#if WX_MINMAX
      a.win_min[b] = 0xffffffffu;
      a.win_max[b] = 0u;
#endif
      ++pos;
    }
  }
  const wx_i64 out_pos = nlo + wsum;
  // hash entries: below-window ones first, the rest after the window
  for (wx_i64 i = tid; i < nh; i += NT) {
    const wx_u64 e = WX_ENT(i);
    const wx_u32 slot = a.h_used[(wx_u32)e];
    const wx_i64 pos = (i < nlo) ? i : out_pos + (i - nlo);
    if (pos < a.capacity) {
      a.out_keys[pos] = (int)((wx_u32)(e >> 32) ^ 0x80000000u);
      a.out_sums[pos] = a.h_sum[slot];
      a.out_counts[pos] = (wx_i64)a.h_cnt[slot];
#if WX_MINMAX
      if (a.out_mins) a.out_mins[pos] = wx_mm_out(a.h_min[slot], true);
      if (a.out_maxs) a.out_maxs[pos] = wx_mm_out(a.h_max[slot], false);
#endif
    }
  }
  // one-collective exchange slots (partials mode): this shard's slot holds
  // its out-of-window group count (-1: table overflow) and the first
  // slot_groups of those groups, ascending (they sit at positions 0..nh of
  // the key order here); every other shard's slot is zero, so a SUM
  // all-reduce of the shards' buffers gathers the slots
  if (part && a.slots) {
    const int sl = 1 + 3 * a.slot_groups;
    const int nd = a.n_slots * sl;
    for (int q = tid; q < nd; q += NT) {
      const int r = q / sl, o = q - r * sl;
      double v = 0.0;
      if (r == a.slot_rank) {
        if (o == 0) {
          v = too_many ? -1.0 : (double)nh;
        } else {
          const int j = (o - 1) / 3, fld = (o - 1) - 3 * j;
          if (j < nh) {
            const wx_u64 e = WX_ENT(j);
            const wx_u32 slot = a.h_used[(wx_u32)e];
            v = fld == 0 ? (double)(int)((wx_u32)(e >> 32) ^ 0x80000000u)
                         : (fld == 1 ? a.h_sum[slot] : (double)a.h_cnt[slot]);
          }
        }
      }
      a.slots[q] = v;
    }
  }
  __syncthreads();
  const wx_i64 total = out_pos + (nh - nlo);
  // return the general-key table to its clean state
  for (wx_i64 i = tid; i < n_hash; i += NT) {
    const wx_u32 slot = a.h_used[i];
    a.h_tag[slot] = 0ull;
    a.h_sum[slot] = 0.0;
    a.h_cnt[slot] = 0ull;
#if WX_MINMAX
    a.h_min[slot] = 0xffffffffu;
    a.h_max[slot] = 0u;
#endif
  }
  if (tid == 0) {
    a.ctrs[0] = 0ull;
    *a.n_groups_out = too_many ? -1 : total;
    if (part) a.win_out[2 * WX_GWIN] = too_many ? 0.0 : (double)total;
    if (total > a.capacity) atomicOr(reinterpret_cast<unsigned int *>(&a.ctrs[1]), WX_DEVERR_CAPACITY);
  }
#undef WX_ENT
}

extern "C" __global__ __launch_bounds__(WX_GFIN_BLOCK) void wx_group_finalize(WxGroupFinArgs a) {
  __shared__ wx_u64 s_ent[WX_HSORT_MAX];  // (key ^ sign) << 32 | used-list position
  __shared__ wx_u32 s_wtot[WX_GFIN_BLOCK / 64];
  __shared__ wx_i64 s_nlo;
  wx_group_finalize_body<WX_GFIN_BLOCK>(a, s_ent, s_wtot, s_nlo);
}
#endif
