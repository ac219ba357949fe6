// wx_util.hip -- the util module: exchange merges, sort utilities, heads, row-order fold
// (one of the kernel sources warpexec concatenates after wx_common.hip, whose
// header describes the prelude they expect)

// ===========================================================================
#if WX_OP == WX_OP_UTIL
// Synthetic data generator and the stable sort used by the legacy
// jit_sort_* entry points (bitonic network over 64-bit (rank << 32 | pos)
// keys: LDS passes for spans <= 2 * WX_BLOCK * 4, global passes above).
__device__ __forceinline__ wx_u64 wx_splitmix64(wx_u64 x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_fill_synthetic(WxFillArgs a) {
  const wx_i64 stride = (wx_i64)gridDim.x * WX_BLOCK;
  const float flo = (float)a.lo, fspan = (float)a.hi - (float)a.lo;
  const wx_i64 ilo = (wx_i64)a.lo, ispan = (wx_i64)a.hi - (wx_i64)a.lo + 1;
  for (wx_i64 i = (wx_i64)blockIdx.x * WX_BLOCK + threadIdx.x; i < a.n; i += stride) {
    const wx_u64 h = wx_splitmix64((wx_u64)(a.row_base + i) + a.seed * 0xD1B54A32D192ED03ull);
    double v;
    if (a.kind == 0) {
      const float u = (float)(h >> 40) * (1.0f / 16777216.0f);
      const float m = __fmul_rn(u, fspan);
      v = (double)__fadd_rn(flo, m);
    } else {
      v = (double)(ilo + (wx_i64)((h >> 32) % (wx_u64)ispan));
    }
    switch (a.dtype) {
      case 0: static_cast<int *>(a.out)[i] = (int)v; break;
      case 1: static_cast<wx_i64 *>(a.out)[i] = (wx_i64)v; break;
      case 2: static_cast<float *>(a.out)[i] = (float)v; break;
      default: static_cast<double *>(a.out)[i] = v; break;
    }
  }
}

// Final GROUP BY result of a row-sharded query (query_multi_gpu GROUP BY):
// the combined exchange window (sums, counts as f64 -- element-wise sums of
// every shard's wx_group_partials window) and the combined out-of-window
// groups (ascending keys) merged in ascending key order: the groups below
// the window, the non-empty window bins, the groups above.  One 1024-thread
// block, two window bins per thread, ranked by a block scan (as
// wx_group_finalize).
#define WX_GCOMB_BLOCK 1024
static_assert(WX_GROUP_WINDOW == 2 * WX_GCOMB_BLOCK, "two window bins per combine thread");
// x_keys / x_sums / x_counts: global or LDS (flat pointers)
__device__ __forceinline__ void wx_group_combine_body(const WxGroupCombineArgs &a, wx_u32 *s_wtot, wx_i64 *s_nlo) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b0 = 2 * tid;
  const double c0 = a.window[WX_GROUP_WINDOW + b0], c1 = a.window[WX_GROUP_WINDOW + b0 + 1];
  if (tid == 0) {  // out-of-window groups below the window
    wx_i64 lo = 0, hi = a.n_extra;
    while (lo < hi) {
      const wx_i64 mid = (lo + hi) >> 1;
      if (a.x_keys[mid] < a.key_lo) lo = mid + 1;
      else hi = mid;
    }
    *s_nlo = lo;
  }
  const wx_u32 f = (c0 != 0.0 ? 1u : 0u) + (c1 != 0.0 ? 1u : 0u);
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
  for (int w = 0; w < WX_GCOMB_BLOCK / 64; ++w) {
    const wx_u32 v = s_wtot[w];
    wbase += (w < wave) ? v : 0u;
    wsum += v;
  }
  const wx_i64 nlo = *s_nlo;
  wx_i64 pos = nlo + wbase + incl - f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int b = b0 + h;
    const double c = h ? c1 : c0;
    if (c == 0.0) continue;
    if (pos < a.capacity) {
      a.out_keys[pos] = a.key_lo + b;
      a.out_sums[pos] = a.window[b];
      a.out_counts[pos] = (wx_i64)c;
    }
    ++pos;
  }
  const wx_i64 above = nlo + wsum;
  for (wx_i64 i = tid; i < a.n_extra; i += WX_GCOMB_BLOCK) {
    const wx_i64 p = i < nlo ? i : above + (i - nlo);
    if (p < a.capacity) {
      a.out_keys[p] = a.x_keys[i];
      a.out_sums[p] = a.x_sums[i];
      a.out_counts[p] = a.x_counts[i];
    }
  }
  if (tid == 0) *a.n_groups_out = above + (a.n_extra - nlo);
}

extern "C" __global__ __launch_bounds__(WX_GCOMB_BLOCK) void wx_group_combine(WxGroupCombineArgs a) {
  __shared__ wx_u32 s_wtot[WX_GCOMB_BLOCK / 64];
  __shared__ wx_i64 s_nlo;
  wx_group_combine_body(a, s_wtot, &s_nlo);
}

// The one-collective form (wx_group_combine_slots): the exchange buffer is
// the window followed by one slot per shard (count, then (key, sum, count)
// triples, ascending keys).  The slots' groups are sorted in LDS by (key,
// slot), groups of equal key are summed in slot order (so every rank and
// every run adds them in the same order), and the unique groups are merged
// with the window exactly as wx_group_combine does.  A slot whose shard had
// more out-of-window groups than fit (count > slot_groups) makes the result
// -2: the caller merges those groups with a variable-size exchange instead.
extern "C" __global__ __launch_bounds__(WX_GCOMB_BLOCK) void wx_group_combine_slots(WxGroupSlotsArgs a) {
  __shared__ wx_u64 s_ent[WX_GROUP_SLOT_MAX];  // (key ^ sign) << 32 | slot-major entry index
  __shared__ int s_key[WX_GROUP_SLOT_MAX];
  __shared__ double s_sum[WX_GROUP_SLOT_MAX];
  __shared__ wx_i64 s_cnt[WX_GROUP_SLOT_MAX];
  __shared__ int s_off[WX_GCOMB_BLOCK + 1];  // entry offset of each slot (n_slots <= WX_GCOMB_BLOCK)
  __shared__ wx_u32 s_wtot[WX_GCOMB_BLOCK / 64];
  __shared__ wx_i64 s_nlo;
  __shared__ int s_state;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int sl = 1 + 3 * a.slot_groups;
  const double *slots = a.exchange + WX_GROUP_EXCHANGE;
  if (tid == 0) s_state = 0;
  {  // slot counts (thread r: slot r), their prefix by a block scan
    const double c = tid < a.n_slots ? slots[(wx_i64)tid * sl] : 0.0;
    __syncthreads();
    if (c < 0.0) atomicMax(&s_state, 2);
    else if (c > (double)a.slot_groups) atomicMax(&s_state, 1);
    const wx_u32 mine = (c > 0.0 && c <= (double)a.slot_groups) ? (wx_u32)c : 0u;
    wx_u32 incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const wx_u32 t = __shfl_up(incl, o);
      if (lane >= o) incl += t;
    }
    if (lane == 63) s_wtot[wave] = incl;
    __syncthreads();
    wx_u32 base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < WX_GCOMB_BLOCK / 64; ++w) {
      const wx_u32 v = s_wtot[w];
      base += (w < wave) ? v : 0u;
      tot += v;
    }
    s_off[tid] = (int)(base + incl - mine);
    if (tid == 0) s_off[a.n_slots] = (int)tot;
    __syncthreads();
  }
  if (s_state != 0) {
    if (tid == 0) *a.n_groups_out = s_state == 2 ? -1 : -2;
    return;
  }
  const int T = s_off[a.n_slots];
  int npad = 1;
  while (npad < T) npad <<= 1;
  for (int i = tid; i < npad; i += WX_GCOMB_BLOCK) {
    wx_u64 e = ~0ull;
    if (i < T) {
      int lo = 0, hi = a.n_slots - 1;  // the slot holding entry i: last r with s_off[r] <= i
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_off[mid] <= i) lo = mid;
        else hi = mid - 1;
      }
      const int j = i - s_off[lo];
      const int key = (int)slots[(wx_i64)lo * sl + 1 + 3 * j];
      e = ((wx_u64)((wx_u32)key ^ 0x80000000u) << 32) | ((wx_u32)lo * (wx_u32)a.slot_groups + (wx_u32)j);
    }
    s_ent[i] = e;
  }
  __syncthreads();
  for (int k = 2; k <= npad; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < npad; i += WX_GCOMB_BLOCK) {
        const int p = i ^ j;
        if (p > i) {
          const wx_u64 x = s_ent[i], y = s_ent[p];
          const bool up = (i & k) == 0;
          if ((x > y) == up) { s_ent[i] = y; s_ent[p] = x; }
        }
      }
      __syncthreads();
    }
  // unique keys: run heads ranked by a block scan (4 consecutive entries per thread)
  constexpr int PER = WX_GROUP_SLOT_MAX / WX_GCOMB_BLOCK;
  wx_u32 hm = 0u, nh = 0u;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = tid * PER + q;
    if (i < T && (i == 0 || (s_ent[i] >> 32) != (s_ent[i - 1] >> 32))) { hm |= 1u << q; ++nh; }
  }
  wx_u32 incl = nh;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const wx_u32 t = __shfl_up(incl, o);
    if (lane >= o) incl += t;
  }
  if (lane == 63) s_wtot[wave] = incl;
  __syncthreads();
  wx_u32 wbase = 0, usum = 0;
#pragma unroll
  for (int w = 0; w < WX_GCOMB_BLOCK / 64; ++w) {
    const wx_u32 v = s_wtot[w];
    wbase += (w < wave) ? v : 0u;
    usum += v;
  }
  wx_u32 u = wbase + incl - nh;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    if (!(hm & (1u << q))) continue;
    const int i0 = tid * PER + q;
    const wx_u32 kk = (wx_u32)(s_ent[i0] >> 32);
    double sum = 0.0;
    wx_i64 cnt = 0;
    for (int i = i0; i < T && (wx_u32)(s_ent[i] >> 32) == kk; ++i) {  // slot order
      const wx_u32 ent = (wx_u32)s_ent[i];
      const int r = (int)(ent / (wx_u32)a.slot_groups), j = (int)(ent % (wx_u32)a.slot_groups);
      const double *g = slots + (wx_i64)r * sl + 1 + 3 * j;
      sum += g[1];
      cnt += (wx_i64)g[2];
    }
    s_key[u] = (int)(kk ^ 0x80000000u);
    s_sum[u] = sum;
    s_cnt[u] = cnt;
    ++u;
  }
  __syncthreads();
  WxGroupCombineArgs c;
  c.window = a.exchange;
  c.x_keys = s_key;
  c.x_sums = s_sum;
  c.x_counts = s_cnt;
  c.n_extra = usum;
  c.key_lo = a.key_lo;
  c.out_keys = a.out_keys;
  c.out_sums = a.out_sums;
  c.out_counts = a.out_counts;
  c.capacity = a.capacity;
  c.n_groups_out = a.n_groups_out;
  wx_group_combine_body(c, s_wtot + 0, &s_nlo);
}

// Many-key row-sharded GROUP BY (wx_group_merge_lists; replaces a host merge
// of the shards' groups, src/multi_gpu_utils.cpp:23-60 gathers on the host):
// every shard's groups arrive as one fixed-size list record (ascending unique
// keys) from ONE all-gather.  wx_glist_place puts each group at its place in
// (key, list) order -- its index in its own list plus, per other list, the
// groups with a smaller key (and, from an earlier list, an equal one), found
// by binary search -- and marks the first group of each key; wx_glist_count
// counts those heads per WX_GLIST_SPAN places; wx_glist_scan turns the counts
// into offsets, places the window's groups and publishes the totals;
// wx_glist_emit sums each run of equal keys in list order (every rank adds
// them alike) and writes the unique groups below and above the window's.
static_assert(WX_GROUP_WINDOW == 2 * WX_GLIST_BLOCK, "two window bins per list-merge thread");
__device__ __forceinline__ wx_i64 wx_gl_raw(const WxGroupListsArgs &a, int r) {
  return *reinterpret_cast<const wx_i64 *>(a.lists + (wx_i64)r * a.list_bytes);
}
__device__ __forceinline__ wx_i64 wx_gl_valid(const WxGroupListsArgs &a, int r) {  // a bad count reads as empty
  const wx_i64 c = wx_gl_raw(a, r);
  return (c < 0 || c > a.list_cap) ? 0 : c;
}
__device__ __forceinline__ const int *wx_gl_keys(const WxGroupListsArgs &a, int r) {
  return reinterpret_cast<const int *>(a.lists + (wx_i64)r * a.list_bytes + 8);
}
__device__ __forceinline__ wx_i64 wx_gl_lower(const int *keys, wx_i64 n, int k) {  // keys[0..n) below k
  wx_i64 lo = 0, hi = n;
  while (lo < hi) {
    const wx_i64 mid = (lo + hi) >> 1;
    if (keys[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ wx_i64 wx_gl_merged(const WxGroupListsArgs &a) {
  wx_i64 m = 0;
  for (int r = 0; r < a.n_lists; ++r) m += wx_gl_valid(a, r);
  return m;
}

extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_glist_place(WxGroupListsArgs a) {
  const wx_i64 total = (wx_i64)a.n_lists * a.list_cap;
  for (wx_i64 q = (wx_i64)blockIdx.x * WX_BLOCK + threadIdx.x; q < total; q += (wx_i64)gridDim.x * WX_BLOCK) {
    const int r = (int)(q / a.list_cap);
    const wx_i64 i = q - (wx_i64)r * a.list_cap;
    if (i >= wx_gl_valid(a, r)) continue;
    const unsigned char *rec = a.lists + (wx_i64)r * a.list_bytes;
    const int k = wx_gl_keys(a, r)[i];
    wx_i64 pos = i;
    bool head = true;
    for (int s = 0; s < a.n_lists; ++s) {
      if (s == r) continue;
      const int *ks = wx_gl_keys(a, s);
      const wx_i64 ns = wx_gl_valid(a, s);
      const wx_i64 lb = wx_gl_lower(ks, ns, k);
      const bool eq = lb < ns && ks[lb] == k;
      if (s < r) {
        pos += lb + (eq ? 1 : 0);
        head = head && !eq;
      } else {
        pos += lb;
      }
    }
    a.m_keys[pos] = k;
    a.m_sums[pos] = reinterpret_cast<const double *>(rec + a.sums_off)[i];
    a.m_cnts[pos] = reinterpret_cast<const wx_i64 *>(rec + a.counts_off)[i];
    a.m_head[pos] = head ? 1u : 0u;
  }
}

extern "C" __global__ __launch_bounds__(WX_GLIST_BLOCK) void wx_glist_count(WxGroupListsArgs a) {
  __shared__ wx_u32 s_w[WX_GLIST_BLOCK / 64];
  __shared__ wx_i64 s_m;
  const int tid = threadIdx.x;
  if (tid == 0) s_m = wx_gl_merged(a);
  __syncthreads();
  const wx_i64 m = s_m;
  const wx_i64 p0 = (wx_i64)blockIdx.x * WX_GLIST_SPAN + (wx_i64)tid * WX_GLIST_PER;
  wx_u32 c = 0u;
#pragma unroll
  for (int j = 0; j < WX_GLIST_PER; ++j)
    if (p0 + j < m) c += a.m_head[p0 + j];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((tid & 63) == 0) s_w[tid >> 6] = c;
  __syncthreads();
  if (tid == 0) {
    wx_i64 t = 0;
    for (int w = 0; w < WX_GLIST_BLOCK / 64; ++w) t += s_w[w];
    a.blk[blockIdx.x] = t;
  }
}

extern "C" __global__ __launch_bounds__(WX_GLIST_BLOCK) void wx_glist_scan(WxGroupListsArgs a) {
  __shared__ wx_i64 s_w[WX_GLIST_BLOCK / 64];
  __shared__ wx_i64 s_carry, s_p0, s_pb;
  __shared__ int s_bad;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) {
    s_carry = 0;
    s_p0 = 0;
    s_pb = 0;
    s_bad = 0;
  }
  __syncthreads();
  // list validity, and P0 = groups with a key below the window (their places come first)
  for (int r = tid; r < a.n_lists; r += WX_GLIST_BLOCK) {
    const wx_i64 c = wx_gl_raw(a, r);
    if (c < 0 || c > a.list_cap) atomicOr(&s_bad, 1);
    if (a.window)
      atomicAdd(reinterpret_cast<unsigned long long *>(&s_p0),
                (unsigned long long)wx_gl_lower(wx_gl_keys(a, r), wx_gl_valid(a, r), a.key_lo));
  }
  __syncthreads();
  const wx_i64 p0 = s_p0;
  const wx_i64 b0 = p0 / WX_GLIST_SPAN;
  // exclusive prefix of the per-span head counts, 1024 spans per round
  for (wx_i64 base = 0; base < a.n_blk; base += WX_GLIST_BLOCK) {
    const wx_i64 i = base + tid;
    const wx_i64 v = i < a.n_blk ? a.blk[i] : 0;
    wx_i64 incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const wx_i64 t = __shfl_up(incl, o);
      if (lane >= o) incl += t;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    wx_i64 wb = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < WX_GLIST_BLOCK / 64; ++w) {
      const wx_i64 x = s_w[w];
      wb += w < wave ? x : 0;
      tot += x;
    }
    const wx_i64 carry = s_carry;
    if (i < a.n_blk) {
      a.blk[i] = carry + wb + incl - v;
      if (i == b0) s_pb = carry + wb + incl - v;
    }
    __syncthreads();
    if (tid == 0) s_carry = carry + tot;
    __syncthreads();
  }
  const wx_i64 U = s_carry;  // unique keys over all lists
  // unique keys below the window: the heads before place P0
  wx_i64 nlo = 0;
  if (a.window) {
    if (b0 >= a.n_blk) {
      nlo = U;
    } else {
      const wx_i64 q0 = b0 * WX_GLIST_SPAN + (wx_i64)tid * WX_GLIST_PER;
      wx_u32 c = 0u;
#pragma unroll
      for (int j = 0; j < WX_GLIST_PER; ++j)
        if (q0 + j < p0) c += a.m_head[q0 + j];
      wx_i64 cc = c;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) cc += __shfl_xor(cc, o);
      if (lane == 0) s_w[wave] = cc;
      __syncthreads();
      nlo = s_pb;
      for (int w = 0; w < WX_GLIST_BLOCK / 64; ++w) nlo += s_w[w];
      __syncthreads();
    }
  }
  // the window's non-empty bins, in key order, between the groups below and above it
  wx_i64 wn = 0;
  if (a.window) {
    const int b = 2 * tid;
    const double c0 = a.window[WX_GROUP_WINDOW + b], c1 = a.window[WX_GROUP_WINDOW + b + 1];
    const wx_u32 f = (c0 != 0.0 ? 1u : 0u) + (c1 != 0.0 ? 1u : 0u);
    wx_u32 incl = f;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const wx_u32 t = __shfl_up(incl, o);
      if (lane >= o) incl += t;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    wx_i64 wb = 0;
#pragma unroll
    for (int w = 0; w < WX_GLIST_BLOCK / 64; ++w) {
      wb += w < wave ? s_w[w] : 0;
      wn += s_w[w];
    }
    wx_i64 pos = nlo + wb + incl - f;
    if (!s_bad) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const double c = h ? c1 : c0;
        if (c == 0.0) continue;
        if (pos < a.capacity) {
          a.out_keys[pos] = a.key_lo + b + h;
          a.out_sums[pos] = a.window[b + h];
          a.out_counts[pos] = (wx_i64)c;
        }
        ++pos;
      }
    }
  }
  if (tid == 0) {
    a.meta[0] = wx_gl_merged(a);
    a.meta[1] = nlo;
    a.meta[2] = wn;
    a.meta[3] = s_bad ? -1 : 0;
    *a.n_groups_out = s_bad ? -1 : U + wn;
  }
}

extern "C" __global__ __launch_bounds__(WX_GLIST_BLOCK) void wx_glist_emit(WxGroupListsArgs a) {
  __shared__ wx_u32 s_w[WX_GLIST_BLOCK / 64];
  __shared__ wx_i64 s_m;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (a.meta[3] != 0) return;  // a bad list: the scan reported -1, nothing is written
  if (tid == 0) s_m = a.meta[0];
  const wx_i64 nlo = a.meta[1], wn = a.meta[2];
  __syncthreads();
  const wx_i64 m = s_m;
  const wx_i64 p0 = (wx_i64)blockIdx.x * WX_GLIST_SPAN + (wx_i64)tid * WX_GLIST_PER;
  wx_u32 hm = 0u, nh = 0u;
#pragma unroll
  for (int j = 0; j < WX_GLIST_PER; ++j)
    if (p0 + j < m && a.m_head[p0 + j]) {
      hm |= 1u << j;
      ++nh;
    }
  wx_u32 incl = nh;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const wx_u32 t = __shfl_up(incl, o);
    if (lane >= o) incl += t;
  }
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  wx_i64 wb = 0;
#pragma unroll
  for (int w = 0; w < WX_GLIST_BLOCK / 64; ++w) wb += w < wave ? s_w[w] : 0u;
  wx_i64 u = a.blk[blockIdx.x] + wb + incl - nh;
#pragma unroll
  for (int j = 0; j < WX_GLIST_PER; ++j) {
    if (!(hm & (1u << j))) continue;
    const wx_i64 p = p0 + j;
    const int k = a.m_keys[p];
    double sum = a.m_sums[p];  // list order: the first list's sum, then the others' added
    wx_i64 cnt = a.m_cnts[p];
    for (wx_i64 q = p + 1; q < m && a.m_keys[q] == k; ++q) {
      sum += a.m_sums[q];
      cnt += a.m_cnts[q];
    }
    const wx_i64 idx = u < nlo ? u : u + wn;
    if (idx < a.capacity) {
      a.out_keys[idx] = k;
      a.out_sums[idx] = sum;
      a.out_counts[idx] = cnt;
    }
    ++u;
  }
}

// Global ORDER BY .. LIMIT k of a row-sharded query from every shard's
// candidates (wx_topk_merge): n_records records of <= k (key, value, row)
// candidates each.  A candidate's place is the number of candidates that
// beat it in the total order (better key -- NaN last, -0.0 == +0.0 -- then
// the smaller row, then the earlier candidate), counted over all of them in
// LDS; places < k are written.  n_records * k <= WX_TOPK_MERGE_MAX.
extern "C" __global__ __launch_bounds__(1024) void wx_topk_merge(WxTopkMergeArgs a) {
  __shared__ wx_u32 s_r[WX_TOPK_MERGE_MAX];
  __shared__ wx_i64 s_row[WX_TOPK_MERGE_MAX];
  __shared__ float s_key[WX_TOPK_MERGE_MAX], s_val[WX_TOPK_MERGE_MAX];
  __shared__ bool s_ok[WX_TOPK_MERGE_MAX];
  __shared__ int s_tot;
  const int tid = threadIdx.x;
  const int nc = a.n_records * a.k;
  if (tid == 0) s_tot = 0;
  for (int c = tid; c < nc; c += 1024) {
    // one round trip: the record's count and the slot's key, value and row
    // are independent loads (the slot exists whether or not it is used)
    const int r = c / a.k, j = c - r * a.k;
    const unsigned char *rec = a.records + (wx_i64)r * WX_TOPK_REC_BYTES;
    const wx_i64 m = *reinterpret_cast<const wx_i64 *>(rec + WX_TOPK_MAX * 16);
    const float key = reinterpret_cast<const float *>(rec)[j];
    const float val = reinterpret_cast<const float *>(rec + WX_TOPK_MAX * 4)[j];
    const wx_i64 row = reinterpret_cast<const wx_i64 *>(rec + WX_TOPK_MAX * 8)[j];
    const wx_u32 o = wx::f2ord(key);
    s_ok[c] = j < m;
    s_r[c] = (a.descending || o == 0u) ? o : ~o;  // larger is better; NaN (0) worst
    s_row[c] = row;
    s_key[c] = key;
    s_val[c] = val;
  }
  __syncthreads();
  for (int c = tid; c < nc; c += 1024) {
    if (!s_ok[c]) continue;
    atomicAdd(&s_tot, 1);
    const wx_u32 rc = s_r[c];
    const wx_i64 wc = s_row[c];
    int place = 0;
    for (int d = 0; d < nc; ++d) {
      if (!s_ok[d] || d == c) continue;
      const wx_u32 rd = s_r[d];
      const wx_i64 wd = s_row[d];
      place += (rd > rc || (rd == rc && (wd < wc || (wd == wc && d < c)))) ? 1 : 0;
    }
    if (place < a.k) {
      if (a.out_keys) a.out_keys[place] = s_key[c];
      if (a.out_vals) a.out_vals[place] = s_val[c];
      if (a.out_idx) a.out_idx[place] = wc;
    }
  }
  __syncthreads();
  if (tid == 0 && a.count_out) *a.count_out = s_tot < a.k ? s_tot : a.k;
}

// Element-wise C conversion between the column types (wx_cast), e.g. the
// double GROUP BY sums into the float outputs of jit_group_sum.
template <typename S, typename D>
__device__ __forceinline__ void wx_cast_loop(const void *src, void *dst, wx_i64 n) {
  const wx_i64 stride = (wx_i64)gridDim.x * WX_BLOCK;
  for (wx_i64 i = (wx_i64)blockIdx.x * WX_BLOCK + threadIdx.x; i < n; i += stride)
    static_cast<D *>(dst)[i] = (D) static_cast<const S *>(src)[i];
}
template <typename S>
__device__ __forceinline__ void wx_cast_to(const WxCastArgs &a) {
  switch (a.dst_dtype) {
    case 0: wx_cast_loop<S, int>(a.src, a.dst, a.n); break;
    case 1: wx_cast_loop<S, wx_i64>(a.src, a.dst, a.n); break;
    case 2: wx_cast_loop<S, float>(a.src, a.dst, a.n); break;
    default: wx_cast_loop<S, double>(a.src, a.dst, a.n); break;
  }
}
extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_cast(WxCastArgs a) {
  switch (a.src_dtype) {
    case 0: wx_cast_to<int>(a); break;
    case 1: wx_cast_to<wx_i64>(a); break;
    case 2: wx_cast_to<float>(a); break;
    default: wx_cast_to<double>(a); break;
  }
}

// ---------------------------------------------------------------------------
// The row-order fold s = (((s + v0) + v1) + ...) in double, bit for bit, WITHOUT
// one dependent add per value.  While the running sum s stays inside one binade
// [2^k, 2^(k+1)), every double it can take is a multiple of u = 2^(k-52), so
// each step is fl(s + v) = s + round_u(v): a multiple of u plus v rounded to
// the nearest multiple of u (ties to even excepted -- then the parity of s
// decides).  So a block of 64 * WX_XF_J values whose steps provably stay in
// the binade folds to s + u * sum(round_u(v_i)), an exact integer sum, in any
// order: q_i = v_i * 2^(52 - k) (exact), r_i = rint(q_i); the block takes the
// fast path when no q_i is large (|q_i| < 2^44, so every sum of 512 of them is
// an exact double) or non-finite, and every state S + prefix stays strictly
// inside (2^52, 2^53) in magnitude -- checked conservatively against S +-
// sum(|r_i|).  A tie (q_i = m + 1/2) rounds to the even one of S + m and S + m
// + 1, so it depends on the parity of the running integer S and leaves S even:
// XfTies scans the block in row order by ballots and reduces every tie after
// the first to a known +0 / +1, and the first to p_in ^ cf (p_in: S's parity
// where the block starts).  Any other block (s = 0 at the start, a binade
// crossing, NaN / Inf, tiny s) runs the dependent adds in row order through an
// LDS broadcast.  Prices U[0, 40) at ~1e6 rows per group: ~12 of ~2 000 blocks
// per group take the slow path (the first, and one per doubling).
#ifndef WX_FOLD_EXACT
#define WX_FOLD_EXACT 1  // the row-order folds use fold_exact; 0: one dependent add per value (A/B)
#endif
#ifndef WX_XF_J
#define WX_XF_J 8  // values per lane per block (block = 64 * WX_XF_J)
#endif
#ifndef WX_XF_AHEAD
#define WX_XF_AHEAD 4  // blocks whose loads are in flight ahead of the fold (8: 512 VGPRs + scratch)
#endif
#define WX_XF_B (64 * WX_XF_J)
static_assert(WX_XF_B <= 512, "sums of |q| < 2^44 stay exact doubles for at most 512 values");

namespace wx {
// The ties of a row-ordered run of values, 64 at a time (lane l = the l-th
// value of a row), wave-uniform.  b is rint(q), or floor(q) for a tie; a tie
// adds b + ((P + b) & 1) where P is the parity of S before it, and leaves S
// even, so P is known for every tie after the first (the parity of the b's
// since the tie before it), and the first one's +1 is p_in ^ cf.
struct XfTies {
  wx_u32 seen = 0u;  // a tie earlier in this run
  wx_u32 cpar = 0u;  // parity of the b's since the last tie (since the start, relative to p_in, if none)
  wx_u32 has = 0u;   // the run has a tie: its first adds p_in ^ cf
  wx_u32 cf = 0u;
  double adj = 0.0;  // the +1s of the other ties
  __device__ __forceinline__ void row(bool tie, bool bpar) {
    const wx_u64 pm = __builtin_amdgcn_ballot_w64(bpar), tm = __builtin_amdgcn_ballot_w64(tie);
    if (tm == 0ull) {
      cpar ^= (wx_u32)__builtin_popcountll(pm) & 1u;
      return;
    }
    const int lane = threadIdx.x & 63;
    const wx_u64 below = (1ull << lane) - 1ull;
    bool plus = false;
    wx_u32 cf_l = 0u;
    if (tie) {
      const wx_u64 tb = tm & below;
      const wx_u32 bp = bpar ? 1u : 0u;
      if (tb) {  // the tie before it is in this row: the b's strictly between them
        const int lt = 63 - __builtin_clzll(tb);
        plus = ((((wx_u32)__builtin_popcountll(pm & below & ~((2ull << lt) - 1ull))) & 1u) ^ bp) != 0u;
      } else if (seen) {  // in an earlier row
        plus = ((cpar ^ ((wx_u32)__builtin_popcountll(pm & below) & 1u)) ^ bp) != 0u;
      } else {  // the run's first tie
        cf_l = (cpar ^ ((wx_u32)__builtin_popcountll(pm & below) & 1u)) ^ bp;
      }
    }
    adj += (double)__builtin_popcountll(__builtin_amdgcn_ballot_w64(plus));
    if (!seen) {
      has = 1u;
      cf = (wx_u32)__builtin_amdgcn_readlane((int)cf_l, __builtin_ctzll(tm));
    }
    const int lt = 63 - __builtin_clzll(tm);
    cpar = (wx_u32)__builtin_popcountll(pm & ~((2ull << lt) - 1ull)) & 1u;
    seen = 1u;
  }
  // S + R for a run of total R (t + adj, formed off the chain) starting at
  // the running integer S: the first tie's +1 added only when there is a
  // tie, so a tie-free run puts one add on the chain
  __device__ __forceinline__ double apply(double S, double R) const {
    double r = S + R;
    if (has) {  // wave-uniform
      const double h = S * 0.5;
      r += (double)((h != __builtin_floor(h) ? 1u : 0u) ^ cf);
    }
    return r;
  }
};

// one value under the scaling p2: its b and tie flag (r = rint(q) by the
// 1.5 * 2^52 add and subtract, round half to even, exact for |q| < 2^51)
__device__ __forceinline__ double xf_b(double q, bool &tie) {
  constexpr double M = 0x1.8p52;
  const double r = (q + M) - M;
  tie = __builtin_fabs(q - r) == 0.5;
  return tie && r > q ? r - 1.0 : r;  // a tie's lower neighbour m = floor(q)
}
__device__ __forceinline__ bool xf_odd(double b) {
  const double h = b * 0.5;
  return h != __builtin_floor(h);
}

// The sums of a block under binade k: t = sum b_i, a = sum |b_i| + ties (a
// bound on sum |r_i|) as lane partials, ok = no large / non-finite q, T = the
// block's ties (rows j = 0 .. WX_XF_J - 1, value (j, lane) at row j * 64 +
// lane).  q = x * 2^(52 - k) is exact (a power-of-two scaling; an underflow
// is far below a tie, an overflow fails |q| < 2^44).
__device__ __forceinline__ void xf_sums(int k, const float (&x)[WX_XF_J], double &t, double &a, bool &ok,
                                        XfTies &T) {
  const double p2 = __builtin_ldexp(1.0, 52 - k);
  constexpr double M = 0x1.8p52;
  bool lok = true, any = false;
  t = 0.0;
  a = 0.0;
#pragma unroll
  for (int j = 0; j < WX_XF_J; ++j) {
    const double q = (double)x[j] * p2;
    const double r = (q + M) - M;  // rint(q), round half to even
    lok = lok && __builtin_fabs(q) < 0x1p44;  // false for NaN / Inf
    any = any || __builtin_fabs(q - r) == 0.5;
    t += r;
    a += __builtin_fabs(r);
  }
  ok = __builtin_amdgcn_ballot_w64(!lok) == 0ull;
  T = XfTies();
  if (ok && __builtin_amdgcn_ballot_w64(any) != 0ull) {
    // rare: the row scan; a tie's b is floor(q), which is rint(q) or one less
    double dt = 0.0, nt = 0.0;
#pragma unroll
    for (int j = 0; j < WX_XF_J; ++j) {
      const double q = (double)x[j] * p2;
      bool tie;
      const double b = xf_b(q, tie);
      dt += b - ((q + M) - M);
      nt += tie ? 1.0 : 0.0;
      T.row(tie, xf_odd(b));
    }
    t += dt;
    a += 2.0 * nt;  // a tie's final step is b or b + 1, and |b| <= |rint(q)| + 1
  }
}

// one block, value (j, lane) at row j * 64 + lane of the block; every lane
// returns the same s; lds: 64 * WX_XF_J doubles of this wave
__device__ __forceinline__ double xf_block(double s, const float (&x)[WX_XF_J], double *lds) {
  const double as = __builtin_fabs(s);
  if (as >= 0x1p-900 && as < 0x1p1000) {  // wave-uniform; 0, tiny, huge, NaN, Inf: the slow path
    const int k = __builtin_amdgcn_frexp_exp(s) - 1;  // |s| in [2^k, 2^(k+1))
    double t, a;
    bool ok;
    XfTies T;
    xf_sums(k, x, t, a, ok, T);
    if (ok) {
      t = wave_total_f64(t);
      a = wave_total_f64(a);
      const double S = __builtin_ldexp(s, 52 - k);  // the integer s / u, |S| in [2^52, 2^53)
      const bool fits = s > 0.0 ? (S - a > 0x1p52 && S + a < 0x1p53) : (S + a < -0x1p52 && S - a > -0x1p53);
      if (fits) return __builtin_ldexp(T.apply(S, t + T.adj), k - 52);
    }
  }
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < WX_XF_J; ++j) lds[j * 64 + lane] = (double)x[j];
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): one wave, LDS in order
  __builtin_amdgcn_wave_barrier();
  for (int i = 0; i < WX_XF_B; i += 16) {
    double d[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) d[q] = lds[i + q];
#pragma unroll
    for (int q = 0; q < 16; ++q) s += d[q];
  }
  __builtin_amdgcn_wave_barrier();  // every lane's reads done before the next block's writes
  return s;
}

// v[i] for i < c, else +0.0 (padding), without a branch: the load always
// issues, at a clamped index (c >= 1)
__device__ __forceinline__ float xf_load(const float *v, wx_i64 i, wx_i64 c) {
  const float x = v[i < c ? i : c - 1];
  return i < c ? x : 0.0f;
}

// s = ((s0 + v[0]) + v[1]) + ... + v[c - 1] in double, bit for bit; one wave.
// Blocks go WX_XF_AHEAD at a time: their sums are formed together under the
// binade of the running sum at the group's start (independent reductions the
// scheduler interleaves, off the chain), then applied in order, each after
// checking that the running sum is still in that binade and the block fits;
// a block that does not is folded by xf_block from the exact running sum.
// A block past the end is padded with +0.0, which leaves any running sum
// unchanged (it starts at +0.0, so it is never -0.0).
__device__ __forceinline__ double fold_exact(const float *v, wx_i64 c, double *lds, double s0 = 0.0) {
  if (c <= 0) return s0;
  const int lane = threadIdx.x & 63;
  constexpr int D = WX_XF_AHEAD;
  const wx_i64 nb = (c + WX_XF_B - 1) / WX_XF_B;
  float xr[D][WX_XF_J];
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int j = 0; j < WX_XF_J; ++j) {
      const wx_i64 i = (wx_i64)d * WX_XF_B + j * 64 + lane;
      xr[d][j] = xf_load(v, i, c);
    }
  double s = s0;  // +0.0 for a whole group; a running sum is never -0.0 (it starts at +0.0)
  for (wx_i64 b0 = 0; b0 < nb; b0 += D) {
    // this group's values out of the ring, the next group's loads out
    float xc[D][WX_XF_J];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int j = 0; j < WX_XF_J; ++j) {
        xc[d][j] = xr[d][j];
        const wx_i64 i = (b0 + D + d) * WX_XF_B + j * 64 + lane;
        xr[d][j] = xf_load(v, i, c);
      }
    const double as0 = __builtin_fabs(s);
    const bool sok = as0 >= 0x1p-900 && as0 < 0x1p1000;  // wave-uniform
    const int k = sok ? __builtin_amdgcn_frexp_exp(s) - 1 : 0;
    double t[D], a[D];
    bool ok[D];
    XfTies T[D];
#pragma unroll
    for (int d = 0; d < D; ++d) xf_sums(k, xc[d], t[d], a[d], ok[d], T[d]);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      t[d] = wave_total_f64(t[d]) + T[d].adj;
      a[d] = wave_total_f64(a[d]);
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if (b0 + d >= nb) break;  // wave-uniform
      const double as = __builtin_fabs(s);
      bool done = false;
      if (sok && ok[d] && as >= 0x1p-900 && __builtin_amdgcn_frexp_exp(s) - 1 == k) {
        const double S = __builtin_ldexp(s, 52 - k);
        const bool fits =
            s > 0.0 ? (S - a[d] > 0x1p52 && S + a[d] < 0x1p53) : (S + a[d] < -0x1p52 && S - a[d] > -0x1p53);
        if (fits) {
          s = __builtin_ldexp(T[d].apply(S, t[d]), k - 52);
          done = true;
        }
      }
      if (!done) s = xf_block(s, xc[d], lds);
    }
  }
  return s;
}
}  // namespace wx

// ---------------------------------------------------------------------------
// Groups of more than WX_XF_BIG rows: one wave per group would stream the
// whole segment alone (≈ 4 GB/s), so the segment is cut into WX_XF_CHUNK-value
// chunks.  (1) every chunk's sum in any order (an approximation of the
// running sum where each chunk starts); (2) each chunk but the first forms
// its exact integer sums under the binade of that approximate start (q = v *
// 2^(52 - k), |q| < 2^33 so a chunk's sums stay exact doubles; ties by
// XfTies); (3) one wave per group applies the chunks in order: a chunk whose
// guessed binade is the exact running sum's and whose states provably stay
// in it (S -+ sum |r| strictly inside (2^52, 2^53)) adds u * sum r; any
// other chunk (the first; the binade crossings, ≈ one per doubling of the
// sum) is folded by fold_exact from the exact running sum.  The result
// is the dependent chain's, bit for bit.
__device__ __forceinline__ int wx_xf_entry(const WxXfBigArgs &a, wx_i64 chunk) {
  int lo = 0, hi = a.n_ent - 1;  // the last entry whose first chunk is <= chunk
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (a.ent[4 * mid + 3] <= chunk) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// A chunk's values stream through a wave 16 loads per lane at a time (a
// single-wave loop with one load in flight runs at memory latency).
#define WX_XF_U 16
extern "C" __global__ __launch_bounds__(64) void wx_xf_big_approx(WxXfBigArgs a) {
  const int lane = threadIdx.x;
  for (wx_i64 chunk = blockIdx.x; chunk < a.n_chunks; chunk += gridDim.x) {
    const int e = wx_xf_entry(a, chunk);
    const wx_i64 j = chunk - a.ent[4 * e + 3], count = a.ent[4 * e + 2];
    const wx_i64 b = j * WX_XF_CHUNK, len = count - b < WX_XF_CHUNK ? count - b : WX_XF_CHUNK;
    const float *v = a.svals + a.ent[4 * e + 1] + b;
    double acc = 0.0;
    for (wx_i64 i0 = 0; i0 < len; i0 += 64 * WX_XF_U) {
      float x[WX_XF_U];
#pragma unroll
      for (int u = 0; u < WX_XF_U; ++u) x[u] = wx::xf_load(v, i0 + 64 * u + lane, len);
#pragma unroll
      for (int u = 0; u < WX_XF_U; ++u) acc += (double)x[u];
    }
    const double t = wx::wave_total_f64(acc);
    if (lane == 0) a.approx[chunk] = t;
  }
}

extern "C" __global__ __launch_bounds__(64) void wx_xf_big_exact(WxXfBigArgs a) {
  const int lane = threadIdx.x;
  for (wx_i64 chunk = blockIdx.x; chunk < a.n_chunks; chunk += gridDim.x) {
    const int e = wx_xf_entry(a, chunk);
    const wx_i64 first = a.ent[4 * e + 3], j = chunk - first, count = a.ent[4 * e + 2];
    if (j == 0) {  // the group's first chunk starts at 0: always folded by the combine
      if (lane == 0) a.rec[8 * chunk + 3] = 0.0;
      continue;
    }
    double p = 0.0;  // the approximate running sum where this chunk starts
    for (wx_i64 i = lane; i < j; i += 64) p += a.approx[first + i];
    p = wx::wave_total_f64(p);
    const double ap = __builtin_fabs(p);
    const bool pok = ap >= 0x1p-900 && ap < 0x1p1000;  // wave-uniform; also false for NaN / Inf
    const int k = pok ? __builtin_amdgcn_frexp_exp(p) - 1 : 0;
    const double p2 = __builtin_ldexp(1.0, 52 - k);
    const wx_i64 b = j * WX_XF_CHUNK, len = count - b < WX_XF_CHUNK ? count - b : WX_XF_CHUNK;
    const float *v = a.svals + a.ent[4 * e + 1] + b;
    bool lok = pok;
    double t = 0.0, s_abs = 0.0;
    wx::XfTies T;  // the chunk's ties in row order (row u of an iteration = values i0 + 64 u ..)
    for (wx_i64 i0 = 0; i0 < len && pok; i0 += 64 * WX_XF_U) {
      float x[WX_XF_U];
#pragma unroll
      for (int u = 0; u < WX_XF_U; ++u) x[u] = wx::xf_load(v, i0 + 64 * u + lane, len);  // past len: +0.0
#pragma unroll
      for (int u = 0; u < WX_XF_U; ++u) {
        const double q = (double)x[u] * p2;
        bool tie;
        const double b = wx::xf_b(q, tie);
        lok = lok && __builtin_fabs(q) < 0x1p33;
        t += b;
        s_abs += __builtin_fabs(b) + (tie ? 1.0 : 0.0);
        T.row(tie, wx::xf_odd(b));
      }
    }
    const bool ok = __builtin_amdgcn_ballot_w64(!lok) == 0ull;
    t = wx::wave_total_f64(t);
    s_abs = wx::wave_total_f64(s_abs);
    if (lane == 0) {
      double *r = a.rec + 8 * chunk;
      r[0] = (double)k;
      r[1] = t + T.adj;  // + p_in ^ cf when the chunk has a tie (r[4], r[5])
      r[2] = s_abs;
      r[3] = ok ? 1.0 : 0.0;
      r[4] = (double)T.has;
      r[5] = (double)T.cf;
    }
  }
}

// the chunk records are read 64 at a time (lane l: chunk j0 + l) and taken
// from the lanes in order, so the walk over a group's chunks waits on memory
// once per 64 chunks
__device__ __forceinline__ double wx_xf_lane(double v, int l) {
  const wx_u64 u = __double_as_longlong(v);
  const wx_u32 lo = (wx_u32)__builtin_amdgcn_readlane((int)(wx_u32)u, l);
  const wx_u32 hi = (wx_u32)__builtin_amdgcn_readlane((int)(wx_u32)(u >> 32), l);
  return __longlong_as_double((long long)(((wx_u64)hi << 32) | lo));
}

extern "C" __global__ __launch_bounds__(64) void wx_xf_big_combine(WxXfBigArgs a) {
  __shared__ double s_xf[WX_XF_B];
  const int lane = threadIdx.x;
  for (int e = blockIdx.x; e < a.n_ent; e += gridDim.x) {
    const wx_i64 g = a.ent[4 * e], start = a.ent[4 * e + 1], count = a.ent[4 * e + 2], first = a.ent[4 * e + 3];
    const wx_i64 nch = (count + WX_XF_CHUNK - 1) / WX_XF_CHUNK;
    double s = 0.0;
    for (wx_i64 j0 = 0; j0 < nch; j0 += 64) {
      double rk = 0.0, rt = 0.0, ra = 0.0, rok = 0.0, rhas = 0.0, rcf = 0.0;
      if (j0 + lane < nch) {
        const double *r = a.rec + 8 * (first + j0 + lane);
        rk = r[0];
        rt = r[1];
        ra = r[2];
        rok = r[3];
        rhas = r[4];
        rcf = r[5];
      }
      const int nl = nch - j0 < 64 ? (int)(nch - j0) : 64;
      for (int l = 0; l < nl; ++l) {
        const wx_i64 j = j0 + l;
        const wx_i64 b = j * WX_XF_CHUNK, len = count - b < WX_XF_CHUNK ? count - b : WX_XF_CHUNK;
        if (j > 0 && wx_xf_lane(rok, l) != 0.0) {
          const double as = __builtin_fabs(s);
          const int k = (int)wx_xf_lane(rk, l);
          if (as >= 0x1p-900 && as < 0x1p1000 && __builtin_amdgcn_frexp_exp(s) - 1 == k) {
            const double S = __builtin_ldexp(s, 52 - k), A = wx_xf_lane(ra, l);
            const bool fits =
                s > 0.0 ? (S - A > 0x1p52 && S + A < 0x1p53) : (S + A < -0x1p52 && S - A > -0x1p53);
            if (fits) {
              double R = wx_xf_lane(rt, l);
              if (wx_xf_lane(rhas, l) != 0.0) {  // the chunk's first tie: + (S's parity ^ cf)
                const double h = S * 0.5;
                const wx_u32 p_in = h != __builtin_floor(h) ? 1u : 0u;
                R += (double)(p_in ^ (wx_u32)wx_xf_lane(rcf, l));
              }
              s = __builtin_ldexp(S + R, k - 52);
              continue;
            }
          }
        }
        s = wx::fold_exact(a.svals + start + b, len, s_xf, s);
      }
    }
    if (lane == 0) a.out_sums[g] = s;
    __builtin_amdgcn_wave_barrier();
  }
}

// Row-order GROUP BY sums, general path (WX_F_ROW_ORDER, warpexec.cpp
// do_group_sum_rows): the passing rows sorted by key, row order kept within
// a key, so group g's rows are [starts[g], starts[g] + count[g]) -- the
// counts' exclusive prefix, since the groups come in ascending key order and
// the sorted array holds exactly their rows (wx_group_starts_* form it and
// check that the counts add up to the rows).  Then each group's values are
// folded in ascending row order -- the reference's std::map fold
// (src/warpdb.cpp:373-385: `g.sum += val`) to the bit -- small groups one
// lane each (wx_group_fold_small), the rest one wave each (wx_group_fold),
// groups above skip_above in chunks (wx_xf_big_*).  (Before round 6 each
// wave found its group's first row by a binary search of the sorted keys:
// 30 dependent loads per group, 9.1 ms of the 33.6-ms query at 10^6 keys.)

// exclusive prefix over a workgroup of WX_GS_BLOCK threads (s_w: one word
// per wave); the total in tot
__device__ __forceinline__ wx_i64 wx_gs_block_excl(wx_i64 v, wx_i64 *s_w, wx_i64 &tot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  wx_i64 incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const wx_i64 t = __shfl_up(incl, o);
    if (lane >= o) incl += t;
  }
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  wx_i64 wb = 0;
  tot = 0;
#pragma unroll
  for (int w = 0; w < WX_GS_BLOCK / 64; ++w) {
    const wx_i64 x = s_w[w];
    wb += w < wave ? x : 0;
    tot += x;
  }
  __syncthreads();  // s_w reusable
  return wb + incl - v;
}

// (1) chunk b's count total: groups [b * WX_GS_CHUNK, ...), WX_GS_PER per thread
extern "C" __global__ __launch_bounds__(WX_GS_BLOCK) void wx_group_starts_sum(WxGroupFoldArgs a) {
  __shared__ wx_i64 s_w[WX_GS_BLOCK / 64];
  const wx_i64 g0 = (wx_i64)blockIdx.x * WX_GS_CHUNK + (wx_i64)threadIdx.x * WX_GS_PER;
  wx_i64 v = 0;
#pragma unroll
  for (int k = 0; k < WX_GS_PER; ++k)
    if (g0 + k < a.n_groups) v += a.gcounts[g0 + k];
  wx_i64 tot;
  wx_gs_block_excl(v, s_w, tot);
  if (threadIdx.x == 0) a.chunk_sums[blockIdx.x] = tot;
}

// (2) the chunk totals' exclusive prefix, in place (one 1024-thread
// workgroup, 1024 chunks per round); the rows must add up to m
extern "C" __global__ __launch_bounds__(1024) void wx_group_starts_scan(WxGroupFoldArgs a) {
  __shared__ wx_i64 s_w[16];
  __shared__ wx_i64 s_carry;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s_carry = 0;
  __syncthreads();
  for (wx_i64 base = 0; base < a.n_chunks; base += 1024) {
    const wx_i64 i = base + tid;
    const wx_i64 v = i < a.n_chunks ? a.chunk_sums[i] : 0;
    wx_i64 incl = v;
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
    const wx_i64 carry = s_carry;
    if (i < a.n_chunks) a.chunk_sums[i] = carry + wb + incl - v;
    __syncthreads();
    if (tid == 0) s_carry = carry + tot;
    __syncthreads();
  }
  if (tid == 0 && s_carry != a.m) {  // the counts do not cover the sorted rows exactly
    atomicOr(reinterpret_cast<unsigned int *>(&a.ctrs[1]), WX_DEVERR_INTERNAL_KEY);
  }
}

// (3) every group's first row: chunk prefix + the prefix inside the chunk
extern "C" __global__ __launch_bounds__(WX_GS_BLOCK) void wx_group_starts_emit(WxGroupFoldArgs a) {
  __shared__ wx_i64 s_w[WX_GS_BLOCK / 64];
  const wx_i64 g0 = (wx_i64)blockIdx.x * WX_GS_CHUNK + (wx_i64)threadIdx.x * WX_GS_PER;
  wx_i64 c[WX_GS_PER], v = 0;
#pragma unroll
  for (int k = 0; k < WX_GS_PER; ++k) {
    c[k] = g0 + k < a.n_groups ? a.gcounts[g0 + k] : 0;
    v += c[k];
  }
  wx_i64 tot;
  wx_i64 p = a.chunk_sums[blockIdx.x] + wx_gs_block_excl(v, s_w, tot);
#pragma unroll
  for (int k = 0; k < WX_GS_PER; ++k) {
    if (g0 + k < a.n_groups) a.starts[g0 + k] = p;
    p += c[k];
  }
}

// (4) one lane per group of at most small_max rows: the plain sequential
// fold, eight values loaded ahead of their adds; a larger group goes to
// big_list for wx_group_fold.  Every group's first and last sorted key must
// be its key (with the counts adding up to the rows, checked in (2), that
// pins every group's rows).
extern "C" __global__ __launch_bounds__(WX_GS_BLOCK) void wx_group_fold_small(WxGroupFoldArgs a) {
  const wx_i64 g = (wx_i64)blockIdx.x * WX_GS_BLOCK + threadIdx.x;
  if (g >= a.n_groups) return;
  const wx_i64 c = a.gcounts[g], lo = a.starts[g];
  if (c > a.small_max) {
    a.big_list[atomicAdd(a.big_n, 1u)] = g;
    return;
  }
  const int key = a.gkeys[g];
  if (c < 1 || lo < 0 || lo + c > a.m || a.skeys[lo] != key || a.skeys[lo + c - 1] != key) {
    atomicOr(reinterpret_cast<unsigned int *>(&a.ctrs[1]), WX_DEVERR_INTERNAL_KEY);
    a.out_sums[g] = 0.0;
    return;
  }
  // the lanes' groups lie apart, so each load instruction touches 64 lines:
  // 16-B loads (after up to three values to a 16-B boundary) need a quarter
  // of the instructions that 4-B loads do
  typedef float f4 __attribute__((ext_vector_type(4)));
  const float *v = a.svals + lo;
  double s = 0.0;
  const wx_i64 head = c < (wx_i64)((4u - ((wx_u32)(reinterpret_cast<wx_u64>(v) >> 2) & 3u)) & 3u)
                          ? c
                          : (wx_i64)((4u - ((wx_u32)(reinterpret_cast<wx_u64>(v) >> 2) & 3u)) & 3u);
  wx_i64 i = 0;
  for (; i < head; ++i) s += (double)v[i];
  // 16 values per step, the next step's four loads issued before this
  // step's adds (two steps in flight)
  if (i + 16 <= c) {
    f4 n[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) n[q] = *reinterpret_cast<const f4 *>(v + i + 4 * q);
    for (;;) {
      const f4 x[4] = {n[0], n[1], n[2], n[3]};
      const bool more = i + 32 <= c;
      if (more) {
#pragma unroll
        for (int q = 0; q < 4; ++q) n[q] = *reinterpret_cast<const f4 *>(v + i + 16 + 4 * q);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s += (double)x[q].x;
        s += (double)x[q].y;
        s += (double)x[q].z;
        s += (double)x[q].w;
      }
      i += 16;
      if (!more) break;
    }
  }
  for (; i < c; ++i) s += (double)v[i];
  a.out_sums[g] = s;
}

// Run-length encoding of the sorted keys (the general path's groups when
// no ordinary call ran): a run starts at row i when i == 0 or the key
// differs from row i - 1's.  Every wave walks its own range in 64-row
// chunks, WX_RLE_U of them in flight: no barriers.
#define WX_RLE_U 8
// the head flags of rows c + u * 64 + lane, u < WX_RLE_U (rows >= e: none)
__device__ __forceinline__ void wx_rle_heads(const WxRleArgs &a, wx_i64 c, wx_i64 e, bool (&h)[WX_RLE_U]) {
  const int lane = threadIdx.x & 63;
  int k[WX_RLE_U], p[WX_RLE_U];
#pragma unroll
  for (int u = 0; u < WX_RLE_U; ++u) {
    const wx_i64 i = c + u * 64 + lane;
    k[u] = i < e ? a.sk[i] : 0;
    // lane 0's predecessor is the previous chunk's lane 63 (row i - 1)
    p[u] = lane == 0 && i > 0 && i < e ? a.sk[i - 1] : 0;
  }
#pragma unroll
  for (int u = 0; u < WX_RLE_U; ++u) {
    const wx_i64 i = c + u * 64 + lane;
    const int prev = __shfl_up(k[u], 1);
    h[u] = i < e && (i == 0 || k[u] != (lane == 0 ? p[u] : prev));
  }
}

// (R1) the runs starting in each wave's rows
extern "C" __global__ __launch_bounds__(WX_RLE_BLOCK) void wx_rle_count(WxRleArgs a) {
  const wx_i64 r = (wx_i64)blockIdx.x * (WX_RLE_BLOCK / 64) + (threadIdx.x >> 6);
  if (r >= a.n_blk) return;  // wave-uniform
  const wx_i64 b0 = r * a.span, b1 = b0 + a.span < a.m ? b0 + a.span : a.m;
  wx_i64 n = 0;
  for (wx_i64 c = b0; c < b1; c += 64 * WX_RLE_U) {
    bool h[WX_RLE_U];
    wx_rle_heads(a, c, b1, h);
#pragma unroll
    for (int u = 0; u < WX_RLE_U; ++u) n += __builtin_popcountll(__builtin_amdgcn_ballot_w64(h[u]));
  }
  if ((threadIdx.x & 63) == 0) a.blk[r] = n;
}

// (R2) their exclusive prefix (one workgroup, WX_RLE_BLOCK ranges per round) and the total
extern "C" __global__ __launch_bounds__(WX_RLE_BLOCK) void wx_rle_scan(WxRleArgs a) {
  __shared__ wx_i64 s_w[WX_RLE_BLOCK / 64];
  __shared__ wx_i64 s_carry;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s_carry = 0;
  __syncthreads();
  for (wx_i64 base = 0; base < a.n_blk; base += WX_RLE_BLOCK) {  // workgroup-uniform
    const wx_i64 i = base + tid;
    const wx_i64 v = i < a.n_blk ? a.blk[i] : 0;
    wx_i64 incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const wx_i64 t = __shfl_up(incl, o);
      if (lane >= o) incl += t;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    wx_i64 wb = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < WX_RLE_BLOCK / 64; ++w) {
      const wx_i64 x = s_w[w];
      wb += w < wave ? x : 0;
      tot += x;
    }
    const wx_i64 carry = s_carry;
    if (i < a.n_blk) a.blk[i] = carry + wb + incl - v;
    __syncthreads();  // s_w and s_carry read
    if (tid == 0) s_carry = carry + tot;
    __syncthreads();
  }
  if (tid == 0) {
    a.n_out[0] = s_carry;
    if (a.n_groups_out) a.n_groups_out[0] = s_carry;
  }
}

// (R3) each run's key and first row, in order (runs past capacity not written)
extern "C" __global__ __launch_bounds__(WX_RLE_BLOCK) void wx_rle_emit(WxRleArgs a) {
  const wx_i64 r = (wx_i64)blockIdx.x * (WX_RLE_BLOCK / 64) + (threadIdx.x >> 6);
  if (r >= a.n_blk) return;  // wave-uniform
  const wx_i64 b0 = r * a.span, b1 = b0 + a.span < a.m ? b0 + a.span : a.m;
  wx_i64 base = a.blk[r];
  for (wx_i64 c = b0; c < b1; c += 64 * WX_RLE_U) {
    bool h[WX_RLE_U];
    wx_rle_heads(a, c, b1, h);
#pragma unroll
    for (int u = 0; u < WX_RLE_U; ++u) {
      const wx_u64 m = __builtin_amdgcn_ballot_w64(h[u]);
      if (h[u]) {
        const wx_i64 q = base + (wx_i64)::wx::lanes_below(m), i = c + u * 64 + (threadIdx.x & 63);
        if (q < a.capacity) {
          a.out_keys[q] = a.sk[i];
          a.starts[q] = i;
        }
      }
      base += __builtin_popcountll(m);
    }
  }
}

// (R4) each run's length: the next run's first row (or m) minus its own
extern "C" __global__ __launch_bounds__(WX_GS_BLOCK) void wx_rle_counts(WxRleArgs a) {
  const wx_i64 ng = a.n_out[0], r = (wx_i64)blockIdx.x * WX_GS_BLOCK + threadIdx.x;
  if (r >= ng || r >= a.capacity) return;
  a.out_counts[r] = (r + 1 < ng ? a.starts[r + 1] : a.m) - a.starts[r];
}

// (5) one wave per group of big_list (every group when big_list is null),
// by wx::fold_exact; with WX_FOLD_EXACT=0 the lanes stream the group's
// values (coalesced, WX_FOLD_U chunks of 64 in flight) and the chain runs
// over them in lane order (LDS broadcasts, or v_readlane with
// WX_FOLD_LDS=0), so every lane holds the same running sum.
// A chunk past the group's end is padded with +0.0, which leaves any running
// sum unchanged (the sum starts at +0.0, so it is never -0.0).  1e9 rows x
// 1024 keys: 11.4 ms through LDS broadcasts (about 11 ns per dependent
// double add: the chain itself), 12.1 ms with v_readlane per value, 17 ms
// with every lane widened first and two readlanes per add.
#ifndef WX_FOLD_U
#define WX_FOLD_U 8
#endif
#ifndef WX_FOLD_LDS
#define WX_FOLD_LDS 1
#endif
extern "C" __global__ __launch_bounds__(64) void wx_group_fold(WxGroupFoldArgs a) {
  const int lane = threadIdx.x;
  __shared__ double s_fold[64];
  const wx_i64 n_items = a.big_list ? (wx_i64)*a.big_n : a.n_groups;
  for (wx_i64 it = blockIdx.x; it < n_items; it += gridDim.x) {
    const wx_i64 g = a.big_list ? a.big_list[it] : it;
    const int key = a.gkeys[g];
    const wx_i64 c = a.gcounts[g], lo = a.starts[g];
    if (c < 1 || lo < 0 || lo + c > a.m || a.skeys[lo] != key || a.skeys[lo + c - 1] != key) {
      if (lane == 0) {
        atomicOr(reinterpret_cast<unsigned int *>(&a.ctrs[1]), WX_DEVERR_INTERNAL_KEY);
        a.out_sums[g] = 0.0;
      }
      continue;
    }
    const float *v = a.svals + lo;
    if (a.skip_above > 0 && c > a.skip_above) continue;  // wx_xf_big_* (its count was checked above)
#if WX_FOLD_EXACT
    {
      __shared__ double s_xf[WX_XF_B];
      const double xs = wx::fold_exact(v, c, s_xf);
      if (lane == 0) a.out_sums[g] = xs;
      __builtin_amdgcn_wave_barrier();
      continue;
    }
#endif
    double s = 0.0;
    for (wx_i64 base = 0; base < c; base += 64 * WX_FOLD_U) {
      wx_u32 x[WX_FOLD_U];
#pragma unroll
      for (int u = 0; u < WX_FOLD_U; ++u) {
        const wx_i64 i = base + u * 64 + lane;
        x[u] = i < c ? __float_as_uint(v[i]) : 0u;
      }
#pragma unroll
      for (int u = 0; u < WX_FOLD_U; ++u) {
        if (base + u * 64 >= c) break;  // wave-uniform
#if WX_FOLD_LDS
        // the wave's 64 values widened into LDS, then read back by every lane
        // (same address: a broadcast), 16 at a time, ahead of their adds --
        // only the adds are on the chain, with no SGPR hand-off per value
        s_fold[lane] = (double)__uint_as_float(x[u]);
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): one wave, LDS in order
#pragma unroll
        for (int jb = 0; jb < 64; jb += 16) {
          double d[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) d[q] = s_fold[jb + q];
#pragma unroll
          for (int q = 0; q < 16; ++q) s += d[q];
        }
#else
#pragma unroll
        for (int j = 0; j < 64; ++j) s += (double)__uint_as_float(__builtin_amdgcn_readlane(x[u], j));
#endif
      }
    }
    if (lane == 0) a.out_sums[g] = s;
  }
}

// ORDER BY .. LIMIT heads of any length (the k > 32 form of the top-K
// record, wx_order_head / wx_head_merge in warpexec.cpp): positions to carry
// through the stable key sort, then the sorted head gathered into a record;
// across shards the records' candidates concatenated in record order, sorted
// the same way, and the global head emitted.
#define WX_HEAD_KEYS(rec) reinterpret_cast<const float *>((rec) + 8)
#define WX_HEAD_VALS(rec, cap) reinterpret_cast<const float *>((rec) + 8 + 4 * (cap))
#define WX_HEAD_ROWS(rec, cap) reinterpret_cast<const wx_i64 *>((rec) + 8 + 8 * (cap))
extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_iota(WxHeadArgs a) {
  for (wx_i64 i = (wx_i64)blockIdx.x * WX_BLOCK + threadIdx.x; i < a.n; i += (wx_i64)gridDim.x * WX_BLOCK)
    a.idx[i] = (wx_u32)i;
}

extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_head_gather(WxHeadArgs a) {
  const wx_i64 c = *a.count, m = c < a.limit ? c : a.limit;
  float *k = reinterpret_cast<float *>(a.record + 8);
  float *v = k + a.cap;
  wx_i64 *r = reinterpret_cast<wx_i64 *>(a.record + 8 + 8 * a.cap);
  for (wx_i64 j = (wx_i64)blockIdx.x * WX_BLOCK + threadIdx.x; j < m; j += (wx_i64)gridDim.x * WX_BLOCK) {
    const wx_u32 p = a.idx[j];
    k[j] = a.keys[j];
    v[j] = a.vals ? a.vals[p] : a.keys[j];
    r[j] = a.row_base + (wx_i64)a.rows[p];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *reinterpret_cast<wx_i64 *>(a.record) = m;
}

// one workgroup: the records' valid candidates, record after record
extern "C" __global__ __launch_bounds__(1024) void wx_head_concat(WxHeadArgs a) {
  __shared__ wx_i64 s_off[1025];
  const int tid = threadIdx.x;
  if (tid == 0) {
    wx_i64 o = 0;
    for (int r = 0; r < a.n_records; ++r) {
      s_off[r] = o;
      wx_i64 c = *reinterpret_cast<const wx_i64 *>(a.records + (wx_i64)r * (8 + 16 * a.cap));
      c = c < 0 ? 0 : (c > a.cap ? a.cap : c);  // a bad count reads as empty / full
      o += c;
    }
    s_off[a.n_records] = o;
    *a.cat_count = o;
  }
  __syncthreads();
  for (int r = 0; r < a.n_records; ++r) {
    const unsigned char *rec = a.records + (wx_i64)r * (8 + 16 * a.cap);
    const wx_i64 o = s_off[r], c = s_off[r + 1] - o;
    for (wx_i64 j = tid; j < c; j += 1024) {
      a.cat_keys[o + j] = WX_HEAD_KEYS(rec)[j];
      a.cat_idx[o + j] = (wx_u32)((wx_i64)r * a.cap + j);
    }
  }
}

extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_head_emit(WxHeadArgs a) {
  const wx_i64 c = *a.count, m = c < a.limit ? c : a.limit;
  for (wx_i64 j = (wx_i64)blockIdx.x * WX_BLOCK + threadIdx.x; j < m; j += (wx_i64)gridDim.x * WX_BLOCK) {
    const wx_u32 p = a.idx[j];
    const wx_i64 r = (wx_i64)p / a.cap, q = (wx_i64)p % a.cap;
    const unsigned char *rec = a.records + r * (8 + 16 * a.cap);
    if (a.out_keys) a.out_keys[j] = a.keys[j];
    if (a.out_vals) a.out_vals[j] = WX_HEAD_VALS(rec, a.cap)[q];
    if (a.out_rows) a.out_rows[j] = WX_HEAD_ROWS(rec, a.cap)[q];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.count_out) *a.count_out = m;
}

// kind 0: float values, kind 1: int keys.  Descending order inverts the rank
// but not the position, so equal keys keep their input order (stable).
extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_sort_prep(WxSortPrepArgs a) {
  const wx_i64 stride = (wx_i64)gridDim.x * WX_BLOCK;
  for (wx_i64 i = (wx_i64)blockIdx.x * WX_BLOCK + threadIdx.x; i < a.npad; i += stride) {
    wx_u64 e = ~0ull;
    if (i < a.n) {
      wx_u32 r;
      if (a.kind == 0) {
        const float f = static_cast<const float *>(a.src)[i];
        r = wx::f2ord(f);
        if (r == 0u) r = 0xffffffffu;    // NaN sorts last either way
        else if (!a.ascending) r = ~r;   // 0x007fffff..0x7ffffffe
      } else {
        r = (wx_u32)static_cast<const int *>(a.src)[i] ^ 0x80000000u;
        if (!a.ascending) r = ~r;
      }
      e = ((wx_u64)r << 32) | (wx_u32)i;
    }
    a.keys[i] = e;
  }
}

// LDS bitonic steps on one WX_SORT_LDS-element slice per block: for every
// stage k in [a.k, a.j] (a.j = kend) run all partner distances below
// WX_SORT_LDS.  The first launch covers k = 2 .. WX_SORT_LDS; afterwards each
// larger stage runs its long distances globally and finishes here.
extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_bitonic_lds(WxSortPassArgs a) {
  __shared__ wx_u64 s[WX_SORT_LDS];
  const wx_i64 base = (wx_i64)blockIdx.x * WX_SORT_LDS;
  for (int i = threadIdx.x; i < WX_SORT_LDS; i += WX_BLOCK) s[i] = a.keys[base + i];
  __syncthreads();
  for (wx_i64 k = a.k; k <= a.j; k <<= 1) {
    wx_i64 j = k >> 1;
    if (j >= WX_SORT_LDS) j = WX_SORT_LDS >> 1;
    for (; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < WX_SORT_LDS; i += WX_BLOCK) {
        const int p = i ^ (int)j;
        if (p > i) {
          const wx_u64 x = s[i], y = s[p];
          const bool up = ((base + i) & k) == 0;
          if ((x > y) == up) { s[i] = y; s[p] = x; }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < WX_SORT_LDS; i += WX_BLOCK) a.keys[base + i] = s[i];
}

extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_bitonic_global(WxSortPassArgs a) {
  const wx_i64 stride = (wx_i64)gridDim.x * WX_BLOCK;
  for (wx_i64 i = (wx_i64)blockIdx.x * WX_BLOCK + threadIdx.x; i < a.npad; i += stride) {
    const wx_i64 p = i ^ a.j;
    if (p > i) {
      const wx_u64 x = a.keys[i], y = a.keys[p];
      const bool up = (i & a.k) == 0;
      if ((x > y) == up) { a.keys[i] = y; a.keys[p] = x; }
    }
  }
}

// Apply the permutation: dst[r] = src[pos(keys[r])] for 4-byte payloads
// (float values, or int keys plus float values).
extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_sort_apply(WxSortApplyArgs a) {
  const wx_i64 stride = (wx_i64)gridDim.x * WX_BLOCK;
  for (wx_i64 r = (wx_i64)blockIdx.x * WX_BLOCK + threadIdx.x; r < a.n; r += stride) {
    const wx_u32 p = (wx_u32)a.keys[r];
    static_cast<wx_u32 *>(a.dst_a)[r] = static_cast<const wx_u32 *>(a.src_a)[p];
    if (a.src_v) a.dst_v[r] = a.src_v[p];
  }
}

#endif  // WX_OP == WX_OP_UTIL
