// wx_sum.hip -- SUM / COUNT / MIN / MAX over one table
// (one of the kernel sources warpexec concatenates after wx_common.hip, whose
// header describes the prelude they expect)

// ===========================================================================
#if WX_OP == WX_OP_SUM
// SUM((float)expr) WHERE cond in double.  Persistent grid-stride pass with
// WX_UNROLL row quads in flight per thread; one partial per block, combined
// in a fixed order by wx_sum_finalize (bitwise reproducible).
#ifndef WX_UNROLL
#define WX_UNROLL 8  // profiles/r01/ablate_stream.txt: 8 quads in flight, 8 workgroups per CU
#endif
#ifndef WX_MINMAX
#define WX_MINMAX 0  // also MIN / MAX of the passing values (NaN skipped)
#endif
namespace wx {
__device__ __forceinline__ wx_u32 wave_min_u32(wx_u32 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const wx_u32 x = __shfl_xor(v, o); v = x < v ? x : v; }
  return v;
}
__device__ __forceinline__ wx_u32 wave_max_u32(wx_u32 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const wx_u32 x = __shfl_xor(v, o); v = x > v ? x : v; }
  return v;
}
// decoded MIN / MAX; an empty set (no non-NaN value) reads as NaN (SQL NULL)
__device__ __forceinline__ float minmax_out(wx_u32 m, bool is_min) {
  return (is_min ? m == 0xffffffffu : m == 0u) ? __uint_as_float(0x7fc00000u) : ord2f(m);
}
}  // namespace wx

extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_reduce_sum(WxSumArgs wx_a) {
  __shared__ double s_sum[WX_WAVES];
  __shared__ wx_i64 s_cnt[WX_WAVES];
  __shared__ wx_u32 s_min[WX_WAVES], s_max[WX_WAVES];
  double wx_acc = 0.0;
  wx_i64 wx_cnt = 0;
  wx_u32 wx_mn = 0xffffffffu, wx_mx = 0u;
  WX_STRIDE_LOOP_BEGIN
  const bool wx_k = idx < wx_a.n_rows && WX_EVAL_COND();
  const float wx_val = static_cast<float>(WX_EXPR);
  wx_acc += wx_k ? (double)wx_val : 0.0;
  wx_cnt += wx_k ? 1 : 0;
  if (WX_MINMAX) {
    const wx_u32 o = wx::f2ord(wx_val);  // NaN -> 0
    const bool in = wx_k && o != 0u;
    wx_mn = (in && o < wx_mn) ? o : wx_mn;
    wx_mx = (in && o > wx_mx) ? o : wx_mx;
  }
  WX_STRIDE_LOOP_END
  double acc = wx::wave_sum_f64(wx_acc);
  wx_i64 cnt = (wx_i64)wx::wave_sum_u64((wx_u64)wx_cnt);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (WX_MINMAX) {
    wx_mn = wx::wave_min_u32(wx_mn);
    wx_mx = wx::wave_max_u32(wx_mx);
  }
  if (lane == 0) { s_sum[wave] = acc; s_cnt[wave] = cnt; s_min[wave] = wx_mn; s_max[wave] = wx_mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    wx_i64 c = 0;
    wx_u32 mn = 0xffffffffu, mx = 0u;
    for (int w = 0; w < WX_WAVES; ++w) {
      s += s_sum[w];
      c += s_cnt[w];
      mn = s_min[w] < mn ? s_min[w] : mn;
      mx = s_max[w] > mx ? s_max[w] : mx;
    }
    wx_a.part_sum[blockIdx.x] = s;
    wx_a.part_cnt[blockIdx.x] = c;
    if (WX_MINMAX) {
      wx_a.part_min[blockIdx.x] = mn;
      wx_a.part_max[blockIdx.x] = mx;
    }
  }
}

// One 1024-thread block combines the per-workgroup partials in a fixed order
// (bitwise reproducible): loads batched four per thread, wave reductions,
// then the sixteen wave results in order.
#define WX_SFIN_BLOCK 1024
extern "C" __global__ __launch_bounds__(WX_SFIN_BLOCK) void wx_sum_finalize(WxSumFinArgs a) {
  __shared__ double s_sum[WX_SFIN_BLOCK / 64];
  __shared__ wx_i64 s_cnt[WX_SFIN_BLOCK / 64];
  __shared__ wx_u32 s_min[WX_SFIN_BLOCK / 64], s_max[WX_SFIN_BLOCK / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double s = 0.0;
  wx_i64 c = 0;
  wx_u32 mn = 0xffffffffu, mx = 0u;
  for (int i0 = tid; i0 < a.n_parts; i0 += WX_SFIN_BLOCK * 4) {
    double ps[4];
    wx_i64 pc[4];
    wx_u32 pmn[4], pmx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = i0 + j * WX_SFIN_BLOCK;
      const bool ok = i < a.n_parts;
      ps[j] = ok ? a.part_sum[i] : 0.0;
      pc[j] = ok ? a.part_cnt[i] : 0;
      pmn[j] = (WX_MINMAX && ok) ? a.part_min[i] : 0xffffffffu;
      pmx[j] = (WX_MINMAX && ok) ? a.part_max[i] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s += ps[j];
      c += pc[j];
      mn = pmn[j] < mn ? pmn[j] : mn;
      mx = pmx[j] > mx ? pmx[j] : mx;
    }
  }
  s = wx::wave_sum_f64(s);
  c = (wx_i64)wx::wave_sum_u64((wx_u64)c);
  if (WX_MINMAX) {
    mn = wx::wave_min_u32(mn);
    mx = wx::wave_max_u32(mx);
  }
  if (lane == 0) {
    s_sum[wave] = s;
    s_cnt[wave] = c;
    s_min[wave] = mn;
    s_max[wave] = mx;
  }
  __syncthreads();
  if (tid == 0) {
    double ts = 0.0;
    wx_i64 tc = 0;
    wx_u32 tmn = 0xffffffffu, tmx = 0u;
    for (int w = 0; w < WX_SFIN_BLOCK / 64; ++w) {
      ts += s_sum[w];
      tc += s_cnt[w];
      tmn = s_min[w] < tmn ? s_min[w] : tmn;
      tmx = s_max[w] > tmx ? s_max[w] : tmx;
    }
    a.out[0] = ts;
    if (a.count_f64) a.out[1] = (double)tc;  // exact below 2^53
    else reinterpret_cast<wx_i64 *>(a.out)[1] = tc;
    if (WX_MINMAX) {
      reinterpret_cast<float *>(a.out)[4] = wx::minmax_out(tmn, true);
      reinterpret_cast<float *>(a.out)[5] = wx::minmax_out(tmx, false);
    }
  }
}
#endif
