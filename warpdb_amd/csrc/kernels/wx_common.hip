// wx_common.hip -- hand-written gfx950 kernel templates for the WarpDB
// execution path.  warpexec prepends custom.cu (src/jit.cpp:65-73) and a
// generated prelude, then compiles the result with hiprtc for the device's
// arch.  The prelude defines:
//   WX_OP          which kernel family to instantiate (see WX_OP_* below)
//   WX_COLS(X)     X(name, c_type, slot) for every column the expressions use
//   WX_EXPR        projection / SUM value / GROUP BY value / ORDER BY key
//   WX_HAS_COND, WX_COND     optional WHERE predicate
//   WX_KEY         GROUP BY key expression
//   WX_HAS_SELECT, WX_SELECT top-K output expression (evaluated by gather)
//   WX_TOPK_K, WX_TOPK_DESC  top-K size and direction
//   WX_ALIGNED16   1 when every column / output pointer is 16-byte aligned
// Expressions are the reference's lowered strings ("price[idx] * 2.0f",
// include/expression.hpp:32-78): a column name is bound either to a register
// value with operator[] (streaming kernels) or to the column pointer (gather).
//
// The design is HBM-streaming: 256-thread workgroups (4 wave64s), 16-byte
// loads per lane (one 1 KiB access per wave-instruction), everything else
// kept in registers / LDS.  MFMA is not used: nothing here is a contraction.

#if !defined(__HIPCC_RTC__)
#include <hip/hip_runtime.h>  // offline hipcc builds; hiprtc provides these itself
#endif

#ifndef WX_ALIGNED16
#define WX_ALIGNED16 0
#endif

// Diagnostic builds.  Every WX_*DIAG* switch of the kernel sources
// (per-phase timestamps; parts of a kernel removed to time the rest, results
// invalid) takes effect only in a build that also sets WX_DIAG=1, e.g.
// WARPDB_EXTRA_DEFINES="WX_DIAG=1,WX_RS_DIAG_PHASES=1": a product build
// cannot enable one by accident.
#ifndef WX_DIAG
#define WX_DIAG 0
#endif
#if !WX_DIAG
#undef WX_DIAG_PROFILE
#undef WX_DIAG_TIMELINE
#undef WX_DIAG_NO_STORE
#undef WX_DIAG_NO_LOOKBACK
#undef WX_DIAG_NO_FLUSH
#undef WX_RS_DIAG_PHASES
#undef WX_RS_DIAG_LBSTATS
#undef WX_RS_DIAG_NO_LOOKBACK
#undef WX_RS_DIAG_NO_RANK
#undef WX_RS_DIAG_NO_STORE
#undef WX_GP_DIAG
#undef WX_GP_AGG_DIAG_NOADD
#undef WX_GP_AGG_DIAG_NOBIN
#define WX_DIAG_PROFILE 0
#define WX_DIAG_TIMELINE 0
#define WX_DIAG_NO_STORE 0
#define WX_DIAG_NO_LOOKBACK 0
#define WX_DIAG_NO_FLUSH 0
#define WX_RS_DIAG_PHASES 0
#define WX_RS_DIAG_LBSTATS 0
#define WX_RS_DIAG_NO_LOOKBACK 0
#define WX_RS_DIAG_NO_RANK 0
#define WX_RS_DIAG_NO_STORE 0
#define WX_GP_DIAG 0
#define WX_GP_AGG_DIAG_NOADD 0
#define WX_GP_AGG_DIAG_NOBIN 0
#endif
#ifndef WX_HAS_COND
#define WX_HAS_COND 0
#endif
#ifndef WX_COLS
#define WX_COLS(X)
#endif

namespace wx {

// A column value bound in registers: `price[idx]` and plain `price` both read it.
template <typename T>
struct reg {
  T v;
  __device__ __forceinline__ T operator[](wx_i64) const { return v; }
  __device__ __forceinline__ operator T() const { return v; }
};

// Streamed table columns are read once: nontemporal loads (measured +10 %
// read bandwidth on gfx950, tools/bw_probe.hip).  Results are written once
// and consumed by a later launch or the host: nontemporal stores optional.
#ifndef WX_NT_LOAD
#define WX_NT_LOAD 1
#endif
#ifndef WX_NT_STORE
#define WX_NT_STORE 0
#endif
template <typename V>
__device__ __forceinline__ V ldv(const V *p) {
#if WX_NT_LOAD
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}
template <typename V>
__device__ __forceinline__ void stv(V *p, V v) {
#if WX_NT_STORE
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
template <bool B>
struct btag {
  static constexpr bool value = B;
};
template <bool NT, typename V>
__device__ __forceinline__ void st_sel(V *p, V v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// Four consecutive rows [r0, r0+4) of one column into registers.  Full,
// aligned groups use 16-byte loads (global_load_dwordx4); the ragged tail
// falls back to guarded scalar loads and zero-fills.
template <typename T>
__device__ __forceinline__ void load4(const void *base, wx_i64 r0, wx_i64 n, T (&o)[4]) {
  const T *p = static_cast<const T *>(base);
  if (WX_ALIGNED16 && r0 + 4 <= n) {
    if constexpr (sizeof(T) == 4) {
      typedef T v4 __attribute__((ext_vector_type(4)));
      const v4 x = ldv(reinterpret_cast<const v4 *>(p + r0));
      o[0] = x.x; o[1] = x.y; o[2] = x.z; o[3] = x.w;
    } else {
      typedef T v2 __attribute__((ext_vector_type(2)));
      const v2 x = ldv(reinterpret_cast<const v2 *>(p + r0));
      const v2 y = ldv(reinterpret_cast<const v2 *>(p + r0 + 2));
      o[0] = x.x; o[1] = x.y; o[2] = y.x; o[3] = y.y;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (r0 + e < n) ? p[r0 + e] : T(0);
  }
}

// Four rows known to be in range and 16-byte aligned: 16-byte loads only.
template <typename T>
__device__ __forceinline__ void load4_full(const void *base, wx_i64 r0, T (&o)[4]) {
  const T *p = static_cast<const T *>(base);
  if constexpr (sizeof(T) == 4) {
    typedef T v4 __attribute__((ext_vector_type(4)));
    const v4 x = ldv(reinterpret_cast<const v4 *>(p + r0));
    o[0] = x.x; o[1] = x.y; o[2] = x.z; o[3] = x.w;
  } else {
    typedef T v2 __attribute__((ext_vector_type(2)));
    const v2 x = ldv(reinterpret_cast<const v2 *>(p + r0));
    const v2 y = ldv(reinterpret_cast<const v2 *>(p + r0 + 2));
    o[0] = x.x; o[1] = x.y; o[2] = y.x; o[3] = y.y;
  }
}

// Guarded scalar loads (ragged tail or unaligned columns); zero past the end.
template <typename T>
__device__ __forceinline__ void load4_tail(const void *base, wx_i64 r0, wx_i64 n, T (&o)[4]) {
  const T *p = static_cast<const T *>(base);
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = (r0 + e < n) ? p[r0 + e] : T(0);
}

__device__ __forceinline__ wx_u64 ld_agent(const wx_u64 *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(wx_u64 *p, wx_u64 v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Look-back abort report (wx_args.h WX_LBD_*): the first aborting waiter of
// a workspace claims the record and fills it; one lane calls this.
__device__ __forceinline__ void lb_report(wx_u64 *lbd, wx_u64 what, wx_u64 tile, wx_u64 pred, wx_u64 word) {
  if (atomicCAS(&lbd[0], 0ull, 1ull) != 0ull) return;
  st_agent(&lbd[1], what);
  st_agent(&lbd[2], tile);
  st_agent(&lbd[3], pred);
  st_agent(&lbd[4], word);
}

__device__ __forceinline__ wx_u32 lanes_below(wx_u64 m) {
  return __builtin_amdgcn_mbcnt_hi((wx_u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((wx_u32)m, 0u));
}

__device__ __forceinline__ wx_u64 wave_sum_u64(wx_u64 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Wave total of a double, every lane the same value: an inclusive DPP scan
// (row shifts, then row broadcasts; no LDS round trips, unlike __shfl_xor's
// ds_bpermute) and lane 63's result read back.  Every lane must be active.
// (Exact for the row-order fold's integer-valued sums, < 2^53, so the add
// order does not matter there.)
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_f64(double v) {
  const wx_u64 u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(wx_u32)u, CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(wx_u32)(u >> 32), CTRL, ROW_MASK, 0xf, false);
  return __longlong_as_double((long long)(((wx_u64)(wx_u32)hi << 32) | (wx_u32)lo));
}
__device__ __forceinline__ double wave_total_f64(double v) {
  v += dpp_f64<0x111, 0xf>(v);  // row_shr:1
  v += dpp_f64<0x112, 0xf>(v);  // row_shr:2
  v += dpp_f64<0x114, 0xf>(v);  // row_shr:4
  v += dpp_f64<0x118, 0xf>(v);  // row_shr:8
  v += dpp_f64<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp_f64<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
  const wx_u64 u = __double_as_longlong(v);
  const wx_u32 lo = (wx_u32)__builtin_amdgcn_readlane((int)(wx_u32)u, 63);
  const wx_u32 hi = (wx_u32)__builtin_amdgcn_readlane((int)(wx_u32)(u >> 32), 63);
  return __longlong_as_double((long long)(((wx_u64)hi << 32) | lo));
}

// Order-preserving float -> u32 map used by the top-K and sort kernels.
// -0.0 is canonicalised to +0.0 (they compare equal on the CPU); NaN maps to
// 0, below every number.
// Integer-only (the float compares cost a canonicalising add and twice the
// selects): NaN -> 0, -0.0 -> +0.0's image, negatives complemented,
// non-negatives with the sign bit set.  Denormals are ordinary values (IEEE
// mode: nothing here is compiled with flush-to-zero).
__device__ __forceinline__ wx_u32 f2ord(float f) {
  const wx_u32 u = __float_as_uint(f);
  const wx_u32 a = u & 0x7fffffffu;
  if (a > 0x7f800000u) return 0u;
  const wx_u32 v = a == 0u ? 0u : u;
  return v ^ ((wx_u32)((int)v >> 31) | 0x80000000u);
}
__device__ __forceinline__ float ord2f(wx_u32 m) {
  if (m == 0u) return __uint_as_float(0x7fc00000u);
  const wx_u32 u = (m & 0x80000000u) ? (m & 0x7fffffffu) : ~m;
  return __uint_as_float(u);
}

}  // namespace wx

// ---------------------------------------------------------------------------
// Expression binding helpers.  Every identifier in the scope of an evaluated
// expression that is not a column carries a wx_ prefix so user column names
// cannot collide with it.
#define WX_DECL_LOAD(name, T, slot) \
  T wx_v##slot[4];                  \
  ::wx::load4<T>(wx_a.col[slot], wx_r0, wx_a.n_rows, wx_v##slot);
#define WX_BIND_REG(name, T, slot) const ::wx::reg<T> name{wx_v##slot[wx_e]};
#define WX_BIND_PTR(name, T, slot) const T *__restrict__ name = static_cast<const T *>(wx_a.col[slot]);
// one row's values (gathered at `idx`), bound like the streamed registers
#define WX_BIND_ROW(name, T, slot) const ::wx::reg<T> name{static_cast<const T *>(wx_a.col[slot])[idx]};

// Grid-stride kernels: per iteration a workgroup owns one contiguous span of
// WX_BLOCK * WX_UNROLL row quads (thread t takes quads t, t + WX_BLOCK, ...
// of the span) and issues all their loads before evaluating any row (a
// data-dependent branch in the evaluation would otherwise stop the compiler
// from batching them).  Contiguous spans keep the chip's loads in flight
// within few DRAM pages: 6.7-6.85 TB/s at any grid size, against 5.6-6.9 for
// quads a whole grid stride apart (tools/bw_probe.hip, read1c vs read1).
#ifndef WX_STRIDE_SIMPLE
#define WX_STRIDE_SIMPLE 0  // diagnostic: guarded loads only
#endif
#define WX_DECL_U(name, T, slot) T wx_u##slot[WX_UNROLL][4];
#define WX_LOAD_U_FAST(name, T, slot) ::wx::load4_full<T>(wx_a.col[slot], wx_r0u, wx_u##slot[wx_u]);
#define WX_LOAD_U(name, T, slot) ::wx::load4_tail<T>(wx_a.col[slot], wx_r0u, wx_a.n_rows, wx_u##slot[wx_u]);
#define WX_BIND_U(name, T, slot) const ::wx::reg<T> name{wx_u##slot[wx_u][wx_e]};
// WX_LBLOCK: the block size of the kernel using the stride loop (WX_BLOCK
// unless a kernel family redefines it around its kernel)
#define WX_LBLOCK WX_BLOCK
#define WX_SPAN ((wx_i64)WX_LBLOCK * WX_UNROLL)
#define WX_QUAD(u) (wx_base + (wx_i64)(u) * WX_LBLOCK + threadIdx.x)
// When the whole span lies inside the table (a workgroup-uniform test) the
// loads are unconditional 16-byte loads; only the last span takes the
// guarded path.
#define WX_STRIDE_LOOP_BEGIN                                                                             \
  const wx_i64 wx_nq = (wx_a.n_rows + 3) >> 2;                                                           \
  const wx_i64 wx_nfull = wx_a.n_rows >> 2;                                                              \
  for (wx_i64 wx_base = (wx_i64)blockIdx.x * WX_SPAN; wx_base < wx_nq;                                   \
       wx_base += (wx_i64)gridDim.x * WX_SPAN) {                                                         \
    WX_COLS(WX_DECL_U)                                                                                   \
    if (WX_ALIGNED16 && !WX_STRIDE_SIMPLE && wx_base + WX_SPAN <= wx_nfull) {                            \
      _Pragma("unroll") for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {                                  \
        const wx_i64 wx_r0u = WX_QUAD(wx_u) << 2;                                                        \
        WX_COLS(WX_LOAD_U_FAST)                                                                          \
      }                                                                                                  \
    } else {                                                                                             \
      _Pragma("unroll") for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {                                  \
        const wx_i64 wx_r0u = WX_QUAD(wx_u) << 2;                                                        \
        WX_COLS(WX_LOAD_U)                                                                               \
      }                                                                                                  \
    }                                                                                                    \
    _Pragma("unroll") for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {                                    \
      const wx_i64 wx_r0 = WX_QUAD(wx_u) << 2;                                                           \
      if (WX_QUAD(wx_u) < wx_nq) {                                                                       \
        _Pragma("unroll") for (int wx_e = 0; wx_e < 4; ++wx_e) {                                        \
          WX_COLS(WX_BIND_U)                                                                             \
          const wx_i64 idx = wx_r0 + wx_e;
#define WX_STRIDE_LOOP_END \
  }                        \
  }                        \
  }                        \
  }
// Closes the per-row loops but leaves the batch loop open: code after it
// sees the whole span (wx_base, WX_QUAD); the caller closes the span loop.
#define WX_STRIDE_BATCH_END \
  }                         \
  }                         \
  }

#if WX_HAS_COND
#define WX_EVAL_COND() static_cast<bool>(WX_COND)
#else
#define WX_EVAL_COND() true
#endif
