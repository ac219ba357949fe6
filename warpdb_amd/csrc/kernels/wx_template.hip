// wx_template.hip -- hand-written gfx950 kernel templates for the WarpDB
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

// ===========================================================================
#if WX_OP == WX_OP_DENSE
// Dense projection (the reference contract, src/jit.cpp:55-61):
// out[row] = expr where cond holds.  fill = 1 also writes 0.0f elsewhere
// (WarpDB::query's zeroed result in one pass instead of memset + kernel).
// Same contiguous-span loop as the grid-stride reductions: a workgroup owns
// WX_BLOCK * WX_UNROLL row quads per iteration and issues all their loads
// first; each quad's four results leave as one 16-byte store when the quad
// is full (fill, or every row passing) and as guarded dword stores otherwise.
// Nontemporal stores: 2.20 ms per 1e9 rows with fill (12 B/row, 5.45 TB/s),
// against 2.20-2.34 ms for plain stores across grids and unrolls
// (profiles/r01/ablate_dense.txt).  The software-pipelined loop below (4
// quads per thread, 3 workgroups per CU) takes 2.12 ms against 2.165 for the
// best unpipelined geometry (profiles/r02/abl_dense_*.txt).  Without fill
// every partially selected 64-B line was a masked write (3.1 ms); masked mode
// now reads and rewrites whole quads instead, pipelined like fill mode
// (WX_DENSE_BLEND: 2.63 vs 3.00 ms, profiles/r02/abl_dense_masked_1e9.txt).
#ifndef WX_UNROLL
#define WX_UNROLL 4
#endif
#ifndef WX_DENSE_NT_STORE
#define WX_DENSE_NT_STORE 1
#endif
#ifndef WX_DENSE_PIPE
#define WX_DENSE_PIPE 1
#endif
#ifndef WX_DENSE_BLEND
// Masked mode (rows failing the WHERE keep their old value, the reference's
// jit_compile_and_launch contract): whole spans read the output quads with
// the columns and write every quad back whole, old values where the row
// fails.  16 B/row of traffic instead of 12, but no partial-line (masked)
// writes, which cost more than the extra read.
#define WX_DENSE_BLEND 1
#endif
#ifndef WX_DENSE_BLEND_PIPE
#define WX_DENSE_BLEND_PIPE 1  // masked mode through the software-pipelined loop too
#endif
#ifndef WX_DENSE_BLEND_NT
#define WX_DENSE_BLEND_NT 1  // nontemporal loads of the old output quads (2.88 vs 2.97 ms, plain)
#endif
// One span's rows: evaluate and store (full spans: one 16-byte store per quad;
// BLEND: full spans of masked mode, wx_old holds the output quads as read).
#define WX_DENSE_SPAN_OUT(FULL, BLEND)                                                                 \
  _Pragma("unroll") for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {                                   \
    const wx_i64 wx_r0 = WX_QUAD(wx_u) << 2;                                                           \
    if (WX_QUAD(wx_u) >= wx_nq) continue;                                                              \
    float wx_o[4];                                                                                     \
    bool wx_k[4];                                                                                      \
    _Pragma("unroll") for (int wx_e = 0; wx_e < 4; ++wx_e) {                                          \
      WX_COLS(WX_BIND_U)                                                                               \
      const wx_i64 idx = wx_r0 + wx_e;                                                                 \
      (void)idx;                                                                                       \
      wx_k[wx_e] = WX_EVAL_COND();                                                                     \
      wx_o[wx_e] = static_cast<float>(WX_EXPR);                                                        \
    }                                                                                                  \
    const bool wx_all = wx_k[0] && wx_k[1] && wx_k[2] && wx_k[3];                                      \
    if ((FULL) && (BLEND)) {                                                                           \
      f4 v;                                                                                            \
      v.x = wx_k[0] ? wx_o[0] : wx_old[wx_u].x;                                                        \
      v.y = wx_k[1] ? wx_o[1] : wx_old[wx_u].y;                                                        \
      v.z = wx_k[2] ? wx_o[2] : wx_old[wx_u].z;                                                        \
      v.w = wx_k[3] ? wx_o[3] : wx_old[wx_u].w;                                                        \
      ::wx::st_sel<WX_DENSE_NT_STORE>(reinterpret_cast<f4 *>(wx_a.out + wx_r0), v);                   \
    } else if ((FULL) && (wx_a.fill || wx_all)) {                                                      \
      f4 v;                                                                                            \
      v.x = wx_k[0] ? wx_o[0] : 0.0f;                                                                  \
      v.y = wx_k[1] ? wx_o[1] : 0.0f;                                                                  \
      v.z = wx_k[2] ? wx_o[2] : 0.0f;                                                                  \
      v.w = wx_k[3] ? wx_o[3] : 0.0f;                                                                  \
      ::wx::st_sel<WX_DENSE_NT_STORE>(reinterpret_cast<f4 *>(wx_a.out + wx_r0), v);                   \
    } else {                                                                                           \
      _Pragma("unroll") for (int wx_e = 0; wx_e < 4; ++wx_e) if (wx_r0 + wx_e < wx_a.n_rows &&        \
                                                                  (wx_k[wx_e] || wx_a.fill))           \
          wx_a.out[wx_r0 + wx_e] = wx_k[wx_e] ? wx_o[wx_e] : 0.0f;                                    \
    }                                                                                                  \
  }
#if WX_DENSE_PIPE
// Software-pipelined steady state: while this span and the next are whole
// and every row is written (fill, no WHERE, or masked mode's whole-quad
// blend), the next span's loads are issued before this span's stores and
// waited for after them.  On gfx9
// stores count in vmcnt, so the straight-line body lets the wait leave this
// span's stores in flight (a conditional store or load anywhere in the loop
// makes the compiler drain vmcnt to 0).  Ragged spans take the generic loop
// below.
#define WX_DECL_N(name, T, slot) T wx_n##slot[WX_UNROLL][4];
#define WX_LOAD_N_FAST(name, T, slot) ::wx::load4_full<T>(wx_a.col[slot], wx_r0u, wx_n##slot[wx_u]);
#define WX_MOVE_N(name, T, slot)                                  \
  _Pragma("unroll") for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) \
      _Pragma("unroll") for (int wx_e = 0; wx_e < 4; ++wx_e) wx_u##slot[wx_u][wx_e] = wx_n##slot[wx_u][wx_e];
extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_project_dense(WxDenseArgs wx_a) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const wx_i64 wx_nq = (wx_a.n_rows + 3) >> 2;
  const wx_i64 wx_nfull = wx_a.n_rows >> 2;
  const wx_i64 wx_stride = (wx_i64)gridDim.x * WX_SPAN;
  wx_i64 wx_base = (wx_i64)blockIdx.x * WX_SPAN;
  const bool wx_every = wx_a.fill || !WX_HAS_COND;
  const bool wx_blend = WX_DENSE_BLEND && !wx_every;  // masked mode
  // BLEND: masked mode, the output quads load with the columns and failing
  // rows keep their old value (see WX_DENSE_BLEND)
  auto wx_pipe = [&](auto wx_tag) {
    constexpr bool BLEND = decltype(wx_tag)::value;
    WX_COLS(WX_DECL_U)
    WX_COLS(WX_DECL_N)
    f4 wx_old[WX_UNROLL], wx_nold[WX_UNROLL];
#pragma unroll
    for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {
      const wx_i64 wx_r0u = WX_QUAD(wx_u) << 2;
      WX_COLS(WX_LOAD_N_FAST)
      if constexpr (BLEND) wx_nold[wx_u] = ::wx::ldv(reinterpret_cast<const f4 *>(wx_a.out + wx_r0u));
    }
    // Drain here, so the loop head inherits no pending loads: otherwise the
    // wait the compiler places there for this prologue (vmcnt(0)) also
    // drains every later iteration's stores.
    __builtin_amdgcn_s_waitcnt(0x0f70);  // gfx9: vmcnt(0) expcnt(7) lgkmcnt(15)
    WX_COLS(WX_MOVE_N)
    if constexpr (BLEND) {
#pragma unroll
      for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) wx_old[wx_u] = wx_nold[wx_u];
    }
    while (true) {
      const wx_i64 wx_nb = wx_base + wx_stride;
      const bool wx_more = wx_nb + WX_SPAN <= wx_nfull;  // workgroup-uniform
      if (wx_more) {
#pragma unroll
        for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {
          const wx_i64 wx_r0u = (wx_nb + (wx_i64)wx_u * WX_BLOCK + threadIdx.x) << 2;
          WX_COLS(WX_LOAD_N_FAST)
          if constexpr (BLEND) wx_nold[wx_u] = ::wx::ldv(reinterpret_cast<const f4 *>(wx_a.out + wx_r0u));
        }
      }
#pragma unroll
      for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {
        const wx_i64 wx_r0 = WX_QUAD(wx_u) << 2;
        f4 v;
#pragma unroll
        for (int wx_e = 0; wx_e < 4; ++wx_e) {
          WX_COLS(WX_BIND_U)
          const wx_i64 idx = wx_r0 + wx_e;
          (void)idx;
          const bool wx_k = WX_EVAL_COND();
          v[wx_e] = wx_k ? static_cast<float>(WX_EXPR) : (BLEND ? wx_old[wx_u][wx_e] : 0.0f);
        }
        ::wx::st_sel<WX_DENSE_NT_STORE>(reinterpret_cast<f4 *>(wx_a.out + wx_r0), v);
      }
      wx_base = wx_nb;
      if (!wx_more) break;
      WX_COLS(WX_MOVE_N)
      if constexpr (BLEND) {
#pragma unroll
        for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) wx_old[wx_u] = wx_nold[wx_u];
      }
    }
  };
  if (WX_ALIGNED16 && wx_base + WX_SPAN <= wx_nfull) {
    if (wx_every)
      wx_pipe(::wx::btag<false>{});
    else if (WX_DENSE_BLEND_PIPE && wx_blend)
      wx_pipe(::wx::btag<true>{});
  }
  for (; wx_base < wx_nq; wx_base += wx_stride) {
    WX_COLS(WX_DECL_U)
    f4 wx_old[WX_UNROLL];
    const bool wx_full = WX_ALIGNED16 && wx_base + WX_SPAN <= wx_nfull;
    if (wx_full) {
#pragma unroll
      for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {
        const wx_i64 wx_r0u = WX_QUAD(wx_u) << 2;
        WX_COLS(WX_LOAD_U_FAST)
        if (wx_blend)
          wx_old[wx_u] = WX_DENSE_BLEND_NT ? __builtin_nontemporal_load(reinterpret_cast<const f4 *>(wx_a.out + wx_r0u))
                                           : *reinterpret_cast<const f4 *>(wx_a.out + wx_r0u);
      }
    } else {
#pragma unroll
      for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {
        const wx_i64 wx_r0u = WX_QUAD(wx_u) << 2;
        WX_COLS(WX_LOAD_U)
      }
    }
    WX_DENSE_SPAN_OUT(wx_full, wx_blend)
  }
}
#else
extern "C" __global__ __launch_bounds__(WX_BLOCK) void wx_project_dense(WxDenseArgs wx_a) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const wx_i64 wx_nq = (wx_a.n_rows + 3) >> 2;
  const wx_i64 wx_nfull = wx_a.n_rows >> 2;
  for (wx_i64 wx_base = (wx_i64)blockIdx.x * WX_SPAN; wx_base < wx_nq; wx_base += (wx_i64)gridDim.x * WX_SPAN) {
    WX_COLS(WX_DECL_U)
    const bool wx_full = WX_ALIGNED16 && wx_base + WX_SPAN <= wx_nfull;
    if (wx_full) {
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
#pragma unroll
    for (int wx_u = 0; wx_u < WX_UNROLL; ++wx_u) {
      const wx_i64 wx_r0 = WX_QUAD(wx_u) << 2;
      if (WX_QUAD(wx_u) >= wx_nq) continue;
      float wx_o[4];
      bool wx_k[4];
#pragma unroll
      for (int wx_e = 0; wx_e < 4; ++wx_e) {
        WX_COLS(WX_BIND_U)
        const wx_i64 idx = wx_r0 + wx_e;
        (void)idx;
        wx_k[wx_e] = WX_EVAL_COND();
        wx_o[wx_e] = static_cast<float>(WX_EXPR);
      }
      const bool wx_all = wx_k[0] && wx_k[1] && wx_k[2] && wx_k[3];
      if (wx_full && (wx_a.fill || wx_all)) {
        f4 v;
        v.x = wx_k[0] ? wx_o[0] : 0.0f;
        v.y = wx_k[1] ? wx_o[1] : 0.0f;
        v.z = wx_k[2] ? wx_o[2] : 0.0f;
        v.w = wx_k[3] ? wx_o[3] : 0.0f;
#if WX_DENSE_NT_STORE
        __builtin_nontemporal_store(v, reinterpret_cast<f4 *>(wx_a.out + wx_r0));
#else
        *reinterpret_cast<f4 *>(wx_a.out + wx_r0) = v;
#endif
      } else {
#pragma unroll
        for (int wx_e = 0; wx_e < 4; ++wx_e)
          if (wx_r0 + wx_e < wx_a.n_rows && (wx_k[wx_e] || wx_a.fill))
            wx_a.out[wx_r0 + wx_e] = wx_k[wx_e] ? wx_o[wx_e] : 0.0f;
      }
    }
  }
}
#endif  // WX_DENSE_PIPE
#endif

// ===========================================================================
#if WX_OP == WX_OP_COMPACT
// Ordered stream compaction in one pass: decoupled look-back over tiles.
//
// Tile = WX_DTHREADS data threads x WX_GROUPS groups x 4 rows; row
// (g, thread, e) of a tile is at offset g*4*WX_DTHREADS + thread*4 + e, so each group is one 16-byte
// load per lane per column.  In-tile ranks come from 64-bit wavefront ballots
// (v_mbcnt) and a WX_DWAVES x WX_GROUPS LDS table.  A tile's global offset comes
// from its predecessors' 8-byte status words {epoch:6 | flag:2 | value:56}; a status
// word is its own payload (single agent-scope 8-byte stores and loads), so no
// fence is needed, and output rows are never read inside the launch.
//
// wx_project_compact (default) is a persistent, software-pipelined kernel:
// WX_DWAVES data waves + 1 control wave per workgroup, one LDS stage buffer.
// Iteration k: the data waves evaluate tile t_k (loaded one iteration
// earlier), issue t_{k+1}'s loads and rank t_k; the control wave publishes
// t_k's aggregate while the data waves write t_{k-1} out of LDS (coalesced,
// its offset resolved one iteration earlier); then the data waves stage
// (value, tile-local row) of t_k into LDS and evaluate t_{k+1} while the
// control wave runs t_k's look-back.  Block b owns tiles b, b + grid, ... so the grid must be
// co-resident (the host sizes it from the occupancy query).
// wx_project_compact_ticket takes one tile per workgroup from a ticket
// counter: no residency assumption, no pipelining.
#define WX_GROUPS WX_COMPACT_GROUPS
#define WX_DWAVES WX_COMPACT_DWAVES             // data waves per workgroup
#define WX_DTHREADS (WX_DWAVES * 64)
#define WX_TILE (WX_DTHREADS * 4 * WX_GROUPS)  // rows per tile
#define WX_CBLOCK (WX_DTHREADS + 64)            // + 1 control wave
// Status word {epoch:6 | flag:2 | value:56}: a word whose epoch is not this
// launch's reads as "not published", so the host never clears the array
// between queries (a new epoch per launch; one memset every 63 launches).
#define WX_FLAG_A (1ull << 56)
#define WX_FLAG_P (2ull << 56)
#define WX_VAL_MASK ((1ull << 56) - 1ull)
#define WX_EPOCH_SHIFT 58
__device__ __forceinline__ wx_u64 wx_cflag(wx_u64 w, wx_u64 E) {
  return (w >> WX_EPOCH_SHIFT) == (E >> WX_EPOCH_SHIFT) ? (w >> 56) & 3ull : 0ull;
}
#ifndef WX_COMPACT_VSTORE
#define WX_COMPACT_VSTORE 1  // 16-byte aligned stores for the output runs (2.65 -> 2.47 ms)
#endif
#ifndef WX_COMPACT_WHOLE_LOADS
// unguarded loads when the next tile is whole: measured slower in the same
// process (2.71 vs 2.47 ms, profiles/r01/ablate_compact_ab.txt), kept off
#define WX_COMPACT_WHOLE_LOADS 0
#endif
#ifndef WX_STALL_TICKS
// A waiter gives up after this long (s_memrealtime, 100 MHz) without any
// polled word changing: progress, not poll count, so a query slowed down by
// another process sharing the GPU still completes.
#define WX_STALL_TICKS 200000000ull  // 2 s
#endif
#ifndef WX_LB_PER_LANE
#define WX_LB_PER_LANE 1  // predecessors per lane per look-back round (1 measured fastest: each agent-scope poll is costly)
#endif
#ifndef WX_LB_SLEEP
#define WX_LB_SLEEP 2     // s_sleep units (64 clocks) between polls of an unpublished tile
#endif

// Per-column input registers of one tile and the load/bind helpers.
#define WX_DECL_TILE_IN(name, T, slot) T wx_in##slot[WX_GROUPS][4];
#define WX_LOAD_TILE_IN(name, T, slot) \
  ::wx::load4<T>(wx_a.col[slot], wx_tb + (wx_i64)wx_g * (WX_DTHREADS * 4) + (wx_i64)wx_dt * 4, wx_a.n_rows, wx_in##slot[wx_g]);
#define WX_LOAD_TILE_FULL(name, T, slot) \
  ::wx::load4_full<T>(wx_a.col[slot], wx_tb + (wx_i64)wx_g * (WX_DTHREADS * 4) + (wx_i64)wx_dt * 4, wx_in##slot[wx_g]);
#define WX_BIND_TILE_IN(name, T, slot) const ::wx::reg<T> name{wx_in##slot[wx_g][wx_e]};

// Exclusive prefix of `tile` from its predecessors' status words; one wave.
// Load j of lane l reads tile look - 64*j - l: every load instruction covers
// 64 adjacent status words (agent-scope loads are served beyond L2, so poll
// traffic competes with the table stream).  A timed-out wait raises the error
// bit, and every waiter that sees the bit gives up, so a broken residency
// assumption drains the grid quickly instead of hanging it.
__device__ __forceinline__ wx_i64 wx_lookback(const WxCompactArgs &a, wx_i64 tile) {
  const int lane = threadIdx.x & 63;
  const wx_u64 E = (wx_u64)a.epoch << WX_EPOCH_SHIFT;
  const wx_u64 abort_word = E | 1ull;  // flag 0, value 1: never a tile word
  wx_i64 excl = 0;
  wx_i64 look = tile - 1;
  wx_u32 spins = 0;
  bool moved = false;
  wx_u64 t_last = 0;
  while (true) {
    wx_u64 st[WX_LB_PER_LANE];
#pragma unroll
    for (int j = 0; j < WX_LB_PER_LANE; ++j) {
      const wx_i64 t = look - 64 * j - lane;
      st[j] = t >= 0 ? wx::ld_agent(&a.status[t]) : (E | WX_FLAG_P);  // "tile -1": inclusive 0
    }
    // Wait only for the entries nearer than the nearest inclusive prefix
    // already visible (distance order (j, lane)); farther ones do not matter.
    int near_p = 64 * WX_LB_PER_LANE;  // distance of the nearest P, or window size
    while (true) {
      near_p = 64 * WX_LB_PER_LANE;
      bool pending = false;
#pragma unroll
      for (int j = WX_LB_PER_LANE - 1; j >= 0; --j) {
        const wx_u64 pm = __builtin_amdgcn_ballot_w64(wx_cflag(st[j], E) == 2ull);
        if (pm) near_p = 64 * j + __builtin_ctzll(pm);
      }
#pragma unroll
      for (int j = 0; j < WX_LB_PER_LANE; ++j) {
        const bool need = wx_cflag(st[j], E) == 0ull && 64 * j + lane < near_p;
        pending |= __builtin_amdgcn_ballot_w64(need) != 0ull;
      }
      if (!pending) break;
      __builtin_amdgcn_s_sleep(WX_LB_SLEEP);
#pragma unroll
      for (int j = 0; j < WX_LB_PER_LANE; ++j) {
        if (wx_cflag(st[j], E) == 0ull && 64 * j + lane < near_p) {
          const wx_u64 w = wx::ld_agent(&a.status[look - 64 * j - lane]);
          moved |= w != st[j];
          st[j] = w;
        }
      }
      if ((++spins & 63u) == 0u) {
        const wx_u64 now = __builtin_amdgcn_s_memrealtime();
        if (__builtin_amdgcn_ballot_w64(moved) != 0ull || t_last == 0ull) {
          t_last = now;
          moved = false;
        } else if (now - t_last > WX_STALL_TICKS) {  // sticky error for the host + this launch's abort word
          atomicOr(reinterpret_cast<unsigned int *>(&a.ctrs[1]), WX_DEVERR_LOOKBACK);
          wx::st_agent(&a.status[a.n_tiles], abort_word);
        }
        if (wx::ld_agent(&a.status[a.n_tiles]) == abort_word) {
#pragma unroll
          for (int j = 0; j < WX_LB_PER_LANE; ++j) st[j] = E | WX_FLAG_P;
        }
      }
    }
    wx_u64 v = 0;
#pragma unroll
    for (int j = 0; j < WX_LB_PER_LANE; ++j)
      if (64 * j + lane <= near_p && 64 * j + lane < 64 * WX_LB_PER_LANE) v += st[j] & WX_VAL_MASK;
    excl += (wx_i64)wx::wave_sum_u64(v);
    if (near_p < 64 * WX_LB_PER_LANE) break;
    look -= 64 * WX_LB_PER_LANE;
    t_last = 0ull;  // the window moved: progress
  }
  return excl;
}

// The last workgroup of a compaction launch to retire returns the tile
// ticket to 0 for the next launch on this workspace (no host memset per
// query).  Every workgroup calls it once after its last ticket fetch.
// Relaxed is enough: every ticket fetch of a workgroup has RETURNED (its
// value went through LDS and a barrier) before that workgroup's increment
// is issued, the increments are ordered on their one address, so the reset
// follows every fetch of the launch; the next launch sees it across the
// kernel boundary.  (acq_rel here is a buffer_wbl2 + buffer_inv at agent
// scope, a few µs at the end of every launch.)
#ifndef WX_RETIRE_ACQ_REL
#define WX_RETIRE_ACQ_REL 0
#endif
__device__ __forceinline__ void wx_retire(wx_u64 *ctrs) {
  const wx_u64 done = WX_RETIRE_ACQ_REL
                          ? __hip_atomic_fetch_add(&ctrs[2], 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT)
                          : __hip_atomic_fetch_add(&ctrs[2], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (done == (wx_u64)gridDim.x - 1ull) {
    __hip_atomic_store(&ctrs[0], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&ctrs[2], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Evaluate one tile held in wx_in* registers and rank its passing rows.
// Writes per-wave totals to s_cnt and returns per-lane ranks in lane_pre.
#define WX_EVAL_AND_RANK(S_CNT)                                                                          \
  _Pragma("unroll") for (int wx_g = 0; wx_g < WX_GROUPS; ++wx_g) {                                     \
    _Pragma("unroll") for (int wx_e = 0; wx_e < 4; ++wx_e) {                                           \
      WX_COLS(WX_BIND_TILE_IN)                                                                           \
      const wx_i64 idx = tile_base + (wx_i64)wx_g * (WX_DTHREADS * 4) + (wx_i64)wx_dt * 4 + wx_e;          \
      bool wx_k = idx < wx_a.n_rows;                                                                     \
      wx_k = wx_k && WX_EVAL_COND();                                                                     \
      wx_keep[wx_g][wx_e] = wx_k;                                                                        \
      wx_val[wx_g][wx_e] = static_cast<float>(WX_EXPR);                                                  \
    }                                                                                                    \
  }                                                                                                      \
  _Pragma("unroll") for (int g = 0; g < WX_GROUPS; ++g) {                                              \
    wx_u32 pre = 0, tot = 0;                                                                             \
    _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                                    \
      const wx_u64 m = __builtin_amdgcn_ballot_w64(wx_keep[g][e]);                                       \
      pre += wx::lanes_below(m);                                                                         \
      tot += (wx_u32)__builtin_popcountll(m);                                                            \
    }                                                                                                    \
    lane_pre[g] = pre;                                                                                   \
    if (lane == 0) S_CNT[wave][g] = tot;                                                                 \
  }

#define WX_BASES(S_CNT)                                        \
  _Pragma("unroll") for (int g = 0; g < WX_GROUPS; ++g) {    \
    wx_u32 before = 0, gsum = 0;                               \
    _Pragma("unroll") for (int w = 0; w < WX_DWAVES; ++w) {   \
      const wx_u32 c = S_CNT[w][g];                            \
      before += (w < wave) ? c : 0u;                           \
      gsum += c;                                               \
    }                                                          \
    grp_base[g] = block_total + before;                        \
    block_total += gsum;                                       \
  }

#ifndef WX_DIAG_PROFILE
#define WX_DIAG_PROFILE 0  // per-phase time of data wave 0 / the control wave
#endif
#if WX_DIAG_PROFILE
#define WX_PT(slot)                                              \
  do {                                                          \
    const wx_u64 wx_now = __builtin_amdgcn_s_memrealtime();     \
    wx_prof[slot] += wx_now - wx_prof_t;                        \
    wx_prof_t = wx_now;                                         \
  } while (0)
#else
#define WX_PT(slot) \
  do {              \
  } while (0)
#endif
#ifndef WX_COMPACT_TICKETS
// Tiles from an atomic ticket counter (two iterations ahead) instead of the
// static b, b + grid, ... schedule: a tile is only ever taken by a running
// workgroup, so the look-back progresses whatever else shares the GPU (the
// static schedule deadlocked when two processes' compactions overlapped).
#define WX_COMPACT_TICKETS 1
#endif
#ifndef WX_COMPACT_MINBLOCKS
#define WX_COMPACT_MINBLOCKS 1  // workgroups per CU the register budget must allow
#endif
extern "C" __global__ __launch_bounds__(WX_CBLOCK, WX_COMPACT_MINBLOCKS) void wx_project_compact(WxCompactArgs wx_a) {
  const wx_u64 wx_E = (wx_u64)wx_a.epoch << WX_EPOCH_SHIFT;
  __shared__ wx_u32 s_cnt[WX_DWAVES][WX_GROUPS];
  __shared__ float s_val[WX_TILE];
  __shared__ unsigned short s_off[WX_TILE];
  __shared__ wx_i64 s_excl;
  __shared__ wx_i64 s_tiles[4];  // ticket ring: slot k & 3 holds iteration k's tile
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool control = wave == WX_DWAVES;
  const int wx_dt = tid;  // data-thread index (data waves only)
  const wx_i64 grid = gridDim.x;
#if WX_COMPACT_TICKETS
  if (tid == 0) {
    s_tiles[0] = (wx_i64)__hip_atomic_fetch_add(&wx_a.ctrs[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_tiles[1] = (wx_i64)__hip_atomic_fetch_add(&wx_a.ctrs[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  wx_i64 tile = s_tiles[0];
#else
  wx_i64 tile = blockIdx.x;
#endif
  wx_i64 prev_tile = -1;
  WX_COLS(WX_DECL_TILE_IN)
  if (!control && tile < wx_a.n_tiles) {
    const wx_i64 wx_tb = tile * WX_TILE;
#pragma unroll
    for (int wx_g = 0; wx_g < WX_GROUPS; ++wx_g) { WX_COLS(WX_LOAD_TILE_IN) }
  }
  wx_u32 prev_total = 0;
#if WX_DIAG_PROFILE
  wx_u64 wx_prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  wx_u64 wx_prof_t = __builtin_amdgcn_s_memrealtime();
#endif
  for (int k = 0;; ++k) {
    const bool have = tile < wx_a.n_tiles;
    const bool have_prev = k > 0 && prev_tile < wx_a.n_tiles;
    if (!have && !have_prev) break;
#if WX_COMPACT_TICKETS
    const wx_i64 next_tile = s_tiles[(k + 1) & 3];  // fetched two iterations ahead
#else
    const wx_i64 next_tile = tile + grid;
#endif
    const wx_i64 tile_base = tile * WX_TILE;
    wx_u32 wx_kb = 0;  // bit 4g + e: row (g, e) passes (a VGPR, not 16 SGPR-pair lane masks)
    float wx_val[WX_GROUPS][4];
    wx_u32 lane_pre[WX_GROUPS];
    // phase 1 (data): evaluate t_k, issue t_{k+1}'s loads, rank t_k
    // (issuing each group's loads right after its evaluation measured slower:
    // 2.72 vs 2.53 ms, profiles/r01/ablate_compact_interleave.txt)
    if (!control && have) {
      // rows of this tile inside the table (workgroup-uniform, 32-bit)
      const wx_u32 wx_rows = (wx_u32)(wx_a.n_rows - tile_base < WX_TILE ? wx_a.n_rows - tile_base : WX_TILE);
#pragma unroll
      for (int wx_g = 0; wx_g < WX_GROUPS; ++wx_g) {
#pragma unroll
        for (int wx_e = 0; wx_e < 4; ++wx_e) {
          WX_COLS(WX_BIND_TILE_IN)
          const wx_u32 wx_lrow = (wx_u32)(wx_g * (WX_DTHREADS * 4) + wx_dt * 4 + wx_e);
          const wx_i64 idx = tile_base + wx_lrow;  // dead unless the expression names idx
          (void)idx;
          bool wx_k = wx_lrow < wx_rows;
          wx_k = wx_k && WX_EVAL_COND();
          wx_kb |= (wx_k ? 1u : 0u) << (wx_g * 4 + wx_e);
          wx_val[wx_g][wx_e] = static_cast<float>(WX_EXPR);
        }
      }
      WX_PT(0);  // evaluation, including the wait for t_k's loads
      const wx_i64 next = next_tile;
      const wx_i64 wx_tb = next * WX_TILE;
      if (WX_COMPACT_WHOLE_LOADS && WX_ALIGNED16 && wx_tb + WX_TILE <= wx_a.n_rows) {  // workgroup-uniform
#pragma unroll
        for (int wx_g = 0; wx_g < WX_GROUPS; ++wx_g) { WX_COLS(WX_LOAD_TILE_FULL) }
      } else if (next < wx_a.n_tiles) {
#pragma unroll
        for (int wx_g = 0; wx_g < WX_GROUPS; ++wx_g) { WX_COLS(WX_LOAD_TILE_IN) }
      }
#pragma unroll
      for (int g = 0; g < WX_GROUPS; ++g) {
        wx_u32 pre = 0, tot = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const wx_u64 m = __builtin_amdgcn_ballot_w64(((wx_kb >> (g * 4 + e)) & 1u) != 0u);
          pre += wx::lanes_below(m);
          tot += (wx_u32)__builtin_popcountll(m);
        }
        lane_pre[g] = pre;
        if (lane == 0) s_cnt[wave][g] = tot;
      }
      WX_PT(1);  // issue t_{k+1} loads + rank
    }
    __syncthreads();
    WX_PT(2);  // barrier 1
    // phase 2: control publishes t_k's aggregate; data waves write t_{k-1} out of LDS
    wx_u32 block_total = 0;
    wx_u32 grp_base[WX_GROUPS];
    if (have) { WX_BASES(s_cnt) }
    if (control) {
      if (have && lane == 0)
        wx::st_agent(&wx_a.status[tile], wx_E | (tile == 0 ? WX_FLAG_P : WX_FLAG_A) | (wx_u64)block_total);
#if WX_COMPACT_TICKETS
      // the tile of iteration k + 2 (slot last read as `prev` in iteration k - 1)
      if (lane == 0)
        s_tiles[(k + 2) & 3] = next_tile < wx_a.n_tiles
                                   ? (wx_i64)__hip_atomic_fetch_add(&wx_a.ctrs[0], 1ull, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT)
                                   : wx_a.n_tiles;  // past the end: stop taking tickets
#endif
    } else if (have_prev) {
      const wx_i64 excl = s_excl;
      const wx_i64 prev_base = wx_a.row_base + prev_tile * WX_TILE;
#if !WX_DIAG_NO_STORE
      // The tile's output run [excl, excl + total): a scalar head up to the
      // next 32-element boundary (128 B of f32 / i32), aligned 16-byte stores
      // of four outputs per lane, a scalar tail of < 4.  For this kernel's
      // 8 B read + 5 B write mix the probe gives 6.2 TB/s with aligned 16-B
      // stores (r2wt) against 5.1-5.4 with 4-B stores (r2wd4) and 3.6 with
      // 4-B stores off a 16-B boundary (tools/bw_probe.hip).
      const wx_i64 end = excl + (wx_i64)prev_total;
      wx_i64 b0 = WX_COMPACT_VSTORE ? (excl + 31) & ~(wx_i64)31 : end;
      if (b0 > end) b0 = end;
      const wx_i64 b1 = b0 + ((end - b0) & ~(wx_i64)3);
      const int n_head = (int)(b0 - excl), n_edge = n_head + (int)(end - b1);
      for (int j = wx_dt; j < n_edge; j += WX_DTHREADS) {
        const wx_i64 pos = j < n_head ? excl + j : b1 + (j - n_head);
        const int i = (int)(pos - excl);
        if (wx_a.out_val) wx_a.out_val[pos] = s_val[i];
        if (wx_a.out_idx) {
          const wx_i64 gi = prev_base + s_off[i];
          if (wx_a.idx64) static_cast<wx_i64 *>(wx_a.out_idx)[pos] = gi;
          else static_cast<int *>(wx_a.out_idx)[pos] = (int)gi;
        }
      }
      for (wx_i64 q = b0 + 4 * (wx_i64)wx_dt; q < b1; q += 4 * (wx_i64)WX_DTHREADS) {
        const int i = (int)(q - excl);
        if (wx_a.out_val) {
          typedef float v4f __attribute__((ext_vector_type(4)));
          const v4f v = {s_val[i], s_val[i + 1], s_val[i + 2], s_val[i + 3]};
          wx::stv(reinterpret_cast<v4f *>(wx_a.out_val + q), v);
        }
        if (wx_a.out_idx) {
          if (wx_a.idx64) {
            typedef long long v2l __attribute__((ext_vector_type(2)));
            wx_i64 *o = static_cast<wx_i64 *>(wx_a.out_idx) + q;
            const v2l x = {(long long)(prev_base + s_off[i]), (long long)(prev_base + s_off[i + 1])};
            const v2l y = {(long long)(prev_base + s_off[i + 2]), (long long)(prev_base + s_off[i + 3])};
            wx::stv(reinterpret_cast<v2l *>(o), x);
            wx::stv(reinterpret_cast<v2l *>(o + 2), y);
          } else {
            typedef int v4i __attribute__((ext_vector_type(4)));
            const unsigned base = (unsigned)prev_base;  // int32 indices: (int)(row) as the scalar path
            const v4i x = {(int)(base + s_off[i]), (int)(base + s_off[i + 1]), (int)(base + s_off[i + 2]),
                           (int)(base + s_off[i + 3])};
            wx::stv(reinterpret_cast<v4i *>(static_cast<int *>(wx_a.out_idx) + q), x);
          }
        }
      }
#else
      if (excl == -1 && wx_a.out_val) wx_a.out_val[0] = s_val[wx_dt];
#endif
    }
    WX_PT(3);  // data: stores of t_{k-1}; control: publish
    __syncthreads();
    WX_PT(4);  // barrier 2
    // phase 3: data waves stage t_k; the control wave resolves t_k's offset
    // (overlapping the staging and phase 1 of the next iteration)
    if (control) {
      if (have) {
        wx_i64 excl = 0;
#if WX_DIAG_NO_LOOKBACK
        excl = WX_DIAG_NO_LOOKBACK == 2 ? tile_base * 5 / 8 + 3 : tile_base / 2;  // diagnostic: timing only
#else
        if (tile > 0) {
          excl = wx_lookback(wx_a, tile);
          if (lane == 0) wx::st_agent(&wx_a.status[tile], wx_E | WX_FLAG_P | (wx_u64)(excl + block_total));
        }
#endif
        if (lane == 0) {
          s_excl = excl;
          if (tile == wx_a.n_tiles - 1 && wx_a.count_out) *wx_a.count_out = excl + block_total;
        }
      }
    } else if (have) {
#pragma unroll
      for (int g = 0; g < WX_GROUPS; ++g) {
        wx_u32 pos = grp_base[g] + lane_pre[g];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if ((wx_kb >> (g * 4 + e)) & 1u) {
            s_val[pos] = wx_val[g][e];
            s_off[pos] = (unsigned short)(g * (WX_DTHREADS * 4) + wx_dt * 4 + e);
            ++pos;
          }
        }
      }
    }
    WX_PT(5);  // data: LDS staging of t_k; control: look-back
    prev_total = block_total;
    prev_tile = tile;
    tile = next_tile;
  }
  if (tid == 0) wx_retire(wx_a.ctrs);
#if WX_DIAG_PROFILE
  if (wx_a.diag && (tid == 0 || tid == WX_DTHREADS)) {
    wx_u64 *d = wx_a.diag + (wx_u64)blockIdx.x * 16 + (tid == 0 ? 0 : 8);
    for (int i = 0; i < 6; ++i) d[i] = wx_prof[i];
  }
#endif
}

// Deeper pipeline (WARPDB_COMPACT_SCHED=deep): tile t_j is evaluated and
// staged in iteration j, its offset resolved by the control wave in
// iteration j + 1 (its predecessors' aggregates have long landed), and its
// output written in iteration j + 2 — the look-back gets a whole iteration
// of slack instead of half of one.  Two stage buffers (2 x 6 B per tile row),
// so only compiled when selected.  Its output runs leave with nontemporal
// stores: 2.23 vs 2.29 ms per 1e9 rows in one process
// (profiles/r01/ablate_compact_deep_nt.txt; the single-buffer kernel was
// slower with them, ablate_compact_nt.txt).
#ifndef WX_DEEP_NT_STORE
#define WX_DEEP_NT_STORE 1
#endif
#ifndef WX_TICKET_PAIR
#define WX_TICKET_PAIR 1
#endif
#if defined(WX_COMPACT_STATIC) && WX_COMPACT_STATIC == 3
// (Measured and dropped, round 4, profiles/r04/: half-height tiles for each
// workgroup's last iterations, +2 us per extra tile at 1e8 rows,
// abl_compact_half_tail.txt; resolving a workgroup's last tile in the
// iteration that evaluates it, 234.9 vs 233.9 us at 1e8 and 2255 vs 2250 us
// at 1e9, abl_compact_early_last.txt; store addresses from an opaque thread
// index, 2244 vs 2232 us at 1e9, abl_compact_opaque_dt.txt.)
#ifndef WX_DIAG_TIMELINE
#define WX_DIAG_TIMELINE 0  // diagnostic: per-workgroup entry / first-tile / loop-end times (diag[b * 16 ..])
#endif
extern "C" __global__ __launch_bounds__(WX_CBLOCK, WX_COMPACT_MINBLOCKS) void wx_project_compact_deep(WxCompactArgs wx_a) {
  const wx_u64 wx_E = (wx_u64)wx_a.epoch << WX_EPOCH_SHIFT;
#if WX_DIAG_TIMELINE
  const wx_u64 wx_t_entry = __builtin_amdgcn_s_memrealtime();
  wx_u64 wx_t_first = 0, wx_t_eval0 = 0;
  wx_u32 wx_ntiles = 0;
#endif
  __shared__ wx_u32 s_cnt[WX_DWAVES][WX_GROUPS];
  __shared__ float s_val[2][WX_TILE];
  __shared__ unsigned short s_off[2][WX_TILE];
  __shared__ wx_i64 s_excl[2];
  __shared__ wx_i64 s_tiles[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool control = wave == WX_DWAVES;
  const int wx_dt = tid;
  if (tid == 0) {
    if (WX_TICKET_PAIR) {  // one dequeue for both first tiles (the counter word serialises every dequeue)
      const wx_i64 t0 = (wx_i64)__hip_atomic_fetch_add(&wx_a.ctrs[0], 2ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_tiles[0] = t0;
      s_tiles[1] = t0 + 1;
    } else {
      s_tiles[0] = (wx_i64)__hip_atomic_fetch_add(&wx_a.ctrs[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_tiles[1] = (wx_i64)__hip_atomic_fetch_add(&wx_a.ctrs[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
#if WX_DIAG_TIMELINE
  wx_t_first = __builtin_amdgcn_s_memrealtime();
#endif
  wx_i64 tile = s_tiles[0];
  wx_i64 tile1 = -1, tile2 = -1;   // tiles of iterations k - 1 and k - 2
  wx_u32 tot1 = 0, tot2 = 0;       // their passing counts
  WX_COLS(WX_DECL_TILE_IN)
  if (!control && tile < wx_a.n_tiles) {
    const wx_i64 wx_tb = tile * WX_TILE;
#pragma unroll
    for (int wx_g = 0; wx_g < WX_GROUPS; ++wx_g) { WX_COLS(WX_LOAD_TILE_IN) }
  }
  for (int k = 0;; ++k) {
    const bool have = tile < wx_a.n_tiles;
    const bool have1 = k >= 1 && tile1 < wx_a.n_tiles;
    const bool have2 = k >= 2 && tile2 < wx_a.n_tiles;
    if (!have && !have1 && !have2) break;
    const wx_i64 next_tile = s_tiles[(k + 1) & 3];
    const wx_i64 tile_base = tile * WX_TILE;
    const int cur = k & 1;  // t_k is staged in buffer cur, t_{k-2} is read from it first
    wx_u32 wx_kb = 0;
    float wx_val[WX_GROUPS][4];
    wx_u32 lane_pre[WX_GROUPS];
    // phase 1 (data): evaluate t_k, issue t_{k+1}'s loads, rank t_k
    if (!control && have) {
      const wx_u32 wx_rows = (wx_u32)(wx_a.n_rows - tile_base < WX_TILE ? wx_a.n_rows - tile_base : WX_TILE);
#pragma unroll
      for (int wx_g = 0; wx_g < WX_GROUPS; ++wx_g) {
#pragma unroll
        for (int wx_e = 0; wx_e < 4; ++wx_e) {
          WX_COLS(WX_BIND_TILE_IN)
          const wx_u32 wx_lrow = (wx_u32)(wx_g * (WX_DTHREADS * 4) + wx_dt * 4 + wx_e);
          const wx_i64 idx = tile_base + wx_lrow;
          (void)idx;
          bool wx_k = wx_lrow < wx_rows;
          wx_k = wx_k && WX_EVAL_COND();
          wx_kb |= (wx_k ? 1u : 0u) << (wx_g * 4 + wx_e);
          wx_val[wx_g][wx_e] = static_cast<float>(WX_EXPR);
        }
      }
#if WX_DIAG_TIMELINE
      if (k == 0) wx_t_eval0 = __builtin_amdgcn_s_memrealtime();
      ++wx_ntiles;
#endif
      if (next_tile < wx_a.n_tiles) {
        const wx_i64 wx_tb = next_tile * WX_TILE;
#pragma unroll
        for (int wx_g = 0; wx_g < WX_GROUPS; ++wx_g) { WX_COLS(WX_LOAD_TILE_IN) }
      }
#pragma unroll
      for (int g = 0; g < WX_GROUPS; ++g) {
        wx_u32 pre = 0, tot = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const wx_u64 m = __builtin_amdgcn_ballot_w64(((wx_kb >> (g * 4 + e)) & 1u) != 0u);
          pre += wx::lanes_below(m);
          tot += (wx_u32)__builtin_popcountll(m);
        }
        lane_pre[g] = pre;
        if (lane == 0) s_cnt[wave][g] = tot;
      }
    }
    __syncthreads();
    // phase 2: control publishes t_k's aggregate and fetches the tile of
    // iteration k + 2; data waves write t_{k-2} out of buffer cur
    wx_u32 block_total = 0;
    wx_u32 grp_base[WX_GROUPS];
    if (have) { WX_BASES(s_cnt) }
    if (control) {
      if (lane == 0) {
        if (have) wx::st_agent(&wx_a.status[tile], wx_E | (tile == 0 ? WX_FLAG_P : WX_FLAG_A) | (wx_u64)block_total);
        s_tiles[(k + 2) & 3] = next_tile < wx_a.n_tiles
                                   ? (wx_i64)__hip_atomic_fetch_add(&wx_a.ctrs[0], 1ull, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT)
                                   : wx_a.n_tiles;
      }
    } else if (have2) {
      // write one staged tile's passing rows at its resolved offset
      auto wx_store = [&](const wx_i64 excl, const wx_u32 tot, const wx_i64 tl, const int buf) {
      const int wx_sdt = wx_dt;
      const wx_i64 prev_base = wx_a.row_base + tl * WX_TILE;
      const float *sv = s_val[buf];
      const unsigned short *so = s_off[buf];
#if WX_DIAG_NO_STORE  // diagnostic: timing only (results invalid), the LDS stage still read
      if (excl == -1 && wx_a.out_val) wx_a.out_val[0] = sv[wx_sdt] + (float)so[wx_sdt];
#else
      const wx_i64 end = excl + (wx_i64)tot;
      wx_i64 b0 = (excl + 31) & ~(wx_i64)31;
      if (b0 > end) b0 = end;
      const wx_i64 b1 = b0 + ((end - b0) & ~(wx_i64)3);
      const int n_head = (int)(b0 - excl), n_edge = n_head + (int)(end - b1);
      for (int j = wx_sdt; j < n_edge; j += WX_DTHREADS) {
        const wx_i64 pos = j < n_head ? excl + j : b1 + (j - n_head);
        const int i = (int)(pos - excl);
        if (wx_a.out_val) wx_a.out_val[pos] = sv[i];
        if (wx_a.out_idx) {
          const wx_i64 gi = prev_base + so[i];
          if (wx_a.idx64) static_cast<wx_i64 *>(wx_a.out_idx)[pos] = gi;
          else static_cast<int *>(wx_a.out_idx)[pos] = (int)gi;
        }
      }
      for (wx_i64 q = b0 + 4 * (wx_i64)wx_sdt; q < b1; q += 4 * (wx_i64)WX_DTHREADS) {
        const int i = (int)(q - excl);
        const float v0 = sv[i], v1 = sv[i + 1], v2 = sv[i + 2], v3 = sv[i + 3];
        const wx_u32 o0 = so[i], o1 = so[i + 1], o2 = so[i + 2], o3 = so[i + 3];
        if (wx_a.out_val) {
          typedef float v4f __attribute__((ext_vector_type(4)));
          const v4f v = {v0, v1, v2, v3};
          wx::st_sel<WX_DEEP_NT_STORE>(reinterpret_cast<v4f *>(wx_a.out_val + q), v);
        }
        if (wx_a.out_idx) {
          if (wx_a.idx64) {
            typedef long long v2l __attribute__((ext_vector_type(2)));
            wx_i64 *o = static_cast<wx_i64 *>(wx_a.out_idx) + q;
            const v2l x = {(long long)(prev_base + o0), (long long)(prev_base + o1)};
            const v2l y = {(long long)(prev_base + o2), (long long)(prev_base + o3)};
            wx::st_sel<WX_DEEP_NT_STORE>(reinterpret_cast<v2l *>(o), x);
            wx::st_sel<WX_DEEP_NT_STORE>(reinterpret_cast<v2l *>(o + 2), y);
          } else {
            typedef int v4i __attribute__((ext_vector_type(4)));
            const unsigned base = (unsigned)prev_base;
            const v4i x = {(int)(base + o0), (int)(base + o1), (int)(base + o2), (int)(base + o3)};
            wx::st_sel<WX_DEEP_NT_STORE>(reinterpret_cast<v4i *>(static_cast<int *>(wx_a.out_idx) + q), x);
          }
        }
      }
#endif
      };
      wx_store(s_excl[cur], tot2, tile2, cur);  // t_{k-2} (its offset resolved in iteration k - 1)
    }
    __syncthreads();
    // phase 3: data waves stage t_k into buffer cur; the control wave
    // resolves t_{k-1}'s offset (published one iteration ago)
    if (control) {
      if (have1) {
        wx_i64 excl = 0;
#if WX_DIAG_NO_LOOKBACK  // diagnostic: timing only (results invalid)
        excl = WX_DIAG_NO_LOOKBACK == 2 ? tile1 * WX_TILE * 5 / 8 + 3 : tile1 * WX_TILE / 2;
#else
        if (tile1 > 0) {
          excl = wx_lookback(wx_a, tile1);
          if (lane == 0) wx::st_agent(&wx_a.status[tile1], wx_E | WX_FLAG_P | (wx_u64)(excl + tot1));
        }
#endif
        if (lane == 0) {
          s_excl[cur ^ 1] = excl;  // read when t_{k-1} is written, in iteration k + 1
          if (tile1 == wx_a.n_tiles - 1 && wx_a.count_out) *wx_a.count_out = excl + tot1;
        }
      }
    } else if (have) {
#pragma unroll
      for (int g = 0; g < WX_GROUPS; ++g) {
        wx_u32 pos = grp_base[g] + lane_pre[g];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if ((wx_kb >> (g * 4 + e)) & 1u) {
            s_val[cur][pos] = wx_val[g][e];
            s_off[cur][pos] = (unsigned short)(g * (WX_DTHREADS * 4) + wx_dt * 4 + e);
            ++pos;
          }
        }
      }
    }
    tile2 = tile1;
    tot2 = tot1;
    tile1 = tile;
    tot1 = have ? block_total : 0u;
    tile = next_tile;
  }
#if WX_DIAG_TIMELINE
  if (tid == 0 && wx_a.diag) {
    wx_u64 *d = wx_a.diag + (wx_u64)blockIdx.x * 16;
    d[0] = wx_t_entry;
    d[1] = wx_t_first;
    d[2] = wx_t_eval0;
    d[3] = __builtin_amdgcn_s_memrealtime();
    d[4] = wx_ntiles;
  }
#endif
  if (tid == 0) wx_retire(wx_a.ctrs);
}
#endif

// One tile per workgroup, taken from a ticket counter (robust fallback).
extern "C" __global__ __launch_bounds__(WX_DTHREADS) void wx_project_compact_ticket(WxCompactArgs wx_a) {
  const wx_u64 wx_E = (wx_u64)wx_a.epoch << WX_EPOCH_SHIFT;
  __shared__ wx_u32 s_cnt[WX_DWAVES][WX_GROUPS];
  __shared__ wx_i64 s_excl;
  __shared__ wx_u32 s_tile;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wx_dt = tid;
  if (tid == 0)
    s_tile = (wx_u32)__hip_atomic_fetch_add(&wx_a.ctrs[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const wx_i64 tile = s_tile;
  const wx_i64 tile_base = tile * WX_TILE;
  WX_COLS(WX_DECL_TILE_IN)
  {
    const wx_i64 wx_tb = tile_base;
#pragma unroll
    for (int wx_g = 0; wx_g < WX_GROUPS; ++wx_g) { WX_COLS(WX_LOAD_TILE_IN) }
  }
  bool wx_keep[WX_GROUPS][4];
  float wx_val[WX_GROUPS][4];
  wx_u32 lane_pre[WX_GROUPS];
  WX_EVAL_AND_RANK(s_cnt)
  __syncthreads();
  wx_u32 block_total = 0;
  wx_u32 grp_base[WX_GROUPS];
  WX_BASES(s_cnt)
  if (wave == 0) {
    wx_i64 excl = 0;
    if (tile == 0) {
      if (lane == 0) wx::st_agent(&wx_a.status[0], wx_E | WX_FLAG_P | (wx_u64)block_total);
    } else {
      if (lane == 0) wx::st_agent(&wx_a.status[tile], wx_E | WX_FLAG_A | (wx_u64)block_total);
      excl = wx_lookback(wx_a, tile);
      if (lane == 0) wx::st_agent(&wx_a.status[tile], wx_E | WX_FLAG_P | (wx_u64)(excl + block_total));
    }
    if (lane == 0) s_excl = excl;
  }
  __syncthreads();
  const wx_i64 excl = s_excl;
#pragma unroll
  for (int g = 0; g < WX_GROUPS; ++g) {
    const wx_i64 r0 = tile_base + (wx_i64)g * (WX_DTHREADS * 4) + (wx_i64)tid * 4;
    wx_i64 pos = excl + grp_base[g] + lane_pre[g];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (wx_keep[g][e]) {
        if (wx_a.out_val) wx_a.out_val[pos] = wx_val[g][e];
        if (wx_a.out_idx) {
          const wx_i64 gi = wx_a.row_base + r0 + e;
          if (wx_a.idx64) static_cast<wx_i64 *>(wx_a.out_idx)[pos] = gi;
          else static_cast<int *>(wx_a.out_idx)[pos] = (int)gi;
        }
        ++pos;
      }
    }
  }
  if (tid == 0 && tile == wx_a.n_tiles - 1 && wx_a.count_out) *wx_a.count_out = excl + block_total;
  if (tid == 0) wx_retire(wx_a.ctrs);
}
#endif

// ===========================================================================
#if WX_OP == WX_OP_SUM
// SUM((float)expr) WHERE cond in double.  Persistent grid-stride pass with
// WX_UNROLL row quads in flight per thread; one partial per block, combined
// in a fixed order by wx_sum_finalize (bitwise reproducible).
#ifndef WX_UNROLL
#define WX_UNROLL 8  // tools/ablate_stream.py: 8 quads in flight, 8 workgroups per CU
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

#ifndef WX_MINMAX
#define WX_MINMAX 0  // also per-group MIN / MAX (NaN skipped)
#endif
__device__ __forceinline__ float wx_mm_out(wx_u32 m, bool is_min) {
  return (is_min ? m == 0xffffffffu : m == 0u) ? __uint_as_float(0x7fc00000u) : wx::ord2f(m);
}

// Accumulator reads of the finalize: plain across a kernel boundary, agent
// scope (past the non-coherent L2 of another XCD) inside the launch that wrote them
template <bool COH>
__device__ __forceinline__ wx_u64 wx_gld(const wx_u64 *p) {
  return COH ? wx::ld_agent(p) : *p;
}
template <bool COH>
__device__ __forceinline__ double wx_gldd(const double *p) {
  return COH ? __longlong_as_double((long long)wx::ld_agent(reinterpret_cast<const wx_u64 *>(p))) : *p;
}
template <bool COH>
__device__ __forceinline__ wx_u32 wx_gld32(const wx_u32 *p) {
  return COH ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
}
template <int NT, bool COH>
__device__ __forceinline__ void wx_group_finalize_body(const WxGroupFinArgs &a, wx_u64 *s_ent, wx_u32 *s_wtot,
                                                       wx_i64 &s_nlo);

__device__ __forceinline__ void wx_hash_add(const WxGroupArgs &a, int key, double v, wx_u32 o) {
  const wx_u64 tag = (wx_u64)(wx_u32)key | (1ull << 32);
  wx_u32 h = ((wx_u32)key * 2654435761u) & a.hmask;
  for (wx_u32 probe = 0; probe <= a.hmask; ++probe) {
    wx_u64 cur = wx::ld_agent(&a.h_tag[h]);
    if (cur == 0ull) {
      const wx_u64 prev = atomicCAS(&a.h_tag[h], 0ull, tag);
      if (prev == 0ull) {
        const wx_u64 u = __hip_atomic_fetch_add(&a.ctrs[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // agent scope: a fused finalize in another XCD's workgroup reads it in this launch
        __hip_atomic_store(&a.h_used[u], h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
#ifndef WX_GROUP_FUSED_FIN
// 1: the last workgroup to finish runs the finalize itself (no second launch
// and no launch gap) when the host asks for it (wx_a.fused: no device-wide
// key sort can be needed, capacity <= WX_GROUP_HSORT_MAX)
#define WX_GROUP_FUSED_FIN (!WX_MINMAX)
#endif
extern "C" __global__ __launch_bounds__(WX_GBLOCK) void wx_group_sum(WxGroupArgs wx_a) {
#if WX_GROUP_FUSED_FIN
  // the window during the scan, the finalize's key sort after the flush
  __shared__ wx_u64 wx_s_raw[WX_HSORT_MAX > (WX_GWIN * 12 + 7) / 8 ? WX_HSORT_MAX : (WX_GWIN * 12 + 7) / 8];
  double *wx_s_sum = reinterpret_cast<double *>(wx_s_raw);
  wx_u32 *wx_s_cnt = reinterpret_cast<wx_u32 *>(wx_s_sum + WX_GWIN);
  __shared__ wx_u32 wx_s_wtot[WX_GBLOCK / 64];
  __shared__ wx_i64 wx_s_nlo;
  __shared__ int wx_s_last;
#else
  __shared__ double wx_s_sum[WX_GWIN];
  __shared__ wx_u32 wx_s_cnt[WX_GWIN];
#endif
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
  WX_STRIDE_LOOP_BEGIN
  if (idx < wx_a.n_rows && WX_EVAL_COND()) {
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
#if WX_GROUP_FUSED_FIN
  if (!wx_a.fused) return;
  // this workgroup's flush and hash atomics performed, then its count: the
  // workgroup that counts last sees every other one's accumulators
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    const wx_u64 done = __hip_atomic_fetch_add(&wx_a.ctrs[2], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    wx_s_last = done == (wx_u64)gridDim.x - 1ull;
    if (wx_s_last) __hip_atomic_store(&wx_a.ctrs[2], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!wx_s_last) return;
  wx_group_finalize_body<WX_GBLOCK, true>(wx_a.fin, wx_s_raw, wx_s_wtot, wx_s_nlo);
#endif
}

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

// The finalize on NT threads: the 1024-thread kernel below, or (COH) the last
// workgroup of wx_group_sum itself, which reads the accumulators the other
// workgroups' atomics left with agent-scope loads.  s_ent: WX_HSORT_MAX
// entries ((key ^ sign) << 32 | used-list position), s_wtot: NT / 64 words.
template <int NT, bool COH>
__device__ __forceinline__ void wx_group_finalize_body(const WxGroupFinArgs &a, wx_u64 *s_ent, wx_u32 *s_wtot,
                                                       wx_i64 &s_nlo) {
  constexpr int BPT = WX_GWIN / NT;  // window bins per thread
  static_assert(WX_GWIN == BPT * NT, "the window divides over the threads");
  const int tid = threadIdx.x;
  const wx_i64 n_hash = (wx_i64)wx_gld<COH>(&a.ctrs[0]);
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
  for (int h = 0; h < BPT; ++h) wc[h] = wx_gld<COH>(&a.win_cnt[b0 + h]);
  for (int i = tid; !presorted && i < npad; i += NT) {
    wx_u64 e = ~0ull;
    if (i < nh) {
      const wx_u32 slot = wx_gld32<COH>(&a.h_used[i]);
      const wx_u32 key = (wx_u32)wx_gld<COH>(&a.h_tag[slot]);
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
        a.win_out[b] = c ? wx_gldd<COH>(&a.win_sum[b]) : 0.0;
        a.win_out[WX_GWIN + b] = (double)c;
        if (!c) continue;
        a.win_sum[b] = 0.0;
        a.win_cnt[b] = 0ull;
        continue;
      }
      if (!c) continue;
      if (pos < a.capacity) {
        a.out_keys[pos] = a.key_lo + b;
        a.out_sums[pos] = wx_gldd<COH>(&a.win_sum[b]);
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
    const wx_u32 slot = wx_gld32<COH>(&a.h_used[(wx_u32)e]);
    const wx_i64 pos = (i < nlo) ? i : out_pos + (i - nlo);
    if (pos < a.capacity) {
      a.out_keys[pos] = (int)((wx_u32)(e >> 32) ^ 0x80000000u);
      a.out_sums[pos] = wx_gldd<COH>(&a.h_sum[slot]);
      a.out_counts[pos] = (wx_i64)wx_gld<COH>(&a.h_cnt[slot]);
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
            const wx_u32 slot = wx_gld32<COH>(&a.h_used[(wx_u32)e]);
            v = fld == 0 ? (double)(int)((wx_u32)(e >> 32) ^ 0x80000000u)
                         : (fld == 1 ? wx_gldd<COH>(&a.h_sum[slot]) : (double)wx_gld<COH>(&a.h_cnt[slot]));
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
    const wx_u32 slot = wx_gld32<COH>(&a.h_used[i]);
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
  wx_group_finalize_body<WX_GFIN_BLOCK, false>(a, s_ent, s_wtot, s_nlo);
}
#endif

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
#pragma unroll
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

// Row-order GROUP BY sums (WX_F_ROW_ORDER, warpexec.cpp do_group_sum_rows):
// one wave per group.  The wave finds the group's first row in the
// key-sorted array (lower bound), checks that exactly its count of rows
// carry the key, and folds their values in ascending row order, one
// dependent double add per row -- the reference's std::map fold
// (src/warpdb.cpp:373-385) to the bit.  The lanes stream the group's values
// (coalesced, WX_FOLD_U chunks of 64 in flight); the chain runs over them in
// lane order (LDS broadcasts, or v_readlane with WX_FOLD_LDS=0), so every
// lane holds the same running sum.
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
  for (wx_i64 g = blockIdx.x; g < a.n_groups; g += gridDim.x) {
    const int key = a.gkeys[g];
    const wx_i64 c = a.gcounts[g];
    wx_i64 lo = 0, hi = a.m;
    while (lo < hi) {
      const wx_i64 mid = (lo + hi) >> 1;
      if (a.skeys[mid] < key) lo = mid + 1;
      else hi = mid;
    }
    if (c < 1 || lo + c > a.m || a.skeys[lo + c - 1] != key || (lo + c < a.m && a.skeys[lo + c] == key)) {
      if (lane == 0) {
        atomicOr(reinterpret_cast<unsigned int *>(&a.ctrs[1]), WX_DEVERR_INTERNAL_KEY);
        a.out_sums[g] = 0.0;
      }
      continue;
    }
    const float *v = a.svals + lo;
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

// ---------------------------------------------------------------------------
// LSD radix sort for the jit_sort_* entry points (src/jit.cpp:248-307): four
// stable passes of 8-bit digits over a 32-bit order key computed on the fly
// from the element itself (floats: the order map with -0.0 == +0.0 and NaN
// last; ints: sign flip; descending: the complement), so float sorts move
// only their 4-byte values and pair sorts their key + payload.
//
// wx_radix_hist: one read of the input builds the histograms of all four
// digits (per-workgroup LDS counters; a wave whose lanes share a digit adds
// once).  The host scans them into per-digit output bases and skips a pass
// whose digit is the same for every key.
//
// wx_radix_sweep_* (one pass, "onesweep"): a workgroup takes tile t from a
// ticket counter, loads WX_RS_ITEMS keys per lane wave-striped (key i of
// lane l of wave w at t*TILE + w*64*ITEMS + i*64 + l, so rank order is input
// order), and ranks each key inside its wave by matching digits with eight
// ballots: the lowest lane of every digit group bumps the wave's LDS counter
// and broadcasts the old count.  Threads 0..255 then own one digit each:
// prefix over the waves, publish the tile's count {A}, look back over the
// preceding tiles' words of the same digit until an inclusive {P} word, and
// publish {P}.  Keys are permuted into digit order in LDS and written out
// from there, so consecutive lanes write consecutive addresses of a digit's
// run.  Every wait is bounded: a timed-out waiter raises WX_DEVERR_LOOKBACK
// and the abort word, and the launch drains.
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

#ifndef WX_RS_HCOPIES
#define WX_RS_HCOPIES 8  // LDS histogram copies, picked by lane % copies: few-valued digits conflict 8x less
#endif
#ifndef WX_RS_HUNROLL
#define WX_RS_HUNROLL 4  // 16-byte loads in flight per thread (64 B): the kernel is latency-bound below that
#endif
template <int KIND, bool ASC>
__device__ __forceinline__ void wx_rs_count(wx_u32 *h, wx_u32 x, int lane, int copy) {
  const wx_u32 k = wx_rs_key_t<KIND, ASC>(x);
  const wx_u64 act = __builtin_amdgcn_ballot_w64(true);
  const int first = __builtin_ctzll(act);
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const wx_u32 d = (k >> (8 * p)) & 255u;
    const wx_u32 d0 = __builtin_amdgcn_readfirstlane(d);
    // (Aggregating the first lane's digit group on every wave, not only on a
    // wave-uniform digit, did not pay: as a second LDS add 18.6 vs 17.7 ms
    // per 1e9 keys, folded into the lane's own add 17.5 vs 17.5.)
    if (__builtin_amdgcn_ballot_w64(d != d0) == 0ull) {
      if (lane == first) atomicAdd(&h[(p * 256 + d0) * WX_RS_HCOPIES], (wx_u32)__builtin_popcountll(act));
    } else {
      atomicAdd(&h[(p * 256 + d) * WX_RS_HCOPIES + copy], 1u);
    }
  }
}

#ifndef WX_RS_HWIDE
#define WX_RS_HWIDE 1  // 1.30 -> 0.66 ms per 1e9 keys with the unconditional, pipelined loads (abl_sort_hwide*.txt)
#endif
#ifndef WX_RS_HPIPE
#define WX_RS_HPIPE 1
#endif
#if WX_RS_HWIDE
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
#else
#define WX_RS_HBLOCK WX_BLOCK
#define WX_RS_HC WX_RS_HCOPIES
#define WX_RS_COUNT(x) (wx_sp = 1u, wx_rs_count<KIND, ASC>(h, (x), lane, copy))  // no check: the general map
#endif

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
#if WX_RS_HPIPE
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
#endif
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

#ifndef WX_RS_SKIP
// Skip words: a tile still walking back publishes {S: span, sum} for the
// tiles (p, tile] it has summed (its own count included), so that a
// successor reading its word jumps the whole span in one read instead of
// walking the same aggregates again (flag 3; sum in bits 0..39, span - 1 in
// bits 40..55).  Published when the span reaches WX_RS_SKIP_MIN, then each
// time it has grown WX_RS_SKIP_GROW-fold.  Measured slower (15.5 vs 13.9 ms
// per 1e9 keys, profiles/r02/abl_sort_skip.txt): off.
#define WX_RS_SKIP 0
#endif
#ifndef WX_RS_SKIP_MIN
#define WX_RS_SKIP_MIN 4
#endif
#ifndef WX_RS_SKIP_GROW
#define WX_RS_SKIP_GROW 3
#endif
#define WX_RS_SKIP_SUM ((1ull << 40) - 1ull)
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
#ifndef WX_RS_LB_FIRST
#define WX_RS_LB_FIRST 1  // load the first predecessor word before the in-tile scan's barrier (13.61-13.75 vs 13.83 ms, abl_sort_lbfirst.txt)
#endif
#ifndef WX_RS_DIAG_NO_RANK
#define WX_RS_DIAG_NO_RANK 0  // diagnostic: no in-wave ranking, keys keep their slots (results invalid)
#endif
#ifndef WX_RS_NT_STORE
#define WX_RS_NT_STORE 1  // nontemporal stores: keys 14.27 -> 14.01 ms per 1e9 (abl_sort_nt.txt); the pair module sets 0
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
  wx_u32 tt[256];  // the tile's count of digit d (paired look-back)
  wx_u32 inc[256];  // its wave-inclusive prefix over the digits (paired look-back)
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

#ifndef WX_RS_FOLD_LD
// the digit's tile-local base folded into the per-wave counts once per tile
// (2 048 adds), so the permutation reads one LDS word per key, not two:
// 12.6 vs 12.8 ms per 1e9 float keys with the atomic ranking, 13.45 vs 13.75
// without (abl_sort_fold.txt)
#define WX_RS_FOLD_LD 1
#endif
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

// Threads 0..255, digit d = tid: publish the tile's count of digit d ({A},
// or {P} for tile 0) as soon as the per-wave counts are summed, then the
// exclusive prefix over the waves and over the digits, look back to an
// inclusive {P}, publish it; fills S.gb / S.ld.  Called by every thread (it
// holds a barrier).  Publishing before the in-tile scan and its barrier
// rather than after: 17.0 vs 17.5 ms per 1e9 keys (ablate_sort.txt).
__device__ __forceinline__ void wx_rs_digits(const WxRadixPassArgs &a, WxRsShared &S, wx_u32 tile) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const wx_u64 E = (wx_u64)a.epoch << 58;
  wx_u64 *row = a.status + (wx_u64)tile * 256;
  const bool look = tile != 0 && !WX_RS_DIAG_NO_LOOKBACK;
  wx_u32 tot = 0u, inc = 0u;
  wx_u64 first = 0ull;  // the first predecessor word, loaded before the barrier
  if (tid < 256) {
#pragma unroll
    for (int w = 0; w < WX_RS_WAVES; ++w) {
      const wx_u32 c = S.wc[w][tid];
      S.wc[w][tid] = tot;
      tot += c;
    }
    wx::st_agent(&row[tid], E | (look ? WX_RS_FLAG_A : WX_RS_FLAG_P) | tot);
    if (WX_RS_LB_FIRST && look) first = wx::ld_agent(&a.status[(wx_u64)(tile - 1) * 256 + tid]);
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
    if (WX_RS_FOLD_LD) {
#pragma unroll
      for (int w = 0; w < WX_RS_WAVES; ++w) S.wc[w][tid] += ld;  // the scatter's slot base in one word
    }
    wx_u64 excl = 0;
    if (look) {
      // WX_RS_LBW predecessors per round, loads in flight together; stop at
      // the first unpublished word (re-polled from there) or the first {P}
      wx_i64 p = (wx_i64)tile - 1;
      wx_u32 spins = 0;
      wx_u64 t_last = 0ull;  // time of the last progress (0: not yet sampled)
      bool fresh = WX_RS_LB_FIRST;
#if WX_RS_DIAG_LBSTATS
      wx_u32 lb_rounds = 0, lb_sleeps = 0;
#endif
#if WX_RS_SKIP
      wx_i64 skip_next = WX_RS_SKIP_MIN;  // span at which the next {S} word is published
#endif
      while (true) {
        wx_u64 wv[WX_RS_LBW];
#pragma unroll
        for (int j = 0; j < WX_RS_LBW; ++j)
          wv[j] = (j == 0 && fresh) ? first
                  : p - j >= 0    ? wx::ld_agent(&a.status[(wx_u64)(p - j) * 256 + tid])
                                  : (E | WX_RS_FLAG_P);
        fresh = false;
        int stop = WX_RS_LBW;  // index of the first unpublished word
        bool done = false;
#if WX_RS_SKIP
        wx_i64 jump = 0;  // a skip word ends the round: the walk resumes at p - jump
#endif
#pragma unroll
        for (int j = 0; j < WX_RS_LBW; ++j) {
#if WX_RS_SKIP
          if (stop == WX_RS_LBW && !done && jump == 0) {
            const wx_u64 flag = (wv[j] >> 56) & 3ull;
            if ((wv[j] >> 58) != (wx_u64)a.epoch || flag == 0ull) {
              stop = j;
            } else if (flag == 3ull) {  // {S}: tiles (p - j - span, p - j] summed by a walker
              excl += wv[j] & WX_RS_SKIP_SUM;
              jump = j + 1 + (wx_i64)((wv[j] >> 40) & 0xffffull);
            } else {
              excl += wv[j] & WX_RS_VAL_MASK;
              done = flag == 2ull;
            }
          }
#else
          if (stop == WX_RS_LBW && !done) {
            const wx_u64 flag = (wv[j] >> 56) & 3ull;
            if ((wv[j] >> 58) != (wx_u64)a.epoch || flag == 0ull) {
              stop = j;
            } else {
              excl += wv[j] & WX_RS_VAL_MASK;
              done = flag == 2ull;
            }
          }
#endif
        }
#if WX_RS_DIAG_LBSTATS
        ++lb_rounds;
#endif
        if (done) break;
#if WX_RS_SKIP
        if (jump != 0 || stop == WX_RS_LBW) {
          p -= jump != 0 ? jump : WX_RS_LBW;
          t_last = 0ull;  // progress
          // publish what this walk has summed, own count included, so that
          // a successor reading this tile's word jumps over the whole span
          const wx_i64 span = (wx_i64)tile - p;  // tiles (p, tile]
          if (span >= skip_next && span <= 65536) {
            wx::st_agent(&row[tid], E | (3ull << 56) | ((wx_u64)(span - 1) << 40) | (excl + tot));
            skip_next = span * WX_RS_SKIP_GROW;
          }
          continue;
        }
#else
        if (stop == WX_RS_LBW) {
          p -= WX_RS_LBW;
          t_last = 0ull;  // progress
          continue;
        }
#endif
        if (stop > 0) t_last = 0ull;
        p -= stop;
#if WX_RS_DIAG_LBSTATS
        ++lb_sleeps;
#endif
        if (WX_RS_SLEEP) __builtin_amdgcn_s_sleep(WX_RS_SLEEP);
        if ((++spins & 63u) == 0u) {
          // abort only after WX_STALL_TICKS with this digit's chain not moving
          const wx_u64 now = __builtin_amdgcn_s_memrealtime();
          if (t_last == 0ull) {
            t_last = now;
          } else if (now - t_last > WX_STALL_TICKS) {
            atomicOr(a.err, WX_DEVERR_LOOKBACK);
            atomicExch(&a.ctl[1], 1u);
          }
          if (__hip_atomic_load(&a.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
        }
      }
      wx::st_agent(&row[tid], E | WX_RS_FLAG_P | (excl + tot));
#if WX_RS_DIAG_LBSTATS
      if (tid == 0) {
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
    }
    S.gb[tid] = a.digit_base[tid] + (wx_u32)excl - ld;
    S.ld[tid] = ld;
  }
}

#ifndef WX_RS_LB_PAIR
// Paired look-back (key tiles): digit d's walk is shared by lanes 2d and
// 2d + 1 of the whole 512-thread tile (waves 4-7 used to idle through it),
// each loading WX_RS_LBW predecessor words per round -- half 0 the nearer,
// half 1 the next ones -- and combining their partial results with one
// lane shuffle, so a round covers 2 x WX_RS_LBW predecessors at the
// registers of WX_RS_LBW (128 VGPRs, no spill).  Correct, and slower: 14.60
// vs 13.72 ms per 1e9 float keys in one process, three alternating rounds
// (profiles/r03/abl_sort_lbpair.txt) -- the walk waits on predecessors that
// have not published yet far more than it walks published ones, and the
// doubled poll traffic costs more than the halved round count saves.  Off.
#define WX_RS_LB_PAIR 0
#endif
// As wx_rs_digits, with the look-back of digit tid >> 1 on lane pair
// (tid & ~1, tid | 1): every thread of the tile holds this function's barrier.
__device__ __forceinline__ void wx_rs_digits_pair(const WxRadixPassArgs &a, WxRsShared &S, wx_u32 tile) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const wx_u64 E = (wx_u64)a.epoch << 58;
  const bool look = tile != 0 && !WX_RS_DIAG_NO_LOOKBACK;
  if (tid < 256) {
    wx_u32 tot = 0u;
#pragma unroll
    for (int w = 0; w < WX_RS_WAVES; ++w) {
      const wx_u32 c = S.wc[w][tid];
      S.wc[w][tid] = tot;
      tot += c;
    }
    wx::st_agent(&a.status[(wx_u64)tile * 256 + tid], E | (look ? WX_RS_FLAG_A : WX_RS_FLAG_P) | tot);
    wx_u32 inc = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const wx_u32 t = __shfl_up(inc, o);
      if (lane >= o) inc += t;
    }
    if (lane == 63) S.wsum[wave] = inc;
    S.tt[tid] = tot;
    S.inc[tid] = inc;
  }
  const int d = tid >> 1, h = tid & 1;
  // this half's first round, in flight across the barrier
  wx_i64 p = (wx_i64)tile - 1;
  wx_u64 wv[WX_RS_LBW];
#pragma unroll
  for (int j = 0; j < WX_RS_LBW; ++j) {
    const wx_i64 q = p - h * WX_RS_LBW - j;
    wv[j] = (look && q >= 0) ? wx::ld_agent(&a.status[(wx_u64)q * 256 + d]) : (E | WX_RS_FLAG_P);
  }
  __syncthreads();
  wx_u64 excl = 0;
  if (look) {
    wx_u32 spins = 0;
    wx_u64 t_last = 0ull;
    bool fresh = true;
    while (true) {
      if (!fresh) {
#pragma unroll
        for (int j = 0; j < WX_RS_LBW; ++j) {
          const wx_i64 q = p - h * WX_RS_LBW - j;
          wv[j] = q >= 0 ? wx::ld_agent(&a.status[(wx_u64)q * 256 + d]) : (E | WX_RS_FLAG_P);
        }
      }
      fresh = false;
      // this half: index of its first unpublished word, whether a {P} comes
      // before it, the sum up to either
      int stop = WX_RS_LBW;
      bool done = false;
      wx_u64 sum = 0;
#pragma unroll
      for (int j = 0; j < WX_RS_LBW; ++j) {
        if (stop == WX_RS_LBW && !done) {
          const wx_u64 flag = (wv[j] >> 56) & 3ull;
          if ((wv[j] >> 58) != (wx_u64)a.epoch || flag == 0ull) {
            stop = j;
          } else {
            sum += wv[j] & WX_RS_VAL_MASK;
            done = flag == 2ull;
          }
        }
      }
      const int o_stop = __shfl_xor(stop, 1);
      const int o_done = __shfl_xor((int)done, 1);
      const wx_u64 o_sum = __shfl_xor(sum, 1);
      // near = half 0's words, far = half 1's
      const int n_stop = h ? o_stop : stop, f_stop = h ? stop : o_stop;
      const bool n_done = h ? o_done != 0 : done, f_done = h ? done : o_done != 0;
      const wx_u64 n_sum = h ? o_sum : sum, f_sum = h ? sum : o_sum;
      excl += n_sum;
      int adv;  // predecessors consumed this round
      bool fin = false;
      if (n_stop < WX_RS_LBW) {
        adv = n_stop;
      } else if (n_done) {
        fin = true;
        adv = 0;
      } else {
        excl += f_sum;
        if (f_stop < WX_RS_LBW) adv = WX_RS_LBW + f_stop;
        else if (f_done) { fin = true; adv = 0; }
        else adv = 2 * WX_RS_LBW;
      }
      if (fin) break;
      p -= adv;
      if (adv == 2 * WX_RS_LBW) {
        t_last = 0ull;  // progress
        continue;
      }
      if (adv > 0) t_last = 0ull;
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 63u) == 0u) {
        const wx_u64 now = __builtin_amdgcn_s_memrealtime();
        if (t_last == 0ull) {
          t_last = now;
        } else if (now - t_last > WX_STALL_TICKS) {
          atomicOr(a.err, WX_DEVERR_LOOKBACK);
          atomicExch(&a.ctl[1], 1u);
        }
        if (__hip_atomic_load(&a.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
      }
    }
  }
  if (h == 0) {
    const wx_u32 tot = S.tt[d];
    wx_u32 ld = S.inc[d] - tot;
    for (int w = 0; w < (d >> 6); ++w) ld += S.wsum[w];
    if (WX_RS_FOLD_LD) {
#pragma unroll
      for (int w = 0; w < WX_RS_WAVES; ++w) S.wc[w][d] += ld;
    }
    if (look) wx::st_agent(&a.status[(wx_u64)tile * 256 + d], E | WX_RS_FLAG_P | (excl + tot));
    S.gb[d] = a.digit_base[d] + (wx_u32)excl - ld;
    S.ld[d] = ld;
  }
}

#ifndef WX_RS_SPLIT
// 1: the keys (and payloads) are permuted into LDS by their tile-local
// slots, which need only this tile's counts, before the look-back resolves
// the tile's global offsets: the permutation overlaps the look-back's first
// poll instead of waiting behind the whole look-back.  Key + payload tiles:
// 19.8 vs 21.8 ms per 1e9 pairs; keys alone lose the extra barrier's worth
// (15.4 vs 14.9 ms), so only the pair module sets it (abl_sort_split.txt).
#define WX_RS_SPLIT 0
#endif
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
    if (WX_RS_FOLD_LD) {
#pragma unroll
      for (int w = 0; w < WX_RS_WAVES; ++w) S.wc[w][tid] += ld;
    }
  }
  return tot;
}

// Split form, part 2 (threads 0..255): look back over the preceding tiles'
// words of digit tid to an inclusive {P} (`first` is predecessor tile - 1's
// word, loaded earlier), publish {P}, set S.gb.
__device__ __forceinline__ void wx_rs_resolve(const WxRadixPassArgs &a, WxRsShared &S, wx_u32 tile, wx_u32 tot,
                                              wx_u64 first) {
  const int tid = threadIdx.x;
  const wx_u64 E = (wx_u64)a.epoch << 58;
  const bool look = tile != 0 && !WX_RS_DIAG_NO_LOOKBACK;
  wx_u64 excl = 0;
  if (look) {
    wx_i64 p = (wx_i64)tile - 1;
    wx_u32 spins = 0;
    wx_u64 t_last = 0ull;
    bool fresh = true;
    while (true) {
      wx_u64 wv[WX_RS_LBW];
#pragma unroll
      for (int j = 0; j < WX_RS_LBW; ++j)
        wv[j] = (j == 0 && fresh) ? first
                : p - j >= 0    ? wx::ld_agent(&a.status[(wx_u64)(p - j) * 256 + tid])
                                : (E | WX_RS_FLAG_P);
      fresh = false;
      int stop = WX_RS_LBW;
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
      if (done) break;
      if (stop == WX_RS_LBW) {
        p -= WX_RS_LBW;
        t_last = 0ull;
        continue;
      }
      if (stop > 0) t_last = 0ull;
      p -= stop;
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 63u) == 0u) {
        const wx_u64 now = __builtin_amdgcn_s_memrealtime();
        if (t_last == 0ull) {
          t_last = now;
        } else if (now - t_last > WX_STALL_TICKS) {
          atomicOr(a.err, WX_DEVERR_LOOKBACK);
          atomicExch(&a.ctl[1], 1u);
        }
        if (__hip_atomic_load(&a.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
      }
    }
    wx::st_agent(&a.status[(wx_u64)tile * 256 + tid], E | WX_RS_FLAG_P | (excl + tot));
  }
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
      p = (WX_RS_FOLD_LD ? 0u : S.ld[d]) + S.wc[wave][d] + rk[i];
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
      else if (WX_RS_NT_STORE)
        __builtin_nontemporal_store(xk, a.dst_k + g);
      else
        a.dst_k[g] = xk;
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
    if (WHOLE || p < tile_n) {
      if (WX_RS_NT_STORE)
        __builtin_nontemporal_store(s_k[p], a.dst_v + gdst[j]);
      else
        a.dst_v[gdst[j]] = s_k[p];
    }
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
  if (WX_RS_SPLIT) {
    const wx_u32 tot = wx_rs_local(a, S, tile);
    __syncthreads();  // S.ld
    wx_u64 first = 0ull;
    if (tid < 256 && tile != 0 && !WX_RS_DIAG_NO_LOOKBACK)
      first = wx::ld_agent(&a.status[(wx_u64)(tile - 1) * 256 + tid]);  // in flight during the permutation
    wx_rs_scatter<KIND, ASC, WHOLE>(a, S, wb, x, rk, pos, s_k);
    if (tid < 256) wx_rs_resolve(a, S, tile, tot, first);
  } else {
    if (WX_RS_LB_PAIR && !PAY && WX_RS_BLOCK == 512)
      wx_rs_digits_pair(a, S, tile);
    else
      wx_rs_digits(a, S, tile);
    __syncthreads();
    WX_RS_STAMP(4);
    wx_rs_scatter<KIND, ASC, WHOLE>(a, S, wb, x, rk, pos, s_k);
  }
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

