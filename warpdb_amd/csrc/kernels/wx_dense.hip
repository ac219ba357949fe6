// wx_dense.hip -- the dense projection (WarpDB::query, jit_compile_and_launch)
// (one of the kernel sources warpexec concatenates after wx_common.hip, whose
// header describes the prelude they expect)

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
