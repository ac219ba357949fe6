// wx_compact.hip -- the ordered stream compaction (WHERE, query_compact)
// (one of the kernel sources warpexec concatenates after wx_common.hip, whose
// header describes the prelude they expect)

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
// wx_project_compact_deep (default) is a persistent, software-pipelined
// kernel: WX_DWAVES data waves + 1 control wave per workgroup, two LDS stage
// buffers, tiles from a ticket counter (described at the kernel).
// wx_project_compact_ticket takes one tile per workgroup from the same
// counter: no pipelining (the robust fallback, WARPDB_COMPACT_SCHED=ticket).
// (A single-buffer persistent kernel, the round-1 default, was measured
// slower than the deep one and removed in round 5: profiles/r01/
// ablate_compact_deep.txt.)
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
#ifndef WX_STALL_TICKS
// A waiter gives up after this long (s_memrealtime, 100 MHz) without any
// polled word changing: progress, not poll count, so a query slowed down by
// another process sharing the GPU still completes.
#define WX_STALL_TICKS 200000000ull  // 2 s
#endif
// ... and only after this many polls without progress as well: a wave that
// is descheduled (the queue preempted) polls nothing, so a long preemption
// alone never reads as a stall (>= 65 ms of polling at >= 1 us per poll)
#define WX_STALL_SPINS (1u << 16)
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
          spins = 0;
        } else if (now - t_last > WX_STALL_TICKS && spins >= WX_STALL_SPINS) {  // sticky error for the host + this launch's abort word
          // report the nearest predecessor still unpublished, and its word
          int rj = 0, rl = 0;
          wx_u64 rw = 0ull;
#pragma unroll
          for (int j = WX_LB_PER_LANE - 1; j >= 0; --j) {
            const wx_u64 pm = __builtin_amdgcn_ballot_w64(wx_cflag(st[j], E) == 0ull && 64 * j + lane < near_p);
            if (pm) {
              rj = j;
              rl = __builtin_ctzll(pm);
              rw = __shfl(st[j], rl);
            }
          }
          if (lane == 0) {
            wx::lb_report(a.ctrs + WX_LBD_BASE, WX_LBD_COMPACT | ((wx_u64)a.epoch << 8), (wx_u64)tile,
                          (wx_u64)(look - 64 * rj - rl), rw);
            atomicOr(reinterpret_cast<unsigned int *>(&a.ctrs[1]), WX_DEVERR_LOOKBACK);
            wx::st_agent(&a.status[a.n_tiles], abort_word);
          }
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
    spins = 0;
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
__device__ __forceinline__ void wx_retire(wx_u64 *ctrs) {
  const wx_u64 done = __hip_atomic_fetch_add(&ctrs[2], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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


// The pipelined compaction.  Iteration k: the data waves evaluate tile t_k
// (loaded one iteration earlier), issue t_{k+1}'s loads and rank t_k; the
// control wave publishes t_k's aggregate and takes the ticket of iteration
// k + 2 while the data waves write t_{k-2} out of LDS (coalesced, its offset
// resolved one iteration earlier); then the data waves stage (value,
// tile-local row) of t_k while the control wave resolves t_{k-1}'s offset —
// the look-back gets a whole iteration of slack.  Two stage buffers
// (2 x 6 B per tile row).  Any grid size is correct: a workgroup that starts
// late finds the tickets taken and exits.  Output runs: a scalar head up to
// the next 32-element boundary (128 B), aligned 16-byte stores of four
// outputs per lane (2.65 -> 2.47 ms against 4-byte stores,
// tools/bw_probe.hip), a scalar tail of < 4, all nontemporal: 2.23 vs
// 2.29 ms per 1e9 rows (profiles/r01/ablate_compact_deep_nt.txt).
#ifndef WX_DEEP_NT_STORE
#define WX_DEEP_NT_STORE 1
#endif
// (Measured and dropped, round 4, profiles/r04/: half-height tiles for each
// workgroup's last iterations, +2 us per extra tile at 1e8 rows,
// abl_compact_half_tail.txt; resolving a workgroup's last tile in the
// iteration that evaluates it, 234.9 vs 233.9 us at 1e8 and 2255 vs 2250 us
// at 1e9, abl_compact_early_last.txt; store addresses from an opaque thread
// index, 2244 vs 2232 us at 1e9, abl_compact_opaque_dt.txt.)
#ifndef WX_DIAG_TIMELINE
#define WX_DIAG_TIMELINE 0  // diagnostic: per-workgroup entry / first-tile / loop-end times (diag[b * 16 ..])
#endif
extern "C" __global__ __launch_bounds__(WX_CBLOCK, 1) void wx_project_compact_deep(WxCompactArgs wx_a) {
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
    // one dequeue for both first tiles (the counter word serialises every dequeue)
    const wx_i64 t0 = (wx_i64)__hip_atomic_fetch_add(&wx_a.ctrs[0], 2ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_tiles[0] = t0;
    s_tiles[1] = t0 + 1;
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
