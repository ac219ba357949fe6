// HBM ceiling probe for the streaming shapes the engine's kernels have:
//   read2   : read two 4-byte columns (the SUM / top-K / GROUP BY input side)
//   copy    : read one column, write one column
//   r2w     : read two columns, write 8 B for 5 of every 8 rows into a dense
//             output (the compaction's traffic mix without the scan)
// Variants: workgroups per CU, 16-byte loads in flight per lane, nontemporal.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bw_probe tools/bw_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void read2(const v4f *__restrict__ a, const v4f *__restrict__ b, size_t nq,
                                             float *out) {
  float acc = 0.f;
  size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < nq; i += U * stride) {
    v4f va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) {
        va[u] = __builtin_nontemporal_load(a + i + u * stride);
        vb[u] = __builtin_nontemporal_load(b + i + u * stride);
      } else {
        va[u] = a[i + u * stride];
        vb[u] = b[i + u * stride];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += va[u].x * vb[u].x + va[u].y * vb[u].y + va[u].z * vb[u].z + va[u].w * vb[u].w;
  }
  for (; i < nq; i += stride) acc += a[i].x * b[i].y;
  if (acc == 1234.5f) out[0] = acc;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void read1(const v4f *__restrict__ a, size_t nq, float *out) {
  float acc = 0.f;
  size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < nq; i += U * stride) {
    v4f va[U];
#pragma unroll
    for (int u = 0; u < U; ++u) va[u] = NT ? __builtin_nontemporal_load(a + i + u * stride) : a[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += va[u].x + va[u].y + va[u].z + va[u].w;
  }
  for (; i < nq; i += stride) acc += a[i].x;
  if (acc == 1234.5f) out[0] = acc;
}

// block-contiguous: per iteration a workgroup reads U * 4 KiB in one span
template <int U, bool NT>
__global__ __launch_bounds__(256) void read1c(const v4f *__restrict__ a, size_t nq, float *out) {
  float acc = 0.f;
  const size_t span = (size_t)256 * U;
  for (size_t base = (size_t)blockIdx.x * span; base < nq; base += (size_t)gridDim.x * span) {
    v4f va[U];
    if (base + span <= nq) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t i = base + u * 256 + threadIdx.x;
        va[u] = NT ? __builtin_nontemporal_load(a + i) : a[i];
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t i = base + u * 256 + threadIdx.x;
        va[u] = i < nq ? a[i] : v4f{0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += va[u].x + va[u].y + va[u].z + va[u].w;
  }
  if (acc == 1234.5f) out[0] = acc;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy1(const v4f *__restrict__ a, v4f *__restrict__ o, size_t nq) {
  size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < nq; i += U * stride) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(a + i + u * stride) : a[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], o + i + u * stride);
      else o[i + u * stride] = v[u];
    }
  }
  for (; i < nq; i += stride) o[i] = a[i];
}

// reads 2 x 16 B per lane per step; writes 2 x 10 B-equivalent: out vals and
// idx arrays each receive 5/8 of the input rows' worth of bytes, written as
// contiguous v4f/v4u so the write volume matches compaction (5 GB per 1B rows)
template <int U, bool NT>
__global__ __launch_bounds__(256) void r2w(const v4f *__restrict__ a, const v4f *__restrict__ b,
                                           v4f *__restrict__ ov, v4u *__restrict__ oi, size_t nq) {
  size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < nq; i += U * stride) {
    v4f va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      va[u] = NT ? __builtin_nontemporal_load(a + i + u * stride) : a[i + u * stride];
      vb[u] = NT ? __builtin_nontemporal_load(b + i + u * stride) : b[i + u * stride];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t j = i + u * stride;
      // 5 of 8 quads store (j % 8 < 5), output position j*5/8 (dense)
      if ((j & 7) < 5) {
        size_t p = (j >> 3) * 5 + (j & 7);
        v4f r = va[u] * vb[u];
        v4u ix = (v4u){(unsigned)j * 4, (unsigned)j * 4 + 1, (unsigned)j * 4 + 2, (unsigned)j * 4 + 3};
        if (NT) {
          __builtin_nontemporal_store(r, ov + p);
          __builtin_nontemporal_store(ix, oi + p);
        } else {
          ov[p] = r;
          oi[p] = ix;
        }
      }
    }
  }
}

// block-contiguous read 8 B + write 5 B per row (compaction mix)
template <int U, bool NT>
__global__ __launch_bounds__(256) void r2wc(const v4f *__restrict__ a, const v4f *__restrict__ b,
                                            v4f *__restrict__ ov, v4u *__restrict__ oi, size_t nq) {
  const size_t span = (size_t)256 * U;
  for (size_t base = (size_t)blockIdx.x * span; base + span <= nq; base += (size_t)gridDim.x * span) {
    v4f va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * 256 + threadIdx.x;
      va[u] = NT ? __builtin_nontemporal_load(a + i) : a[i];
      vb[u] = NT ? __builtin_nontemporal_load(b + i) : b[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t j = base + u * 256 + threadIdx.x;
      if ((j & 7) < 5) {
        const size_t p = (j >> 3) * 5 + (j & 7);
        ov[p] = va[u] * vb[u];
        oi[p] = (v4u){(unsigned)j * 4, (unsigned)j * 4 + 1, (unsigned)j * 4 + 2, (unsigned)j * 4 + 3};
      }
    }
  }
}

// block-contiguous, output written as one dense run per span (like a
// compacted tile): lanes store consecutive 16-B words of the span's output
template <int U>
__global__ __launch_bounds__(256) void r2wd(const v4f *__restrict__ a, const v4f *__restrict__ b,
                                            v4f *__restrict__ ov, v4u *__restrict__ oi, size_t nq) {
  const size_t span = (size_t)256 * U;
  const size_t ospan = span * 5 / 8;
  for (size_t base = (size_t)blockIdx.x * span, ob = (size_t)blockIdx.x * ospan; base + span <= nq;
       base += (size_t)gridDim.x * span, ob += (size_t)gridDim.x * ospan) {
    v4f va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * 256 + threadIdx.x;
      va[u] = __builtin_nontemporal_load(a + i);
      vb[u] = __builtin_nontemporal_load(b + i);
    }
    v4f acc = va[0] * vb[0];
#pragma unroll
    for (int u = 1; u < U; ++u) acc += va[u] * vb[u];  // every load stays live
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t k = u * 256 + threadIdx.x;
      if (k < ospan) {
        ov[ob + k] = acc;
        oi[ob + k] = (v4u){(unsigned)k, (unsigned)k + 1, (unsigned)k + 2, (unsigned)k + 3};
      }
    }
  }
}

// as r2wd, but the output run goes through buffer stores with an explicit
// cache policy (aux: 0 plain, 2 nt, 16 sc1, 17 sc0 sc1, 18 sc1 nt); the
// buffer base is the workgroup's output run, lanes store at 16-B offsets
template <int U, int AUX, bool READ>
__global__ __launch_bounds__(256) void r2wdb(const v4f *__restrict__ a, const v4f *__restrict__ b,
                                             v4f *__restrict__ ov, v4u *__restrict__ oi, size_t nq) {
  const size_t span = (size_t)256 * U;
  const size_t ospan = span * 5 / 8;
  for (size_t base = (size_t)blockIdx.x * span, ob = (size_t)blockIdx.x * ospan; base + span <= nq;
       base += (size_t)gridDim.x * span, ob += (size_t)gridDim.x * ospan) {
    v4f acc = {1.f, 2.f, 3.f, (float)base};
    if (READ) {
      v4f va[U], vb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t i = base + u * 256 + threadIdx.x;
        va[u] = __builtin_nontemporal_load(a + i);
        vb[u] = __builtin_nontemporal_load(b + i);
      }
      acc = va[0] * vb[0];
#pragma unroll
      for (int u = 1; u < U; ++u) acc += va[u] * vb[u];
    }
    __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(ov + ob, 0, 0x7fffffff, 0x00020000);
    __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc(oi + ob, 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned k = u * 256 + threadIdx.x;
      if (k < ospan) {
        const v4u x = __builtin_bit_cast(v4u, acc);
        const v4u y = (v4u){k, k + 1, k + 2, k + 3};
        __builtin_amdgcn_raw_buffer_store_b128(x, rv, (int)(k * 16), 0, AUX);
        __builtin_amdgcn_raw_buffer_store_b128(y, ri, (int)(k * 16), 0, AUX);
      }
    }
  }
}

// as r2wd, but the output run is written with 4-byte stores (one value per
// lane, like the compaction's LDS drain), starting `shift` floats past a
// 16-byte boundary
template <int U>
__global__ __launch_bounds__(256) void r2wd4(const v4f *__restrict__ a, const v4f *__restrict__ b,
                                             float *__restrict__ ov, unsigned *__restrict__ oi, size_t nq, int shift) {
  const size_t span = (size_t)256 * U;
  const size_t orows = span * 4 * 5 / 8;  // output values per span
  for (size_t base = (size_t)blockIdx.x * span, ob = (size_t)blockIdx.x * orows + shift; base + span <= nq;
       base += (size_t)gridDim.x * span, ob += (size_t)gridDim.x * orows) {
    v4f va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * 256 + threadIdx.x;
      va[u] = __builtin_nontemporal_load(a + i);
      vb[u] = __builtin_nontemporal_load(b + i);
    }
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) acc += va[u].x * vb[u].y + va[u].z * vb[u].w;
    for (size_t k = threadIdx.x; k < orows; k += 256) {
      ov[ob + k] = acc + (float)k;
      oi[ob + k] = (unsigned)(base * 4 + k);
    }
  }
}

// the compaction's shape step by step: 1024-thread workgroups (960 data
// threads), a tile of G groups x 16 B per lane per column, loads of tile k+1
// issued right after tile k is consumed, the (dense, aligned) output of tile
// k-1 stored one iteration later, optional barriers between the phases
template <int G, bool BAR>
__global__ __launch_bounds__(1024) void r2wt(const v4f *__restrict__ a, const v4f *__restrict__ b,
                                             v4f *__restrict__ ov, v4u *__restrict__ oi, size_t nq) {
  const int t = threadIdx.x;
  const bool data = t < 960;
  const size_t tq = (size_t)960 * G;        // quads per tile
  const size_t oq = tq * 5 / 8;             // output quads per tile
  const size_t ntiles = nq / tq;
  v4f va[G], vb[G];
  size_t tile = blockIdx.x;
  if (data && tile < ntiles)
#pragma unroll
    for (int g = 0; g < G; ++g) {
      va[g] = __builtin_nontemporal_load(a + tile * tq + g * 960 + t);
      vb[g] = __builtin_nontemporal_load(b + tile * tq + g * 960 + t);
    }
  v4f keep[G];
  bool have_prev = false;
  size_t prev = 0;
  for (; tile < ntiles + gridDim.x; tile += gridDim.x) {
    const bool have = tile < ntiles;
    if (data && have) {
#pragma unroll
      for (int g = 0; g < G; ++g) keep[g] = va[g] * vb[g];
      const size_t nx = tile + gridDim.x;
      if (nx < ntiles)
#pragma unroll
        for (int g = 0; g < G; ++g) {
          va[g] = __builtin_nontemporal_load(a + nx * tq + g * 960 + t);
          vb[g] = __builtin_nontemporal_load(b + nx * tq + g * 960 + t);
        }
    }
    if (BAR) __syncthreads();
    v4f acc = keep[0];
#pragma unroll
    for (int g = 1; g < G; ++g) acc += keep[g];  // every group's loads stay live
    if (data && have_prev) {
      for (size_t k = t; k < oq; k += 960) {
        ov[prev * oq + k] = acc;
        oi[prev * oq + k] = (v4u){(unsigned)k, 1u, 2u, 3u};
      }
    }
    if (BAR) __syncthreads();
    have_prev = have;
    prev = tile;
    if (!have) break;
  }
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  f();
  CK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main(int argc, char **argv) {
  size_t n = argc > 1 ? (size_t)atof(argv[1]) : 1000000000ull;
  size_t nq = n / 4;
  float *a, *b, *ov, *out;
  unsigned *oi;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  CK(hipMalloc(&ov, n * 4));
  CK(hipMalloc(&oi, n * 4));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 0, n * 4));
  CK(hipMemset(b, 0, n * 4));
  int cus = 256;
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  cus = pr.multiProcessorCount;
  const int reps = 15;
  int wpcs[] = {1, 2, 4, 8};
#define RUN(name, KER, bytes, ...)                                                                            \
  for (int w : wpcs) {                                                                                        \
    int g = cus * w;                                                                                          \
    float ms = time_it([&] { KER<<<g, 256>>>(__VA_ARGS__); }, reps);                                          \
    printf("%-28s wg/CU %2d  %7.3f ms  %7.1f GB/s\n", name, w, ms, (double)(bytes) / ms / 1e6);               \
  }
  RUN("read1c u8 nt", (read1c<8, true>), n * 4, (const v4f *)a, nq, out);
  RUN("r2wd u8", (r2wd<8>), n * 13, (const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq);
  if (getenv("BW_POLICY")) {
    RUN("r2wdb plain", (r2wdb<8, 0, true>), n * 13, (const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq);
    RUN("r2wdb nt", (r2wdb<8, 2, true>), n * 13, (const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq);
    RUN("r2wdb sc1", (r2wdb<8, 16, true>), n * 13, (const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq);
    RUN("r2wdb sc0sc1", (r2wdb<8, 17, true>), n * 13, (const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq);
    RUN("r2wdb sc1nt", (r2wdb<8, 18, true>), n * 13, (const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq);
    RUN("w-only plain", (r2wdb<8, 0, false>), n * 5, (const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq);
    RUN("w-only nt", (r2wdb<8, 2, false>), n * 5, (const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq);
    RUN("w-only sc1", (r2wdb<8, 16, false>), n * 5, (const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq);
    RUN("w-only sc0sc1", (r2wdb<8, 17, false>), n * 5, (const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq);
    RUN("r2wd u8 (again)", (r2wd<8>), n * 13, (const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq);
    return 0;
  }
  {
    int wp1[] = {1};
    for (int w : wp1) {
      float ms = time_it([&] { r2wt<4, false><<<cus * w, 1024>>>((const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq); }, reps);
      printf("%-28s wg/CU %2d  %7.3f ms  %7.1f GB/s\n", "r2wt g4 nobar", w, ms, n * 13.0 / ms / 1e6);
      ms = time_it([&] { r2wt<4, true><<<cus * w, 1024>>>((const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq); }, reps);
      printf("%-28s wg/CU %2d  %7.3f ms  %7.1f GB/s\n", "r2wt g4 bar", w, ms, n * 13.0 / ms / 1e6);
      ms = time_it([&] { r2wt<2, true><<<cus * w, 1024>>>((const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq); }, reps);
      printf("%-28s wg/CU %2d  %7.3f ms  %7.1f GB/s\n", "r2wt g2 bar", w, ms, n * 13.0 / ms / 1e6);
      ms = time_it([&] { r2wt<8, true><<<cus * w, 1024>>>((const v4f *)a, (const v4f *)b, (v4f *)ov, (v4u *)oi, nq); }, reps);
      printf("%-28s wg/CU %2d  %7.3f ms  %7.1f GB/s\n", "r2wt g8 bar", w, ms, n * 13.0 / ms / 1e6);
    }
  }
  return 0;
}
