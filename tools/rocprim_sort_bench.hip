// Baseline for wx_sort_float: rocPRIM's radix_sort_keys (the vendor library
// sort) on the same 1e9 uniform float32 keys, timed with HIP events.
// Comparison tool only; the product sort is wx_radix_* (warpdb_amd/csrc/kernels/wx_radix.hip).
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); std::exit(1); } } while (0)

__global__ void fill(float *p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned long long x = i + 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    p[i] = (float)(x >> 40) * (40.0f / 16777216.0f);
  }
}

int main(int argc, char **argv) {
  const size_t n = argc > 1 ? (size_t)std::atof(argv[1]) : 1000000000ull;
  float *a, *b, *c;
  unsigned *va, *vb;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  CK(hipMalloc(&c, n * 4));
  CK(hipMalloc(&va, n * 4));
  CK(hipMalloc(&vb, n * 4));
  fill<<<4096, 256>>>(a, n);
  size_t tmp_bytes = 0, tmp2 = 0;
  CK(rocprim::radix_sort_keys(nullptr, tmp_bytes, c, b, n));
  CK(rocprim::radix_sort_pairs(nullptr, tmp2, c, b, va, vb, n));
  void *tmp;
  CK(hipMalloc(&tmp, std::max(tmp_bytes, tmp2)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int mode = 0; mode < 2; ++mode) {
    std::vector<float> ts;
    for (int r = 0; r < 6; ++r) {
      CK(hipMemcpy(c, a, n * 4, hipMemcpyDeviceToDevice));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      if (mode == 0) CK(rocprim::radix_sort_keys(tmp, tmp_bytes, c, b, n));
      else CK(rocprim::radix_sort_pairs(tmp, tmp2, c, b, va, vb, n));
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const float med = ts[ts.size() / 2];
    std::printf("rocprim radix_sort_%s n=%zu  %.3f ms  %.2f G keys/s\n", mode ? "pairs" : "keys ", n, med, n / med / 1e6);
  }
  return 0;
}
