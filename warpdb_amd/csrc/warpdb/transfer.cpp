// transfer.cpp -- host <-> HBM copies for the loaders and the multi-GPU paths
// (the reference copies pageable memory with one blocking cudaMemcpy per
// column, src/csv_loader.cpp:126-161, src/multi_gpu_utils.cpp:34-58).
//
// hipMemcpyAsync straight from the caller's pageable memory: on MI355X hosts
// the runtime moves pageable memory at the full PCIe rate (56 GB/s H2D and
// D2H, tools/pcie_bench.cpp).  A pinned staging ring (host copy overlapping
// the DMA: 20-31 GB/s, bound by one host memcpy) and pinning the caller's
// range in place were measured slower and removed in round 5.
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>

#include <algorithm>
#include <cstdlib>
#include <thread>
#include <vector>

#include "internal.hpp"

namespace warpdb {

std::vector<float> host_result(size_t n) {
  // Large host results: back the allocation with transparent huge pages
  // before first touch (a 400 MB value-initialised vector costs ≈63 ms of
  // 4 KiB page faults on the GPU box; huge pages: 21.9 ms), and populate the
  // pages from four threads (MADV_POPULATE_WRITE over disjoint ranges of the
  // reserved storage) before resize() zero-fills them: 8.8 ms
  // (tools/host_alloc_bench.cpp, profiles/r01/host_alloc.txt; 8 or 16
  // threads contend on the address-space lock: 15-17 ms).  A kernel without
  // MADV_POPULATE_WRITE (Linux < 5.14) rejects the call and resize() faults
  // the pages in as before.
  std::vector<float> v;
  v.reserve(n);
  if (n * sizeof(float) >= (size_t(64) << 20)) {
    const uintptr_t page = uintptr_t(2) << 20;
    const uintptr_t b = (reinterpret_cast<uintptr_t>(v.data()) + page - 1) & ~(page - 1);
    const uintptr_t e = (reinterpret_cast<uintptr_t>(v.data() + n)) & ~(page - 1);
    if (e > b) {
      (void)madvise(reinterpret_cast<void *>(b), e - b, MADV_HUGEPAGE);
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
      const size_t pages = (e - b) / page;
      const int T = 4;
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t)
        th.emplace_back([=] {
          const size_t p0 = pages * t / T, p1 = pages * (t + 1) / T;
          if (p1 > p0) (void)madvise(reinterpret_cast<void *>(b + p0 * page), (p1 - p0) * page, MADV_POPULATE_WRITE);
        });
      for (auto &x : th) x.join();
    }
  }
  v.resize(n);
  return v;
}

void copy_h2d(int device, hipStream_t s, void *dst, const void *src, size_t bytes) {
  if (!bytes) return;
  DevGuard g(device);
  hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s), "hipMemcpyAsync");
}

void copy_d2h(int device, hipStream_t s, void *dst, const void *src, size_t bytes) {
  if (!bytes) return;
  DevGuard g(device);
  hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
  hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
}

}  // namespace warpdb
