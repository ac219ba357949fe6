// transfer.cpp -- host <-> HBM copies for the loaders and the multi-GPU paths
// (the reference copies pageable memory with one blocking cudaMemcpy per
// column, src/csv_loader.cpp:126-161, src/multi_gpu_utils.cpp:34-58).
//
// Three modes, chosen by $WARPDB_H2D (default "pageable"):
//   pageable  hipMemcpyAsync straight from the caller's memory.  On MI355X
//             hosts the runtime moves pageable memory at the full PCIe rate
//             (measured 56 GB/s H2D and D2H, tools/pcie_bench.cpp), so this
//             is the default;
//   staged    a per-device ring of pinned buffers: the host thread copies
//             chunk i into a free slot while the DMA engine moves chunk i-1,
//             so host copy and PCIe overlap; D2H runs the ring the other way
//             (bound by one host memcpy: 20-31 GB/s measured);
//   register  pin the caller's range in place (hipHostRegister) for the
//             duration of the copy: no host copy at all, but pays page pinning.
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "internal.hpp"

namespace warpdb {
namespace {

constexpr size_t kSlotBytes = size_t(32) << 20;  // 32 MiB per pinned slot
constexpr int kSlots = 4;

struct Ring {
  std::mutex mu;
  int device = 0;
  void *slot[kSlots] = {};
  hipEvent_t ev[kSlots] = {};
  bool armed[kSlots] = {};
};

Ring &ring_for(int device) {
  static std::mutex mu;
  static std::map<int, std::unique_ptr<Ring>> rings;
  std::lock_guard<std::mutex> lk(mu);
  auto &r = rings[device];
  if (!r) {
    r.reset(new Ring);
    r->device = device;
    DevGuard g(device);
    for (int i = 0; i < kSlots; ++i) {
      hip_ok(hipHostMalloc(&r->slot[i], kSlotBytes, hipHostMallocDefault), "hipHostMalloc");
      hip_ok(hipEventCreateWithFlags(&r->ev[i], hipEventDisableTiming), "hipEventCreate");
    }
  }
  return *r;
}

}  // namespace

TransferMode transfer_mode() {
  const char *v = std::getenv("WARPDB_H2D");
  const std::string m = v ? v : "";
  if (m == "staged") return TransferMode::Staged;
  if (m == "register") return TransferMode::Register;
  return TransferMode::Pageable;
}

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
  const TransferMode mode = transfer_mode();
  if (mode == TransferMode::Pageable) {
    hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s), "hipMemcpyAsync");
    return;
  }
  if (mode == TransferMode::Register) {
    void *p = const_cast<void *>(src);
    const bool pinned = hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess;
    hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s), "hipMemcpyAsync");
    if (pinned) {
      hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
      (void)hipHostUnregister(p);
    }
    return;
  }
  Ring &r = ring_for(device);
  std::lock_guard<std::mutex> lk(r.mu);
  const char *in = static_cast<const char *>(src);
  char *out = static_cast<char *>(dst);
  int k = 0;
  for (size_t off = 0; off < bytes; off += kSlotBytes, k = (k + 1) % kSlots) {
    const size_t n = std::min(kSlotBytes, bytes - off);
    if (r.armed[k]) hip_ok(hipEventSynchronize(r.ev[k]), "hipEventSynchronize");  // slot's last DMA done
    std::memcpy(r.slot[k], in + off, n);
    hip_ok(hipMemcpyAsync(out + off, r.slot[k], n, hipMemcpyHostToDevice, s), "hipMemcpyAsync");
    hip_ok(hipEventRecord(r.ev[k], s), "hipEventRecord");
    r.armed[k] = true;
  }
  // the caller's buffer may be reused as soon as we return: every byte is in
  // a pinned slot or already on the device, so no wait is needed here
}

void copy_d2h(int device, hipStream_t s, void *dst, const void *src, size_t bytes) {
  if (!bytes) return;
  DevGuard g(device);
  const TransferMode mode = transfer_mode();
  if (mode == TransferMode::Pageable) {
    hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
    hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
    return;
  }
  if (mode == TransferMode::Register) {
    const bool pinned = hipHostRegister(dst, bytes, hipHostRegisterDefault) == hipSuccess;
    hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
    hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
    if (pinned) (void)hipHostUnregister(dst);
    return;
  }
  Ring &r = ring_for(device);
  std::lock_guard<std::mutex> lk(r.mu);
  const char *in = static_cast<const char *>(src);
  char *out = static_cast<char *>(dst);
  struct Pending {
    int slot;
    size_t off, n;
  };
  std::deque<Pending> q;
  auto drain_one = [&] {
    const Pending p = q.front();
    q.pop_front();
    hip_ok(hipEventSynchronize(r.ev[p.slot]), "hipEventSynchronize");
    std::memcpy(out + p.off, r.slot[p.slot], p.n);
  };
  int k = 0;
  for (size_t off = 0; off < bytes; off += kSlotBytes, k = (k + 1) % kSlots) {
    if (static_cast<int>(q.size()) == kSlots) drain_one();  // frees slot k (ring order)
    else if (r.armed[k]) hip_ok(hipEventSynchronize(r.ev[k]), "hipEventSynchronize");  // a previous H2D
    const size_t n = std::min(kSlotBytes, bytes - off);
    hip_ok(hipMemcpyAsync(r.slot[k], in + off, n, hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
    hip_ok(hipEventRecord(r.ev[k], s), "hipEventRecord");
    r.armed[k] = true;
    q.push_back({k, off, n});
  }
  while (!q.empty()) drain_one();
}

}  // namespace warpdb
