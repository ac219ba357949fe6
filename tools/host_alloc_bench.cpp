// host_alloc_bench.cpp -- how fast can a host std::vector<float> result of n
// floats be made ready?  (WarpDB::query / query_multi_gpu return one; on the
// GPU box its first touch is the critical path of host-resident queries.)
//   plain      std::vector<float>(n)
//   thp        reserve + MADV_HUGEPAGE + resize (transfer.cpp host_result)
//   thp_pop_T  reserve + MADV_HUGEPAGE + MADV_POPULATE_WRITE on T threads over
//              disjoint ranges of the reserved storage + resize
// Prints one line per variant (best of 5).  Host only, no GPU.
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static std::vector<float> make(size_t n, int mode, int threads) {
  std::vector<float> v;
  if (mode == 0) {
    v.resize(n);
    return v;
  }
  v.reserve(n);
  const uintptr_t page = uintptr_t(2) << 20;
  const uintptr_t b = (reinterpret_cast<uintptr_t>(v.data()) + page - 1) & ~(page - 1);
  const uintptr_t e = reinterpret_cast<uintptr_t>(v.data() + n) & ~(page - 1);
  if (e > b) madvise(reinterpret_cast<void *>(b), e - b, MADV_HUGEPAGE);
  if (mode == 2 && e > b) {
    const size_t pages = (e - b) / page;
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
      th.emplace_back([=] {
        const size_t p0 = pages * t / threads, p1 = pages * (t + 1) / threads;
        if (p1 > p0) madvise(reinterpret_cast<void *>(b + p0 * page), (p1 - p0) * page, MADV_POPULATE_WRITE);
      });
    for (auto &x : th) x.join();
  }
  v.resize(n);
  return v;
}

int main(int argc, char **argv) {
  const size_t n = argc > 1 ? (size_t)std::atof(argv[1]) : 100000000;
  struct V { const char *name; int mode, threads; };
  const V vs[] = {{"plain", 0, 1}, {"thp", 1, 1}, {"thp_pop_1", 2, 1}, {"thp_pop_4", 2, 4}, {"thp_pop_8", 2, 8},
                  {"thp_pop_16", 2, 16}};
  for (const V &x : vs) {
    double best = 1e9;
    for (int r = 0; r < 5; ++r) {
      const double t0 = now();
      std::vector<float> v = make(n, x.mode, x.threads);
      const double t1 = now();
      best = std::min(best, t1 - t0);
      if (v[n / 2] != 0.0f) std::printf("bad\n");
    }
    std::printf("{\"variant\": \"%s\", \"bytes\": %zu, \"ms\": %.2f, \"GB_per_s\": %.1f}\n", x.name, n * 4, best * 1e3,
                n * 4 / best / 1e9);
  }
  return 0;
}
