// pcie_bench.cpp -- PCIe-inclusive rates of the host-resident paths, per
// transfer mode ($WARPDB_H2D = pageable | staged | register):
//   upload     upload_to_gpu of a 2-column float table (8 B/row H2D)
//   multi_gpu  run_multi_gpu_jit_host("price * quantity", "price > 15"):
//              H2D 8 B/row + compaction-free dense kernel + D2H 4 B/row
//   resident_multi_gpu  WarpDB::query_multi_gpu's path: shards kept in HBM
//              after the first call, D2H 4 B/row per query
//   csv        WarpDB::query_multi_gpu_csv over a generated CSV (parse-bound)
// Prints one JSON line per (mode, path).  Build: make -C tools pcie_bench
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "warpdb/csv_loader.hpp"
#include "warpdb/internal.hpp"
#include "warpdb/multi_gpu_utils.hpp"
#include "warpdb/warpdb.hpp"

namespace {
double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

HostTable synth(int64_t n) {
  std::vector<float> p(n), q(n);
  uint64_t x = 42;
  for (int64_t i = 0; i < n; ++i) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    p[i] = static_cast<float>((x >> 40) * (40.0 / 16777216.0));
    q[i] = static_cast<float>(1 + ((x >> 20) % 100));
  }
  HostTable h;
  h.columns.push_back({"price", DataType::Float32, std::move(p)});
  h.columns.push_back({"quantity", DataType::Float32, std::move(q)});
  return h;
}
}  // namespace

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? static_cast<int64_t>(std::atof(argv[1])) : 100000000;
  const int64_t csv_rows = argc > 2 ? static_cast<int64_t>(std::atof(argv[2])) : 5000000;
  const int reps = 3;
  HostTable h = synth(n);
  const char *modes[] = {"pageable", "staged", "register"};
  int ndev = 0;
  (void)hipGetDeviceCount(&ndev);
  for (const char *m : modes) {
    setenv("WARPDB_H2D", m, 1);
    // warm: allocate rings, compile the kernel
    {
      Table t = upload_to_gpu(h, 0);
      free_table(t);
      (void)run_multi_gpu_jit_host(h, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)");
    }
    double best_up = 1e30, best_mg = 1e30;
    for (int r = 0; r < reps; ++r) {
      double t0 = now();
      Table t = upload_to_gpu(h, 0);
      double t1 = now();
      free_table(t);
      best_up = std::min(best_up, t1 - t0);
      t0 = now();
      auto out = run_multi_gpu_jit_host(h, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)");
      t1 = now();
      best_mg = std::min(best_mg, t1 - t0);
      if (out.size() != static_cast<size_t>(n)) return 2;
    }
    std::printf("{\"mode\": \"%s\", \"path\": \"upload\", \"rows\": %lld, \"s\": %.4f, \"GB_per_s\": %.2f}\n", m,
                (long long)n, best_up, n * 8.0 / best_up / 1e9);
    std::printf("{\"mode\": \"%s\", \"path\": \"multi_gpu\", \"gpus\": %d, \"rows\": %lld, \"s\": %.4f, "
                "\"rows_per_s\": %.3e, \"pcie_GB_per_s\": %.2f}\n",
                m, ndev, (long long)n, best_mg, n / best_mg, n * 12.0 / best_mg / 1e9);
    std::fflush(stdout);
  }
  // WarpDB::query_multi_gpu on the same table: shards resident after the
  // first call, so a query moves only its 4 B/row result over PCIe
  {
    setenv("WARPDB_H2D", "pageable", 1);
    warpdb::ResidentShards rs(h);
    (void)rs.dense("(price[idx] * quantity[idx])", "(price[idx] > 15.0f)");
    double best = 1e30;
    for (int r = 0; r < reps; ++r) {
      const double t0 = now();
      auto out = rs.dense("(price[idx] * quantity[idx])", "(price[idx] > 15.0f)");
      best = std::min(best, now() - t0);
      if (out.size() != static_cast<size_t>(n)) return 2;
    }
    std::printf("{\"mode\": \"pageable\", \"path\": \"resident_multi_gpu\", \"gpus\": %d, \"rows\": %lld, \"s\": %.4f, "
                "\"rows_per_s\": %.3e, \"pcie_GB_per_s\": %.2f}\n",
                ndev, (long long)n, best, n / best, n * 4.0 / best / 1e9);
    std::fflush(stdout);
  }
  // components of the dense multi-GPU path (one device, 4 B/row result)
  {
    const size_t bytes = sizeof(float) * static_cast<size_t>(n);
    void *d = nullptr;
    double t0 = now();
    (void)hipMalloc(&d, bytes);
    (void)hipMemset(d, 0, bytes);
    (void)hipDeviceSynchronize();
    double t1 = now();
    std::printf("{\"path\": \"hipMalloc+memset\", \"bytes\": %zu, \"s\": %.4f}\n", bytes, t1 - t0);
    t0 = now();
    std::vector<float> fresh(static_cast<size_t>(n), 0.0f);
    t1 = now();
    std::printf("{\"path\": \"vector_zero_init\", \"bytes\": %zu, \"s\": %.4f}\n", bytes, t1 - t0);
    t0 = now();
    std::vector<float> huge = warpdb::host_result(static_cast<size_t>(n));
    t1 = now();
    std::printf("{\"path\": \"host_result (THP)\", \"bytes\": %zu, \"s\": %.4f}\n", bytes, t1 - t0);
    for (const char *m : modes) {
      setenv("WARPDB_H2D", m, 1);
      warpdb::copy_d2h(0, nullptr, fresh.data(), d, bytes);  // warm
      double best = 1e30;
      for (int r = 0; r < reps; ++r) {
        t0 = now();
        warpdb::copy_d2h(0, nullptr, fresh.data(), d, bytes);
        best = std::min(best, now() - t0);
      }
      std::printf("{\"mode\": \"%s\", \"path\": \"d2h_touched\", \"bytes\": %zu, \"s\": %.4f, \"GB_per_s\": %.2f}\n",
                  m, bytes, best, bytes / best / 1e9);
      std::vector<float> cold(static_cast<size_t>(n));
      t0 = now();
      warpdb::copy_d2h(0, nullptr, cold.data(), d, bytes);
      t1 = now();
      std::printf("{\"mode\": \"%s\", \"path\": \"d2h_fresh_vector\", \"s\": %.4f}\n", m, t1 - t0);
    }
    t0 = now();
    (void)hipFree(d);
    std::printf("{\"path\": \"hipFree\", \"s\": %.4f}\n", now() - t0);
    std::fflush(stdout);
  }
  // streaming CSV (staged transfers): parse-bound, pipelined with the GPUs
  {
    setenv("WARPDB_H2D", "staged", 1);
    const std::string path = "/tmp/warpdb_pcie_bench.csv";
    {
      std::ofstream f(path);
      f << "price,quantity\n";
      const auto &p = std::get<std::vector<float>>(h.columns[0].data);
      const auto &q = std::get<std::vector<float>>(h.columns[1].data);
      for (int64_t i = 0; i < csv_rows && i < n; ++i) f << p[i] << ',' << q[i] << '\n';
    }
    const double t0 = now();
    auto r = WarpDB::query_multi_gpu_csv(path, "price * quantity WHERE price > 15", 1000000);
    const double t1 = now();
    std::printf("{\"mode\": \"staged\", \"path\": \"csv_stream\", \"rows\": %zu, \"s\": %.4f, \"rows_per_s\": %.3e}\n",
                r.size(), t1 - t0, r.size() / (t1 - t0));
    std::remove(path.c_str());
  }
  return 0;
}
