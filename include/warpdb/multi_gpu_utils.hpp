// multi_gpu_utils.hpp -- row-sharded execution over every visible GPU
// (reference include/multi_gpu_utils.hpp:10-12).
#pragma once
#include <string>
#include <vector>

#include "csv_loader.hpp"
#include "jit.hpp"

// Dense result of N floats in row order (non-passing rows are 0.0f).  Shards
// are contiguous ranges of ceil(N / devices) rows (src/multi_gpu_utils.cpp:24-32);
// unlike the reference, the per-device upload, launch and download run
// concurrently (one stream per device) and the module is built once per arch.
std::vector<float> run_multi_gpu_jit_host(const HostTable &host, const std::string &expr_cuda,
                                          const std::string &cond_cuda);

namespace warpdb {

struct ShardRange {
  int device;
  int64_t begin, end;
};
// ceil(N / devices) contiguous rows per device; empty shards are dropped.
std::vector<ShardRange> plan_shards(int64_t n_rows, int devices);

// SUM((float)expr) WHERE cond over a host table sharded across every GPU,
// combined with one RCCL all-reduce (ncclFloat64) over the devices.  Returns
// the sum and the passing row count.
std::pair<double, int64_t> run_multi_gpu_sum(const HostTable &host, const std::string &expr_cuda,
                                             const std::string &cond_cuda);

}  // namespace warpdb
