// multi_gpu.cpp -- row-sharded execution across every GPU of the node
// (replaces the reference's sequential device loop, src/multi_gpu_utils.cpp:5-63).
//
// One host thread per device uploads its shard, launches on its own stream
// and downloads its slice of the result, so the devices run concurrently.
// The only cross-device exchange is the final aggregate of
// run_multi_gpu_sum: one RCCL all-reduce over a communicator built once with
// ncclCommInitAll (xGMI on MI355X nodes).
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <exception>
#include <future>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <vector>

#include "warpdb/internal.hpp"
#include "warpdb/multi_gpu_utils.hpp"

namespace warpdb {

std::vector<ShardRange> plan_shards(int64_t n_rows, int devices) {
  std::vector<ShardRange> out;
  if (devices < 1) devices = 1;
  const int64_t chunk = (n_rows + devices - 1) / devices;
  for (int d = 0; d < devices; ++d) {
    const int64_t b = d * chunk, e = std::min(n_rows, b + chunk);
    if (b >= e) break;
    out.push_back({d, b, e});
  }
  return out;
}

namespace {

int device_count() {
  int n = 0;
  hip_ok(hipGetDeviceCount(&n), "hipGetDeviceCount");
  if (n < 1) throw std::runtime_error("no HIP device visible");
  return n;
}

size_t width(DataType t) { return (t == DataType::Int64 || t == DataType::Float64) ? 8 : 4; }

// Device copy of rows [b, e) of every numeric column.
struct Shard {
  std::vector<DeviceBuffer> bufs;
  Table table;
};

Shard upload_shard(const HostTable &h, int device, int64_t b, int64_t e, hipStream_t s) {
  Shard sh;
  sh.table.num_rows = e - b;
  sh.table.device = device;
  for (const auto &c : h.columns) {
    if (c.type == DataType::String) {
      sh.table.columns.push_back({c.name, c.type, nullptr, e - b});
      continue;
    }
    const size_t w = width(c.type);
    sh.bufs.emplace_back(device, w * static_cast<size_t>(e - b));
    const char *src = static_cast<const char *>(std::visit([](auto &&v) -> const void * { return v.data(); }, c.data));
    copy_h2d(device, s, sh.bufs.back().ptr, src + w * b, w * static_cast<size_t>(e - b));
    sh.table.columns.push_back({c.name, c.type, sh.bufs.back().ptr, e - b});
  }
  return sh;
}

template <typename F>
void run_per_device(const std::vector<ShardRange> &shards, F &&fn) {
  std::vector<std::exception_ptr> errs(shards.size());
  std::vector<std::thread> th;
  for (size_t i = 0; i < shards.size(); ++i)
    th.emplace_back([&, i] {
      try {
        DevGuard g(shards[i].device);
        fn(i, shards[i]);
      } catch (...) {
        errs[i] = std::current_exception();
      }
    });
  for (auto &t : th) t.join();
  for (auto &e : errs)
    if (e) std::rethrow_exception(e);
}

// One long-lived stream per device: the execution layer keys its workspaces
// by (device, stream), so reusing the streams reuses the workspaces.
hipStream_t device_stream(int device) {
  static std::mutex mu;
  static std::vector<hipStream_t> streams;
  std::lock_guard<std::mutex> lk(mu);
  if ((int)streams.size() <= device) streams.resize(device + 1, nullptr);
  if (!streams[device]) {
    DevGuard g(device);
    hip_ok(hipStreamCreateWithFlags(&streams[device], hipStreamNonBlocking), "hipStreamCreate");
  }
  return streams[device];
}

struct Comms {
  std::mutex mu;
  std::vector<ncclComm_t> comms;
};
Comms &comms_for(int ndev) {
  static Comms c;
  std::lock_guard<std::mutex> lk(c.mu);
  if ((int)c.comms.size() != ndev) {
    for (auto cm : c.comms) ncclCommDestroy(cm);
    c.comms.assign(ndev, nullptr);
    std::vector<int> devs(ndev);
    for (int i = 0; i < ndev; ++i) devs[i] = i;
    if (ncclCommInitAll(c.comms.data(), ndev, devs.data()) != ncclSuccess) {
      c.comms.clear();
      throw std::runtime_error("ncclCommInitAll failed");
    }
  }
  return c;
}

}  // namespace

std::pair<double, int64_t> run_multi_gpu_sum(const HostTable &host, const std::string &expr_cuda,
                                             const std::string &cond_cuda) {
  const int ndev = device_count();
  auto shards = plan_shards(host.num_rows(), ndev);
  if (shards.empty()) return {0.0, 0};
  std::vector<DeviceBuffer> outs(shards.size());
  std::vector<hipStream_t> streams(shards.size(), nullptr);
  std::vector<Shard> keep(shards.size());
  run_per_device(shards, [&](size_t i, const ShardRange &r) {
    streams[i] = device_stream(r.device);
    keep[i] = upload_shard(host, r.device, r.begin, r.end, streams[i]);
    outs[i] = DeviceBuffer(r.device, 16);
    WxTableView v(keep[i].table);
    wx_launch L = sync_launch(r.device, streams[i]);
    L.flags = 0;  // asynchronous; synchronised after the collective
    char err[8192];
    throw_on(wx_reduce_sum(&v.table, expr_cuda.c_str(), cond_cuda.c_str(), &L, outs[i].ptr, nullptr, nullptr, err,
                           sizeof(err)),
             err);
  });
  // one all-reduce of {sum (f64), count (i64)} across the shards' devices
  const int nshard = static_cast<int>(shards.size());
  Comms &c = comms_for(nshard);
  {
    std::lock_guard<std::mutex> lk(c.mu);
    if (ncclGroupStart() != ncclSuccess) throw std::runtime_error("ncclGroupStart failed");
    for (int i = 0; i < nshard; ++i) {
      DevGuard g(shards[i].device);
      double *p = static_cast<double *>(outs[i].ptr);
      ncclAllReduce(p, p, 1, ncclFloat64, ncclSum, c.comms[i], streams[i]);
      ncclAllReduce(p + 1, p + 1, 1, ncclInt64, ncclSum, c.comms[i], streams[i]);
    }
    if (ncclGroupEnd() != ncclSuccess) throw std::runtime_error("RCCL all-reduce failed");
  }
  double res[2] = {0, 0};
  for (int i = 0; i < nshard; ++i) {
    DevGuard g(shards[i].device);
    hip_ok(hipStreamSynchronize(streams[i]), "hipStreamSynchronize");
    wx_launch L = sync_launch(shards[i].device, streams[i]);
    char err[1024];
    throw_on(wx_check(&L, err, sizeof(err)), err);
    if (i == 0) hip_ok(hipMemcpy(res, outs[i].ptr, 16, hipMemcpyDeviceToHost), "hipMemcpy");
  }
  for (int i = 0; i < nshard; ++i) {
    DevGuard g(shards[i].device);
    keep[i] = Shard();
  }
  int64_t cnt;
  std::memcpy(&cnt, &res[1], 8);
  return {res[0], cnt};
}

}  // namespace warpdb

std::vector<float> run_multi_gpu_jit_host(const HostTable &host, const std::string &expr_cuda,
                                          const std::string &cond_cuda) {
  using namespace warpdb;
  const int64_t n = host.num_rows();
  auto shards = plan_shards(n, device_count());
  // The host result (4 B/row, first-touch bound) is allocated on its own
  // thread while the devices upload and compute; D2H waits for it.
  std::vector<float> result;
  std::promise<void> ready;
  std::shared_future<void> result_ready = ready.get_future().share();
  std::thread alloc([&] {
    try {
      result = host_result(static_cast<size_t>(n));
      ready.set_value();
    } catch (...) {
      ready.set_exception(std::current_exception());
    }
  });
  struct Join {
    std::thread &t;
    ~Join() { t.join(); }
  } join{alloc};
  run_per_device(shards, [&](size_t, const ShardRange &r) {
    hipStream_t s = device_stream(r.device);
    Shard sh = upload_shard(host, r.device, r.begin, r.end, s);
    DeviceBuffer out(r.device, sizeof(float) * static_cast<size_t>(r.end - r.begin));
    WxTableView v(sh.table);
    wx_launch L = sync_launch(r.device, s);
    L.flags = 0;
    char err[8192];
    throw_on(wx_project_filter(&v.table, expr_cuda.c_str(), cond_cuda.c_str(), &L, WX_MODE_DENSE_FILL,
                               static_cast<float *>(out.ptr), nullptr, 0, 0, nullptr, nullptr, err, sizeof(err)),
             err);
    result_ready.get();
    copy_d2h(r.device, s, result.data() + r.begin, out.ptr, sizeof(float) * static_cast<size_t>(r.end - r.begin));
    throw_on(wx_check(&L, err, sizeof(err)), err);
  });
  result_ready.get();  // n == 0: no device ran
  return result;
}
