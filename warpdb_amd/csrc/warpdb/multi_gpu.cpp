// multi_gpu.cpp -- row-sharded execution across every GPU of the node
// (replaces the reference's sequential device loop, src/multi_gpu_utils.cpp:5-63).
//
// One host thread per device uploads its shard, launches on its own stream
// and downloads its slice of the result, so the devices run concurrently.
// The cross-device exchanges are the aggregates' (SURVEY.md 8(e)), each ONE
// RCCL all-reduce over a communicator built once with ncclCommInitAll (xGMI
// on MI355X nodes): SUM {sum, count} as two doubles, GROUP BY the key window
// plus one slot of out-of-window groups per shard (wx_group_partials_slots),
// top-K one all-gather of wx_topk_record candidates.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <condition_variable>
#include <cstring>
#include <exception>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <vector>

#include "warpdb/internal.hpp"
#include "warpdb/multi_gpu_utils.hpp"

namespace warpdb {

namespace {

int device_count() {
  int n = 0;
  hip_ok(hipGetDeviceCount(&n), "hipGetDeviceCount");
  if (n < 1) throw std::runtime_error("no HIP device visible");
  return n;
}

// Test hook: WARPDB_VIRTUAL_SHARDS=k plans k shards over the visible devices
// round robin, so with k above the device count several shards share a
// device and the multi-shard code (a thread per shard, the shard plan,
// per-shard scratch, the exchanges, the merges) runs on a one-GPU box.
// Shards that share a device cannot form an RCCL communicator; their
// exchanges stage through the host (see allreduce_f64, ResidentShards::topk).
int virtual_shards() {
  const char *v = std::getenv("WARPDB_VIRTUAL_SHARDS");
  return v ? std::max(0, std::atoi(v)) : 0;
}

// Test hook: WARPDB_EXCHANGE_ONE_RANK=1 runs the RCCL exchanges even for a
// single shard (a one-device communicator), so a one-GPU box executes the
// ncclAllReduce / ncclAllGather calls and the buffers they hand over.
bool exchange_one_rank() {
  const char *v = std::getenv("WARPDB_EXCHANGE_ONE_RANK");
  return v && v[0] == '1' && v[1] == 0;
}

// shards to plan when the caller asks for every device
int shard_count() {
  const int v = virtual_shards();
  return v > 0 ? v : device_count();
}

// one shard per device (the RCCL case)
bool distinct_devices(const std::vector<ShardRange> &shards) {
  std::vector<int> d;
  for (const auto &r : shards) d.push_back(r.device);
  std::sort(d.begin(), d.end());
  return std::adjacent_find(d.begin(), d.end()) == d.end();
}

}  // namespace

std::vector<ShardRange> plan_shards(int64_t n_rows, int devices) {
  std::vector<ShardRange> out;
  if (devices < 1) devices = 1;
  const int physical = virtual_shards() > 0 ? device_count() : devices;
  const int64_t chunk = (n_rows + devices - 1) / devices;
  for (int d = 0; d < devices; ++d) {
    const int64_t b = d * chunk, e = std::min(n_rows, b + chunk);
    if (b >= e) break;
    out.push_back({d % physical, b, e});
  }
  return out;
}

namespace {

// `want` shards (0 = every visible device), checked against what is there
int devices_for(int want) {
  const int have = shard_count();
  if (want <= 0) return have;
  if (want > have) throw std::runtime_error("requested " + std::to_string(want) + " devices, " +
                                            std::to_string(have) + " visible");
  return want;
}

size_t width(DataType t) { return (t == DataType::Int64 || t == DataType::Float64) ? 8 : 4; }

}  // namespace

// Device copy of rows [b, e) of every numeric column (bufs empty: the
// columns are borrowed from a Table the caller keeps alive).
struct Shard {
  std::vector<DeviceBuffer> bufs;
  Table table;
};

namespace {

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
  if (shards.size() == 1) {  // one device: on this thread (a thread per query costs tens of µs)
    DevGuard g(shards[0].device);
    fn(0, shards[0]);
    return;
  }
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

// Long-lived streams per device (role 0: uploads + kernels, role 1:
// downloads): the execution layer keys its workspaces by (device, stream),
// so reusing the streams reuses the workspaces.
hipStream_t device_stream(int device, int role = 0) {
  static std::mutex mu;
  static std::vector<hipStream_t> streams[2];
  std::lock_guard<std::mutex> lk(mu);
  auto &v = streams[role];
  if ((int)v.size() <= device) v.resize(device + 1, nullptr);
  if (!v[device]) {
    DevGuard g(device);
    hip_ok(hipStreamCreateWithFlags(&v[device], hipStreamNonBlocking), "hipStreamCreate");
  }
  return v[device];
}

// Per-device scratch HBM for the host-resident pipeline, kept across calls
// and grown on demand: hipMalloc + hipFree of a 1.2 GB shard took 7-14 ms of
// a 31 ms query (1e8 rows, 1 GPU).  The lock is held for a whole call, so
// concurrent host callers take turns per device.
struct Scratch {
  std::mutex mu;
  DeviceBuffer buf;
  size_t bytes = 0;
};
Scratch &scratch_for(int device) {
  static std::mutex mu;
  // never destroyed: freeing HBM from a static destructor would run after
  // the HIP runtime's own teardown
  static auto *all = new std::map<int, std::unique_ptr<Scratch>>();
  std::lock_guard<std::mutex> lk(mu);
  auto &p = (*all)[device];
  if (!p) p.reset(new Scratch);
  return *p;
}

// One communicator set per shard count over devices 0..n-1 (plan_shards'
// assignment), built once and never destroyed: ResidentShards objects with
// different shard counts each use their own set, and no set is torn down
// while another thread may enqueue on it.  A caller holds `mu` for the whole
// ncclGroupStart .. ncclGroupEnd of one collective.
struct Comms {
  std::mutex mu;
  std::vector<ncclComm_t> comms;
};
Comms &comms_for(int ndev) {
  static std::mutex mu;
  static auto *all = new std::map<int, std::unique_ptr<Comms>>();  // never freed (outlives HIP teardown)
  std::lock_guard<std::mutex> lk(mu);
  auto &p = (*all)[ndev];
  if (!p) {
    std::unique_ptr<Comms> c(new Comms);
    c->comms.assign(ndev, nullptr);
    std::vector<int> devs(ndev);
    for (int i = 0; i < ndev; ++i) devs[i] = i;
    if (ncclCommInitAll(c->comms.data(), ndev, devs.data()) != ncclSuccess) throw std::runtime_error("ncclCommInitAll failed");
    p = std::move(c);
  }
  return *p;
}

}  // namespace

namespace {

// Host -> device copy ordered on the shard's stream, where the kernels that
// read it run (a null-stream hipMemcpy from pageable memory may return before
// the data lands, and the shard streams are non-blocking); synchronous, so the
// host buffer may go out of scope.
void h2d_ordered(void *dst, const void *src, size_t bytes, hipStream_t s) {
  hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s), "hipMemcpyAsync");
  hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
}

// ncclAllGather of `bytes` bytes per shard: every shard's `recv` receives
// all shards' `send` buffers in shard order (co-located virtual shards go
// through the host; one shard copies unless the one-rank test hook is on).
void allgather_bytes(const std::vector<ShardRange> &shards, const std::vector<void *> &send,
                     const std::vector<void *> &recv, const std::vector<hipStream_t> &streams, size_t bytes) {
  const size_t ns = shards.size();
  if (ns == 1 && !exchange_one_rank()) {
    DevGuard g(shards[0].device);
    hip_ok(hipMemcpyAsync(recv[0], send[0], bytes, hipMemcpyDeviceToDevice, streams[0]), "hipMemcpyAsync");
    return;
  }
  if (ns > 1 && !distinct_devices(shards)) {
    std::vector<char> all(bytes * ns);
    for (size_t i = 0; i < ns; ++i) {
      DevGuard g(shards[i].device);
      hip_ok(hipStreamSynchronize(streams[i]), "hipStreamSynchronize");
      hip_ok(hipMemcpy(all.data() + bytes * i, send[i], bytes, hipMemcpyDeviceToHost), "hipMemcpy");
    }
    for (size_t i = 0; i < ns; ++i) {
      DevGuard g(shards[i].device);
      h2d_ordered(recv[i], all.data(), all.size(), streams[i]);
    }
    return;
  }
  Comms &cm = comms_for(static_cast<int>(ns));
  std::lock_guard<std::mutex> clk(cm.mu);
  if (ncclGroupStart() != ncclSuccess) throw std::runtime_error("ncclGroupStart failed");
  for (size_t i = 0; i < ns; ++i) {
    DevGuard g(shards[i].device);
    if (ncclAllGather(send[i], recv[i], bytes, ncclUint8, cm.comms[i], streams[i]) != ncclSuccess) {
      (void)ncclGroupEnd();
      throw std::runtime_error("ncclAllGather failed");
    }
  }
  if (ncclGroupEnd() != ncclSuccess) throw std::runtime_error("RCCL all-gather failed");
}

// In-place ncclAllReduce(SUM, ncclFloat64) of `count` doubles of every
// shard's buffer, one call per device inside one group (devices 0..n-1, as
// plan_shards assigns them).  A single shard has nothing to exchange.
void allreduce_f64(const std::vector<ShardRange> &shards, const std::vector<double *> &bufs,
                   const std::vector<hipStream_t> &streams, size_t count) {
  const int nshard = static_cast<int>(shards.size());
  if (nshard < 1 || (nshard < 2 && !exchange_one_rank())) return;
  if (!distinct_devices(shards)) {  // co-located shards (WARPDB_VIRTUAL_SHARDS): sum through the host
    std::vector<double> acc(count, 0.0), part(count);
    for (int i = 0; i < nshard; ++i) {
      DevGuard g(shards[i].device);
      hip_ok(hipStreamSynchronize(streams[i]), "hipStreamSynchronize");
      hip_ok(hipMemcpy(part.data(), bufs[i], count * sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
      for (size_t j = 0; j < count; ++j) acc[j] += part[j];
    }
    for (int i = 0; i < nshard; ++i) {
      DevGuard g(shards[i].device);
      h2d_ordered(bufs[i], acc.data(), count * sizeof(double), streams[i]);
    }
    return;
  }
  Comms &c = comms_for(nshard);
  std::lock_guard<std::mutex> lk(c.mu);
  if (ncclGroupStart() != ncclSuccess) throw std::runtime_error("ncclGroupStart failed");
  for (int i = 0; i < nshard; ++i) {
    DevGuard g(shards[i].device);
    double *p = bufs[i];
    if (ncclAllReduce(p, p, count, ncclFloat64, ncclSum, c.comms[i], streams[i]) != ncclSuccess) {
      (void)ncclGroupEnd();
      throw std::runtime_error("ncclAllReduce failed");
    }
  }
  if (ncclGroupEnd() != ncclSuccess) throw std::runtime_error("RCCL all-reduce failed");
}

// SUM over shards already in HBM: one reduce per device, then one RCCL
// all-reduce of {sum (f64), count (i64)} across the shards' devices.
// Exchange timing of resident-shard queries: an event pair per device and
// query, recorded on the shard's stream around the collective and the merge.
struct ExchangeTimer {
  bool kernels = false, exchange = false;
  std::vector<std::vector<std::pair<hipEvent_t, hipEvent_t>>> ev;  // [shard][query]
  std::vector<hipEvent_t> open;                                     // [shard] the pending start event
  void begin(const std::vector<ShardRange> &ranges, const std::vector<hipStream_t> &streams) {
    if (!exchange) return;
    ev.resize(ranges.size());
    open.assign(ranges.size(), nullptr);
    for (size_t i = 0; i < ranges.size(); ++i) {
      DevGuard g(ranges[i].device);
      hip_ok(hipEventCreateWithFlags(&open[i], hipEventDisableSystemFence), "hipEventCreate");
      hip_ok(hipEventRecord(open[i], streams[i]), "hipEventRecord");
    }
  }
  void end(const std::vector<ShardRange> &ranges, const std::vector<hipStream_t> &streams) {
    if (!exchange || open.size() != ranges.size()) return;
    for (size_t i = 0; i < ranges.size(); ++i) {
      DevGuard g(ranges[i].device);
      hipEvent_t e = nullptr;
      hip_ok(hipEventCreateWithFlags(&e, hipEventDisableSystemFence), "hipEventCreate");
      hip_ok(hipEventRecord(e, streams[i]), "hipEventRecord");
      ev[i].push_back({open[i], e});
    }
    open.clear();
  }
  int32_t flags() const { return kernels ? WX_F_TIME : 0; }
};

std::pair<double, int64_t> sum_over_shards(const std::vector<ShardRange> &shards, std::vector<Shard> &keep,
                                           const std::string &expr_cuda, const std::string &cond_cuda,
                                           const HostTable *upload_from, std::vector<DeviceBuffer> *cached = nullptr,
                                           ExchangeTimer *timer = nullptr) {
  if (shards.empty()) return {0.0, 0};
  std::vector<DeviceBuffer> local;
  std::vector<DeviceBuffer> &outs = cached ? *cached : local;  // {sum, count} per shard (kept by resident shards)
  if (outs.size() != shards.size()) {
    outs.clear();
    outs.resize(shards.size());
  }
  std::vector<hipStream_t> streams(shards.size(), nullptr);
  run_per_device(shards, [&](size_t i, const ShardRange &r) {
    streams[i] = device_stream(r.device);
    if (upload_from) keep[i] = upload_shard(*upload_from, r.device, r.begin, r.end, streams[i]);
    if (!outs[i].ptr) outs[i] = DeviceBuffer(r.device, 16);
    WxTableView v(keep[i].table);
    wx_launch L = sync_launch(r.device, streams[i]);
    L.flags = WX_F_F64_COUNTS | (timer ? timer->flags() : 0);  // {sum, count} as two doubles; asynchronous until after the collective
    char err[8192];
    throw_on(wx_reduce_sum(&v.table, expr_cuda.c_str(), cond_cuda.c_str(), &L, outs[i].ptr, nullptr, nullptr, err,
                           sizeof(err)),
             err);
  });
  const int nshard = static_cast<int>(shards.size());
  std::vector<double *> ptrs;
  for (auto &o : outs) ptrs.push_back(static_cast<double *>(o.ptr));
  const bool coll = nshard > 1 || exchange_one_rank();
  if (coll && timer) timer->begin(shards, streams);
  allreduce_f64(shards, ptrs, streams, 2);
  if (coll && timer) timer->end(shards, streams);
  double res[2] = {0, 0};
  for (int i = 0; i < nshard; ++i) {
    DevGuard g(shards[i].device);
    hip_ok(hipStreamSynchronize(streams[i]), "hipStreamSynchronize");
    wx_launch L = sync_launch(shards[i].device, streams[i]);
    char err[1024];
    throw_on(wx_check(&L, err, sizeof(err)), err);
    if (i == 0) hip_ok(hipMemcpy(res, outs[i].ptr, 16, hipMemcpyDeviceToHost), "hipMemcpy");
  }
  return {res[0], static_cast<int64_t>(res[1])};
}

}  // namespace

std::pair<double, int64_t> run_multi_gpu_sum(const HostTable &host, const std::string &expr_cuda,
                                             const std::string &cond_cuda) {
  auto shards = plan_shards(host.num_rows(), shard_count());
  std::vector<Shard> keep(shards.size());
  auto r = sum_over_shards(shards, keep, expr_cuda, cond_cuda, &host);
  for (size_t i = 0; i < keep.size(); ++i) {
    DevGuard g(shards[i].device);
    keep[i] = Shard();
  }
  return r;
}

// ------------------------------------------------------- resident shards
// Per-shard device buffers of the GROUP BY exchange, kept across queries.
struct GroupScratch {
  int64_t cap = 0;
  size_t win_doubles = 0;  // the one-collective exchange buffer (window + slots)
  int lists = 0;           // records `all` holds
  // rec: this shard's out-of-window groups as one list record
  // (WX_GROUP_LIST_BYTES(cap): count | keys | sums | counts); all: every
  // shard's record after the all-gather of the many-key fallback
  DeviceBuffer win, rec, all, ok, os, oc, ng;
  char *r() const { return static_cast<char *>(rec.ptr); }
  int32_t *xk() const { return reinterpret_cast<int32_t *>(r() + 8); }
  double *xs() const { return reinterpret_cast<double *>(r() + WX_GROUP_LIST_SUMS_OFF(cap)); }
  int64_t *xc() const { return reinterpret_cast<int64_t *>(r() + WX_GROUP_LIST_COUNTS_OFF(cap)); }
  int64_t *nx() const { return reinterpret_cast<int64_t *>(r()); }
};

// Per-shard top-K candidates and their all-gathered copies (k <= 32).
struct TopkScratch {
  // wx_topk_record: [keys f32 x 32 | vals f32 x 32 | rows i64 x 32 | count i64], x shards for `all`;
  // `out` the merged global top-K in the same layout
  DeviceBuffer cand, all, out;
  int shards = 0;
  // k > 32: head records of capacity hcap (WX_HEAD_RECORD_BYTES), all shards'
  // after the all-gather, and the merged head (keys f32 | rows i64 | vals f32)
  DeviceBuffer hrec, hall, hkeys, hrows, hvals;
  int64_t hcap = 0, hout = 0;
  int hshards = 0;
};
constexpr size_t kTopkMax = 32;
constexpr size_t kTopkRec = kTopkMax * 4 + kTopkMax * 4 + kTopkMax * 8 + 8;  // bytes per shard record

struct ResidentShards::Impl {
  int64_t n = 0;
  ExchangeTimer timer;
  std::vector<ShardRange> ranges;
  std::vector<Shard> shards;
  std::vector<GroupScratch> group;
  std::vector<TopkScratch> topk;
  std::vector<DeviceBuffer> sum_out;  // {sum, count} per shard, kept across queries
  // pinned host staging for the first kStage groups of a GROUP BY result (one
  // stream sync per query instead of one per small pageable copy)
  char *stage = nullptr;
  std::mutex mu;  // one query at a time per object (shared workspaces and scratch)
};

ResidentShards::ResidentShards() : impl_(new Impl) {}

ResidentShards::ResidentShards(const HostTable &host, int devices) : impl_(new Impl) {
  impl_->n = host.num_rows();
  impl_->ranges = plan_shards(impl_->n, devices_for(devices));
  impl_->shards.resize(impl_->ranges.size());
  run_per_device(impl_->ranges, [&](size_t i, const ShardRange &r) {
    hipStream_t s = device_stream(r.device);
    impl_->shards[i] = upload_shard(host, r.device, r.begin, r.end, s);
    hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
  });
}

std::unique_ptr<ResidentShards> ResidentShards::borrow(const Table &table) {
  std::unique_ptr<ResidentShards> r(new ResidentShards());
  r->impl_->n = table.num_rows;
  if (table.num_rows > 0) {
    r->impl_->ranges.push_back({table.device, 0, table.num_rows});
    r->impl_->shards.resize(1);
    r->impl_->shards[0].table = table;  // column pointers only; the caller owns the memory
  }
  return r;
}

std::unique_ptr<ResidentShards> ResidentShards::synthetic(int64_t n_rows, const std::vector<SyntheticColumn> &cols,
                                                          int devices) {
  std::unique_ptr<ResidentShards> r(new ResidentShards());
  Impl &im = *r->impl_;
  im.n = n_rows;
  im.ranges = plan_shards(n_rows, devices_for(devices));
  im.shards.resize(im.ranges.size());
  run_per_device(im.ranges, [&](size_t i, const ShardRange &sr) {
    hipStream_t s = device_stream(sr.device);
    Shard &sh = im.shards[i];
    const int64_t rows = sr.end - sr.begin;
    sh.table.num_rows = rows;
    sh.table.device = sr.device;
    for (const auto &c : cols) {
      if (c.type == DataType::String) throw std::runtime_error("synthetic string columns are not supported");
      sh.bufs.emplace_back(sr.device, width(c.type) * static_cast<size_t>(rows));
      wx_launch L = sync_launch(sr.device, s);
      char err[1024];
      // rows are generated at their global row numbers: every shard holds
      // exactly the rows a single-device table would have
      throw_on(wx_fill_synthetic(sh.bufs.back().ptr, static_cast<int32_t>(c.type), rows, c.seed, c.kind, c.lo, c.hi,
                                 sr.begin, &L, err, sizeof(err)),
               err);
      sh.table.columns.push_back({c.name, c.type, sh.bufs.back().ptr, rows});
    }
  });
  return r;
}

ResidentShards::~ResidentShards() {
  for (size_t i = 0; i < impl_->shards.size(); ++i) {
    DevGuard g(impl_->ranges[i].device);
    impl_->shards[i] = Shard();
    if (i < impl_->group.size()) impl_->group[i] = GroupScratch();
    if (i < impl_->topk.size()) impl_->topk[i] = TopkScratch();
    if (i < impl_->sum_out.size()) impl_->sum_out[i] = DeviceBuffer();
  }
  if (impl_->stage) (void)hipHostFree(impl_->stage);
}

int64_t ResidentShards::num_rows() const { return impl_->n; }

int ResidentShards::num_shards() const { return static_cast<int>(impl_->ranges.size()); }

std::vector<ShardRange> ResidentShards::ranges() const { return impl_->ranges; }

std::vector<float> ResidentShards::dense(const std::string &expr_cuda, const std::string &cond_cuda) const {
  std::lock_guard<std::mutex> lk(impl_->mu);
  std::vector<float> result = host_result(static_cast<size_t>(impl_->n));
  run_per_device(impl_->ranges, [&](size_t i, const ShardRange &r) {
    hipStream_t s = device_stream(r.device);
    const int64_t rows = r.end - r.begin;
    Scratch &scr = scratch_for(r.device);
    std::lock_guard<std::mutex> scr_lock(scr.mu);
    const size_t bytes = sizeof(float) * static_cast<size_t>(rows);
    if (scr.bytes < bytes) {
      scr.buf = DeviceBuffer();
      scr.buf = DeviceBuffer(r.device, bytes);
      scr.bytes = bytes;
    }
    float *out = static_cast<float *>(scr.buf.ptr);
    WxTableView v(impl_->shards[i].table);
    wx_launch L = sync_launch(r.device, s);
    L.flags = 0;
    char err[8192];
    throw_on(wx_project_filter(&v.table, expr_cuda.c_str(), cond_cuda.c_str(), &L, WX_MODE_DENSE_FILL, out, nullptr,
                               0, 0, nullptr, nullptr, err, sizeof(err)),
             err);
    copy_d2h(r.device, s, result.data() + r.begin, out, bytes);
    throw_on(wx_check(&L, err, sizeof(err)), err);
  });
  return result;
}

// ORDER BY .. LIMIT k over the shards: wx_topk per device
// (global row numbers via the shard's row base) into one wx_topk_record,
// ONE ncclAllGather of the records (bytes), then wx_topk_merge of the
// <= 32 x shards candidates on the first shard's device.
// ORDER BY .. LIMIT k > 32 over the shards: wx_order_head per device (this
// shard's first k rows in ORDER BY order, global rows) into a head record of
// capacity k, ONE ncclAllGather of the records, wx_head_merge on the first
// shard's device (the same stable order: ties by ascending row).
TopkResult ResidentShards::topk_heads(const std::string &order_cuda, const std::string &cond_cuda,
                                      const std::string &select_cuda, int64_t k, bool descending) const {
  TopkResult res;
  const auto &ranges = impl_->ranges;
  const size_t ns = ranges.size();
  if (ns == 0) return res;
  if (impl_->topk.size() < ns) impl_->topk.resize(ns);
  const size_t rec = static_cast<size_t>(WX_HEAD_RECORD_BYTES(k));
  std::vector<hipStream_t> streams(ns, nullptr);
  run_per_device(ranges, [&](size_t i, const ShardRange &r) {
    streams[i] = device_stream(r.device);
    TopkScratch &t = impl_->topk[i];
    if (t.hcap != k || t.hshards != static_cast<int>(ns)) {
      t.hrec = DeviceBuffer(r.device, rec);
      t.hall = DeviceBuffer(r.device, rec * ns);
      t.hcap = k;
      t.hshards = static_cast<int>(ns);
    }
    WxTableView v(impl_->shards[i].table);
    wx_launch L = sync_launch(r.device, streams[i]);
    L.flags = 0;
    char err[8192];
    throw_on(wx_order_head(&v.table, order_cuda.c_str(), cond_cuda.c_str(),
                           select_cuda.empty() ? nullptr : select_cuda.c_str(), k, descending ? 1 : 0, &L, r.begin,
                           t.hrec.ptr, k, err, sizeof(err)),
             err);
  });
  bool gathered = ns > 1;
  if (ns > 1 && !distinct_devices(ranges)) {  // co-located shards (WARPDB_VIRTUAL_SHARDS): through the host
    std::vector<char> all(rec * ns);
    for (size_t i = 0; i < ns; ++i) {
      DevGuard g(ranges[i].device);
      hip_ok(hipStreamSynchronize(streams[i]), "hipStreamSynchronize");
      hip_ok(hipMemcpy(all.data() + rec * i, impl_->topk[i].hrec.ptr, rec, hipMemcpyDeviceToHost), "hipMemcpy");
    }
    DevGuard g(ranges[0].device);
    h2d_ordered(impl_->topk[0].hall.ptr, all.data(), all.size(), streams[0]);
  } else if (ns > 1 || exchange_one_rank()) {
    gathered = true;
    impl_->timer.begin(ranges, streams);
    Comms &cm = comms_for(static_cast<int>(ns));
    std::lock_guard<std::mutex> clk(cm.mu);
    if (ncclGroupStart() != ncclSuccess) throw std::runtime_error("ncclGroupStart failed");
    for (size_t i = 0; i < ns; ++i) {
      DevGuard g(ranges[i].device);
      if (ncclAllGather(impl_->topk[i].hrec.ptr, impl_->topk[i].hall.ptr, rec, ncclUint8, cm.comms[i], streams[i]) !=
          ncclSuccess) {
        (void)ncclGroupEnd();
        throw std::runtime_error("ncclAllGather failed");
      }
    }
    if (ncclGroupEnd() != ncclSuccess) throw std::runtime_error("RCCL all-gather failed");
  }
  TopkScratch &t0 = impl_->topk[0];
  const int dev0 = ranges[0].device;
  if (t0.hout < k) {
    t0.hkeys = DeviceBuffer(dev0, sizeof(float) * k);
    t0.hrows = DeviceBuffer(dev0, sizeof(int64_t) * k);
    t0.hvals = DeviceBuffer(dev0, sizeof(float) * k);
    t0.hout = k;
  }
  int64_t m = 0;
  {
    DevGuard dg(dev0);
    wx_launch L = sync_launch(dev0, streams[0]);
    L.flags = 0;
    char err[1024];
    throw_on(wx_head_merge(gathered ? t0.hall.ptr : t0.hrec.ptr, static_cast<int32_t>(ns), k, k, descending ? 1 : 0,
                           &L, static_cast<float *>(t0.hkeys.ptr), static_cast<int64_t *>(t0.hrows.ptr),
                           static_cast<float *>(t0.hvals.ptr), nullptr, &m, err, sizeof(err)),
             err);
    impl_->timer.end(ranges, streams);  // no-op unless begin ran (a collective), as in topk()
    for (size_t i = 0; i < ns; ++i) {
      DevGuard g(ranges[i].device);
      hip_ok(hipStreamSynchronize(streams[i]), "hipStreamSynchronize");
      wx_launch Li = sync_launch(ranges[i].device, streams[i]);
      throw_on(wx_check(&Li, err, sizeof(err)), err);
    }
    res.keys.resize(static_cast<size_t>(m));
    res.rows.resize(static_cast<size_t>(m));
    res.values.resize(static_cast<size_t>(m));
    if (m > 0) {
      hip_ok(hipMemcpy(res.keys.data(), t0.hkeys.ptr, sizeof(float) * m, hipMemcpyDeviceToHost), "hipMemcpy");
      hip_ok(hipMemcpy(res.rows.data(), t0.hrows.ptr, sizeof(int64_t) * m, hipMemcpyDeviceToHost), "hipMemcpy");
      hip_ok(hipMemcpy(res.values.data(), t0.hvals.ptr, sizeof(float) * m, hipMemcpyDeviceToHost), "hipMemcpy");
    }
  }
  return res;
}

TopkResult ResidentShards::topk(const std::string &order_cuda, const std::string &cond_cuda,
                                const std::string &select_cuda, int64_t k, bool descending) const {
  if (k < 1) throw std::runtime_error("top-K needs k >= 1");
  if (k > static_cast<int64_t>(kTopkMax)) {
    std::lock_guard<std::mutex> lk(impl_->mu);
    return topk_heads(order_cuda, cond_cuda, select_cuda, k, descending);
  }
  std::lock_guard<std::mutex> lk(impl_->mu);
  TopkResult res;
  const auto &ranges = impl_->ranges;
  const size_t ns = ranges.size();
  if (ns == 0) return res;
  if (impl_->topk.size() < ns) impl_->topk.resize(ns);
  std::vector<hipStream_t> streams(ns, nullptr);
  run_per_device(ranges, [&](size_t i, const ShardRange &r) {
    streams[i] = device_stream(r.device);
    TopkScratch &t = impl_->topk[i];
    if (t.shards != static_cast<int>(ns)) {
      t.cand = DeviceBuffer(r.device, kTopkRec);
      t.all = DeviceBuffer(r.device, kTopkRec * ns);
      t.shards = static_cast<int>(ns);
    }
    char *c = static_cast<char *>(t.cand.ptr);
    WxTableView v(impl_->shards[i].table);
    wx_launch L = sync_launch(r.device, streams[i]);
    L.flags = impl_->timer.flags();  // asynchronous until after the collective
    char err[8192];
    throw_on(wx_topk(&v.table, order_cuda.c_str(), cond_cuda.c_str(), select_cuda.empty() ? nullptr : select_cuda.c_str(),
                     static_cast<int32_t>(k), descending ? 1 : 0, &L, r.begin, reinterpret_cast<float *>(c),
                     reinterpret_cast<int64_t *>(c + kTopkMax * 8), reinterpret_cast<float *>(c + kTopkMax * 4),
                     reinterpret_cast<int64_t *>(c + kTopkMax * 16), nullptr, err, sizeof(err)),
             err);
  });
  bool gathered = ns > 1;  // the records of every shard are in each shard's `all`
  if (ns > 1 && !distinct_devices(ranges)) {  // co-located shards (WARPDB_VIRTUAL_SHARDS): gather through the host
    std::vector<char> all(kTopkRec * ns);
    for (size_t i = 0; i < ns; ++i) {
      DevGuard g(ranges[i].device);
      hip_ok(hipStreamSynchronize(streams[i]), "hipStreamSynchronize");
      hip_ok(hipMemcpy(all.data() + kTopkRec * i, impl_->topk[i].cand.ptr, kTopkRec, hipMemcpyDeviceToHost),
             "hipMemcpy");
    }
    for (size_t i = 0; i < ns; ++i) {
      DevGuard g(ranges[i].device);
      h2d_ordered(impl_->topk[i].all.ptr, all.data(), all.size(), streams[i]);
    }
  } else if (ns > 1 || exchange_one_rank()) {
    gathered = true;
    impl_->timer.begin(ranges, streams);
    Comms &cm = comms_for(static_cast<int>(ns));
    std::lock_guard<std::mutex> clk(cm.mu);
    if (ncclGroupStart() != ncclSuccess) throw std::runtime_error("ncclGroupStart failed");
    for (size_t i = 0; i < ns; ++i) {
      DevGuard g(ranges[i].device);
      if (ncclAllGather(impl_->topk[i].cand.ptr, impl_->topk[i].all.ptr, kTopkRec, ncclUint8, cm.comms[i],
                        streams[i]) != ncclSuccess) {
        (void)ncclGroupEnd();
        throw std::runtime_error("ncclAllGather failed");
      }
    }
    if (ncclGroupEnd() != ncclSuccess) throw std::runtime_error("RCCL all-gather failed");
  }
  // the global top-K on the first shard's device: wx_topk_merge over the
  // gathered records (better key, NaN last, then the smaller row), k results
  // read back with the count
  TopkScratch &t0 = impl_->topk[0];
  const int dev0 = ranges[0].device;
  if (!t0.out.ptr) t0.out = DeviceBuffer(dev0, kTopkRec);
  char *o = static_cast<char *>(t0.out.ptr);
  char err[1024];
  {
    DevGuard dg(dev0);
    wx_launch L = sync_launch(dev0, streams[0]);
    L.flags = 0;
    throw_on(wx_topk_merge(static_cast<const wx_topk_record *>(gathered ? t0.all.ptr : t0.cand.ptr),
                           static_cast<int32_t>(ns), static_cast<int32_t>(k), descending ? 1 : 0, &L,
                           reinterpret_cast<float *>(o),
                           reinterpret_cast<int64_t *>(o + kTopkMax * 8), reinterpret_cast<float *>(o + kTopkMax * 4),
                           reinterpret_cast<int64_t *>(o + kTopkMax * 16), nullptr, err, sizeof(err)),
             err);
  }
  impl_->timer.end(ranges, streams);  // no-op unless begin ran (a collective)
  for (size_t i = 0; i < ns; ++i) {
    DevGuard dg(ranges[i].device);
    hip_ok(hipStreamSynchronize(streams[i]), "hipStreamSynchronize");
    wx_launch L = sync_launch(ranges[i].device, streams[i]);
    throw_on(wx_check(&L, err, sizeof(err)), err);
  }
  wx_topk_record h;
  {
    DevGuard dg(dev0);
    hip_ok(hipMemcpy(&h, o, sizeof(h), hipMemcpyDeviceToHost), "hipMemcpy");
  }
  for (int64_t j = 0; j < h.count; ++j) {
    res.keys.push_back(h.keys[j]);
    res.rows.push_back(h.rows[j]);
    res.values.push_back(h.vals[j]);
  }
  return res;
}

std::pair<double, int64_t> ResidentShards::sum(const std::string &expr_cuda, const std::string &cond_cuda) const {
  std::lock_guard<std::mutex> lk(impl_->mu);
  return sum_over_shards(impl_->ranges, impl_->shards, expr_cuda, cond_cuda, nullptr, &impl_->sum_out,
                         &impl_->timer);
}

void ResidentShards::set_timing(bool kernels, bool exchange) {
  std::lock_guard<std::mutex> lk(impl_->mu);
  impl_->timer.kernels = kernels;
  impl_->timer.exchange = exchange;
}

ApiTiming ResidentShards::take_timing() {
  std::lock_guard<std::mutex> lk(impl_->mu);
  ApiTiming out;
  for (size_t i = 0; i < impl_->ranges.size(); ++i) {
    const int dev = impl_->ranges[i].device;
    bool seen = false;
    for (size_t j = 0; j < i; ++j) seen = seen || impl_->ranges[j].device == dev;
    if (seen) continue;  // virtual shards on one device: its launches are read once
    double ms = 0;
    int64_t n = 0;
    char err[1024];
    throw_on(wx_timing_read_device(dev, &ms, &n, err, sizeof(err)), err);
    if (n > 0 && ms / n > out.kernel_ms) {
      out.kernel_ms = ms / n;
      out.launches = n;
    }
  }
  auto &ev = impl_->timer.ev;
  for (size_t i = 0; i < ev.size() && i < impl_->ranges.size(); ++i) {
    DevGuard g(impl_->ranges[i].device);
    double tot = 0;
    for (auto &p : ev[i]) {
      hip_ok(hipEventSynchronize(p.second), "hipEventSynchronize");
      float ms = 0;
      hip_ok(hipEventElapsedTime(&ms, p.first, p.second), "hipEventElapsedTime");
      tot += ms;
      (void)hipEventDestroy(p.first);
      (void)hipEventDestroy(p.second);
    }
    if (!ev[i].empty()) {
      out.exchanges = static_cast<int64_t>(ev[i].size());
      out.exchange_ms = std::max(out.exchange_ms, tot / ev[i].size());
    }
    ev[i].clear();
  }
  return out;
}

// GROUP BY over the shards in ONE collective: per device
// wx_group_partials_slots (the dense 2048-key window and this shard's slot of
// up to 64 out-of-window groups, zeros in the others), ONE ncclAllReduce of
// the exchange buffers (it reduces the windows and gathers the slots), then
// wx_group_combine_slots on the first shard's device.  Only when a shard had
// more out-of-window groups than its slot holds (WX_GROUP_NEEDS_MERGE) does a
// second collective follow: an all-gather of every shard's whole list of
// out-of-window groups (one fixed-size record each), merged with the window
// by wx_group_merge_lists on the first shard's device.
GroupResult ResidentShards::group_sum(const std::string &val_cuda, const std::string &key_cuda,
                                      const std::string &cond_cuda, int32_t key_lo) const {
  std::lock_guard<std::mutex> lk(impl_->mu);
  GroupResult res;
  const auto &ranges = impl_->ranges;
  const size_t ns = ranges.size();
  if (ns == 0) return res;
  constexpr int64_t kCap = 1 << 16;  // out-of-window groups per shard / final groups
  constexpr int kSlotMax = 4096;     // n_slots * slot_groups bound of wx_group_combine_slots
  const int S = std::max(1, std::min(64, kSlotMax / static_cast<int>(ns)));
  const size_t WD = static_cast<size_t>(WX_GROUP_SLOTS_DOUBLES(ns, S));
  if (impl_->group.size() < ns) impl_->group.resize(ns);
  std::vector<double *> wins(ns, nullptr);
  std::vector<hipStream_t> streams(ns, nullptr);
  run_per_device(ranges, [&](size_t i, const ShardRange &r) {
    streams[i] = device_stream(r.device);
    GroupScratch &g = impl_->group[i];
    if (g.cap < kCap || g.win_doubles != WD) {
      g.win = DeviceBuffer(r.device, WD * 8);
      g.win_doubles = WD;
    }
    if (g.cap < kCap) {
      g.rec = DeviceBuffer(r.device, static_cast<size_t>(WX_GROUP_LIST_BYTES(kCap)));
      g.ok = DeviceBuffer(r.device, kCap * 4);
      g.os = DeviceBuffer(r.device, kCap * 8);
      g.oc = DeviceBuffer(r.device, kCap * 8);
      g.ng = DeviceBuffer(r.device, 8);
      g.cap = kCap;
    }
    WxTableView v(impl_->shards[i].table);
    wx_launch L = sync_launch(r.device, streams[i]);
    L.flags = impl_->timer.flags();  // asynchronous until after the collective
    char err[8192];
    throw_on(wx_group_partials_slots(&v.table, val_cuda.c_str(), key_cuda.c_str(), cond_cuda.c_str(), &L, key_lo,
                                     static_cast<double *>(g.win.ptr), static_cast<int32_t>(ns),
                                     static_cast<int32_t>(i), S, kCap, g.xk(), g.xs(), g.xc(), g.nx(), nullptr, err,
                                     sizeof(err)),
             err);
    wins[i] = static_cast<double *>(g.win.ptr);
  });
  const bool coll = ns > 1 || exchange_one_rank();
  if (coll) impl_->timer.begin(ranges, streams);
  allreduce_f64(ranges, wins, streams, WD);
  GroupScratch &g0 = impl_->group[0];
  const int dev0 = ranges[0].device;
  char err[8192];
  wx_launch L0 = sync_launch(dev0, streams[0]);
  L0.flags = 0;
  throw_on(wx_group_combine_slots(static_cast<double *>(g0.win.ptr), static_cast<int32_t>(ns), S, key_lo, &L0, kCap,
                                  static_cast<int32_t *>(g0.ok.ptr), static_cast<double *>(g0.os.ptr),
                                  static_cast<int64_t *>(g0.oc.ptr), static_cast<int64_t *>(g0.ng.ptr), nullptr, err,
                                  sizeof(err)),
           err);
  if (coll) impl_->timer.end(ranges, streams);
  // the group count and the first kStage groups, in one batch of
  // asynchronous copies behind the combine
  constexpr int64_t kStage = 4096;
  if (!impl_->stage) {
    DevGuard dg(dev0);
    hip_ok(hipHostMalloc(reinterpret_cast<void **>(&impl_->stage), 16 + kStage * 20), "hipHostMalloc");
  }
  char *st = impl_->stage;
  {
    DevGuard dg(dev0);
    hip_ok(hipMemcpyAsync(st + 8, g0.ng.ptr, 8, hipMemcpyDeviceToHost, streams[0]), "hipMemcpyAsync");
    hip_ok(hipMemcpyAsync(st + 16, g0.ok.ptr, kStage * 4, hipMemcpyDeviceToHost, streams[0]), "hipMemcpyAsync");
    hip_ok(hipMemcpyAsync(st + 16 + kStage * 4, g0.os.ptr, kStage * 8, hipMemcpyDeviceToHost, streams[0]),
           "hipMemcpyAsync");
    hip_ok(hipMemcpyAsync(st + 16 + kStage * 12, g0.oc.ptr, kStage * 8, hipMemcpyDeviceToHost, streams[0]),
           "hipMemcpyAsync");
  }
  // every shard's stream (and the collective) complete; the decisions below
  // come from the combined buffer only, so a shard's own capacity flag is
  // reported through it (the same error whichever shard hit it)
  std::exception_ptr shard_err;
  for (size_t i = 0; i < ns; ++i) {
    DevGuard dg(ranges[i].device);
    hip_ok(hipStreamSynchronize(streams[i]), "hipStreamSynchronize");
    wx_launch L = sync_launch(ranges[i].device, streams[i]);
    if (wx_check(&L, err, sizeof(err)) != WX_OK && !shard_err)
      shard_err = std::make_exception_ptr(std::runtime_error(err));
  }
  int64_t ng = 0;
  std::memcpy(&ng, st + 8, 8);
  if (ng == -1) throw std::runtime_error("group table / output capacity exceeded (general-key table overflow)");
  if (shard_err) std::rethrow_exception(shard_err);
  const bool merged_extra = ng == WX_GROUP_NEEDS_MERGE;
  if (merged_extra) {
    // every shard's whole out-of-window list (already in its record): ONE
    // all-gather of the fixed-size records, merged with the combined window
    // on the first shard's device (wx_group_merge_lists)
    const size_t rb = static_cast<size_t>(WX_GROUP_LIST_BYTES(kCap));
    std::vector<void *> send(ns), recv(ns);
    for (size_t i = 0; i < ns; ++i) {
      GroupScratch &g = impl_->group[i];
      if (g.lists != static_cast<int>(ns)) {
        g.all = DeviceBuffer(ranges[i].device, rb * ns);
        g.lists = static_cast<int>(ns);
      }
      send[i] = g.rec.ptr;
      recv[i] = g.all.ptr;
    }
    allgather_bytes(ranges, send, recv, streams, rb);
    DevGuard dg(dev0);
    wx_launch L = sync_launch(dev0, streams[0]);
    throw_on(wx_group_merge_lists(g0.all.ptr, static_cast<int32_t>(ns), kCap, static_cast<double *>(g0.win.ptr), key_lo,
                                  &L, kCap, static_cast<int32_t *>(g0.ok.ptr), static_cast<double *>(g0.os.ptr),
                                  static_cast<int64_t *>(g0.oc.ptr), static_cast<int64_t *>(g0.ng.ptr), &ng, err,
                                  sizeof(err)),
             err);
  }
  DevGuard dg(dev0);
  if (ng > kCap) throw std::runtime_error("group table / output capacity exceeded");
  res.keys.resize(ng);
  res.sums.resize(ng);
  res.counts.resize(ng);
  if (ng && !merged_extra && ng <= kStage) {  // the staged copies hold the whole result
    std::memcpy(res.keys.data(), st + 16, ng * 4);
    std::memcpy(res.sums.data(), st + 16 + kStage * 4, ng * 8);
    std::memcpy(res.counts.data(), st + 16 + kStage * 12, ng * 8);
  } else if (ng) {
    hip_ok(hipMemcpy(res.keys.data(), g0.ok.ptr, ng * 4, hipMemcpyDeviceToHost), "hipMemcpy");
    hip_ok(hipMemcpy(res.sums.data(), g0.os.ptr, ng * 8, hipMemcpyDeviceToHost), "hipMemcpy");
    hip_ok(hipMemcpy(res.counts.data(), g0.oc.ptr, ng * 8, hipMemcpyDeviceToHost), "hipMemcpy");
  }
  return res;
}

}  // namespace warpdb

std::vector<float> run_multi_gpu_jit_host(const HostTable &host, const std::string &expr_cuda,
                                          const std::string &cond_cuda) {
  using namespace warpdb;
  const int64_t n = host.num_rows();
  auto shards = plan_shards(n, shard_count());
  // The host result (4 B/row, first-touch bound) is allocated and populated
  // before the uploads: populating it on a thread of its own while the
  // runtime stages the pageable uploads slowed both, 31 vs 27-29 ms per 1e8
  // rows (profiles/r01/host_pipeline_alloc_mode.txt).
  std::vector<float> result = host_result(static_cast<size_t>(n));
  // Per device, a chunked pipeline over its shard: this thread uploads chunk
  // c and runs the dense kernel on it (stream 0) while a second thread
  // downloads chunk c - 1 (stream 1), so the two PCIe directions overlap
  // (the reference uploads, runs and downloads each shard in turn,
  // src/multi_gpu_utils.cpp:34-58).  Chunks are multiples of 4 rows, so the
  // chunk views keep the columns' 16-byte alignment.
  const int64_t chunk_rows = std::max<int64_t>(
      4, (std::atoll(std::getenv("WARPDB_HOST_CHUNK_ROWS") ? std::getenv("WARPDB_HOST_CHUNK_ROWS") : "16777216") + 3) &
             ~int64_t(3));
  const bool debug = std::getenv("WARPDB_DEBUG") != nullptr;
  const auto t_start = std::chrono::steady_clock::now();
  auto stamp = [&](const char *what, int dev, int64_t c) {
    if (!debug) return;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    std::fprintf(stderr, "[multi_gpu] %8.3f ms dev %d chunk %lld %s\n", ms, dev, (long long)c, what);
  };
  run_per_device(shards, [&](size_t, const ShardRange &r) {
    hipStream_t s = device_stream(r.device, 0), s2 = device_stream(r.device, 1);
    const int64_t rows = r.end - r.begin;
    const int64_t n_chunks = (rows + chunk_rows - 1) / chunk_rows;
    // device copies of the numeric columns of this shard and its output, in
    // the device's scratch HBM (256-byte aligned slices)
    Scratch &scr = scratch_for(r.device);
    std::lock_guard<std::mutex> scr_lock(scr.mu);
    std::vector<const char *> src;
    std::vector<size_t> width, offset;
    size_t total = 0;
    auto slice = [&](size_t bytes) {
      const size_t at = total;
      total += (bytes + 255) & ~size_t(255);
      return at;
    };
    for (const auto &c : host.columns) {
      const size_t w = (c.type == DataType::Int64 || c.type == DataType::Float64) ? 8 : 4;
      width.push_back(w);
      src.push_back(c.type == DataType::String
                        ? nullptr
                        : static_cast<const char *>(std::visit([](auto &&v) -> const void * { return v.data(); }, c.data)));
      offset.push_back(c.type == DataType::String ? 0 : slice(w * static_cast<size_t>(rows)));
    }
    const size_t out_off = slice(sizeof(float) * static_cast<size_t>(rows));
    if (scr.bytes < total) {
      scr.buf = DeviceBuffer();
      scr.buf = DeviceBuffer(r.device, total);
      scr.bytes = total;
    }
    char *base = static_cast<char *>(scr.buf.ptr);
    float *out = reinterpret_cast<float *>(base + out_off);
    stamp("device buffers", r.device, -1);
    std::vector<hipEvent_t> done(static_cast<size_t>(n_chunks), nullptr);
    for (auto &e : done) hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    struct Events {
      std::vector<hipEvent_t> &v;
      ~Events() {
        for (auto e : v)
          if (e) (void)hipEventDestroy(e);
      }
    } ev_guard{done};
    std::mutex mu;
    std::condition_variable cv;
    int64_t recorded = 0;
    bool failed = false;
    std::exception_ptr d2h_err;
    std::thread down([&] {
      try {
        DevGuard g(r.device);
        for (int64_t c = 0; c < n_chunks; ++c) {
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return recorded > c || failed; });
            if (failed) return;
          }
          hip_ok(hipStreamWaitEvent(s2, done[c], 0), "hipStreamWaitEvent");
          const int64_t c0 = c * chunk_rows, cr = std::min(chunk_rows, rows - c0);
          copy_d2h(r.device, s2, result.data() + r.begin + c0, out + c0, sizeof(float) * static_cast<size_t>(cr));
          stamp("downloaded", r.device, c);
        }
      } catch (...) {
        d2h_err = std::current_exception();
      }
    });
    try {
      char err[8192];
      for (int64_t c = 0; c < n_chunks; ++c) {
        const int64_t c0 = c * chunk_rows, cr = std::min(chunk_rows, rows - c0);
        Table chunk;
        chunk.num_rows = cr;
        chunk.device = r.device;
        for (size_t k = 0; k < host.columns.size(); ++k) {
          const auto &hc = host.columns[k];
          if (hc.type == DataType::String) {
            chunk.columns.push_back({hc.name, hc.type, nullptr, cr});
            continue;
          }
          char *dst = base + offset[k] + width[k] * static_cast<size_t>(c0);
          copy_h2d(r.device, s, dst, src[k] + width[k] * static_cast<size_t>(r.begin + c0),
                   width[k] * static_cast<size_t>(cr));
          chunk.columns.push_back({hc.name, hc.type, dst, cr});
        }
        WxTableView v(chunk);
        wx_launch L = sync_launch(r.device, s);
        L.flags = 0;
        throw_on(wx_project_filter(&v.table, expr_cuda.c_str(), cond_cuda.c_str(), &L, WX_MODE_DENSE_FILL, out + c0,
                                   nullptr, 0, 0, nullptr, nullptr, err, sizeof(err)),
                 err);
        hip_ok(hipEventRecord(done[c], s), "hipEventRecord");
        stamp("uploaded + launched", r.device, c);
        {
          std::lock_guard<std::mutex> lk(mu);
          recorded = c + 1;
        }
        cv.notify_one();
      }
      wx_launch L = sync_launch(r.device, s);
      throw_on(wx_check(&L, err, sizeof(err)), err);
    } catch (...) {
      {
        std::lock_guard<std::mutex> lk(mu);
        failed = true;
      }
      cv.notify_one();
      down.join();
      throw;
    }
    down.join();
    if (d2h_err) std::rethrow_exception(d2h_err);
    hip_ok(hipStreamSynchronize(s2), "hipStreamSynchronize");
  });
  return result;
}
