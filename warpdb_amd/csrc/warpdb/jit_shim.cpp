// jit_shim.cpp -- the reference's JIT entry points (include/jit.hpp) over
// the C ABI.  Each call is synchronous and throws std::runtime_error on
// failure with the reference's messages (src/jit.cpp:11-28, :123-129).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <iostream>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "warpdb/jit.hpp"
#include "warpdb/internal.hpp"
#include "warpexec.h"

namespace warpdb {

WxTableView::WxTableView(const Table &t) {
  names.reserve(t.columns.size());
  for (const auto &c : t.columns) names.push_back(c.name);
  for (size_t i = 0; i < t.columns.size(); ++i)
    cols.push_back({names[i].c_str(), static_cast<int32_t>(t.columns[i].type), t.columns[i].device_ptr});
  table.n_rows = t.num_rows;
  table.n_cols = static_cast<int32_t>(cols.size());
  table.cols = cols.empty() ? nullptr : cols.data();
}

wx_launch sync_launch(int device, void *stream) {
  wx_launch L;
  L.device = device;
  L.stream = stream;
  L.custom_src = nullptr;  // ./custom.cu, as the reference (src/jit.cpp:65-73)
  L.flags = WX_F_SYNC;
  return L;
}

void throw_on(wx_status st, const char *err) {
  if (st == WX_OK) return;
  if (st == WX_ERR_COMPILE) {
    std::cerr << "HIPRTC Compile Log:\n" << err << "\n";
    throw std::runtime_error("Kernel compilation failed.");
  }
  throw std::runtime_error(err);
}

}  // namespace warpdb

using namespace warpdb;

void jit_compile_and_launch(const std::string &expr_code, const std::string &condition_code, const Table &table,
                            float *d_output, int device_id) {
  WxTableView v(table);
  wx_launch L = sync_launch(device_id);
  char err[8192];
  throw_on(wx_project_filter(&v.table, expr_code.c_str(), condition_code.c_str(), &L, WX_MODE_DENSE, d_output,
                             nullptr, 0, 0, nullptr, nullptr, err, sizeof(err)),
           err);
}

namespace {
// Double sums / int64 counts behind jit_group_sum, per device, kept across
// calls and grown only when a query has more groups than it holds: O(groups)
// of HBM, not O(rows) (the reference's caller sizes its outputs for N rows,
// src/warpdb.cpp:356-358, but a GROUP BY yields at most a few thousand).
struct GroupScratch {
  std::mutex mu;
  DeviceBuffer sums, counts;
  int64_t cap = 0;
};
GroupScratch &group_scratch(int device) {
  static std::mutex mu;
  static auto *all = new std::map<int, std::unique_ptr<GroupScratch>>();  // never destroyed (HIP teardown order)
  std::lock_guard<std::mutex> lk(mu);
  auto &p = (*all)[device];
  if (!p) p.reset(new GroupScratch);
  return *p;
}
}  // namespace

void jit_group_sum(const std::string &val_expr_code, const std::string &key_expr_code, float *d_price,
                   int *d_quantity, float *d_out_vals, int *d_out_keys, int *d_count, int N, int device_id) {
  // the reference kernel binds exactly these two columns (src/jit.cpp:194)
  Table t;
  t.num_rows = N;
  t.device = device_id;
  t.columns.push_back({"price", DataType::Float32, d_price, N});
  t.columns.push_back({"quantity", DataType::Int32, d_quantity, N});
  WxTableView v(t);
  wx_launch L = sync_launch(device_id);
  GroupScratch &scr = group_scratch(device_id);
  std::lock_guard<std::mutex> lk(scr.mu);
  int64_t cap = std::max<int64_t>(scr.cap, 4096);
  int64_t groups = 0;
  char err[8192];
  for (;;) {
    if (scr.cap < cap) {
      scr.sums = DeviceBuffer();
      scr.counts = DeviceBuffer();
      scr.sums = DeviceBuffer(device_id, cap * sizeof(double));
      scr.counts = DeviceBuffer(device_id, cap * sizeof(int64_t));
      scr.cap = cap;
    }
    const wx_status st = wx_group_sum(&v.table, val_expr_code.c_str(), key_expr_code.c_str(), nullptr, &L, 0, cap,
                                      d_out_keys, static_cast<double *>(scr.sums.ptr),
                                      static_cast<int64_t *>(scr.counts.ptr), nullptr, &groups, err, sizeof(err));
    if (st == WX_ERR_CAPACITY) {  // more groups than the scratch holds: grow and run again
      cap = std::max<int64_t>(2 * cap, groups + 1);
      continue;
    }
    throw_on(st, err);
    break;
  }
  // the reference's outputs are float sums and an int count: converted on
  // the device, nothing but the count crosses to the host
  throw_on(wx_cast(scr.sums.ptr, WX_FLOAT64, d_out_vals, WX_FLOAT32, groups, &L, err, sizeof(err)), err);
  DevGuard g(device_id);
  hip_ok(hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(d_count), static_cast<int>(groups), 1), "hipMemsetD32");
}

void jit_sort_pairs(int *d_keys, float *d_vals, int count, bool ascending, int device_id) {
  wx_launch L = sync_launch(device_id);
  char err[1024];
  throw_on(wx_sort_pairs(d_keys, d_vals, count, ascending ? 1 : 0, &L, err, sizeof(err)), err);
}

void jit_sort_float(float *d_vals, int count, bool ascending, int device_id) {
  wx_launch L = sync_launch(device_id);
  char err[1024];
  throw_on(wx_sort_float(d_vals, count, ascending ? 1 : 0, &L, err, sizeof(err)), err);
}
