// internal.hpp -- helpers shared by the C++ host layer (not installed).
#pragma once
#include <hip/hip_runtime_api.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "warpdb/csv_loader.hpp"
#include "warpexec.h"

namespace warpdb {

inline void hip_ok(hipError_t e, const char *what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + what + ": " + hipGetErrorString(e));
}

class DevGuard {
 public:
  explicit DevGuard(int dev) {
    if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
    if (prev_ != dev) hip_ok(hipSetDevice(dev), "hipSetDevice");
    dev_ = dev;
  }
  ~DevGuard() {
    if (prev_ >= 0 && prev_ != dev_) (void)hipSetDevice(prev_);
  }

 private:
  int prev_ = -1, dev_ = 0;
};

// RAII device allocation.
struct DeviceBuffer {
  void *ptr = nullptr;
  int device = 0;
  DeviceBuffer() = default;
  DeviceBuffer(int dev, size_t bytes) : device(dev) {
    DevGuard g(dev);
    hip_ok(hipMalloc(&ptr, bytes ? bytes : 1), "hipMalloc");
  }
  DeviceBuffer(const DeviceBuffer &) = delete;
  DeviceBuffer &operator=(const DeviceBuffer &) = delete;
  DeviceBuffer(DeviceBuffer &&o) noexcept : ptr(o.ptr), device(o.device) { o.ptr = nullptr; }
  DeviceBuffer &operator=(DeviceBuffer &&o) noexcept {
    std::swap(ptr, o.ptr);
    std::swap(device, o.device);
    return *this;
  }
  ~DeviceBuffer() {
    if (ptr) {
      DevGuard g(device);
      (void)hipFree(ptr);
    }
  }
  void *release() {
    void *p = ptr;
    ptr = nullptr;
    return p;
  }
};

// A wx_table view over a Table's columns (names kept alive here).
struct WxTableView {
  explicit WxTableView(const Table &t);
  std::vector<std::string> names;
  std::vector<wx_col> cols;
  wx_table table{};
};

// Host <-> HBM copies (transfer.cpp).  copy_h2d may return before the DMA
// finishes (the source is already staged); copy_d2h returns with `dst` filled.
void copy_h2d(int device, hipStream_t s, void *dst, const void *src, size_t bytes);
void copy_d2h(int device, hipStream_t s, void *dst, const void *src, size_t bytes);
// A zero-filled host result of n floats (huge-page backed when large).
std::vector<float> host_result(size_t n);

// CSV data rows in [b, e) appended to `out` (typed columns already set up),
// parsed on up to `threads` threads (csv_parse.cpp).
int parse_threads();  // $WARPDB_PARSE_THREADS, default hardware threads, at most 16
void parse_csv_rows(const char *b, const char *e, HostTable &out, int threads);

wx_launch sync_launch(int device, void *stream = nullptr);
void throw_on(wx_status st, const char *err);

}  // namespace warpdb
