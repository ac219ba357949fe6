// arrow_export.cpp -- results through the Arrow C Data Interface
// (reference src/arrow_utils.cpp:37-94) and, new, a zero-copy
// ArrowDeviceArray on ROCm (ARROW_DEVICE_ROCM).
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>

#include "warpdb/arrow_utils.hpp"

namespace {

struct HostResult {
  void *data = nullptr;
  size_t bytes = 0;
  bool shared = false;
  int fd = -1;
  std::string shm_name;
  const void *buffers[2] = {nullptr, nullptr};
};

void release_host_array(ArrowArray *a) {
  if (!a || !a->release) return;
  auto *r = static_cast<HostResult *>(a->private_data);
  if (r) {
    if (r->shared) {
      if (r->data && r->data != MAP_FAILED) munmap(r->data, r->bytes ? r->bytes : 1);
      if (r->fd >= 0) {
        close(r->fd);
        shm_unlink(r->shm_name.c_str());
      }
    } else {
      std::free(r->data);
    }
    delete r;
  }
  a->release = nullptr;
}

void release_schema(ArrowSchema *s) {
  if (s) s->release = nullptr;
}

void fill_schema(ArrowSchema *s) {
  s->format = "f";  // float32
  s->name = "result";
  s->metadata = nullptr;
  s->flags = ARROW_FLAG_NULLABLE;
  s->n_children = 0;
  s->children = nullptr;
  s->dictionary = nullptr;
  s->release = release_schema;
  s->private_data = nullptr;
}

struct DeviceResult {
  void *data = nullptr;
  int device = 0;
  const void *buffers[2] = {nullptr, nullptr};
};

void release_device_array(ArrowArray *a) {
  if (!a || !a->release) return;
  auto *r = static_cast<DeviceResult *>(a->private_data);
  if (r) {
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(r->device);
    if (r->data) (void)hipFree(r->data);
    (void)hipSetDevice(prev);
    delete r;
  }
  a->release = nullptr;
}

}  // namespace

void export_to_arrow(const float *data, int64_t length, bool use_shared_memory, ArrowArray *out_array,
                     ArrowSchema *out_schema) {
  if (!out_array || !out_schema) throw std::invalid_argument("Null output");
  if (length < 0) throw std::invalid_argument("negative length");
  auto *r = new HostResult();
  r->bytes = sizeof(float) * static_cast<size_t>(length);
  r->shared = use_shared_memory;
  if (use_shared_memory) {
    r->shm_name = "/warpdb_result";  // the name consumers of the reference open
    r->fd = shm_open(r->shm_name.c_str(), O_CREAT | O_RDWR, 0600);
    if (r->fd < 0) {
      delete r;
      throw std::runtime_error("shm_open failed");
    }
    if (ftruncate(r->fd, static_cast<off_t>(r->bytes)) != 0) {
      close(r->fd);
      shm_unlink(r->shm_name.c_str());
      delete r;
      throw std::runtime_error("ftruncate failed");
    }
    r->data = mmap(nullptr, r->bytes ? r->bytes : 1, PROT_READ | PROT_WRITE, MAP_SHARED, r->fd, 0);
    if (r->data == MAP_FAILED) {
      close(r->fd);
      shm_unlink(r->shm_name.c_str());
      delete r;
      throw std::runtime_error("mmap failed");
    }
  } else {
    r->data = std::malloc(r->bytes ? r->bytes : 1);
    if (!r->data) {
      delete r;
      throw std::bad_alloc();
    }
  }
  if (r->bytes) std::memcpy(r->data, data, r->bytes);
  r->buffers[0] = nullptr;  // no validity bitmap
  r->buffers[1] = r->data;
  out_array->length = length;
  out_array->null_count = 0;
  out_array->offset = 0;
  out_array->n_buffers = 2;
  out_array->n_children = 0;
  out_array->buffers = r->buffers;
  out_array->children = nullptr;
  out_array->dictionary = nullptr;
  out_array->release = release_host_array;
  out_array->private_data = r;
  fill_schema(out_schema);
}

void export_device_to_arrow(float *d_data, int64_t length, int device, ArrowDeviceArray *out, ArrowSchema *schema) {
  if (!out || !schema) throw std::invalid_argument("Null output");
  auto *r = new DeviceResult();
  r->data = d_data;
  r->device = device;
  r->buffers[0] = nullptr;
  r->buffers[1] = d_data;
  std::memset(out, 0, sizeof(*out));
  out->array.length = length;
  out->array.null_count = 0;
  out->array.offset = 0;
  out->array.n_buffers = 2;
  out->array.buffers = r->buffers;
  out->array.release = release_device_array;
  out->array.private_data = r;
  out->device_id = device;
  out->device_type = ARROW_DEVICE_ROCM;
  out->sync_event = nullptr;  // the producer synchronised before returning
  fill_schema(schema);
}
