// arrow_export.cpp -- results through the Arrow C Data Interface
// (reference src/arrow_utils.cpp:37-94) and, new, zero-copy
// ArrowDeviceArrays on ROCm (ARROW_DEVICE_ROCM, include/arrow_c_abi.h:126,
// 140-155 of the reference): the dense float32 result, and the compacted
// result as struct<value: float32, row: int64> (passing rows only).
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>
#include <unistd.h>

#include <cstdlib>
#include <vector>
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

// struct<value: float32, row: int64>: the parent array (no validity bitmap)
// owns its two children and their buffers (host: malloc, device: hipFree).
struct CompactResult {
  bool device = false;
  int device_id = 0;
  void *values = nullptr;
  void *rows = nullptr;
  const void *parent_buffers[1] = {nullptr};
  const void *value_buffers[2] = {nullptr, nullptr};
  const void *row_buffers[2] = {nullptr, nullptr};
  ArrowArray child_arrays[2];
  ArrowArray *children[2] = {&child_arrays[0], &child_arrays[1]};
};

void release_child_array(ArrowArray *a) {
  if (a) a->release = nullptr;  // buffers belong to the parent
}

void release_compact_array(ArrowArray *a) {
  if (!a || !a->release) return;
  auto *r = static_cast<CompactResult *>(a->private_data);
  if (r) {
    for (int i = 0; i < 2; ++i)
      if (r->child_arrays[i].release) r->child_arrays[i].release(&r->child_arrays[i]);
    if (r->device) {
      int prev = 0;
      (void)hipGetDevice(&prev);
      (void)hipSetDevice(r->device_id);
      if (r->values) (void)hipFree(r->values);
      if (r->rows) (void)hipFree(r->rows);
      (void)hipSetDevice(prev);
    } else {
      std::free(r->values);
      std::free(r->rows);
    }
    delete r;
  }
  a->release = nullptr;
}

struct CompactSchema {
  ArrowSchema child_schemas[2];
  ArrowSchema *children[2] = {&child_schemas[0], &child_schemas[1]};
};

void release_child_schema(ArrowSchema *s) {
  if (s) s->release = nullptr;
}

void release_compact_schema(ArrowSchema *s) {
  if (!s || !s->release) return;
  auto *c = static_cast<CompactSchema *>(s->private_data);
  if (c) {
    for (auto &ch : c->child_schemas)
      if (ch.release) ch.release(&ch);
    delete c;
  }
  s->release = nullptr;
}

void fill_leaf_schema(ArrowSchema *s, const char *format, const char *name, int64_t flags) {
  s->format = format;
  s->name = name;
  s->metadata = nullptr;
  s->flags = flags;
  s->n_children = 0;
  s->children = nullptr;
  s->dictionary = nullptr;
  s->release = release_child_schema;
  s->private_data = nullptr;
}

void fill_compact_schema(ArrowSchema *s) {
  auto *c = new CompactSchema();
  fill_leaf_schema(&c->child_schemas[0], "f", "value", 0);
  fill_leaf_schema(&c->child_schemas[1], "l", "row", 0);
  s->format = "+s";
  s->name = "result";
  s->metadata = nullptr;
  s->flags = 0;
  s->n_children = 2;
  s->children = c->children;
  s->dictionary = nullptr;
  s->release = release_compact_schema;
  s->private_data = c;
}

void fill_leaf_array(ArrowArray *a, const void **buffers, int64_t length) {
  a->length = length;
  a->null_count = 0;
  a->offset = 0;
  a->n_buffers = 2;
  a->n_children = 0;
  a->buffers = buffers;
  a->children = nullptr;
  a->dictionary = nullptr;
  a->release = release_child_array;
  a->private_data = nullptr;
}

void fill_compact_array(CompactResult *r, int64_t length, ArrowArray *a) {
  r->value_buffers[1] = r->values;
  r->row_buffers[1] = r->rows;
  fill_leaf_array(&r->child_arrays[0], r->value_buffers, length);
  fill_leaf_array(&r->child_arrays[1], r->row_buffers, length);
  a->length = length;
  a->null_count = 0;
  a->offset = 0;
  a->n_buffers = 1;  // struct: validity bitmap only (none)
  a->n_children = 2;
  a->buffers = r->parent_buffers;
  a->children = r->children;
  a->dictionary = nullptr;
  a->release = release_compact_array;
  a->private_data = r;
}

}  // namespace

void export_compact_to_arrow(const float *values, const int64_t *rows, int64_t length, ArrowArray *out_array,
                             ArrowSchema *out_schema) {
  if (!out_array || !out_schema) throw std::invalid_argument("Null output");
  if (length < 0) throw std::invalid_argument("negative length");
  auto *r = new CompactResult();
  const size_t n = static_cast<size_t>(length);
  r->values = std::malloc(n * sizeof(float) + 1);
  r->rows = std::malloc(n * sizeof(int64_t) + 1);
  if (!r->values || !r->rows) {
    std::free(r->values);
    std::free(r->rows);
    delete r;
    throw std::bad_alloc();
  }
  if (n) {
    std::memcpy(r->values, values, n * sizeof(float));
    std::memcpy(r->rows, rows, n * sizeof(int64_t));
  }
  fill_compact_array(r, length, out_array);
  fill_compact_schema(out_schema);
}

void export_device_compact_to_arrow(float *d_values, int64_t *d_rows, int64_t length, int device,
                                    ArrowDeviceArray *out, ArrowSchema *schema) {
  if (!out || !schema) throw std::invalid_argument("Null output");
  auto *r = new CompactResult();
  r->device = true;
  r->device_id = device;
  r->values = d_values;
  r->rows = d_rows;
  std::memset(out, 0, sizeof(*out));
  fill_compact_array(r, length, &out->array);
  out->device_id = device;
  out->device_type = ARROW_DEVICE_ROCM;
  out->sync_event = nullptr;  // the producer synchronised before returning
  fill_compact_schema(schema);
}

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
