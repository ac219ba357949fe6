// arrow_utils.hpp -- export query results through the Arrow C Data Interface
// (reference include/arrow_utils.hpp, src/arrow_utils.cpp:37-94).
#pragma once
#include <cstdint>

#include "arrow_c_abi.h"

// Copy `length` host floats into a malloc'd buffer (or POSIX shm
// "/warpdb_result" when use_shared_memory) and describe it as a float32
// ("f") array named "result" with no validity bitmap.  release() frees it.
void export_to_arrow(const float *data, int64_t length, bool use_shared_memory, ArrowArray *out_array,
                     ArrowSchema *out_schema);

// Zero-copy export of a device buffer as an ArrowDeviceArray with
// device_type ARROW_DEVICE_ROCM.  Ownership of d_data passes to the array:
// its release() calls hipFree.
void export_device_to_arrow(float *d_data, int64_t length, int device, ArrowDeviceArray *out, ArrowSchema *schema);

// The compacted result (passing rows only, ascending row order) as an Arrow
// struct<value: float32, row: int64> array named "result"; host buffers are
// copied into malloc'd memory that release() frees.
void export_compact_to_arrow(const float *values, const int64_t *rows, int64_t length, ArrowArray *out_array,
                             ArrowSchema *out_schema);

// Zero-copy device export of a compacted result (ARROW_DEVICE_ROCM):
// ownership of both device buffers passes to the array (release() hipFrees them).
void export_device_compact_to_arrow(float *d_values, int64_t *d_rows, int64_t length, int device,
                                    ArrowDeviceArray *out, ArrowSchema *schema);
