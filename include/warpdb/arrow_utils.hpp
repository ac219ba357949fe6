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
