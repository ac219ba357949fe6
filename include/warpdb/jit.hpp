// jit.hpp -- the reference's JIT entry points (include/jit.hpp:7-27), kept
// with their signatures and implemented over the C ABI (include/warpexec.h):
// hiprtc + gfx950 kernel templates instead of NVRTC.  All calls are
// synchronous, like the reference (cuCtxSynchronize, src/jit.cpp:171), and
// throw std::runtime_error on failure ("Kernel compilation failed." for a
// compile error, with the hiprtc log on stderr, as src/jit.cpp:123-129).
#pragma once
#include <string>

#include "csv_loader.hpp"

// output[idx] = expr where condition holds (empty condition = every row);
// other rows are left untouched.  Columns come from `table` in schema order.
void jit_compile_and_launch(const std::string &expr_code, const std::string &condition_code, const Table &table,
                            float *d_output, int device_id = 0);

// GROUP BY SUM over N rows of (price, quantity).  Groups come out in
// ascending key order (the reference emits first-seen order from a serial
// scan; its tests expect std::map order).  *d_count receives the group count.
// Sums accumulate in double and are rounded to float on the device; the
// double scratch holds O(groups), cached per device.
void jit_group_sum(const std::string &val_expr_code, const std::string &key_expr_code, float *d_price,
                   int *d_quantity, float *d_out_vals, int *d_out_keys, int *d_count, int N, int device_id = 0);

// In-place stable sorts (LSD radix sort on the device; NaN last, -0.0 == +0.0).
void jit_sort_pairs(int *d_keys, float *d_vals, int count, bool ascending, int device_id = 0);
void jit_sort_float(float *d_vals, int count, bool ascending, int device_id = 0);
