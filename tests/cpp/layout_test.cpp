// layout_test.cpp -- pins the boundary's compatibility level at compile time
// (INTEGRATION.md 1.1).  The drop-in is SOURCE-level: reference call sites
// compile unchanged against include/warpdb/, but the row counts are 64-bit
// and Table / WarpDB carry a device, so a binary built against the
// reference's headers (include/csv_loader.hpp:15-51, include/warpdb.hpp:13-14)
// cannot link against libwarpdb.  What the C++ shims rely on is asserted here;
// main() only exercises the reference's own idioms.
#include <cstddef>
#include <cstdint>
#include <string>
#include <type_traits>
#include <vector>

#include "warpdb/warpdb.hpp"
#include "warpexec.h"

// WxTableView (jit_shim.cpp) hands DataType to the C ABI by value cast
static_assert(static_cast<int>(DataType::Int32) == WX_INT32, "DataType / wx_dtype numbering");
static_assert(static_cast<int>(DataType::Int64) == WX_INT64, "DataType / wx_dtype numbering");
static_assert(static_cast<int>(DataType::Float32) == WX_FLOAT32, "DataType / wx_dtype numbering");
static_assert(static_cast<int>(DataType::Float64) == WX_FLOAT64, "DataType / wx_dtype numbering");
static_assert(static_cast<int>(DataType::String) == WX_STRING, "DataType / wx_dtype numbering");

// ... and the row count without narrowing
static_assert(std::is_same<decltype(Table::num_rows), int64_t>::value, "Table::num_rows is 64-bit");
static_assert(std::is_same<decltype(Table::num_rows), decltype(wx_table::n_rows)>::value,
              "Table::num_rows carries wx_table::n_rows unchanged");
static_assert(std::is_same<decltype(ColumnDesc::length), int64_t>::value, "ColumnDesc::length is 64-bit");
static_assert(std::is_same<decltype(ColumnDesc::device_ptr), void *>::value, "device_ptr is a plain HIP pointer");
static_assert(std::is_same<decltype(Table::device), int>::value, "Table::device (not in the reference)");

// the reference's members, in its order (source compatibility for aggregate
// initialisation as its tests write it)
static_assert(offsetof(ColumnDesc, name) < offsetof(ColumnDesc, type), "member order");
static_assert(offsetof(ColumnDesc, type) < offsetof(ColumnDesc, device_ptr), "member order");
static_assert(offsetof(ColumnDesc, device_ptr) < offsetof(ColumnDesc, length), "member order");

// the reference's constructor calls still compile (the device argument is defaulted)
static_assert(std::is_constructible<WarpDB, const std::string &>::value, "WarpDB(path)");
static_assert(std::is_constructible<WarpDB, const std::string &, const std::vector<DataType> &>::value,
              "WarpDB(path, schema)");
static_assert(std::is_constructible<WarpDB, const std::string &, const std::vector<DataType> &, int>::value,
              "WarpDB(path, schema, device)");

int main() {
  // reference idioms (tests/jit_arch_test.cpp builds a Table by hand)
  Table t;
  t.columns.push_back({"price", DataType::Float32, nullptr, 10});
  t.num_rows = 10;
  int n = static_cast<int>(t.num_rows);  // reference callers hold row counts in int
  float *p = t.get_column_ptr<float>("price");
  return (n == 10 && p == nullptr && t.device == 0) ? 0 : 1;
}
