// csv_loader.hpp -- table types and loaders (drop-in for the reference's
// include/csv_loader.hpp).  Same names and members; row counts are 64-bit
// (the reference uses int, which caps a table at 2^31 rows).
#pragma once
#include <cstdint>
#include <istream>
#include <string>
#include <variant>
#include <vector>

enum class DataType { Int32, Int64, Float32, Float64, String };

struct ColumnDesc {
  std::string name;
  DataType type;
  void *device_ptr;  // HBM, caller-owned (or WarpDB-owned inside the facade)
  int64_t length;
};

struct ColumnStatsFloat {
  float min = 0.0f;
  float max = 0.0f;
  int null_count = 0;
};

struct ColumnStatsInt {
  int min = 0;
  int max = 0;
  int null_count = 0;
};

struct TableStats {
  ColumnStatsFloat price;
  ColumnStatsInt quantity;
};

// Device table: column descriptors in schema order + row count.
struct Table {
  std::vector<ColumnDesc> columns;
  int64_t num_rows = 0;
  int device = 0;  // HIP device that holds the columns

  template <typename T>
  T *get_column_ptr(const std::string &name) const {
    for (const auto &c : columns)
      if (c.name == name) return static_cast<T *>(c.device_ptr);
    return nullptr;
  }
};

using ColumnData = std::variant<std::vector<int32_t>, std::vector<int64_t>, std::vector<float>,
                                std::vector<double>, std::vector<std::string>>;

struct HostColumn {
  std::string name;
  DataType type;
  ColumnData data;
};

struct HostTable {
  std::vector<HostColumn> columns;
  int64_t num_rows() const {
    if (columns.empty()) return 0;
    return std::visit([](auto &&v) { return static_cast<int64_t>(v.size()); }, columns[0].data);
  }
  const HostColumn *get_column(const std::string &name) const {
    for (const auto &c : columns)
      if (c.name == name) return &c;
    return nullptr;
  }
};

// Header line = column names; default schema all Float32 (reference
// src/csv_loader.cpp:49-124).  Throws std::runtime_error on I/O errors,
// schema mismatch or unparsable cells.
HostTable load_csv_to_host(const std::string &filepath, const std::vector<DataType> &schema = {});

// Copy every numeric column into freshly allocated HBM on `device` (String
// columns stay host-only: device_ptr = nullptr).  Free with free_table().
Table upload_to_gpu(const HostTable &table, int device = 0);
Table load_csv_to_gpu(const std::string &filepath, const std::vector<DataType> &schema = {});
void free_table(Table &table);

// Read up to max_rows data rows from a stream positioned after the header.
// Column names and types come from `header` (the reference re-reads a data row
// as the header of every chunk, src/csv_loader.cpp:186-223; fixed here).
HostTable load_csv_chunk(std::istream &stream, int64_t max_rows, bool &finished,
                         const std::vector<std::string> &names, const std::vector<DataType> &schema = {});
// Reference signature: the first line read is taken as the header.
HostTable load_csv_chunk(std::istream &stream, int max_rows, bool &finished);
