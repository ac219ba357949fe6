// loaders.cpp -- CSV / JSON loading into host tables and HBM.
// Semantics follow the reference loaders (src/csv_loader.cpp:49-223,
// src/json_loader.cpp:16-53): header row of names, default schema all
// Float32, one value per comma-separated cell.
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "warpdb/csv_loader.hpp"
#include "internal.hpp"
#include "warpdb/json_loader.hpp"

namespace {

void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + what + ": " + hipGetErrorString(e));
}

std::vector<std::string> split_commas(const std::string &line) {
  std::vector<std::string> out;
  std::string cell;
  std::stringstream ss(line);
  while (std::getline(ss, cell, ',')) out.push_back(cell);
  return out;
}

void strip_cr(std::string &s) {
  if (!s.empty() && s.back() == '\r') s.pop_back();
}

ColumnData empty_column(DataType t) {
  switch (t) {
    case DataType::Int32: return std::vector<int32_t>();
    case DataType::Int64: return std::vector<int64_t>();
    case DataType::Float32: return std::vector<float>();
    case DataType::Float64: return std::vector<double>();
    case DataType::String: return std::vector<std::string>();
  }
  return std::vector<float>();
}

HostTable make_table(const std::vector<std::string> &names, const std::vector<DataType> &schema) {
  if (!schema.empty() && schema.size() != names.size())
    throw std::runtime_error("Schema size does not match column count");
  HostTable h;
  for (size_t i = 0; i < names.size(); ++i) {
    const DataType t = schema.empty() ? DataType::Float32 : schema[i];
    h.columns.push_back({names[i], t, empty_column(t)});
  }
  return h;
}

size_t width(DataType t) {
  switch (t) {
    case DataType::Int32:
    case DataType::Float32: return 4;
    case DataType::Int64:
    case DataType::Float64: return 8;
    default: return 0;
  }
}

const void *host_data(const HostColumn &c) {
  return std::visit([](auto &&v) -> const void * { return v.data(); }, c.data);
}

}  // namespace

HostTable load_csv_to_host(const std::string &filepath, const std::vector<DataType> &schema) {
  // the whole file is mapped and its rows parsed in parallel
  const int fd = ::open(filepath.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("Unable to open file: " + filepath);
  struct stat st;
  if (::fstat(fd, &st) != 0) {
    ::close(fd);
    throw std::runtime_error("Unable to open file: " + filepath);
  }
  const size_t size = static_cast<size_t>(st.st_size);
  if (size == 0) {
    ::close(fd);
    throw std::runtime_error("Empty CSV file");
  }
  void *map = ::mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
  ::close(fd);
  if (map == MAP_FAILED) throw std::runtime_error("Unable to map file: " + filepath);
  struct Unmap {
    void *p;
    size_t n;
    ~Unmap() { ::munmap(p, n); }
  } unmap{map, size};
  const char *b = static_cast<const char *>(map), *e = b + size;
  const char *nl = static_cast<const char *>(std::memchr(b, '\n', size));
  std::string header(b, nl ? nl : e);
  strip_cr(header);
  HostTable h = make_table(split_commas(header), schema);
  if (nl) warpdb::parse_csv_rows(nl + 1, e, h, warpdb::parse_threads());
  return h;
}

Table upload_to_gpu(const HostTable &host, int device) {
  int prev = 0;
  hip_check(hipGetDevice(&prev), "hipGetDevice");
  hip_check(hipSetDevice(device), "hipSetDevice");
  Table t;
  t.num_rows = host.num_rows();
  t.device = device;
  try {
    for (const auto &c : host.columns) {
      void *p = nullptr;
      const size_t w = width(c.type);
      if (w && t.num_rows > 0) {
        hip_check(hipMalloc(&p, w * static_cast<size_t>(t.num_rows)), "hipMalloc");
        t.columns.push_back({c.name, c.type, p, t.num_rows});
        warpdb::copy_h2d(device, nullptr, p, host_data(c), w * static_cast<size_t>(t.num_rows));
      } else {
        t.columns.push_back({c.name, c.type, nullptr, t.num_rows});  // strings stay on the host
      }
    }
    hip_check(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
  } catch (...) {
    free_table(t);
    (void)hipSetDevice(prev);
    throw;
  }
  (void)hipSetDevice(prev);
  return t;
}

Table load_csv_to_gpu(const std::string &filepath, const std::vector<DataType> &schema) {
  return upload_to_gpu(load_csv_to_host(filepath, schema));
}

void free_table(Table &t) {
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(t.device);
  for (auto &c : t.columns)
    if (c.device_ptr) (void)hipFree(c.device_ptr);
  t.columns.clear();
  t.num_rows = 0;
  (void)hipSetDevice(prev);
}

HostTable load_csv_chunk(std::istream &stream, int64_t max_rows, bool &finished, const std::vector<std::string> &names,
                         const std::vector<DataType> &schema) {
  HostTable h = make_table(names, schema);
  // gather up to max_rows non-empty lines, then parse them in parallel
  std::string text, line;
  int64_t n = 0;
  while (n < max_rows && std::getline(stream, line)) {
    strip_cr(line);
    if (line.empty()) continue;
    text.append(line).push_back('\n');
    ++n;
  }
  finished = !stream.good();
  warpdb::parse_csv_rows(text.data(), text.data() + text.size(), h, warpdb::parse_threads());
  return h;
}

HostTable load_csv_chunk(std::istream &stream, int max_rows, bool &finished) {
  std::string header;
  if (!std::getline(stream, header)) {
    finished = true;
    return {};
  }
  strip_cr(header);
  return load_csv_chunk(stream, static_cast<int64_t>(max_rows), finished, split_commas(header), {});
}

HostTable load_json_to_host(const std::string &filepath) {
  std::ifstream file(filepath);
  if (!file.is_open()) throw std::runtime_error("Unable to open file: " + filepath);
  HostTable h;
  h.columns.push_back({"price", DataType::Float32, std::vector<float>()});
  h.columns.push_back({"quantity", DataType::Int32, std::vector<int32_t>()});
  auto &price = std::get<std::vector<float>>(h.columns[0].data);
  auto &qty = std::get<std::vector<int32_t>>(h.columns[1].data);
  std::string line;
  while (std::getline(file, line)) {
    const size_t p = line.find("\"price\"");
    const size_t q = line.find("\"quantity\"");
    if (p == std::string::npos || q == std::string::npos) continue;
    const size_t pc = line.find(':', p), qc = line.find(':', q);
    if (pc == std::string::npos || qc == std::string::npos) continue;
    price.push_back(std::strtof(line.c_str() + pc + 1, nullptr));
    qty.push_back(static_cast<int32_t>(std::strtol(line.c_str() + qc + 1, nullptr, 10)));
  }
  return h;
}

Table load_json_to_gpu(const std::string &filepath, int device) { return upload_to_gpu(load_json_to_host(filepath), device); }
