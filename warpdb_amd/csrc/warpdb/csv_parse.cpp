// csv_parse.cpp -- multi-threaded CSV row parsing for the loaders and the
// streaming multi-GPU path (the reference parses one line at a time with
// std::getline + std::sto*, src/csv_loader.cpp:49-124, 186-223).
//
// The text is cut into line-aligned ranges, one per thread.  Pass 1 counts
// each range's non-empty lines, the columns grow once, pass 2 parses every
// range straight into its final rows.  Cells keep the std::strto* meaning of
// the sequential loader: std::from_chars handles the common case, and any
// cell it does not consume whole (leading blanks, '+', hex, trailing text,
// out-of-range) is re-read with strto* so the value and the error are the
// ones the sequential parser gives.
#include <cerrno>
#include <charconv>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "internal.hpp"

namespace warpdb {
namespace {

[[noreturn]] void bad_cell(const char *b, const char *e) {
  throw std::runtime_error("Invalid numeric value in CSV: '" + std::string(b, e) + "'");
}

template <typename T>
bool fast_int(const char *b, const char *e, T &out) {
  if (b == e || *b == '+' || *b == ' ' || *b == '\t') return false;
  auto r = std::from_chars(b, e, out, 10);
  return r.ec == std::errc() && r.ptr == e;
}

template <typename T>
bool fast_float(const char *b, const char *e, T &out) {
  if (b == e || *b == '+' || *b == ' ' || *b == '\t') return false;
  auto r = std::from_chars(b, e, out, std::chars_format::general);
  return r.ec == std::errc() && r.ptr == e;
}

void parse_cell(const HostColumn &col, void *dst_base, int64_t row, const char *b, const char *e) {
  switch (col.type) {
    case DataType::Int32: {
      int32_t v;
      if (!fast_int(b, e, v)) {
        const std::string s(b, e);
        char *end = nullptr;
        errno = 0;
        const long x = std::strtol(s.c_str(), &end, 10);
        if (end == s.c_str() || errno == ERANGE || x < INT32_MIN || x > INT32_MAX) bad_cell(b, e);
        v = static_cast<int32_t>(x);
      }
      static_cast<int32_t *>(dst_base)[row] = v;
      break;
    }
    case DataType::Int64: {
      int64_t v;
      if (!fast_int(b, e, v)) {
        const std::string s(b, e);
        char *end = nullptr;
        errno = 0;
        const long long x = std::strtoll(s.c_str(), &end, 10);
        if (end == s.c_str() || errno == ERANGE) bad_cell(b, e);
        v = x;
      }
      static_cast<int64_t *>(dst_base)[row] = v;
      break;
    }
    case DataType::Float32: {
      float v;
      if (!fast_float(b, e, v)) {
        const std::string s(b, e);
        char *end = nullptr;
        v = std::strtof(s.c_str(), &end);
        if (end == s.c_str()) bad_cell(b, e);
      }
      static_cast<float *>(dst_base)[row] = v;
      break;
    }
    case DataType::Float64: {
      double v;
      if (!fast_float(b, e, v)) {
        const std::string s(b, e);
        char *end = nullptr;
        v = std::strtod(s.c_str(), &end);
        if (end == s.c_str()) bad_cell(b, e);
      }
      static_cast<double *>(dst_base)[row] = v;
      break;
    }
    case DataType::String: static_cast<std::string *>(dst_base)[row].assign(b, e); break;
  }
}

// next line [b, le) (without '\n' / '\r'); returns the start of the line after
inline const char *next_line(const char *b, const char *e, const char *&le) {
  const char *nl = static_cast<const char *>(std::memchr(b, '\n', static_cast<size_t>(e - b)));
  const char *stop = nl ? nl : e;
  le = (stop > b && stop[-1] == '\r') ? stop - 1 : stop;
  return nl ? nl + 1 : e;
}

int64_t count_rows(const char *b, const char *e) {
  int64_t n = 0;
  while (b < e) {
    const char *le;
    const char *nb = next_line(b, e, le);
    if (le > b) ++n;
    b = nb;
  }
  return n;
}

void parse_range(const char *b, const char *e, std::vector<HostColumn> &cols, const std::vector<void *> &base,
                 int64_t row) {
  const size_t nc = cols.size();
  while (b < e) {
    const char *le;
    const char *nb = next_line(b, e, le);
    if (le > b) {
      const char *p = b;
      for (size_t c = 0; c < nc; ++c) {
        const char *q = p;
        if (p <= le) {
          q = static_cast<const char *>(std::memchr(p, ',', static_cast<size_t>(le - p)));
          if (!q) q = le;
        }
        const char *cb = p <= le ? p : le, *ce = p <= le ? q : le;  // missing cell: empty
        if (ce == cb && cols[c].type != DataType::String) bad_cell(cb, ce);
        parse_cell(cols[c], base[c], row, cb, ce);
        p = q + 1;  // past the comma (or past le: later cells are missing)
      }
      ++row;
    }
    b = nb;
  }
}

}  // namespace

int parse_threads() {
  const char *v = std::getenv("WARPDB_PARSE_THREADS");
  int t = v ? std::atoi(v) : static_cast<int>(std::thread::hardware_concurrency());
  return std::max(1, std::min(t, 16));
}

void parse_csv_rows(const char *b, const char *e, HostTable &out, int threads) {
  if (b >= e) return;
  // line-aligned ranges, at least 1 MiB each
  const size_t bytes = static_cast<size_t>(e - b);
  int T = std::max(1, std::min<int>(threads, static_cast<int>(bytes >> 20) + 1));
  std::vector<const char *> cut(T + 1, e);
  cut[0] = b;
  for (int t = 1; t < T; ++t) {
    const char *p = b + bytes * t / T;
    if (p < cut[t - 1]) p = cut[t - 1];
    const char *nl = static_cast<const char *>(std::memchr(p, '\n', static_cast<size_t>(e - p)));
    cut[t] = nl ? nl + 1 : e;
  }
  std::vector<int64_t> rows(T + 1, 0);
  std::vector<std::exception_ptr> errs(T);
  auto run = [&](auto &&fn) {
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back([&, t] {
      try {
        fn(t);
      } catch (...) {
        errs[t] = std::current_exception();
      }
    });
    try {
      fn(0);
    } catch (...) {
      errs[0] = std::current_exception();
    }
    for (auto &x : th) x.join();
    for (auto &x : errs)  // the first range's error is the sequential parser's error
      if (x) std::rethrow_exception(x);
  };
  run([&](int t) { rows[t + 1] = count_rows(cut[t], cut[t + 1]); });
  for (int t = 0; t < T; ++t) rows[t + 1] += rows[t];
  const int64_t old_n = out.num_rows();
  std::vector<void *> base(out.columns.size());
  for (size_t c = 0; c < out.columns.size(); ++c) {
    std::visit(
        [&](auto &v) {
          v.resize(static_cast<size_t>(old_n + rows[T]));
          base[c] = v.data() + old_n;
        },
        out.columns[c].data);
  }
  try {
    run([&](int t) { parse_range(cut[t], cut[t + 1], out.columns, base, rows[t]); });
  } catch (...) {
    for (auto &col : out.columns) std::visit([&](auto &v) { v.resize(static_cast<size_t>(old_n)); }, col.data);
    throw;
  }
}

}  // namespace warpdb
