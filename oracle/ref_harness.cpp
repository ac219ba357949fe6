// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Driver around the reference's own CPU code, compiled by oracle/build_ref.sh
// straight from /root/reference (nothing is copied into this repository):
//   src/expression.cpp:1-268   tokenize / parse_expression / parse_logical_*
//   src/warpdb.cpp:109-157     get_value / eval_node / eval_condition
//   src/csv_loader.cpp:49-124  load_csv_to_host
// The slices are the parts of those files that compile without CUDA; the
// rest of each file is left out because the snapshot does not build
// (SURVEY.md section 0).  This file supplies only main(): it never restates
// reference logic, it calls it.
//
// Modes:
//   ref_harness lower  "<expr>"                -> lowered CUDA-C string
//   ref_harness tokens "<expr>"                -> one token per line
//   ref_harness eval   <csv> "<query>" [schema] -> "idx hexfloat" per passing row
//   ref_harness bench  <rows> "<query>" [threads]
//                                              -> JSON timing of the reference
//                                                 evaluator over synthetic rows
//                                                 (threads > 1: contiguous row
//                                                 ranges on std::threads, the
//                                                 per-range row lists joined in
//                                                 order; the reference itself is
//                                                 single-threaded)
//   ref_harness groupsum <csv> "<val>" "<key>" [schema]
//                                              -> "key hexdouble count" per group:
//                                                 the reference query_sql's CPU
//                                                 aggregation (std::map<int,
//                                                 AggData>, double sums,
//                                                 src/warpdb.cpp:375-385) over
//                                                 the reference's eval_node
//   ref_harness topk <csv> "<order>" k desc [schema]
//                                              -> "row hexfloat" of the first k
//                                                 rows of a stable sort by the
//                                                 reference's eval_node value
//                                                 (the intent of ORDER BY .. LIMIT,
//                                                 tests/sql_features_test.cpp:24-30)
#include <algorithm>
#include <chrono>
#include <cmath>
#include <map>
#include <thread>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_set>
#include <variant>
#include <vector>

#include "csv_loader.hpp"
#include "expression.hpp"

#include "slice_expression.inc"
#include "slice_eval.inc"
#include "slice_csv.inc"

namespace {

void split_where(const std::string &q, std::string &e, std::string &c) {
  // The same split WarpDB::query performs (src/warpdb.cpp:204-213); kept in
  // the harness because that function body also uploads to the GPU.
  std::string up = q;
  for (auto &ch : up) ch = static_cast<char>(std::toupper(static_cast<unsigned char>(ch)));
  auto p = up.find("WHERE");
  if (p == std::string::npos) {
    e = q;
    c.clear();
  } else {
    e = q.substr(0, p);
    c = q.substr(p + 5);
  }
}

uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Synthetic generator shared with warpexec's wx_fill_synthetic.
float gen_uniform(uint64_t seed, uint64_t row, float lo, float hi) {
  uint64_t h = splitmix64(row + seed * 0xD1B54A32D192ED03ull);
  float u = static_cast<float>(h >> 40) * (1.0f / 16777216.0f);
  volatile float span = hi - lo;
  volatile float m = u * span;
  return lo + m;
}
int64_t gen_int(uint64_t seed, uint64_t row, int64_t lo, int64_t hi) {
  uint64_t h = splitmix64(row + seed * 0xD1B54A32D192ED03ull);
  return lo + static_cast<int64_t>((h >> 32) % static_cast<uint64_t>(hi - lo + 1));
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: ref_harness lower|tokens|eval|bench ...\n");
    return 2;
  }
  std::string mode = argv[1];
  try {
    if (mode == "lower") {
      auto ast = parse_expression(tokenize(argv[2]));
      std::printf("%s\n", ast->to_cuda_expr().c_str());
      return 0;
    }
    if (mode == "tokens") {
      for (auto &t : tokenize(argv[2]))
        std::printf("%d %s %d %d\n", static_cast<int>(t.type), t.value.c_str(), t.line, t.column);
      return 0;
    }
    if (mode == "eval" && argc >= 4) {
      std::vector<DataType> schema;
      if (argc >= 5)
        for (const char *s = argv[4]; *s; ++s) schema.push_back(static_cast<DataType>(*s - '0'));
      HostTable h = load_csv_to_host(argv[2], schema);
      std::string e, c;
      split_where(argv[3], e, c);
      auto ex = parse_expression(tokenize(e));
      std::unique_ptr<ASTNode> cx;
      if (!c.empty()) cx = parse_expression(tokenize(c));
      for (int i = 0; i < h.num_rows(); ++i) {
        if (cx && !eval_condition(cx.get(), h, i)) continue;
        std::printf("%d %a\n", i, static_cast<double>(eval_node(ex.get(), h, i)));
      }
      return 0;
    }
    if (mode == "bench" && argc >= 4) {
      long long n = std::atoll(argv[2]);
      HostTable h;
      h.columns.resize(2);
      h.columns[0].name = "price";
      h.columns[0].type = DataType::Float32;
      h.columns[1].name = "quantity";
      h.columns[1].type = DataType::Float32;
      std::vector<float> p(n), q(n);
      for (long long i = 0; i < n; ++i) {
        p[i] = gen_uniform(1, i, 0.0f, 40.0f);
        q[i] = static_cast<float>(gen_int(2, i, 1, 100));
      }
      h.columns[0].data = std::move(p);
      h.columns[1].data = std::move(q);
      std::string e, c;
      split_where(argv[3], e, c);
      auto ex = parse_expression(tokenize(e));
      std::unique_ptr<ASTNode> cx;
      if (!c.empty()) cx = parse_expression(tokenize(c));
      const int threads = argc >= 5 ? std::max(1, std::atoi(argv[4])) : 1;
      // Output pages are touched before the clock starts (both modes): the
      // timing is the evaluator's, not the kernel's page-fault path, which
      // serialises threads on the address-space lock.
      std::vector<float> out(n);
      std::vector<int> rows(n);
      std::vector<long long> filled(threads, 0);
      const long long chunk = (n + threads - 1) / threads;
      auto t0 = std::chrono::steady_clock::now();
      // The reference CPU path: ascending row list of passing rows
      // (src/warpdb.cpp:336-344) then eval_node per row (:457-459).
      auto scan = [&](int t) {
        const long long b = std::min(n, t * chunk), e = std::min(n, b + chunk);
        long long k = b;
        for (long long i = b; i < e; ++i) {
          if (cx && !eval_condition(cx.get(), h, static_cast<int>(i))) continue;
          rows[k] = static_cast<int>(i);
          out[k++] = eval_node(ex.get(), h, static_cast<int>(i));
        }
        filled[t] = k - b;
      };
      if (threads == 1) {
        scan(0);
      } else {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t) th.emplace_back(scan, t);
        for (auto &x : th) x.join();
      }
      // close the gaps between the ranges: the row list in ascending order
      long long total = filled[0];
      for (int t = 1; t < threads; ++t) {
        const long long b = std::min(n, t * chunk);
        std::memmove(&rows[total], &rows[b], sizeof(int) * filled[t]);
        std::memmove(&out[total], &out[b], sizeof(float) * filled[t]);
        total += filled[t];
      }
      rows.resize(total);
      out.resize(total);
      auto t1 = std::chrono::steady_clock::now();
      double s = std::chrono::duration<double>(t1 - t0).count();
      double chk = 0;
      for (float v : out) chk += v;
      std::printf("{\"rows\": %lld, \"threads\": %d, \"seconds\": %.6f, \"rows_per_s\": %.1f, \"passing\": %zu, "
                  "\"checksum\": %.6f}\n",
                  n, threads, s, n / s, rows.size(), chk);
      return 0;
    }
    if (mode == "groupsum" && argc >= 5) {
      std::vector<DataType> schema;
      if (argc >= 6)
        for (const char *c = argv[5]; *c; ++c) schema.push_back(static_cast<DataType>(*c - '0'));
      HostTable h = load_csv_to_host(argv[2], schema);
      auto val = parse_expression(tokenize(argv[3]));
      auto key = parse_expression(tokenize(argv[4]));
      std::map<int, std::pair<double, long long>> groups;  // AggData's sum / count
      for (int i = 0; i < h.num_rows(); ++i) {
        auto &g = groups[static_cast<int>(eval_node(key.get(), h, i))];
        g.first += eval_node(val.get(), h, i);
        g.second += 1;
      }
      for (auto &kv : groups) std::printf("%d %a %lld\n", kv.first, kv.second.first, kv.second.second);
      return 0;
    }
    if (mode == "topk" && argc >= 6) {
      std::vector<DataType> schema;
      if (argc >= 7)
        for (const char *c = argv[6]; *c; ++c) schema.push_back(static_cast<DataType>(*c - '0'));
      HostTable h = load_csv_to_host(argv[2], schema);
      auto ord = parse_expression(tokenize(argv[3]));
      const int k = std::atoi(argv[4]);
      const bool desc = std::atoi(argv[5]) != 0;
      std::vector<std::pair<float, int>> v;
      for (int i = 0; i < h.num_rows(); ++i) v.push_back({eval_node(ord.get(), h, i), i});
      // NaN last in either direction, ties keep row order (a stable sort)
      std::stable_sort(v.begin(), v.end(), [&](const std::pair<float, int> &a, const std::pair<float, int> &b) {
        if (std::isnan(a.first) || std::isnan(b.first)) return !std::isnan(a.first) && std::isnan(b.first);
        return desc ? a.first > b.first : a.first < b.first;
      });
      for (int i = 0; i < k && i < static_cast<int>(v.size()); ++i)
        std::printf("%d %a\n", v[i].second, static_cast<double>(v[i].first));
      return 0;
    }
  } catch (const std::exception &ex) {
    std::printf("ERROR: %s\n", ex.what());
    return 1;
  }
  std::fprintf(stderr, "bad arguments\n");
  return 2;
}
