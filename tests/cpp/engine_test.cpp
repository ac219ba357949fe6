// engine_test.cpp -- GPU checks of the C++ API (WarpDB facade and the
// legacy jit_* entry points) with the expectations of the reference's
// jit_arch_test, jit_error_test, sql_features_test, extended_types_test and
// having_distinct_test.  Run from the repository root.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <iostream>
#include <sstream>
#include <functional>
#include <map>
#include <vector>

#include "warpdb/jit.hpp"
#include "warpdb/optimizer.hpp"
#include "warpdb/warpdb.hpp"

static int failures = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::printf("FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);   \
      ++failures;                                                  \
    }                                                              \
  } while (0)

static bool near(float a, float b) { return std::fabs(a - b) < 1e-5f; }

int main() {
  const std::string csv = "tests/golden/test.csv";
  // --- jit_compile_and_launch on a hand-built Table (jit_arch_test)
  {
    float h_price = 2.0f, h_out = 0.0f;
    int h_qty = 0;
    float *d_price, *d_out;
    int *d_qty;
    hipMalloc(&d_price, 4);
    hipMalloc(&d_qty, 4);
    hipMalloc(&d_out, 4);
    hipMemcpy(d_price, &h_price, 4, hipMemcpyHostToDevice);
    hipMemcpy(d_qty, &h_qty, 4, hipMemcpyHostToDevice);
    Table t;
    t.num_rows = 1;
    t.columns.push_back({"price", DataType::Float32, d_price, 1});
    t.columns.push_back({"quantity", DataType::Int32, d_qty, 1});
    bool threw = false;
    try {
      jit_compile_and_launch("price", "", t, d_out);
    } catch (...) {
      threw = true;
    }
    CHECK(!threw);
    hipMemcpy(&h_out, d_out, 4, hipMemcpyDeviceToHost);
    CHECK(h_out == h_price);
    // jit_error_test: a failed compile, then a successful call
    threw = false;
    try {
      jit_compile_and_launch("invalid@", "", t, d_out);
    } catch (const std::exception &) {
      threw = true;
    }
    CHECK(threw);
    threw = false;
    try {
      jit_compile_and_launch("price + 1", "", t, d_out);
    } catch (...) {
      threw = true;
    }
    CHECK(!threw);
    hipMemcpy(&h_out, d_out, 4, hipMemcpyDeviceToHost);
    CHECK(h_out == 3.0f);
    hipFree(d_price);
    hipFree(d_qty);
    hipFree(d_out);
  }
  // --- jit_group_sum / jit_sort_pairs / jit_sort_float with the reference
  // signatures (include/jit.hpp:15-27): test.csv's sql_features_test
  // expectations (keys 2,3,4,5 -> 15.25, 10.5, 20, 30), then 1e6 rows of
  // 1000 keys against a host std::map (the reference query_sql's AggData)
  {
    const float hp[4] = {10.5f, 20.0f, 15.25f, 30.0f};
    const int hq[4] = {3, 4, 2, 5};
    float *d_p, *d_vals;
    int *d_q, *d_keys, *d_count;
    hipMalloc(&d_p, 16);
    hipMalloc(&d_q, 16);
    hipMalloc(&d_vals, 16);
    hipMalloc(&d_keys, 16);
    hipMalloc(&d_count, 4);
    hipMemcpy(d_p, hp, 16, hipMemcpyHostToDevice);
    hipMemcpy(d_q, hq, 16, hipMemcpyHostToDevice);
    jit_group_sum("price[idx]", "quantity[idx]", d_p, d_q, d_vals, d_keys, d_count, 4);
    int cnt = 0;
    float v[4];
    int k[4];
    hipMemcpy(&cnt, d_count, 4, hipMemcpyDeviceToHost);
    hipMemcpy(v, d_vals, 16, hipMemcpyDeviceToHost);
    hipMemcpy(k, d_keys, 16, hipMemcpyDeviceToHost);
    CHECK(cnt == 4 && k[0] == 2 && k[1] == 3 && k[2] == 4 && k[3] == 5);
    CHECK(v[0] == 15.25f && v[1] == 10.5f && v[2] == 20.0f && v[3] == 30.0f);
    // ORDER BY the group key DESC: jit_sort_pairs (query_sql, src/warpdb.cpp:365-371)
    jit_sort_pairs(d_keys, d_vals, cnt, false);
    hipMemcpy(v, d_vals, 16, hipMemcpyDeviceToHost);
    hipMemcpy(k, d_keys, 16, hipMemcpyDeviceToHost);
    CHECK(k[0] == 5 && k[3] == 2 && v[0] == 30.0f && v[3] == 15.25f);
    // ORDER BY price DESC (LIMIT 2 -> 30, 20: sql_features_test.cpp:24-30)
    hipMemcpy(d_vals, hp, 16, hipMemcpyHostToDevice);
    jit_sort_float(d_vals, 4, false);
    hipMemcpy(v, d_vals, 16, hipMemcpyDeviceToHost);
    CHECK(v[0] == 30.0f && v[1] == 20.0f && v[2] == 15.25f && v[3] == 10.5f);
    hipFree(d_p);
    hipFree(d_q);
    hipFree(d_vals);
    hipFree(d_keys);
    hipFree(d_count);

    const int n = 1000000, groups = 1000;
    std::vector<float> p(n);
    std::vector<int> q(n);
    uint64_t x = 42;
    for (int i = 0; i < n; ++i) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      p[i] = static_cast<float>((x >> 40) & 0xffff) / 1024.0f;
      q[i] = static_cast<int>((x >> 20) % groups) - 200;  // keys -200..799: both sides of 0
    }
    std::map<int, double> expect;
    for (int i = 0; i < n; ++i) expect[q[i]] += p[i];
    hipMalloc(&d_p, n * 4);
    hipMalloc(&d_q, n * 4);
    hipMalloc(&d_vals, n * 4);  // sized for N rows, as query_sql allocates (src/warpdb.cpp:356-358)
    hipMalloc(&d_keys, n * 4);
    hipMalloc(&d_count, 4);
    hipMemcpy(d_p, p.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_q, q.data(), n * 4, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; ++rep) {  // the second call reuses the cached scratch
      jit_group_sum("(price[idx] * 2.0f)", "quantity[idx]", d_p, d_q, d_vals, d_keys, d_count, n);
      hipMemcpy(&cnt, d_count, 4, hipMemcpyDeviceToHost);
      CHECK(cnt == static_cast<int>(expect.size()));
      std::vector<float> gv(cnt);
      std::vector<int> gk(cnt);
      hipMemcpy(gv.data(), d_vals, cnt * 4, hipMemcpyDeviceToHost);
      hipMemcpy(gk.data(), d_keys, cnt * 4, hipMemcpyDeviceToHost);
      int i = 0;
      bool ok = true;
      for (auto &kv : expect) {
        ok = ok && i < cnt && gk[i] == kv.first && gv[i] == static_cast<float>(2.0 * kv.second);
        ++i;
      }
      CHECK(ok);
    }
    // jit_sort_float on 1e6 values vs std::stable_sort; jit_sort_pairs stability
    hipMemcpy(d_vals, p.data(), n * 4, hipMemcpyHostToDevice);
    jit_sort_float(d_vals, n, true);
    std::vector<float> sorted(n), ref = p;
    hipMemcpy(sorted.data(), d_vals, n * 4, hipMemcpyDeviceToHost);
    std::stable_sort(ref.begin(), ref.end());
    CHECK(sorted == ref);
    std::vector<float> payload(n);
    for (int i = 0; i < n; ++i) payload[i] = static_cast<float>(i);
    hipMemcpy(d_vals, payload.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_keys, q.data(), n * 4, hipMemcpyHostToDevice);
    jit_sort_pairs(d_keys, d_vals, n, true);
    std::vector<int> order(n);
    for (int i = 0; i < n; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return q[a] < q[b]; });
    std::vector<float> pv(n);
    std::vector<int> pk(n);
    hipMemcpy(pv.data(), d_vals, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(pk.data(), d_keys, n * 4, hipMemcpyDeviceToHost);
    bool stable = true;
    for (int i = 0; i < n; ++i) stable = stable && pk[i] == q[order[i]] && pv[i] == static_cast<float>(order[i]);
    CHECK(stable);
    hipFree(d_p);
    hipFree(d_q);
    hipFree(d_vals);
    hipFree(d_keys);
    hipFree(d_count);
  }
  // --- WarpDB facade (sql_features_test, having_distinct_test)
  {
    WarpDB db(csv);
    auto r = db.query("price * quantity WHERE price > 10");
    CHECK(r.size() == 4 && r[0] == 31.5f && r[1] == 80.0f && r[2] == 30.5f && r[3] == 150.0f);
    HostTable h = load_csv_to_host(csv);
    const auto &price = std::get<std::vector<float>>(h.columns[0].data);
    const auto &qty = std::get<std::vector<float>>(h.columns[1].data);
    std::map<int, double> groups;
    for (size_t i = 0; i < price.size(); ++i) groups[static_cast<int>(qty[i])] += price[i];
    auto res = db.query_sql("SELECT SUM(price) FROM test GROUP BY quantity ORDER BY quantity ASC");
    CHECK(res.size() == groups.size());
    size_t i = 0;
    for (auto &kv : groups) CHECK(i < res.size() && near(res[i++], static_cast<float>(kv.second)));
    auto limited = db.query_sql("SELECT price FROM test ORDER BY price DESC LIMIT 2");
    std::vector<float> sorted = price;
    std::sort(sorted.begin(), sorted.end(), std::greater<float>());
    CHECK(limited.size() == 2 && near(limited[0], sorted[0]) && near(limited[1], sorted[1]));
    auto offset = db.query_sql("SELECT price FROM test ORDER BY price DESC OFFSET 1 LIMIT 2");
    CHECK(offset.size() == 2 && near(offset[0], sorted[1]) && near(offset[1], sorted[2]));
    auto having = db.query_sql("SELECT SUM(price) FROM test GROUP BY quantity HAVING SUM(price) > 15 ORDER BY quantity ASC");
    CHECK(having.size() == 3);
    auto none = db.query_sql("SELECT SUM(price) FROM test GROUP BY quantity HAVING COUNT(price) > 1");
    CHECK(none.empty());
    auto distinct = db.query_sql("SELECT DISTINCT quantity FROM test ORDER BY quantity DESC");
    CHECK(distinct.size() == 4 && distinct.front() > distinct.back());
    auto top = db.query_sql("SELECT price FROM test ORDER BY price DESC LIMIT 5");
    CHECK(top.size() == 4 && top[0] == 30.0f && top[3] == 10.5f);
    auto sum = db.query_sum("price * 0.9 WHERE price > 20");
    CHECK(sum.second == 1 && near(static_cast<float>(sum.first), 27.0f));
    // the row-sharded aggregates (every visible GPU)
    auto msum = db.query_multi_gpu_sum("price * 0.9 WHERE price > 20");
    CHECK(msum.second == 1 && near(static_cast<float>(msum.first), 27.0f));
    auto mg = db.query_multi_gpu_group("SELECT SUM(price) FROM test GROUP BY quantity");
    CHECK(mg.keys.size() == groups.size());
    i = 0;
    for (auto &kv : groups) {
      CHECK(i < mg.keys.size() && mg.keys[i] == kv.first && mg.sums[i] == kv.second && mg.counts[i] == 1);
      ++i;
    }
  }
  // --- extended_types_test: schema {F32, I32, F32}
  {
    WarpDB db("tests/golden/extended.csv", {DataType::Float32, DataType::Int32, DataType::Float32});
    auto res = db.query("price * discount");
    CHECK(res.size() == 4 && static_cast<int>(res[0]) == 1);
  }
  // --- JSON input (src/json_loader.cpp)
  {
    WarpDB db("tests/golden/test.json");
    auto r = db.query("price * quantity WHERE price > 15");
    CHECK(r.size() == 4 && r[0] == 0.0f && r[1] == 80.0f && r[3] == 150.0f);
  }
  // --- optimizer (src/optimizer.cpp): execute_query_optimized output
  {
    WarpDB db("tests/golden/test.csv");
    Table &t = const_cast<Table &>(db.table());
    std::ostringstream cap;
    auto *old = std::cout.rdbuf(cap.rdbuf());
    execute_query_optimized("price * quantity", "price > 100", t);
    execute_query_optimized("price * 2", "price > 15", t);
    std::cout.rdbuf(old);
    CHECK(cap.str() == "[Optimizer] Filter eliminates all rows.\nResult[0] = 0\nResult[1] = 40\n"
                       "Result[2] = 30.5\nResult[3] = 60\n");
    bool at = false, af = false;
    TableStats ts;
    ts.price.min = 10.5f;
    ts.price.max = 30.0f;
    ts.quantity.min = 2;
    ts.quantity.max = 5;
    auto cond = parse_expression(tokenize("price > 10 AND quantity < 6"));
    analyze_condition(cond.get(), ts, at, af);
    CHECK(at && !af);
  }
  if (failures) return 1;
  std::printf("engine_test: all passed\n");
  return 0;
}
