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
