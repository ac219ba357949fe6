// sanitize_test.cpp -- host code of the product under AddressSanitizer and
// UndefinedBehaviorSanitizer (no GPU): the expression / SQL front end on
// random token soup and pathological nesting, and the parallel CSV parser
// (csv_parse.cpp) against a sequential std::getline + strto* reading of the
// same text, including blanks, '+', hex, CRLF, blank lines, missing cells.
// Built by `make -C tests/cpp sanitize_test` with -fsanitize=address,undefined.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "warpdb/expression.hpp"
#include "../../warpdb_amd/csrc/warpdb/internal.hpp"

static int failures = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::printf("FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);   \
      ++failures;                                                  \
    }                                                              \
  } while (0)

static void fuzz_front_end() {
  const char *atoms[] = {"price", "quantity", "1", "2.5", ".5", "10.", "(", ")", "+", "-", "*", "/", ">", "<",
                         ">=", "<=", "==", "!=", "=", "AND", "OR", "discount", ",", "a.b", "SUM", "COUNT", "*",
                         "WHERE", "SELECT", "FROM", "GROUP", "BY", "ORDER", "DESC", "LIMIT", "OFFSET", "HAVING",
                         "DISTINCT", "JOIN", "ON", "t", "99999999999", "@", "\n", " "};
  const int na = sizeof(atoms) / sizeof(atoms[0]);
  std::mt19937 rng(12345);
  int parsed = 0, rejected = 0;
  for (int it = 0; it < 40000; ++it) {
    std::string s;
    const int len = 1 + static_cast<int>(rng() % 14);
    if (it % 2) s = "SELECT ";
    for (int k = 0; k < len; ++k) s += std::string(atoms[rng() % na]) + (rng() % 3 ? " " : "");
    try {
      if (it % 2) {
        QueryAST q = parse_query(tokenize(s));
        for (auto &e : q.select_list) (void)e->to_cuda_expr();
      } else {
        (void)parse_expression(tokenize(s))->to_cuda_expr();
      }
      ++parsed;
    } catch (const std::runtime_error &) {
      ++rejected;
    }
  }
  CHECK(parsed > 100 && rejected > 100);
  // nesting: a deep nest is an error, not a stack overflow
  for (const char *open : {"(", "f("}) {
    std::string deep;
    for (int i = 0; i < 100000; ++i) deep += open;
    deep += "1";
    bool threw = false;
    try {
      (void)parse_expression(tokenize(deep));
    } catch (const std::runtime_error &e) {
      threw = std::string(e.what()).find("nested too deeply") != std::string::npos;
    }
    CHECK(threw);
  }
  std::string ok = "1";
  for (int i = 0; i < 200; ++i) ok = "(" + ok + " + 1)";
  CHECK(parse_expression(tokenize(ok))->to_cuda_expr().size() > 200);
  bool threw = false;
  try {
    (void)parse_query(tokenize("SELECT price FROM t LIMIT 99999999999"));
  } catch (const std::runtime_error &) {
    threw = true;
  }
  CHECK(threw);
}

// Sequential reading of the same text: std::getline, split on ',', strto*.
static bool sequential(const std::string &text, std::vector<float> &f, std::vector<int32_t> &i,
                       std::vector<double> &d) {
  std::istringstream in(text);
  std::string line;
  while (std::getline(in, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.empty()) continue;
    std::vector<std::string> cells;
    std::stringstream ss(line);
    std::string c;
    while (std::getline(ss, c, ',')) cells.push_back(c);
    if (cells.size() < 3) return false;
    char *end = nullptr;
    const float fv = std::strtof(cells[0].c_str(), &end);
    if (end == cells[0].c_str()) return false;
    const long iv = std::strtol(cells[1].c_str(), &end, 10);
    if (end == cells[1].c_str()) return false;
    const double dv = std::strtod(cells[2].c_str(), &end);
    if (end == cells[2].c_str()) return false;
    f.push_back(fv);
    i.push_back(static_cast<int32_t>(iv));
    d.push_back(dv);
  }
  return true;
}

static HostTable empty_table() {
  HostTable t;
  t.columns.push_back({"a", DataType::Float32, std::vector<float>{}});
  t.columns.push_back({"b", DataType::Int32, std::vector<int32_t>{}});
  t.columns.push_back({"c", DataType::Float64, std::vector<double>{}});
  return t;
}

static void fuzz_csv() {
  std::mt19937 rng(777);
  const char *odd_f[] = {" 1.5", "+2", "0x1p3", "1e3", "-0", "nan", "inf", "3.25 ", "1e-50"};
  std::string text;
  for (int r = 0; r < 120000; ++r) {  // > 2 MiB: several parser ranges
    const unsigned k = rng() % 50;
    if (k == 0) {
      text += (rng() % 2) ? "\n" : "\r\n";  // blank line
      continue;
    }
    char buf[128];
    if (k == 1) std::snprintf(buf, sizeof buf, "%s,%d,%s", odd_f[rng() % 9], static_cast<int>(rng() % 1000) - 500,
                              odd_f[rng() % 9]);
    else std::snprintf(buf, sizeof buf, "%.9g,%d,%.17g", (rng() % 100000) / 7.0, static_cast<int>(rng() % 2000001) - 1000000,
                       (rng() % 1000000) / 3.0);
    text += buf;
    text += (rng() % 5) ? "\n" : "\r\n";
  }
  std::vector<float> rf;
  std::vector<int32_t> ri;
  std::vector<double> rd;
  CHECK(sequential(text, rf, ri, rd));
  for (int threads : {1, 3, 8}) {
    HostTable t = empty_table();
    warpdb::parse_csv_rows(text.data(), text.data() + text.size(), t, threads);
    const auto &f = std::get<std::vector<float>>(t.columns[0].data);
    const auto &i = std::get<std::vector<int32_t>>(t.columns[1].data);
    const auto &d = std::get<std::vector<double>>(t.columns[2].data);
    CHECK(f.size() == rf.size() && i == ri);
    bool same = f.size() == rf.size() && d.size() == rd.size();
    for (size_t r = 0; same && r < f.size(); ++r)
      same = (std::memcmp(&f[r], &rf[r], 4) == 0 || (std::isnan(f[r]) && std::isnan(rf[r]))) &&
             (std::memcmp(&d[r], &rd[r], 8) == 0 || (std::isnan(d[r]) && std::isnan(rd[r])));
    CHECK(same);
  }
  // an unparsable cell is an error (the sequential loader's message), and the
  // table is left as it was
  const std::string bad = text + "1.5,abc,2\n";
  HostTable t = empty_table();
  bool threw = false;
  try {
    warpdb::parse_csv_rows(bad.data(), bad.data() + bad.size(), t, 4);
  } catch (const std::runtime_error &e) {
    threw = std::string(e.what()).find("Invalid numeric value in CSV: 'abc'") != std::string::npos;
  }
  CHECK(threw && t.num_rows() == 0);
  // missing cells and an empty text
  const std::string short_row = "1.5,2\n";
  threw = false;
  try {
    warpdb::parse_csv_rows(short_row.data(), short_row.data() + short_row.size(), t, 2);
  } catch (const std::runtime_error &) {
    threw = true;
  }
  CHECK(threw);
  warpdb::parse_csv_rows(short_row.data(), short_row.data(), t, 2);
  CHECK(t.num_rows() == 0);
}

int main() {
  fuzz_front_end();
  fuzz_csv();
  if (failures) return 1;
  std::printf("sanitize_test: all passed\n");
  return 0;
}
