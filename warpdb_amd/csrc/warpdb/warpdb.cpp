// warpdb.cpp -- the WarpDB facade on the MI355X execution layer.
// Reference: src/warpdb.cpp:159-590.  query() keeps the reference's result
// contract (dense vector of num_rows floats); the work runs through the C
// ABI (include/warpexec.h) on the table resident in HBM.
#include "warpdb/warpdb.hpp"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdlib>
#include <cctype>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <exception>
#include <fstream>
#include <functional>
#include <map>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <thread>
#include <unordered_set>

#include "warpdb/internal.hpp"
#include "warpdb/multi_gpu_utils.hpp"

using warpdb::DeviceBuffer;
using warpdb::DevGuard;
using warpdb::hip_ok;
using warpdb::sync_launch;
using warpdb::throw_on;
using warpdb::WxTableView;

namespace {

// Every column reference must name a table column (src/warpdb.cpp:19-44).
void validate_ast(const ASTNode *node, const std::unordered_set<std::string> &cols) {
  if (!node) return;
  if (auto v = dynamic_cast<const VariableNode *>(node)) {
    if (!cols.count(v->name)) throw std::runtime_error("Unknown column: " + v->name);
  } else if (auto b = dynamic_cast<const BinaryOpNode *>(node)) {
    validate_ast(b->left.get(), cols);
    validate_ast(b->right.get(), cols);
  } else if (auto f = dynamic_cast<const FunctionCallNode *>(node)) {
    for (const auto &a : f->args) validate_ast(a.get(), cols);
  } else if (auto a = dynamic_cast<const AggregationNode *>(node)) {
    validate_ast(a->expr.get(), cols);
  } else if (auto w = dynamic_cast<const WindowFunctionNode *>(node)) {
    validate_ast(w->expr.get(), cols);
    for (const auto &p : w->partition_by) validate_ast(p.get(), cols);
    if (w->order_by) validate_ast(w->order_by->expr.get(), cols);
  }
}

std::unordered_set<std::string> names_of(const Table &t) {
  std::unordered_set<std::string> s;
  for (const auto &c : t.columns) s.insert(c.name);
  return s;
}

std::unordered_set<std::string> names_of(const HostTable &t) {
  std::unordered_set<std::string> s;
  for (const auto &c : t.columns) s.insert(c.name);
  return s;
}

bool blank(const std::string &s) {
  return std::all_of(s.begin(), s.end(), [](char c) { return std::isspace(static_cast<unsigned char>(c)); });
}

// split + parse + validate + lower, with the reference's error prefixes
void lower_query(const std::string &query, const std::unordered_set<std::string> &cols, std::string &expr_c,
                 std::string &cond_c) {
  if (query.empty()) throw std::runtime_error("Empty query expression");
  std::string e, c;
  warpdb::split_where(query, e, c);
  ASTNodePtr ex;
  try {
    ex = parse_expression(tokenize(e));
  } catch (const std::exception &err) {
    throw std::runtime_error(std::string("Failed to parse expression: ") + err.what());
  }
  validate_ast(ex.get(), cols);
  expr_c = ex->to_cuda_expr();
  cond_c.clear();
  if (!blank(c)) {
    try {
      auto cx = parse_expression(tokenize(c));
      validate_ast(cx.get(), cols);
      cond_c = cx->to_cuda_expr();
    } catch (const std::exception &err) {
      throw std::runtime_error(std::string("Failed to parse WHERE clause: ") + err.what());
    }
  }
}

std::string lower_ext(const std::string &path) {
  const auto dot = path.find_last_of('.');
  std::string ext = dot == std::string::npos ? "" : path.substr(dot + 1);
  for (char &ch : ext) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
  return ext;
}

std::vector<float> download(const void *d, int64_t n, int device) {
  std::vector<float> h = warpdb::host_result(static_cast<size_t>(n));
  DevGuard g(device);
  if (n) warpdb::copy_d2h(device, nullptr, h.data(), d, sizeof(float) * static_cast<size_t>(n));
  return h;
}

bool same_expr(const ASTNode *a, const ASTNode *b) { return a && b && a->to_cuda_expr() == b->to_cuda_expr(); }

}  // namespace

WarpDB::WarpDB(const std::string &filepath, const std::vector<DataType> &schema, int device) {
  const std::string ext = lower_ext(filepath);
  if (ext == "csv") {
    host_table_ = load_csv_to_host(filepath, schema);
  } else if (ext == "json") {
    host_table_ = load_json_to_host(filepath);
  } else if (ext == "parquet" || ext == "arrow" || ext == "feather" || ext == "orc") {
    throw std::runtime_error("Arrow support is not compiled into WarpDB");
  } else {
    throw std::runtime_error("Unsupported file format: " + filepath);
  }
  table_ = upload_to_gpu(host_table_, device);
}

WarpDB::~WarpDB() { free_table(table_); }

void WarpDB::lower(const std::string &query, std::string &expr_c, std::string &cond_c) const {
  lower_query(query, names_of(table_), expr_c, cond_c);
}

std::vector<float> WarpDB::query(const std::string &expr) {
  std::string e, c;
  lower(expr, e, c);
  const int64_t n = table_.num_rows;
  DeviceBuffer out(table_.device, sizeof(float) * static_cast<size_t>(n ? n : 1));
  WxTableView v(table_);
  wx_launch L = sync_launch(table_.device);
  char err[8192];
  throw_on(wx_project_filter(&v.table, e.c_str(), c.c_str(), &L, WX_MODE_DENSE_FILL, static_cast<float *>(out.ptr),
                             nullptr, 0, 0, nullptr, nullptr, err, sizeof(err)),
           err);
  return download(out.ptr, n, table_.device);
}

std::pair<std::vector<float>, std::vector<int64_t>> WarpDB::query_compact(const std::string &expr) {
  std::string e, c;
  lower(expr, e, c);
  const int64_t n = table_.num_rows;
  DeviceBuffer vals(table_.device, sizeof(float) * static_cast<size_t>(n ? n : 1));
  DeviceBuffer idx(table_.device, sizeof(int64_t) * static_cast<size_t>(n ? n : 1));
  WxTableView v(table_);
  wx_launch L = sync_launch(table_.device);
  int64_t count = 0;
  char err[8192];
  throw_on(wx_project_filter(&v.table, e.c_str(), c.c_str(), &L, WX_MODE_COMPACT, static_cast<float *>(vals.ptr),
                             idx.ptr, 8, 0, nullptr, &count, err, sizeof(err)),
           err);
  std::vector<float> hv = download(vals.ptr, count, table_.device);
  std::vector<int64_t> hi(static_cast<size_t>(count));
  DevGuard g(table_.device);
  if (count) hip_ok(hipMemcpy(hi.data(), idx.ptr, sizeof(int64_t) * count, hipMemcpyDeviceToHost), "hipMemcpy");
  return {std::move(hv), std::move(hi)};
}

std::pair<double, int64_t> WarpDB::query_sum(const std::string &expr) {
  std::string e, c;
  lower(expr, e, c);
  WxTableView v(table_);
  wx_launch L = sync_launch(table_.device);
  double s = 0;
  int64_t n = 0;
  char err[8192];
  throw_on(wx_reduce_sum(&v.table, e.c_str(), c.c_str(), &L, nullptr, &s, &n, err, sizeof(err)), err);
  return {s, n};
}

void WarpDB::query_arrow(const std::string &expr, ArrowArray *out_array, ArrowSchema *out_schema,
                         bool use_shared_memory) {
  auto r = query(expr);
  export_to_arrow(r.data(), static_cast<int64_t>(r.size()), use_shared_memory, out_array, out_schema);
}

void WarpDB::query_arrow_device(const std::string &expr, ArrowDeviceArray *out_array, ArrowSchema *out_schema) {
  std::string e, c;
  lower(expr, e, c);
  const int64_t n = table_.num_rows;
  DeviceBuffer out(table_.device, sizeof(float) * static_cast<size_t>(n ? n : 1));
  WxTableView v(table_);
  wx_launch L = sync_launch(table_.device);
  char err[8192];
  throw_on(wx_project_filter(&v.table, e.c_str(), c.c_str(), &L, WX_MODE_DENSE_FILL, static_cast<float *>(out.ptr),
                             nullptr, 0, 0, nullptr, nullptr, err, sizeof(err)),
           err);
  const int dev = table_.device;
  export_device_to_arrow(static_cast<float *>(out.release()), n, dev, out_array, out_schema);
}

// The row shards of query_multi_gpu*, built on first use.  With one visible
// GPU holding table_ the shard IS table_ (borrowed, no second HBM copy).
warpdb::ResidentShards &WarpDB::shards() {
  if (host_table_.num_rows() == 0) throw std::runtime_error("Host table not available for multi-GPU query");
  // call_once: two threads' first multi-GPU calls (GIL released) build one set
  // of shards; a throwing build leaves the flag unset, so the next call retries
  std::call_once(shards_once_, [this] {
    int ndev = 0;
    hip_ok(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    if (ndev == 1 && table_.device == 0 && !std::getenv("WARPDB_VIRTUAL_SHARDS"))  // (test hook: multi_gpu.cpp)
      shards_ = warpdb::ResidentShards::borrow(table_);
    else
      shards_ = std::make_unique<warpdb::ResidentShards>(host_table_);
  });
  return *shards_;
}

void WarpDB::query_arrow_compact(const std::string &expr, ArrowArray *out_array, ArrowSchema *out_schema) {
  auto r = query_compact(expr);
  export_compact_to_arrow(r.first.data(), r.second.data(), static_cast<int64_t>(r.first.size()), out_array,
                          out_schema);
}

void WarpDB::query_arrow_device_compact(const std::string &expr, ArrowDeviceArray *out_array,
                                        ArrowSchema *out_schema) {
  std::string e, c;
  lower(expr, e, c);
  const int64_t n = table_.num_rows;
  // sized for every row passing; the array's length is the passing count
  DeviceBuffer vals(table_.device, sizeof(float) * static_cast<size_t>(n ? n : 1));
  DeviceBuffer rows(table_.device, sizeof(int64_t) * static_cast<size_t>(n ? n : 1));
  WxTableView v(table_);
  wx_launch L = sync_launch(table_.device);
  int64_t count = 0;
  char err[8192];
  throw_on(wx_project_filter(&v.table, e.c_str(), c.c_str(), &L, WX_MODE_COMPACT, static_cast<float *>(vals.ptr),
                             rows.ptr, 8, 0, nullptr, &count, err, sizeof(err)),
           err);
  const int dev = table_.device;
  export_device_compact_to_arrow(static_cast<float *>(vals.release()), static_cast<int64_t *>(rows.release()), count,
                                 dev, out_array, out_schema);
}

std::vector<float> WarpDB::query_multi_gpu(const std::string &expr) {
  std::string e, c;
  lower_query(expr, names_of(host_table_), e, c);
  return shards().dense(e, c);
}

std::pair<double, int64_t> WarpDB::query_multi_gpu_sum(const std::string &expr) {
  std::string e, c;
  lower_query(expr, names_of(host_table_), e, c);
  return shards().sum(e, c);
}

warpdb::GroupResult WarpDB::query_multi_gpu_group(const std::string &sql, int32_t key_window_lo) {
  QueryAST ast;
  try {
    ast = parse_query(tokenize(sql));
  } catch (const std::exception &e) {
    throw std::runtime_error(std::string("Failed to parse SQL: ") + e.what());
  }
  const auto cols = names_of(host_table_);
  auto *agg = ast.select_list.empty() ? nullptr : dynamic_cast<const AggregationNode *>(ast.select_list[0].get());
  if (!ast.group_by || !agg) throw std::runtime_error("query_multi_gpu_group expects SELECT <agg>(expr) ... GROUP BY key");
  if (ast.group_by->keys.size() != 1) throw std::runtime_error("GROUP BY supports one key expression");
  if (!ast.joins.empty()) throw std::runtime_error("JOIN is not supported by the execution engine");
  const std::string kind = agg->agg_kernel();
  if (kind != "sum" && kind != "count" && kind != "avg")  // the shards exchange (sum, count) only
    throw std::runtime_error("query_multi_gpu_group supports SUM / COUNT / AVG, not " + kind);
  validate_ast(agg->expr.get(), cols);
  validate_ast(ast.group_by->keys[0].get(), cols);
  std::string cond;
  if (ast.where) {
    validate_ast(ast.where->get(), cols);
    cond = (*ast.where)->to_cuda_expr();
  }
  // SUM / COUNT / AVG all derive from the (sum, count) the shards exchange
  return shards().group_sum(agg->expr->to_cuda_expr(), ast.group_by->keys[0]->to_cuda_expr(), cond, key_window_lo);
}

warpdb::TopkResult WarpDB::query_multi_gpu_topk(const std::string &sql) {
  QueryAST ast;
  try {
    ast = parse_query(tokenize(sql));
  } catch (const std::exception &e) {
    throw std::runtime_error(std::string("Failed to parse SQL: ") + e.what());
  }
  if (ast.select_list.size() != 1 || ast.group_by || ast.distinct || !ast.order_by || !ast.limit)
    throw std::runtime_error("query_multi_gpu_topk expects SELECT expr FROM t [WHERE c] ORDER BY o [DESC] LIMIT k");
  if (dynamic_cast<const AggregationNode *>(ast.select_list[0].get()))
    throw std::runtime_error("query_multi_gpu_topk takes a plain SELECT expression");
  if (!ast.joins.empty()) throw std::runtime_error("JOIN is not supported by the execution engine");
  const int64_t off = ast.offset ? ast.offset->count : 0;
  int64_t lim = ast.limit->count;
  if (off < 0 || lim < 0) throw std::runtime_error("query_multi_gpu_topk needs OFFSET, LIMIT >= 0");
  const int64_t n_rows = static_cast<int64_t>(host_table_.num_rows());
  // nothing beyond the table: LIMIT 0 or OFFSET >= rows is an empty result
  // (no head is gathered); otherwise off + lim <= rows, computed without
  // overflow, so each shard's head record holds at most the table's rows
  lim = off >= n_rows ? 0 : std::min(lim, n_rows - off);
  const auto cols = names_of(host_table_);
  validate_ast(ast.select_list[0].get(), cols);
  validate_ast(ast.order_by->expr.get(), cols);
  std::string cond;
  if (ast.where) {
    validate_ast(ast.where->get(), cols);
    cond = (*ast.where)->to_cuda_expr();
  }
  warpdb::TopkResult r;
  if (lim == 0) return r;
  r = shards().topk(ast.order_by->expr->to_cuda_expr(), cond, ast.select_list[0]->to_cuda_expr(), off + lim,
                    !ast.order_by->ascending);
  const size_t drop = std::min(r.keys.size(), static_cast<size_t>(off));  // OFFSET
  r.keys.erase(r.keys.begin(), r.keys.begin() + drop);
  r.rows.erase(r.rows.begin(), r.rows.begin() + drop);
  r.values.erase(r.values.begin(), r.values.begin() + drop);
  return r;
}

std::vector<float> WarpDB::query_multi_gpu_csv(const std::string &csv_path, const std::string &expr,
                                               int rows_per_chunk) {
  if (rows_per_chunk <= 0) throw std::runtime_error("rows_per_chunk must be positive");
  std::ifstream file(csv_path);
  if (!file.is_open()) throw std::runtime_error("Failed to open file: " + csv_path);
  std::string header;
  if (!std::getline(file, header)) throw std::runtime_error("Empty CSV file");
  if (!header.empty() && header.back() == '\r') header.pop_back();
  std::vector<std::string> names;
  {
    std::stringstream ss(header);
    std::string n;
    while (std::getline(ss, n, ',')) names.push_back(n);
  }
  std::unordered_set<std::string> cols(names.begin(), names.end());
  std::string e, c;
  lower_query(expr, cols, e, c);
  // Two-stage pipeline: a parser thread reads chunk i+1 while the GPUs run
  // chunk i (the reference parses, uploads and runs each chunk in turn,
  // src/warpdb.cpp:544-590).  At most two parsed chunks wait in the queue.
  std::mutex mu;
  std::condition_variable cv;
  std::deque<HostTable> ready;
  bool done = false;
  std::exception_ptr parse_err;
  // The parser reads the file in large blocks and cuts each chunk after its
  // rows_per_chunk-th non-empty line with memchr (line-by-line std::getline
  // capped the whole pipeline at ≈29-41 M rows/s); the chunk's rows are
  // parsed on parse_threads() threads.  Rows keep the default Float32 schema
  // of the reference's chunk loader (src/csv_loader.cpp:186-223).
  std::thread parser([&] {
    try {
      const size_t block = size_t(64) << 20;
      std::string buf;
      size_t start = 0;
      bool eof = false;
      while (true) {
        // position just past the rows_per_chunk-th non-empty line of buf[start..)
        size_t pos = start, cut = std::string::npos;
        int64_t rows = 0;
        while (true) {
          const char *b = buf.data();
          while (rows < rows_per_chunk && pos < buf.size()) {
            const char *nl = static_cast<const char *>(std::memchr(b + pos, '\n', buf.size() - pos));
            if (!nl) break;
            const size_t len = static_cast<size_t>(nl - (b + pos));
            if (len > 1 || (len == 1 && b[pos] != '\r')) ++rows;
            pos = static_cast<size_t>(nl - b) + 1;
          }
          if (rows == rows_per_chunk) {
            cut = pos;
            break;
          }
          if (eof) {
            cut = buf.size();  // the rest, a last line without '\n' included
            break;
          }
          buf.erase(0, start);  // keep only the unconsumed text, then read on
          pos -= start;
          start = 0;
          const size_t old = buf.size();
          buf.resize(old + block);
          file.read(&buf[old], static_cast<std::streamsize>(block));
          buf.resize(old + static_cast<size_t>(file.gcount()));
          eof = !file;
        }
        HostTable chunk;
        for (const auto &nm : names) chunk.columns.push_back({nm, DataType::Float32, std::vector<float>()});
        warpdb::parse_csv_rows(buf.data() + start, buf.data() + cut, chunk, warpdb::parse_threads());
        start = cut;
        const bool last = eof && start >= buf.size();
        if (chunk.num_rows() > 0) {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return ready.size() < 2 || done; });
          if (done) break;  // consumer gave up
          ready.push_back(std::move(chunk));
          cv.notify_all();
        }
        if (last) break;
      }
    } catch (...) {
      std::lock_guard<std::mutex> lk(mu);
      parse_err = std::current_exception();
    }
    std::lock_guard<std::mutex> lk(mu);
    done = true;
    cv.notify_all();
  });
  std::vector<float> all;
  try {
    while (true) {
      HostTable chunk;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !ready.empty() || done; });
        if (ready.empty()) break;
        chunk = std::move(ready.front());
        ready.pop_front();
        cv.notify_all();
      }
      auto part = run_multi_gpu_jit_host(chunk, e, c);
      all.insert(all.end(), part.begin(), part.end());
    }
  } catch (...) {
    {
      std::lock_guard<std::mutex> lk(mu);
      done = true;
      cv.notify_all();
    }
    parser.join();
    throw;
  }
  parser.join();
  if (parse_err) std::rethrow_exception(parse_err);
  return all;
}

// ------------------------------------------------------------------ SQL
namespace {
bool uses_minmax(const ASTNode *n) {
  if (!n) return false;
  if (auto a = dynamic_cast<const AggregationNode *>(n))
    return a->agg == AggregationType::Min || a->agg == AggregationType::Max;
  if (auto b = dynamic_cast<const BinaryOpNode *>(n)) return uses_minmax(b->left.get()) || uses_minmax(b->right.get());
  return false;
}
}  // namespace

std::vector<float> WarpDB::query_sql(const std::string &sql) {
  QueryAST ast;
  try {
    ast = parse_query(tokenize(sql));
  } catch (const std::exception &e) {
    throw std::runtime_error(std::string("Failed to parse SQL: ") + e.what());
  }
  const auto cols = names_of(table_);
  auto validate_ctx = [&](const ASTNode *n, const std::string &ctx) {
    try {
      validate_ast(n, cols);
    } catch (const std::exception &e) {
      throw std::runtime_error(ctx + ": " + e.what());
    }
  };
  if (ast.select_list.empty()) throw std::runtime_error("Empty SELECT list");
  for (const auto &e : ast.select_list) validate_ctx(e.get(), "SELECT clause");
  for (const auto &j : ast.joins) validate_ctx(j.condition.get(), "JOIN condition");
  if (ast.where) validate_ctx(ast.where->get(), "WHERE clause");
  if (ast.group_by)
    for (const auto &k : ast.group_by->keys) validate_ctx(k.get(), "GROUP BY");
  if (ast.order_by) validate_ctx(ast.order_by->expr.get(), "ORDER BY");
  if (!ast.joins.empty()) throw std::runtime_error("JOIN is not supported by the execution engine");

  const std::string cond = ast.where ? (*ast.where)->to_cuda_expr() : std::string();
  WxTableView v(table_);
  wx_launch L = sync_launch(table_.device);
  char err[8192];
  std::vector<float> result;
  const size_t off = ast.offset ? static_cast<size_t>(std::max(0, ast.offset->count)) : 0;
  const size_t lim = ast.limit ? static_cast<size_t>(std::max(0, ast.limit->count)) : SIZE_MAX;
  auto slice = [&](std::vector<float> r) {
    if (off >= r.size()) return std::vector<float>();
    r.erase(r.begin(), r.begin() + static_cast<long>(off));
    if (r.size() > lim) r.resize(lim);
    return r;
  };
  auto *agg = dynamic_cast<const AggregationNode *>(ast.select_list[0].get());

  if (ast.group_by) {
    if (!agg) throw std::runtime_error("Only aggregation queries supported with GROUP BY");
    if (ast.group_by->keys.size() != 1) throw std::runtime_error("GROUP BY supports one key expression");
    const ASTNode *key = ast.group_by->keys[0].get();
    const int64_t cap = std::max<int64_t>(1, std::min<int64_t>(table_.num_rows, 1 << 22));
    // MIN / MAX anywhere (SELECT, HAVING, ORDER BY) selects the MIN / MAX build
    const bool mm = uses_minmax(agg) || (ast.having && uses_minmax(ast.having->get())) ||
                    (ast.order_by && uses_minmax(ast.order_by->expr.get()));
    DeviceBuffer dk(table_.device, cap * 4), ds(table_.device, cap * 8), dc(table_.device, cap * 8);
    DeviceBuffer dmn(table_.device, mm ? cap * 4 : 4), dmx(table_.device, mm ? cap * 4 : 4);
    int64_t g = 0;
    // WARPDB_GROUP_ROW_ORDER=1: each group's sum folded in row order, the
    // reference's own fold (src/warpdb.cpp:373-385) to the bit (WX_F_ROW_ORDER)
    const char *ro = std::getenv("WARPDB_GROUP_ROW_ORDER");
    if (ro && std::string(ro) == "1") L.flags |= WX_F_ROW_ORDER;
    throw_on(wx_group_agg(&v.table, agg->expr->to_cuda_expr().c_str(), key->to_cuda_expr().c_str(), cond.c_str(), &L,
                          0, cap, static_cast<int32_t *>(dk.ptr), static_cast<double *>(ds.ptr),
                          static_cast<int64_t *>(dc.ptr), mm ? static_cast<float *>(dmn.ptr) : nullptr,
                          mm ? static_cast<float *>(dmx.ptr) : nullptr, nullptr, &g, err, sizeof(err)),
             err);
    std::vector<int32_t> keys(g);
    std::vector<double> sums(g);
    std::vector<int64_t> cnts(g);
    std::vector<float> mins(mm ? g : 0), maxs(mm ? g : 0);
    {
      DevGuard dg(table_.device);
      if (g) {
        hip_ok(hipMemcpy(keys.data(), dk.ptr, g * 4, hipMemcpyDeviceToHost), "hipMemcpy");
        hip_ok(hipMemcpy(sums.data(), ds.ptr, g * 8, hipMemcpyDeviceToHost), "hipMemcpy");
        hip_ok(hipMemcpy(cnts.data(), dc.ptr, g * 8, hipMemcpyDeviceToHost), "hipMemcpy");
        if (mm) {
          hip_ok(hipMemcpy(mins.data(), dmn.ptr, g * 4, hipMemcpyDeviceToHost), "hipMemcpy");
          hip_ok(hipMemcpy(maxs.data(), dmx.ptr, g * 4, hipMemcpyDeviceToHost), "hipMemcpy");
        }
      }
    }
    // per-group aggregate value (AggData, src/warpdb.cpp:375-385)
    auto value_of = [&](AggregationType t, size_t i) -> double {
      switch (t) {
        case AggregationType::Sum: return sums[i];
        case AggregationType::Avg: return sums[i] / static_cast<double>(cnts[i]);
        case AggregationType::Count: return static_cast<double>(cnts[i]);
        case AggregationType::Min: return mins[i];
        case AggregationType::Max: return maxs[i];
      }
      return NAN;
    };
    // HAVING over the (few) aggregated groups, with the reference's
    // comparison semantics (src/warpdb.cpp:387-423)
    std::function<double(const ASTNode *, size_t)> having = [&](const ASTNode *n, size_t i) -> double {
      if (auto c = dynamic_cast<const ConstantNode *>(n)) return std::stod(c->value);
      if (auto a = dynamic_cast<const AggregationNode *>(n)) {
        if (!same_expr(a->expr.get(), agg->expr.get()) && a->agg != AggregationType::Count)
          throw std::runtime_error("HAVING may only aggregate the selected expression");
        return value_of(a->agg, i);
      }
      if (auto b = dynamic_cast<const BinaryOpNode *>(n)) {
        const double l = having(b->left.get(), i), r = having(b->right.get(), i);
        const std::string &op = b->op;
        if (op == "+") return l + r;
        if (op == "-") return l - r;
        if (op == "*") return l * r;
        if (op == "/") return l / r;
        if (op == ">") return l > r;
        if (op == "<") return l < r;
        if (op == ">=") return l >= r;
        if (op == "<=") return l <= r;
        if (op == "==") return l == r;
        if (op == "!=") return l != r;
        if (op == "&&") return l != 0 && r != 0;
        if (op == "||") return l != 0 || r != 0;
      }
      if (same_expr(n, key)) return keys[i];
      throw std::runtime_error("unsupported HAVING term");
    };
    std::vector<size_t> order;
    for (size_t i = 0; i < static_cast<size_t>(g); ++i)
      if (!ast.having || having(ast.having->get(), i) != 0.0) order.push_back(i);
    if (ast.order_by) {  // groups arrive in ascending key order
      const ASTNode *ob = ast.order_by->expr.get();
      auto *oagg = dynamic_cast<const AggregationNode *>(ob);
      if (oagg) {
        std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
          const double x = value_of(oagg->agg, a), y = value_of(oagg->agg, b);
          return ast.order_by->ascending ? x < y : x > y;
        });
      } else if (same_expr(ob, key)) {
        if (!ast.order_by->ascending) std::reverse(order.begin(), order.end());
      } else {
        throw std::runtime_error("ORDER BY with GROUP BY must name the key or an aggregate");
      }
    }
    for (size_t i : order) result.push_back(static_cast<float>(value_of(agg->agg, i)));
    if (ast.distinct) {
      std::sort(result.begin(), result.end());
      result.erase(std::unique(result.begin(), result.end()), result.end());
    }
    return slice(std::move(result));
  }

  if (agg) {  // ungrouped aggregate over the WHERE rows
    wx_stats st{};
    if (uses_minmax(agg)) {
      throw_on(wx_reduce_stats(&v.table, agg->expr->to_cuda_expr().c_str(), cond.c_str(), &L, nullptr, &st, err,
                               sizeof(err)),
               err);
    } else {
      throw_on(wx_reduce_sum(&v.table, agg->expr->to_cuda_expr().c_str(), cond.c_str(), &L, nullptr, &st.sum,
                             &st.count, err, sizeof(err)),
               err);
    }
    double val = NAN;
    switch (agg->agg) {
      case AggregationType::Sum: val = st.sum; break;
      case AggregationType::Avg: val = st.count ? st.sum / static_cast<double>(st.count) : NAN; break;
      case AggregationType::Count: val = static_cast<double>(st.count); break;
      case AggregationType::Min: val = st.min; break;
      case AggregationType::Max: val = st.max; break;
    }
    return slice({static_cast<float>(val)});
  }

  const ASTNode *sel = ast.select_list[0].get();
  const std::string sel_c = sel->to_cuda_expr();
  const ASTNode *ob = ast.order_by ? ast.order_by->expr.get() : nullptr;
  // ORDER BY .. LIMIT k: device top-K (ties by ascending row index)
  if (ob && !ast.distinct && ast.limit && off + lim <= 32) {
    const int k = static_cast<int>(off + lim);
    if (k == 0) return {};
    DeviceBuffer dv(table_.device, sizeof(float) * k);
    int64_t m = 0;
    throw_on(wx_topk(&v.table, ob->to_cuda_expr().c_str(), cond.c_str(), sel_c.c_str(), k,
                     ast.order_by->ascending ? 0 : 1, &L, 0, nullptr, nullptr, static_cast<float *>(dv.ptr), nullptr,
                     &m, err, sizeof(err)),
             err);
    return slice(download(dv.ptr, m, table_.device));
  }
  const int64_t n = table_.num_rows;
  DeviceBuffer dv(table_.device, sizeof(float) * static_cast<size_t>(n ? n : 1));
  // ORDER BY a bare float column, no WHERE, no LIMIT: the projection would be
  // a copy of the column, so the sort reads the column itself
  // (src/warpdb.cpp:450-455 projects, then jit_sort_float sorts the copy)
  if (ob && !ast.distinct && !ast.limit && cond.empty() && same_expr(ob, sel)) {
    if (auto var = dynamic_cast<const VariableNode *>(sel)) {
      for (const auto &c : table_.columns) {
        if (c.name != var->name || c.type != DataType::Float32) continue;
        throw_on(wx_sort_float_from(static_cast<const float *>(c.device_ptr), static_cast<float *>(dv.ptr), n,
                                    ast.order_by->ascending ? 1 : 0, &L, err, sizeof(err)),
                 err);
        return slice(download(dv.ptr, n, table_.device));
      }
    }
  }
  // projection of the WHERE rows in row order (ordered compaction)
  int64_t count = 0;
  throw_on(wx_project_filter(&v.table, sel_c.c_str(), cond.c_str(), &L, WX_MODE_COMPACT, static_cast<float *>(dv.ptr),
                             nullptr, 0, 0, nullptr, &count, err, sizeof(err)),
           err);
  if (ob && !same_expr(ob, sel)) {
    // ORDER BY another expression: its values at the same rows (same WHERE,
    // same ascending row order) are the keys of a keyed sort that carries the
    // SELECT values along (the pairs the reference builds, src/warpdb.cpp:470-476)
    if (ast.distinct) throw std::runtime_error("DISTINCT with ORDER BY a different expression is not supported");
    DeviceBuffer dk(table_.device, sizeof(float) * static_cast<size_t>(n ? n : 1));
    int64_t kcount = 0;
    throw_on(wx_project_filter(&v.table, ob->to_cuda_expr().c_str(), cond.c_str(), &L, WX_MODE_COMPACT,
                               static_cast<float *>(dk.ptr), nullptr, 0, 0, nullptr, &kcount, err, sizeof(err)),
             err);
    if (kcount != count) throw std::runtime_error("ORDER BY rows differ from SELECT rows");
    // with a LIMIT only the first OFFSET + LIMIT rows of the order are needed
    throw_on(wx_sort_by_key_limit(static_cast<float *>(dk.ptr), static_cast<float *>(dv.ptr), count,
                                  ast.limit ? std::min<int64_t>(count, off + lim) : count,
                                  ast.order_by->ascending ? 1 : 0, &L, err, sizeof(err)),
             err);
    if (ast.limit) count = std::min<int64_t>(count, off + lim);
  } else if (ob || ast.distinct) {
    const bool asc = ob ? ast.order_by->ascending : true;
    const bool head_only = ob && !ast.distinct && ast.limit;  // DISTINCT needs every value
    throw_on(wx_sort_float_limit(static_cast<float *>(dv.ptr), count,
                                 head_only ? std::min<int64_t>(count, off + lim) : count, asc ? 1 : 0, &L, err,
                                 sizeof(err)),
             err);
    if (head_only) count = std::min<int64_t>(count, off + lim);
  }
  result = download(dv.ptr, count, table_.device);
  if (ast.distinct) result.erase(std::unique(result.begin(), result.end()), result.end());
  return slice(std::move(result));
}
