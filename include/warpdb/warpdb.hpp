// warpdb.hpp -- the WarpDB facade (drop-in for the reference's
// include/warpdb.hpp:11-48) running on the MI355X execution layer.
#pragma once
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "arrow_utils.hpp"
#include "csv_loader.hpp"
#include "expression.hpp"
#include "jit.hpp"
#include "json_loader.hpp"
#include "multi_gpu_utils.hpp"

class WarpDB {
 public:
  // Loads .csv (optional schema; default all Float32) or .json into HBM of
  // `device` and keeps the host copy for query_multi_gpu.
  explicit WarpDB(const std::string &filepath, const std::vector<DataType> &schema = {}, int device = 0);
  ~WarpDB();
  WarpDB(const WarpDB &) = delete;
  WarpDB &operator=(const WarpDB &) = delete;

  // "expr [WHERE cond]": dense vector of num_rows floats in row order; rows
  // where cond is false are 0.0f (the reference leaves them uninitialised).
  std::vector<float> query(const std::string &expr);

  // SELECT ... [WHERE] [GROUP BY k [HAVING]] [ORDER BY [ASC|DESC]] [LIMIT] [OFFSET]
  // with SUM/AVG/COUNT aggregates, DISTINCT, ORDER BY .. LIMIT (top-K).
  std::vector<float> query_sql(const std::string &sql);

  // Every visible GPU, rows sharded; same result contract as query().
  std::vector<float> query_multi_gpu(const std::string &expr);

  // Stream a CSV file in chunks of rows_per_chunk through query_multi_gpu.
  static std::vector<float> query_multi_gpu_csv(const std::string &csv_path, const std::string &expr,
                                                int rows_per_chunk = 1000000);

  // query() exported as an Arrow float32 array (malloc or POSIX shm).
  void query_arrow(const std::string &expr, ArrowArray *out_array, ArrowSchema *out_schema,
                   bool use_shared_memory = false);

  // --- extensions on the same execution path -------------------------------
  // Ordered compaction: values and ascending row indices of passing rows.
  std::pair<std::vector<float>, std::vector<int64_t>> query_compact(const std::string &expr);
  // SUM(expr) WHERE cond on the device, and its row count.
  std::pair<double, int64_t> query_sum(const std::string &expr);
  // SUM(expr) WHERE cond over every GPU with an RCCL all-reduce.
  std::pair<double, int64_t> query_multi_gpu_sum(const std::string &expr);
  // "SELECT SUM(v) FROM t [WHERE c] GROUP BY k" over every GPU: per-GPU dense
  // key-window partials and per-GPU slots of keys outside [key_window_lo,
  // key_window_lo + 2048) combined by ONE RCCL all-reduce (more than 64 such
  // keys on a GPU: merged on the host).  Groups in ascending key order with
  // double sums and counts: SUM / COUNT / AVG (MIN / MAX are refused).
  warpdb::GroupResult query_multi_gpu_group(const std::string &sql, int32_t key_window_lo = 0);
  // "SELECT e FROM t [WHERE c] ORDER BY o [ASC|DESC] LIMIT k [OFFSET n]" over
  // every GPU: per GPU its best OFFSET + LIMIT rows (top-K candidates up to 32,
  // beyond that the sorted head), one RCCL all-gather, the (key, row) merge on
  // the device.  The winning ORDER BY keys, global row numbers and SELECT
  // values, best first.
  warpdb::TopkResult query_multi_gpu_topk(const std::string &sql);
  // Zero-copy result: dense device buffer as an ArrowDeviceArray (ROCm).
  void query_arrow_device(const std::string &expr, ArrowDeviceArray *out_array, ArrowSchema *out_schema);
  // The compacted result (passing rows only) as struct<value: float32, row: int64>:
  // host copy, and zero-copy in HBM (ARROW_DEVICE_ROCM; buffers sized for n_rows).
  void query_arrow_compact(const std::string &expr, ArrowArray *out_array, ArrowSchema *out_schema);
  void query_arrow_device_compact(const std::string &expr, ArrowDeviceArray *out_array, ArrowSchema *out_schema);

  const Table &table() const { return table_; }
  const HostTable &host_table() const { return host_table_; }

 private:
  void lower(const std::string &query, std::string &expr_c, std::string &cond_c) const;
  warpdb::ResidentShards &shards();
  Table table_;
  HostTable host_table_;
  std::unique_ptr<warpdb::ResidentShards> shards_;  // query_multi_gpu*: built on first use
  std::once_flag shards_once_;                      // the bindings release the GIL: one builder
};
