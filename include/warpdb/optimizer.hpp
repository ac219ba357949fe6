// optimizer.hpp -- statistics pushdown for the projection path (drop-in for
// the reference's include/optimizer.hpp).
//
// The reference declares execute_query_optimized() and an analyze_condition()
// that never decides anything (src/optimizer.cpp:13-17).  Here the WHERE
// clause is checked against per-column ranges computed on the GPU
// (wx_reduce_stats): a filter that no row can pass skips the launch, and one
// that every row passes is dropped from the kernel.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "csv_loader.hpp"
#include "expression.hpp"

// Reference entry point (include/optimizer.hpp:7-8): parse, analyse, run the
// projection and print "Result[i] = v" per row, or
// "[Optimizer] Filter eliminates all rows." when the filter is always false.
void execute_query_optimized(const std::string &expr_part, const std::string &where_part, Table &table);

// The reference's two-column form (price / quantity members of TableStats).
void analyze_condition(const ASTNode *cond, const TableStats &stats, bool &always_true, bool &always_false);

namespace warpdb {

// Range of one column as the kernels see it: values converted to float
// (the lowered expressions compare in float).  min/max exclude NaN;
// null_count counts NaN rows.  `known` is false for columns the analysis
// cannot bound (Float64, String) or that hold no non-NaN value.
struct ColumnRange {
  bool known = false;
  bool is_int = false;
  double min = 0.0, max = 0.0;
  int64_t null_count = 0;
};
using StatsMap = std::map<std::string, ColumnRange>;

// One wx_reduce_stats pass per requested column (all columns when `names` is
// empty), plus one NaN count for float columns.
StatsMap compute_column_stats(const Table &table, const std::vector<std::string> &names = {});
TableStats to_table_stats(const StatsMap &stats);

enum class Verdict { Unknown = 0, AlwaysTrue = 1, AlwaysFalse = 2 };
Verdict analyze_condition(const ASTNode *cond, const StatsMap &stats);
const char *verdict_name(Verdict v);

// Column names an expression references.
std::vector<std::string> referenced_columns(const ASTNode *n);

// The optimised projection: dense results (0.0f where the filter fails, as
// WarpDB::query), with the verdict that was applied.  `stats` may be cached
// by the caller; when null, the WHERE columns' ranges are computed here.
std::vector<float> query_optimized(const std::string &expr_part, const std::string &where_part, const Table &table,
                                   const StatsMap *stats = nullptr, Verdict *verdict_out = nullptr);

}  // namespace warpdb
