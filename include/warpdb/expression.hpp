// expression.hpp -- WarpDB query front end (drop-in for the reference's
// include/expression.hpp): tokens, AST node types, the CUDA-C lowering
// (to_cuda_expr) and the SQL query AST.
//
// Same public names, members and error messages as the reference, so code
// that inspects the AST (dynamic_cast<const VariableNode*> etc.) compiles
// unchanged.  Differences, all documented in DESIGN.md:
//   * the parser keeps its state on the stack (the reference uses globals,
//     src/expression.cpp:123-124), so it is reentrant;
//   * a single '=' is parsed as equality '==' (the reference lowers it to a
//     C assignment, src/expression.cpp:159);
//   * parse_query accepts LIMIT and OFFSET in either order (the reference's
//     OFFSET block is unterminated, src/expression.cpp:515-531).
#pragma once
#include <memory>
#include <optional>
#include <string>
#include <vector>

enum class TokenType { Identifier, Number, Operator, Keyword, End };

struct Token {
  TokenType type;
  std::string value;
  int line = 1;
  int column = 1;
};

// Lexer: identifiers may contain '.', numbers have no exponent, keywords are
// upper-cased (reference src/expression.cpp:22-120).
std::vector<Token> tokenize(const std::string &input);

enum class ASTNodeType { Constant, Variable, BinaryOp, FunctionCall, Aggregation };

struct ASTNode {
  virtual ~ASTNode() {}
  // Lowered C expression over `<column>[idx]` (include/expression.hpp:32-78).
  virtual std::string to_cuda_expr() const = 0;
  virtual ASTNodeType type() const = 0;
};

using ASTNodePtr = std::unique_ptr<ASTNode>;

struct ConstantNode : public ASTNode {
  std::string value;
  explicit ConstantNode(const std::string &val) : value(val) {}
  std::string to_cuda_expr() const override;
  ASTNodeType type() const override { return ASTNodeType::Constant; }
};

struct VariableNode : public ASTNode {
  std::string name;
  explicit VariableNode(const std::string &n) : name(n) {}
  std::string to_cuda_expr() const override;
  ASTNodeType type() const override { return ASTNodeType::Variable; }
};

struct BinaryOpNode : public ASTNode {
  std::string op;
  ASTNodePtr left;
  ASTNodePtr right;
  BinaryOpNode(std::string o, ASTNodePtr l, ASTNodePtr r)
      : op(std::move(o)), left(std::move(l)), right(std::move(r)) {}
  std::string to_cuda_expr() const override;
  ASTNodeType type() const override { return ASTNodeType::BinaryOp; }
};

struct FunctionCallNode : public ASTNode {
  std::string name;
  std::vector<ASTNodePtr> args;
  FunctionCallNode(std::string n, std::vector<ASTNodePtr> a) : name(std::move(n)), args(std::move(a)) {}
  std::string to_cuda_expr() const override;
  ASTNodeType type() const override { return ASTNodeType::FunctionCall; }
};

// Expression parsers.  Precedence (low to high): OR, AND, comparison,
// + -, * /, factor.  parse_expression parses a full expression and requires
// the End token afterwards.
ASTNodePtr parse_expression(const std::vector<Token> &tokens);
ASTNodePtr parse_logical_and(const std::vector<Token> &tokens);
ASTNodePtr parse_logical_or(const std::vector<Token> &tokens);

enum class AggregationType { Sum, Avg, Count, Min, Max };

struct AggregationNode : public ASTNode {
  AggregationType agg;
  ASTNodePtr expr;
  AggregationNode(AggregationType a, ASTNodePtr e) : agg(a), expr(std::move(e)) {}
  std::string to_cuda_expr() const override { return expr->to_cuda_expr(); }
  ASTNodeType type() const override { return ASTNodeType::Aggregation; }
  std::string agg_kernel() const;  // "sum", "avg", "count", "min", "max"
};

struct OrderByClause {
  ASTNodePtr expr;
  bool ascending;
};

struct LimitClause {
  int count;
};

struct OffsetClause {
  int count;
};

struct WindowFunctionNode : public ASTNode {
  AggregationType agg;
  ASTNodePtr expr;
  std::vector<ASTNodePtr> partition_by;
  std::optional<OrderByClause> order_by;
  WindowFunctionNode(AggregationType a, ASTNodePtr e) : agg(a), expr(std::move(e)) {}
  std::string to_cuda_expr() const override { return "<window>"; }
  ASTNodeType type() const override { return ASTNodeType::Aggregation; }
};

struct JoinClause {
  std::string table;
  ASTNodePtr condition;
};

struct GroupByClause {
  std::vector<ASTNodePtr> keys;
};

struct QueryAST {
  std::vector<ASTNodePtr> select_list;
  std::string from_table;
  std::vector<JoinClause> joins;
  std::optional<ASTNodePtr> where;
  std::optional<GroupByClause> group_by;
  std::optional<ASTNodePtr> having;
  std::optional<OrderByClause> order_by;
  std::optional<LimitClause> limit;
  std::optional<OffsetClause> offset;
  bool distinct = false;
};

QueryAST parse_query(const std::vector<Token> &tokens);

namespace warpdb {
// Split "expr WHERE cond" at the first case-insensitive "WHERE"
// (reference src/warpdb.cpp:204-213).  cond is empty when there is none.
void split_where(const std::string &query, std::string &expr, std::string &cond);
}  // namespace warpdb
