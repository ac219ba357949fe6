// frontend_test.cpp -- C++ API checks of the front end through the public
// headers (include/warpdb), covering the expectations of the reference's
// test_expression / precedence / expression / tokenizer / parsing-error /
// parse_query / identifier-validation tests.  No GPU needed.
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <unordered_set>

#include "warpdb/expression.hpp"

static int failures = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::printf("FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);   \
      ++failures;                                                  \
    }                                                              \
  } while (0)

static std::string lower(const std::string &s) { return parse_expression(tokenize(s))->to_cuda_expr(); }

template <typename F>
static std::string error_of(F &&f) {
  try {
    f();
  } catch (const std::runtime_error &e) {
    return e.what();
  }
  return "<no error>";
}

static void walk(const ASTNode *n, const std::unordered_set<std::string> &cols) {
  if (auto v = dynamic_cast<const VariableNode *>(n)) {
    if (!cols.count(v->name)) throw std::runtime_error("Unknown column: " + v->name);
  } else if (auto b = dynamic_cast<const BinaryOpNode *>(n)) {
    walk(b->left.get(), cols);
    walk(b->right.get(), cols);
  } else if (auto a = dynamic_cast<const AggregationNode *>(n)) {
    walk(a->expr.get(), cols);
  }
}

int main() {
  CHECK(lower("price > 10") == "(price[idx] > 10.0f)");
  CHECK(lower("quantity <= 5") == "(quantity[idx] <= 5.0f)");
  CHECK(lower("discount(price, 0.9)") == "discount(price[idx], 0.9f)");
  CHECK(lower("price > 10 AND quantity < 5") == "((price[idx] > 10.0f) && (quantity[idx] < 5.0f))");
  CHECK(lower("price > 10 OR quantity < 5") == "((price[idx] > 10.0f) || (quantity[idx] < 5.0f))");
  CHECK(lower("price + quantity * 2") == "(price[idx] + (quantity[idx] * 2.0f))");
  CHECK(lower("(price + quantity) * 2") == "((price[idx] + quantity[idx]) * 2.0f)");
  CHECK(parse_logical_and(tokenize("a > 1 AND b < 2"))->to_cuda_expr() == "((a[idx] > 1.0f) && (b[idx] < 2.0f))");

  auto toks = tokenize("price > 10");
  CHECK(toks.size() == 4 && toks[0].type == TokenType::Identifier && toks[1].value == ">" &&
        toks[2].type == TokenType::Number && toks[3].type == TokenType::End);

  CHECK(error_of([] { lower("1 2"); }).find("Unexpected token") != std::string::npos);
  CHECK(error_of([] { lower("(price + 5"); }).find("Expected ')'") != std::string::npos);
  CHECK(error_of([] { tokenize("price & 5"); }).find("Unknown character") != std::string::npos);
  const std::string e = error_of([] { tokenize("price # 1\n"); });
  CHECK(e.find("line 1") != std::string::npos && e.find("column") != std::string::npos);
  const std::string q = error_of([] { parse_query(tokenize("SELECT price")); });
  CHECK(q.find("line") != std::string::npos && q.find("column") != std::string::npos);
  CHECK(error_of([] { parse_query(tokenize("SELECT price FROM test EXTRA")); }).find("Unexpected token") !=
        std::string::npos);

  QueryAST ast = parse_query(tokenize("SELECT SUM(price), quantity FROM sales JOIN items ON sales.id = items.id "
                                      "WHERE price > 10 GROUP BY quantity ORDER BY price DESC LIMIT 5"));
  CHECK(ast.select_list.size() == 2 && !ast.joins.empty() && ast.where.has_value() && ast.group_by.has_value() &&
        ast.order_by.has_value() && ast.limit.has_value());
  CHECK(dynamic_cast<AggregationNode *>(ast.select_list[0].get())->agg_kernel() == "sum");

  QueryAST bad = parse_query(tokenize("SELECT foo FROM test"));
  const std::unordered_set<std::string> cols{"price", "quantity"};
  CHECK(error_of([&] { walk(bad.select_list[0].get(), cols); }).find("Unknown column") != std::string::npos);

  std::string ex, cond;
  warpdb::split_where("price * quantity where price > 10", ex, cond);
  CHECK(ex == "price * quantity " && cond == " price > 10");

  if (failures) return 1;
  std::printf("frontend_test: all passed\n");
  return 0;
}
