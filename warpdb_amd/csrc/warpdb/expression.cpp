// expression.cpp -- query front end: lexer, recursive-descent parser,
// lowering to the C expression strings the execution layer compiles.
// Behaviour follows the reference front end (src/expression.cpp:22-531,
// include/expression.hpp:32-78); see include/warpdb/expression.hpp for the
// documented differences.
#include "warpdb/expression.hpp"

#include <array>
#include <cctype>
#include <stdexcept>

namespace {

const std::array<const char *, 23> kKeywords = {
    "SELECT", "FROM", "WHERE", "JOIN",  "ON",  "GROUP",     "BY",  "ORDER",  "ASC",     "DESC", "LIMIT", "OFFSET",
    "SUM",    "AVG",  "COUNT", "MIN",   "MAX", "OVER",      "PARTITION", "AND", "OR", "HAVING", "DISTINCT"};

bool is_keyword(const std::string &upper) {
  for (const char *k : kKeywords)
    if (upper == k) return true;
  return false;
}

const char *type_name(TokenType t) {
  switch (t) {
    case TokenType::Identifier: return "Identifier";
    case TokenType::Number: return "Number";
    case TokenType::Operator: return "Operator";
    case TokenType::Keyword: return "Keyword";
    case TokenType::End: return "End";
  }
  return "Unknown";
}

std::string where_at(const Token &t) {
  return " at line " + std::to_string(t.line) + " column " + std::to_string(t.column);
}

class Lexer {
 public:
  explicit Lexer(const std::string &s) : src_(s) {}

  std::vector<Token> run() {
    std::vector<Token> out;
    while (pos_ < src_.size()) {
      const char c = src_[pos_];
      const unsigned char uc = static_cast<unsigned char>(c);
      if (std::isspace(uc)) {
        step();
        continue;
      }
      const int line = line_, col = col_;
      if (std::isalpha(uc) || c == '_') {
        std::string word;
        while (pos_ < src_.size() && (std::isalnum(static_cast<unsigned char>(src_[pos_])) || src_[pos_] == '_' ||
                                      src_[pos_] == '.'))
          word += step();
        std::string upper = word;
        for (char &ch : upper) ch = static_cast<char>(std::toupper(static_cast<unsigned char>(ch)));
        if (is_keyword(upper)) out.push_back({TokenType::Keyword, upper, line, col});
        else out.push_back({TokenType::Identifier, word, line, col});
      } else if (std::isdigit(uc) || (c == '.' && pos_ + 1 < src_.size() &&
                                      std::isdigit(static_cast<unsigned char>(src_[pos_ + 1])))) {
        std::string num;
        bool dot = false;
        while (pos_ < src_.size()) {
          const char d = src_[pos_];
          if (std::isdigit(static_cast<unsigned char>(d))) num += step();
          else if (d == '.' && !dot) { dot = true; num += step(); }
          else break;
        }
        out.push_back({TokenType::Number, num, line, col});
      } else if (c == '>' || c == '<' || c == '=' || c == '!') {
        std::string op(1, step());
        if (pos_ < src_.size() && src_[pos_] == '=') op += step();
        out.push_back({TokenType::Operator, op, line, col});
      } else if (c == '+' || c == '-' || c == '*' || c == '/' || c == '(' || c == ')' || c == ',' || c == '.') {
        out.push_back({TokenType::Operator, std::string(1, step()), line, col});
      } else {
        throw std::runtime_error("Unknown character '" + std::string(1, c) + "' at line " + std::to_string(line) +
                                 " column " + std::to_string(col));
      }
    }
    out.push_back({TokenType::End, "", line_, col_});
    return out;
  }

 private:
  char step() {
    const char c = src_[pos_++];
    if (c == '\n') {
      ++line_;
      col_ = 1;
    } else {
      ++col_;
    }
    return c;
  }
  const std::string &src_;
  size_t pos_ = 0;
  int line_ = 1, col_ = 1;
};

bool aggregation_keyword(const std::string &kw, AggregationType &out) {
  if (kw == "SUM") out = AggregationType::Sum;
  else if (kw == "AVG") out = AggregationType::Avg;
  else if (kw == "COUNT") out = AggregationType::Count;
  else if (kw == "MIN") out = AggregationType::Min;
  else if (kw == "MAX") out = AggregationType::Max;
  else return false;
  return true;
}

// Recursive descent over a token range [pos, end) (end always holds an End
// token or the range is terminated by the caller).
class Parser {
 public:
  Parser(const std::vector<Token> &toks, bool allow_aggregates) : t_(toks), aggs_(allow_aggregates) {}

  ASTNodePtr full(int level) {
    ASTNodePtr n = level == 0 ? logical_or() : logical_and();
    if (peek().type != TokenType::End) throw std::runtime_error("Unexpected tokens remaining: " + peek().value);
    return n;
  }

 private:
  const Token &peek() const {
    static const Token end{TokenType::End, "", 0, 0};
    return i_ < t_.size() ? t_[i_] : end;
  }
  bool accept_op(const char *op) {
    if (peek().type == TokenType::Operator && peek().value == op) {
      ++i_;
      return true;
    }
    return false;
  }
  bool accept_kw(const char *kw) {
    if (peek().type == TokenType::Keyword && peek().value == kw) {
      ++i_;
      return true;
    }
    return false;
  }

  ASTNodePtr logical_or() {
    ASTNodePtr n = logical_and();
    while (accept_kw("OR")) n = std::make_unique<BinaryOpNode>("||", std::move(n), logical_and());
    return n;
  }
  ASTNodePtr logical_and() {
    ASTNodePtr n = comparison();
    while (accept_kw("AND")) n = std::make_unique<BinaryOpNode>("&&", std::move(n), comparison());
    return n;
  }
  ASTNodePtr comparison() {
    ASTNodePtr n = additive();
    for (;;) {
      const Token &t = peek();
      if (t.type != TokenType::Operator) break;
      std::string op = t.value;
      if (op != ">" && op != "<" && op != ">=" && op != "<=" && op != "==" && op != "!=" && op != "=") break;
      ++i_;
      if (op == "=") op = "==";  // SQL equality
      n = std::make_unique<BinaryOpNode>(op, std::move(n), additive());
    }
    return n;
  }
  ASTNodePtr additive() {
    ASTNodePtr n = term();
    for (;;) {
      if (accept_op("+")) n = std::make_unique<BinaryOpNode>("+", std::move(n), term());
      else if (accept_op("-")) n = std::make_unique<BinaryOpNode>("-", std::move(n), term());
      else return n;
    }
  }
  ASTNodePtr term() {
    ASTNodePtr n = factor();
    for (;;) {
      if (accept_op("*")) n = std::make_unique<BinaryOpNode>("*", std::move(n), factor());
      else if (accept_op("/")) n = std::make_unique<BinaryOpNode>("/", std::move(n), factor());
      else return n;
    }
  }
  ASTNodePtr factor() {
    const Token tok = peek();
    if (tok.type == TokenType::Number) {
      ++i_;
      return std::make_unique<ConstantNode>(tok.value);
    }
    if (tok.type == TokenType::Identifier) {
      ++i_;
      if (!accept_op("(")) return std::make_unique<VariableNode>(tok.value);
      std::vector<ASTNodePtr> args;
      if (++depth_ > kMaxDepth) throw std::runtime_error("Expression nested too deeply");
      struct Leave {
        int &d;
        ~Leave() { --d; }
      } leave{depth_};
      if (!accept_op(")")) {
        do {
          args.push_back(additive());
        } while (accept_op(","));
        if (!accept_op(")")) throw std::runtime_error("Expected ')' after arguments");
      }
      return std::make_unique<FunctionCallNode>(tok.value, std::move(args));
    }
    AggregationType at;
    if (aggs_ && tok.type == TokenType::Keyword && aggregation_keyword(tok.value, at) && i_ + 1 < t_.size() &&
        t_[i_ + 1].type == TokenType::Operator && t_[i_ + 1].value == "(") {
      i_ += 2;
      ASTNodePtr inner;
      if (at == AggregationType::Count && accept_op("*")) inner = std::make_unique<ConstantNode>("1");
      else inner = additive();
      if (!accept_op(")")) throw std::runtime_error("Expected ')'");
      return std::make_unique<AggregationNode>(at, std::move(inner));
    }
    if (accept_op("(")) {
      // the reference recurses without bound; a deep enough nest would
      // overflow the caller's stack, so nesting is capped
      if (++depth_ > kMaxDepth) throw std::runtime_error("Expression nested too deeply");
      ASTNodePtr n = additive();
      --depth_;
      if (!accept_op(")")) throw std::runtime_error("Expected ')'");
      return n;
    }
    throw std::runtime_error(std::string("Unexpected token (") + type_name(tok.type) + ": " + tok.value + ")");
  }

  static constexpr int kMaxDepth = 256;
  const std::vector<Token> &t_;
  size_t i_ = 0;
  int depth_ = 0;
  bool aggs_;
};

// LIMIT / OFFSET count: std::stoi as the reference (src/expression.cpp:509,
// 520), but a count beyond int is a query error, not std::out_of_range.
int count_value(const std::string &text, const char *clause) {
  try {
    return std::stoi(text);
  } catch (const std::out_of_range &) {
    throw std::runtime_error(std::string(clause) + " value out of range: " + text);
  }
}

std::vector<Token> slice(const std::vector<Token> &t, size_t a, size_t b) {
  std::vector<Token> s(t.begin() + static_cast<long>(a), t.begin() + static_cast<long>(b));
  s.push_back({TokenType::End, "", 0, 0});
  return s;
}

ASTNodePtr parse_in_query(const std::vector<Token> &t, size_t a, size_t b) {
  return Parser(slice(t, a, b), true).full(0);
}

}  // namespace

std::vector<Token> tokenize(const std::string &input) { return Lexer(input).run(); }

std::string ConstantNode::to_cuda_expr() const {
  return value.find('.') == std::string::npos ? value + ".0f" : value + "f";
}

std::string VariableNode::to_cuda_expr() const { return name + "[idx]"; }

std::string BinaryOpNode::to_cuda_expr() const {
  return "(" + left->to_cuda_expr() + " " + op + " " + right->to_cuda_expr() + ")";
}

std::string FunctionCallNode::to_cuda_expr() const {
  std::string s = name + "(";
  for (size_t i = 0; i < args.size(); ++i) s += (i ? ", " : "") + args[i]->to_cuda_expr();
  return s + ")";
}

std::string AggregationNode::agg_kernel() const {
  switch (agg) {
    case AggregationType::Sum: return "sum";
    case AggregationType::Avg: return "avg";
    case AggregationType::Count: return "count";
    case AggregationType::Min: return "min";
    case AggregationType::Max: return "max";
  }
  return "";
}

ASTNodePtr parse_expression(const std::vector<Token> &tokens) { return Parser(tokens, false).full(0); }
ASTNodePtr parse_logical_or(const std::vector<Token> &tokens) { return Parser(tokens, false).full(0); }
ASTNodePtr parse_logical_and(const std::vector<Token> &tokens) { return Parser(tokens, false).full(1); }

QueryAST parse_query(const std::vector<Token> &tokens) {
  size_t end = tokens.size();
  if (end && tokens[end - 1].type == TokenType::End) --end;
  size_t pos = 0;
  const Token last = tokens.empty() ? Token{TokenType::End, "", 1, 1} : tokens.back();
  auto at = [&](size_t p) -> const Token & { return p < tokens.size() ? tokens[p] : last; };
  auto is_kw = [&](size_t p, const char *kw) {
    return p < end && tokens[p].type == TokenType::Keyword && tokens[p].value == kw;
  };
  auto is_op = [&](size_t p, const char *op) {
    return p < end && tokens[p].type == TokenType::Operator && tokens[p].value == op;
  };
  auto expect = [&](const char *kw) {
    if (!is_kw(pos, kw)) throw std::runtime_error(std::string("Expected keyword '") + kw + "'" + where_at(at(pos)));
    ++pos;
  };
  // scan to the next top-level stop keyword
  auto until = [&](std::initializer_list<const char *> stops) {
    size_t p = pos;
    int depth = 0;
    while (p < end) {
      if (is_op(p, "(")) ++depth;
      if (is_op(p, ")")) --depth;
      if (depth == 0 && tokens[p].type == TokenType::Keyword) {
        bool stop = false;
        for (const char *s : stops) stop = stop || tokens[p].value == s;
        if (stop) break;
      }
      ++p;
    }
    return p;
  };

  QueryAST q;
  expect("SELECT");
  if (is_kw(pos, "DISTINCT")) {
    q.distinct = true;
    ++pos;
  }
  // select list: items split on top-level commas, up to FROM
  while (pos < end && !is_kw(pos, "FROM")) {
    size_t p = pos;
    int depth = 0;
    while (p < end) {
      if (is_op(p, "(")) ++depth;
      if (is_op(p, ")")) --depth;
      if (depth == 0 && (is_op(p, ",") || is_kw(p, "FROM"))) break;
      ++p;
    }
    AggregationType agg;
    size_t over = pos;
    while (over < p && !is_kw(over, "OVER")) ++over;
    if (tokens[pos].type == TokenType::Keyword && aggregation_keyword(tokens[pos].value, agg)) {
      const bool parens = over > pos + 2 && is_op(pos + 1, "(") && is_op(over - 1, ")");
      if (!parens) throw std::runtime_error("Invalid syntax for " + tokens[pos].value + " aggregation");
      ASTNodePtr inner;
      if (agg == AggregationType::Count && over == pos + 4 && is_op(pos + 2, "*"))
        inner = std::make_unique<ConstantNode>("1");
      else
        inner = parse_in_query(tokens, pos + 2, over - 1);
      if (over < p) q.select_list.push_back(std::make_unique<WindowFunctionNode>(agg, std::move(inner)));
      else q.select_list.push_back(std::make_unique<AggregationNode>(agg, std::move(inner)));
    } else {
      q.select_list.push_back(parse_in_query(tokens, pos, p));
    }
    pos = p;
    if (is_op(pos, ",")) ++pos;
  }
  expect("FROM");
  if (pos >= end || tokens[pos].type != TokenType::Identifier)
    throw std::runtime_error("Expected table name after FROM" + where_at(at(pos)));
  q.from_table = tokens[pos++].value;
  while (is_kw(pos, "JOIN")) {
    ++pos;
    if (pos >= end || tokens[pos].type != TokenType::Identifier)
      throw std::runtime_error("Expected table name after JOIN" + where_at(at(pos)));
    JoinClause j;
    j.table = tokens[pos++].value;
    expect("ON");
    const size_t stop = until({"WHERE", "GROUP", "ORDER", "HAVING", "JOIN", "LIMIT", "OFFSET"});
    j.condition = parse_in_query(tokens, pos, stop);
    pos = stop;
    q.joins.push_back(std::move(j));
  }
  if (is_kw(pos, "WHERE")) {
    ++pos;
    const size_t stop = until({"GROUP", "ORDER", "HAVING", "LIMIT", "OFFSET"});
    q.where = parse_in_query(tokens, pos, stop);
    pos = stop;
  }
  if (is_kw(pos, "GROUP")) {
    ++pos;
    expect("BY");
    GroupByClause g;
    const size_t stop = until({"ORDER", "HAVING", "LIMIT", "OFFSET"});
    while (pos < stop) {
      size_t p = pos;
      int depth = 0;
      while (p < stop && !(depth == 0 && is_op(p, ","))) {
        if (is_op(p, "(")) ++depth;
        if (is_op(p, ")")) --depth;
        ++p;
      }
      g.keys.push_back(parse_in_query(tokens, pos, p));
      pos = p;
      if (is_op(pos, ",")) ++pos;
    }
    q.group_by = std::move(g);
  }
  if (is_kw(pos, "HAVING")) {
    ++pos;
    const size_t stop = until({"ORDER", "LIMIT", "OFFSET"});
    q.having = parse_in_query(tokens, pos, stop);
    pos = stop;
  }
  if (is_kw(pos, "ORDER")) {
    ++pos;
    expect("BY");
    const size_t stop = until({"ASC", "DESC", "LIMIT", "OFFSET"});
    OrderByClause ob;
    ob.expr = parse_in_query(tokens, pos, stop);
    ob.ascending = true;
    pos = stop;
    if (is_kw(pos, "ASC") || is_kw(pos, "DESC")) ob.ascending = tokens[pos++].value == "ASC";
    q.order_by = std::move(ob);
  }
  for (int rep = 0; rep < 2; ++rep) {  // LIMIT n / OFFSET n, either order
    if (is_kw(pos, "LIMIT") && !q.limit) {
      ++pos;
      if (pos >= end || tokens[pos].type != TokenType::Number)
        throw std::runtime_error("Expected numeric value after LIMIT" + where_at(at(pos)));
      q.limit = LimitClause{count_value(tokens[pos++].value, "LIMIT")};
    } else if (is_kw(pos, "OFFSET") && !q.offset) {
      ++pos;
      if (pos >= end || tokens[pos].type != TokenType::Number)
        throw std::runtime_error("Expected numeric value after OFFSET");
      q.offset = OffsetClause{count_value(tokens[pos++].value, "OFFSET")};
    }
  }
  if (pos != end) throw std::runtime_error("Unexpected token in query near: " + tokens[pos].value);
  return q;
}

namespace warpdb {
void split_where(const std::string &query, std::string &expr, std::string &cond) {
  std::string upper = query;
  for (char &c : upper) c = static_cast<char>(std::toupper(static_cast<unsigned char>(c)));
  const auto p = upper.find("WHERE");
  if (p == std::string::npos) {
    expr = query;
    cond.clear();
  } else {
    expr = query.substr(0, p);
    cond = query.substr(p + 5);
  }
}
}  // namespace warpdb
