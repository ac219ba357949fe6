/*
 * warpdb_oracle.c -- TEST INFRASTRUCTURE ONLY (see warpdb_oracle.h).
 *
 * Plain-C restatement of the reference WarpDB CPU query path:
 *   tokenizer            src/expression.cpp:22-120
 *   parser (precedence)  src/expression.cpp:144-248
 *   lowering strings     include/expression.hpp:32-78
 *   WHERE split          src/warpdb.cpp:204-213
 *   row evaluator        src/warpdb.cpp:111-155 (get_value / eval_node /
 *                        eval_condition), incl. the ascending row list of
 *                        src/warpdb.cpp:336-344
 *   GROUP BY SUM intent  tests/sql_features_test.cpp:11-22 (std::map<int,double>)
 *   ORDER BY .. LIMIT    tests/sql_features_test.cpp:24-34
 * Documented deviations (the reference CPU evaluator returns 0.0f for these,
 * src/warpdb.cpp:150): && and || use C truthiness, '=' is equality, and
 * discount(p, r) = p * r mirrors custom.cu:1-3.
 *
 * This file is never linked into the product; it is the checker.
 */
#include "warpdb_oracle.h"

#include <ctype.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ errors */
typedef struct {
  char *buf;
  size_t len;
  int failed;
} errctx;

static void seterr(errctx *e, const char *fmt, ...) {
  if (e->failed) return;
  e->failed = 1;
  if (!e->buf || !e->len) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(e->buf, e->len, fmt, ap);
  va_end(ap);
}

/* ---------------------------------------------------------------- tokens */
enum { TK_IDENT, TK_NUMBER, TK_OP, TK_KEYWORD, TK_END };

typedef struct {
  int type;
  char text[64];
  int line, col;
} token;

typedef struct {
  token *v;
  int n, cap;
} tokvec;

static const char *KEYWORDS[] = {"SELECT", "FROM",  "WHERE",  "JOIN",  "ON",       "GROUP",
                                 "BY",     "ORDER", "ASC",    "DESC",  "LIMIT",    "OFFSET",
                                 "SUM",    "AVG",   "COUNT",  "MIN",   "MAX",      "OVER",
                                 "PARTITION", "AND", "OR",    "HAVING", "DISTINCT", NULL};

static void push_tok(tokvec *tv, int type, const char *s, size_t n, int line, int col) {
  if (tv->n == tv->cap) {
    tv->cap = tv->cap ? tv->cap * 2 : 16;
    tv->v = (token *)realloc(tv->v, sizeof(token) * (size_t)tv->cap);
  }
  token *t = &tv->v[tv->n++];
  t->type = type;
  if (n >= sizeof(t->text)) n = sizeof(t->text) - 1;
  memcpy(t->text, s, n);
  t->text[n] = 0;
  t->line = line;
  t->col = col;
}

/* src/expression.cpp:22-120 */
static int tokenize(const char *in, tokvec *tv, errctx *e) {
  size_t i = 0, n = strlen(in);
  int line = 1, col = 1;
  while (i < n) {
    char c = in[i];
    if (c == '\n') { line++; col = 1; i++; continue; }
    if (isspace((unsigned char)c)) { col++; i++; continue; }
    if (isalpha((unsigned char)c) || c == '_') {
      int sc = col;
      size_t s = i;
      while (i < n && (isalnum((unsigned char)in[i]) || in[i] == '_' || in[i] == '.')) { i++; col++; }
      char up[64];
      size_t len = i - s < 63 ? i - s : 63;
      for (size_t k = 0; k < len; k++) up[k] = (char)toupper((unsigned char)in[s + k]);
      up[len] = 0;
      int kw = 0;
      for (const char **k = KEYWORDS; *k; k++)
        if (strcmp(*k, up) == 0 && (i - s) == strlen(*k)) kw = 1;
      if (kw) push_tok(tv, TK_KEYWORD, up, len, line, sc);
      else push_tok(tv, TK_IDENT, in + s, i - s, line, sc);
    } else if (isdigit((unsigned char)c) || (c == '.' && i + 1 < n && isdigit((unsigned char)in[i + 1]))) {
      int sc = col, dot = 0;
      size_t s = i;
      while (i < n && (isdigit((unsigned char)in[i]) || (!dot && in[i] == '.'))) {
        if (in[i] == '.') dot = 1;
        i++; col++;
      }
      push_tok(tv, TK_NUMBER, in + s, i - s, line, sc);
    } else if (c == '>' || c == '<' || c == '=' || c == '!') {
      int sc = col;
      size_t s = i;
      if (i + 1 < n && in[i + 1] == '=') { i++; col++; }
      i++; col++;
      push_tok(tv, TK_OP, in + s, i - s, line, sc);
    } else if (strchr("+-*/()<>,.", c) && c) {
      push_tok(tv, TK_OP, in + i, 1, line, col);
      i++; col++;
    } else {
      seterr(e, "Unknown character '%c' at line %d column %d", c, line, col);
      return -1;
    }
  }
  push_tok(tv, TK_END, "", 0, line, col);
  return 0;
}

/* ------------------------------------------------------------------- AST */
enum { N_CONST, N_VAR, N_BIN, N_CALL };
enum { OP_ADD, OP_SUB, OP_MUL, OP_DIV, OP_GT, OP_LT, OP_GE, OP_LE, OP_EQ, OP_NE, OP_AND, OP_OR, OP_BAD };

typedef struct node {
  int kind;
  char text[64];   /* constant text / variable / operator / function name */
  int op;          /* resolved operator */
  float cval;      /* std::stof(text) for constants */
  int colidx;      /* resolved column, -1 = unknown */
  struct node *l, *r;
  struct node **args;
  int nargs;
} node;

static node *mk(int kind, const char *text) {
  node *x = (node *)calloc(1, sizeof(node));
  x->kind = kind;
  snprintf(x->text, sizeof(x->text), "%s", text);
  x->colidx = -1;
  x->op = OP_BAD;
  return x;
}

static void freenode(node *x) {
  if (!x) return;
  freenode(x->l);
  freenode(x->r);
  for (int i = 0; i < x->nargs; i++) freenode(x->args[i]);
  free(x->args);
  free(x);
}

typedef struct {
  tokvec *tv;
  int pos;
  errctx *e;
} parser;

static token *peek(parser *p) { return &p->tv->v[p->pos]; }
static int match_op(parser *p, const char *op) {
  token *t = peek(p);
  if (t->type == TK_OP && strcmp(t->text, op) == 0) { p->pos++; return 1; }
  return 0;
}

static node *p_or(parser *p);
static node *p_add(parser *p);

static const char *tkname(int t) {
  switch (t) {
    case TK_IDENT: return "Identifier";
    case TK_NUMBER: return "Number";
    case TK_OP: return "Operator";
    case TK_KEYWORD: return "Keyword";
    default: return "End";
  }
}

static node *binop(const char *op, node *l, node *r) {
  node *b = mk(N_BIN, op);
  b->l = l;
  b->r = r;
  return b;
}

/* factor = number | identifier [ '(' args ')' ] | '(' expr ')'   (:205-235) */
static node *p_factor(parser *p) {
  if (p->e->failed) return NULL;
  token *t = peek(p);
  if (t->type == TK_NUMBER) {
    p->pos++;
    node *c = mk(N_CONST, t->text);
    c->cval = strtof(t->text, NULL);
    return c;
  }
  if (t->type == TK_IDENT) {
    char name[64];
    snprintf(name, sizeof(name), "%s", t->text);
    p->pos++;
    if (match_op(p, "(")) {
      node *f = mk(N_CALL, name);
      if (!match_op(p, ")")) {
        do {
          f->args = (node **)realloc(f->args, sizeof(node *) * (size_t)(f->nargs + 1));
          f->args[f->nargs++] = p_add(p);
          if (p->e->failed) { freenode(f); return NULL; }
        } while (match_op(p, ","));
        if (!match_op(p, ")")) { seterr(p->e, "Expected ')' after arguments"); freenode(f); return NULL; }
      }
      return f;
    }
    return mk(N_VAR, name);
  }
  if (match_op(p, "(")) {
    node *x = p_add(p);
    if (p->e->failed) { freenode(x); return NULL; }
    if (!match_op(p, ")")) { seterr(p->e, "Expected ')'"); freenode(x); return NULL; }
    return x;
  }
  seterr(p->e, "Unexpected token (%s: %s)", tkname(t->type), t->text);
  return NULL;
}

static node *p_term(parser *p) { /* :193-202 */
  node *x = p_factor(p);
  while (!p->e->failed && (match_op(p, "*") || match_op(p, "/"))) {
    const char *op = p->tv->v[p->pos - 1].text;
    x = binop(op, x, p_factor(p));
  }
  return x;
}

static node *p_add(parser *p) { /* :144-153 */
  node *x = p_term(p);
  while (!p->e->failed && (match_op(p, "+") || match_op(p, "-"))) {
    const char *op = p->tv->v[p->pos - 1].text;
    x = binop(op, x, p_term(p));
  }
  return x;
}

static node *p_cmp(parser *p) { /* :156-166 */
  node *x = p_add(p);
  while (!p->e->failed && (match_op(p, ">") || match_op(p, "<") || match_op(p, ">=") ||
                           match_op(p, "<=") || match_op(p, "==") || match_op(p, "!=") ||
                           match_op(p, "="))) {
    const char *op = p->tv->v[p->pos - 1].text;
    /* deviation: '=' is SQL equality (the reference emits a C assignment) */
    x = binop(strcmp(op, "=") == 0 ? "==" : op, x, p_add(p));
  }
  return x;
}

static int kw(parser *p, const char *k) {
  token *t = peek(p);
  return t->type == TK_KEYWORD && strcmp(t->text, k) == 0;
}

static node *p_and(parser *p) { /* :169-178 */
  node *x = p_cmp(p);
  while (!p->e->failed && kw(p, "AND")) {
    p->pos++;
    x = binop("&&", x, p_cmp(p));
  }
  return x;
}

static node *p_or(parser *p) { /* :181-190 */
  node *x = p_and(p);
  while (!p->e->failed && kw(p, "OR")) {
    p->pos++;
    x = binop("||", x, p_and(p));
  }
  return x;
}

static int opcode(const char *s) {
  static const char *ops[] = {"+", "-", "*", "/", ">", "<", ">=", "<=", "==", "!=", "&&", "||"};
  for (int i = 0; i < 12; i++)
    if (strcmp(ops[i], s) == 0) return i;
  return OP_BAD;
}

/* parse_expression (:238-248) */
static node *parse_expr(const char *src, errctx *e) {
  tokvec tv = {0};
  if (tokenize(src, &tv, e) != 0) { free(tv.v); return NULL; }
  parser p = {&tv, 0, e};
  node *x = p_or(&p);
  if (!e->failed && peek(&p)->type != TK_END) seterr(e, "Unexpected tokens remaining: %s", peek(&p)->text);
  free(tv.v);
  if (e->failed) { freenode(x); return NULL; }
  return x;
}

static int resolve(node *x, const ora_table *t, errctx *e) {
  if (!x) return 0;
  if (x->kind == N_BIN) x->op = opcode(x->text);
  if (x->kind == N_VAR) {
    for (int i = 0; i < t->n_cols; i++)
      if (strcmp(t->cols[i].name, x->text) == 0) x->colidx = i;
    if (x->colidx < 0) { seterr(e, "Unknown column: %s", x->text); return -1; }
  }
  if (x->kind == N_CALL) {
    if (strcmp(x->text, "discount") != 0 || x->nargs != 2) {
      seterr(e, "oracle: unsupported function %s/%d", x->text, x->nargs);
      return -1;
    }
  }
  if (resolve(x->l, t, e) || resolve(x->r, t, e)) return -1;
  for (int i = 0; i < x->nargs; i++)
    if (resolve(x->args[i], t, e)) return -1;
  return 0;
}

/* ------------------------------------------------------------- lowering */
static void lower_rec(const node *x, char *out, size_t outlen, size_t *pos) {
#define EMIT(...) (*pos += (size_t)snprintf(out + (*pos < outlen ? *pos : outlen), *pos < outlen ? outlen - *pos : 0, __VA_ARGS__))
  switch (x->kind) {
    case N_CONST: /* include/expression.hpp:32-38 */
      if (strchr(x->text, '.')) EMIT("%sf", x->text);
      else EMIT("%s.0f", x->text);
      break;
    case N_VAR: EMIT("%s[idx]", x->text); break; /* :45 */
    case N_BIN: /* :56-59 */
      EMIT("(");
      lower_rec(x->l, out, outlen, pos);
      EMIT(" %s ", x->text);
      lower_rec(x->r, out, outlen, pos);
      EMIT(")");
      break;
    case N_CALL: /* :69-78 */
      EMIT("%s(", x->text);
      for (int i = 0; i < x->nargs; i++) {
        if (i) EMIT(", ");
        lower_rec(x->args[i], out, outlen, pos);
      }
      EMIT(")");
      break;
  }
#undef EMIT
}

int ora_lower(const char *expr, char *out, size_t outlen, char *err, size_t errlen) {
  errctx e = {err, errlen, 0};
  node *x = parse_expr(expr, &e);
  if (!x) return -1;
  size_t pos = 0;
  if (outlen) out[0] = 0;
  lower_rec(x, out, outlen, &pos);
  freenode(x);
  return 0;
}

void ora_split_where(const char *q, char *expr, size_t elen, char *cond, size_t clen) {
  size_t n = strlen(q);
  long at = -1;
  for (size_t i = 0; i + 5 <= n && at < 0; i++) {
    int ok = 1;
    for (int k = 0; k < 5; k++)
      if (toupper((unsigned char)q[i + k]) != "WHERE"[k]) ok = 0;
    if (ok) at = (long)i;
  }
  if (at < 0) {
    snprintf(expr, elen, "%s", q);
    if (clen) cond[0] = 0;
  } else {
    snprintf(expr, elen, "%.*s", (int)at, q);
    snprintf(cond, clen, "%s", q + at + 5);
  }
}

/* ------------------------------------------------------------ evaluation */
/* ORA_SEM_CPU: src/warpdb.cpp:111-126 get_value casts every column to float. */
static inline float col_as_float(const ora_col *c, int64_t i) {
  switch (c->dtype) {
    case ORA_INT32: return (float)((const int32_t *)c->data)[i];
    case ORA_INT64: return (float)((const int64_t *)c->data)[i];
    case ORA_FLOAT32: return ((const float *)c->data)[i];
    case ORA_FLOAT64: return (float)((const double *)c->data)[i];
    default: return 0.0f;
  }
}

/* src/warpdb.cpp:128-151 */
static float eval_cpu(const node *x, const ora_table *t, int64_t i) {
  switch (x->kind) {
    case N_CONST: return x->cval;
    case N_VAR: return col_as_float(&t->cols[x->colidx], i);
    case N_CALL: { /* deviation: custom.cu discount(price, rate) = price * rate */
      float a = eval_cpu(x->args[0], t, i), b = eval_cpu(x->args[1], t, i);
      return a * b;
    }
    default: break;
  }
  float l = eval_cpu(x->l, t, i), r = eval_cpu(x->r, t, i);
  switch (x->op) {
    case OP_ADD: return l + r;
    case OP_SUB: return l - r;
    case OP_MUL: return l * r;
    case OP_DIV: return l / r;
    case OP_GT: return (float)(l > r);
    case OP_LT: return (float)(l < r);
    case OP_GE: return (float)(l >= r);
    case OP_LE: return (float)(l <= r);
    case OP_EQ: return (float)(l == r);
    case OP_NE: return (float)(l != r);
    case OP_AND: return (float)(l != 0.0f && r != 0.0f); /* deviation */
    case OP_OR: return (float)(l != 0.0f || r != 0.0f);  /* deviation */
    default: return 0.0f;
  }
}

/* ORA_SEM_JIT: C semantics of the generated kernel, src/jit.cpp:31-45,55-61. */
enum { V_I32, V_I64, V_F32, V_F64 };
typedef struct {
  int t;
  long long i;
  double d; /* holds the float for V_F32 (exactly) */
} tval;

static inline tval tv_i32(long long v) { tval r = {V_I32, (int)v, 0}; return r; }
static inline tval tv_f32(float v) { tval r = {V_F32, 0, v}; return r; }

static inline double tv_d(tval v) { return (v.t >= V_F32) ? v.d : (double)v.i; }
static inline float tv_f(tval v) {
  if (v.t == V_F32) return (float)v.d;
  if (v.t == V_F64) return (float)v.d;
  return (float)v.i;
}
static inline int tv_truth(tval v) { return v.t >= V_F32 ? v.d != 0.0 : v.i != 0; }

static tval eval_jit(const node *x, const ora_table *t, int64_t i) {
  switch (x->kind) {
    case N_CONST: return tv_f32(x->cval);
    case N_VAR: {
      const ora_col *c = &t->cols[x->colidx];
      tval r = {0, 0, 0};
      switch (c->dtype) {
        case ORA_INT32: r.t = V_I32; r.i = ((const int32_t *)c->data)[i]; break;
        case ORA_INT64: r.t = V_I64; r.i = ((const int64_t *)c->data)[i]; break;
        case ORA_FLOAT32: r.t = V_F32; r.d = ((const float *)c->data)[i]; break;
        case ORA_FLOAT64: r.t = V_F64; r.d = ((const double *)c->data)[i]; break;
      }
      return r;
    }
    case N_CALL: {
      float a = tv_f(eval_jit(x->args[0], t, i)), b = tv_f(eval_jit(x->args[1], t, i));
      return tv_f32(a * b);
    }
    default: break;
  }
  tval l = eval_jit(x->l, t, i), r = eval_jit(x->r, t, i);
  if (x->op == OP_AND) return tv_i32(tv_truth(l) && tv_truth(r));
  if (x->op == OP_OR) return tv_i32(tv_truth(l) || tv_truth(r));
  int ct = l.t > r.t ? l.t : r.t; /* usual arithmetic conversions */
  if (ct == V_F64) {
    double a = tv_d(l), b = tv_d(r);
    switch (x->op) {
      case OP_ADD: { tval v = {V_F64, 0, a + b}; return v; }
      case OP_SUB: { tval v = {V_F64, 0, a - b}; return v; }
      case OP_MUL: { tval v = {V_F64, 0, a * b}; return v; }
      case OP_DIV: { tval v = {V_F64, 0, a / b}; return v; }
      case OP_GT: return tv_i32(a > b);
      case OP_LT: return tv_i32(a < b);
      case OP_GE: return tv_i32(a >= b);
      case OP_LE: return tv_i32(a <= b);
      case OP_EQ: return tv_i32(a == b);
      case OP_NE: return tv_i32(a != b);
    }
  } else if (ct == V_F32) {
    float a = tv_f(l), b = tv_f(r);
    switch (x->op) {
      case OP_ADD: return tv_f32(a + b);
      case OP_SUB: return tv_f32(a - b);
      case OP_MUL: return tv_f32(a * b);
      case OP_DIV: return tv_f32(a / b);
      case OP_GT: return tv_i32(a > b);
      case OP_LT: return tv_i32(a < b);
      case OP_GE: return tv_i32(a >= b);
      case OP_LE: return tv_i32(a <= b);
      case OP_EQ: return tv_i32(a == b);
      case OP_NE: return tv_i32(a != b);
    }
  } else {
    long long a = l.i, b = r.i, v = 0;
    int is64 = ct == V_I64;
    switch (x->op) {
      case OP_ADD: v = a + b; break;
      case OP_SUB: v = a - b; break;
      case OP_MUL: v = a * b; break;
      case OP_DIV: v = b ? a / b : 0; break;
      case OP_GT: return tv_i32(a > b);
      case OP_LT: return tv_i32(a < b);
      case OP_GE: return tv_i32(a >= b);
      case OP_LE: return tv_i32(a <= b);
      case OP_EQ: return tv_i32(a == b);
      case OP_NE: return tv_i32(a != b);
    }
    tval o = {is64 ? V_I64 : V_I32, is64 ? v : (long long)(int)v, 0};
    return o;
  }
  return tv_i32(0);
}

static inline float eval_val(const node *x, const ora_table *t, int64_t i, int sem) {
  return sem == ORA_SEM_JIT ? tv_f(eval_jit(x, t, i)) : eval_cpu(x, t, i);
}
static inline int eval_cond(const node *x, const ora_table *t, int64_t i, int sem) {
  if (!x) return 1;
  return sem == ORA_SEM_JIT ? tv_truth(eval_jit(x, t, i)) : eval_cpu(x, t, i) != 0.0f;
}
static inline int eval_key(const node *x, const ora_table *t, int64_t i, int sem) {
  if (sem == ORA_SEM_JIT) {
    tval v = eval_jit(x, t, i);
    return v.t >= V_F32 ? (int)v.d : (int)v.i;
  }
  return (int)eval_cpu(x, t, i); /* static_cast<int>(eval_node(...)), src/warpdb.cpp:374 */
}

static node *prep(const char *src, const ora_table *t, errctx *e, int allow_empty) {
  if (!src) return NULL;
  int blank = 1;
  for (const char *s = src; *s; s++)
    if (!isspace((unsigned char)*s)) blank = 0;
  if (blank) {
    if (!allow_empty) seterr(e, "Empty query expression");
    return NULL;
  }
  node *x = parse_expr(src, e);
  if (!x) return NULL;
  if (resolve(x, t, e)) { freenode(x); return NULL; }
  return x;
}

int ora_project_filter(const ora_table *t, const char *expr, const char *cond, int sem,
                       float *out_vals, int64_t *out_idx, int64_t *out_count, float *dense_out,
                       char *err, size_t errlen) {
  errctx e = {err, errlen, 0};
  node *ex = prep(expr, t, &e, 0);
  if (e.failed) return -1;
  node *cx = prep(cond, t, &e, 1);
  if (e.failed) { freenode(ex); return -1; }
  int64_t k = 0;
  for (int64_t i = 0; i < t->n_rows; i++) {
    if (!eval_cond(cx, t, i, sem)) continue;
    float v = eval_val(ex, t, i, sem);
    if (out_vals) out_vals[k] = v;
    if (out_idx) out_idx[k] = i;
    if (dense_out) dense_out[i] = v;
    k++;
  }
  if (out_count) *out_count = k;
  freenode(ex);
  freenode(cx);
  return 0;
}

int ora_sum(const ora_table *t, const char *expr, const char *cond, int sem, double *out_sum,
            int64_t *out_count, char *err, size_t errlen) {
  errctx e = {err, errlen, 0};
  node *ex = prep(expr, t, &e, 0);
  if (e.failed) return -1;
  node *cx = prep(cond, t, &e, 1);
  if (e.failed) { freenode(ex); return -1; }
  double s = 0.0;
  int64_t k = 0;
  for (int64_t i = 0; i < t->n_rows; i++) {
    if (!eval_cond(cx, t, i, sem)) continue;
    s += (double)eval_val(ex, t, i, sem);
    k++;
  }
  *out_sum = s;
  if (out_count) *out_count = k;
  freenode(ex);
  freenode(cx);
  return 0;
}

/* MIN / MAX fold of the reference's AggData (src/warpdb.cpp:375-385: min/max
 * of the group's values).  Stated order-free: NaN values are skipped (the
 * reference's std::min/std::max keep or drop a NaN depending on where it falls
 * in the scan), -0.0 folds to +0.0, and an empty fold reads NaN. */
static inline void mm_fold(float v, int *have, float *mn, float *mx) {
  if (isnan(v)) return;
  if (v == 0.0f) v = 0.0f;
  if (!*have) { *mn = *mx = v; *have = 1; return; }
  if (v < *mn) *mn = v;
  if (v > *mx) *mx = v;
}

int ora_stats(const ora_table *t, const char *expr, const char *cond, int sem, double *out_sum,
              int64_t *out_count, float *out_min, float *out_max, char *err, size_t errlen) {
  errctx e = {err, errlen, 0};
  node *ex = prep(expr, t, &e, 0);
  if (e.failed) return -1;
  node *cx = prep(cond, t, &e, 1);
  if (e.failed) { freenode(ex); return -1; }
  double s = 0.0;
  int64_t k = 0;
  int have = 0;
  float mn = NAN, mx = NAN;
  for (int64_t i = 0; i < t->n_rows; i++) {
    if (!eval_cond(cx, t, i, sem)) continue;
    const float v = eval_val(ex, t, i, sem);
    s += (double)v;
    k++;
    mm_fold(v, &have, &mn, &mx);
  }
  if (out_sum) *out_sum = s;
  if (out_count) *out_count = k;
  if (out_min) *out_min = mn;
  if (out_max) *out_max = mx;
  freenode(ex);
  freenode(cx);
  return 0;
}

/* open-addressing int -> slot map for GROUP BY */
typedef struct {
  int32_t key;
  int used;
  double sum;
  int64_t cnt;
  int have_mm;
  float mn, mx;
} gslot;

static int cmp_gslot(const void *a, const void *b) {
  const gslot *x = (const gslot *)a, *y = (const gslot *)b;
  return (x->key > y->key) - (x->key < y->key);
}

int ora_group_agg(const ora_table *t, const char *val_expr, const char *key_expr, const char *cond,
                  int sem, int64_t capacity, int32_t *out_keys, double *out_sums,
                  int64_t *out_counts, float *out_mins, float *out_maxs, int64_t *out_groups, char *err,
                  size_t errlen) {
  errctx e = {err, errlen, 0};
  node *vx = prep(val_expr, t, &e, 0);
  if (e.failed) return -1;
  node *kx = prep(key_expr, t, &e, 0);
  if (e.failed) { freenode(vx); return -1; }
  node *cx = prep(cond, t, &e, 1);
  if (e.failed) { freenode(vx); freenode(kx); return -1; }
  size_t cap = 1024;
  size_t used = 0;
  gslot *tab = (gslot *)calloc(cap, sizeof(gslot));
  for (int64_t i = 0; i < t->n_rows; i++) {
    if (!eval_cond(cx, t, i, sem)) continue;
    int32_t key = eval_key(kx, t, i, sem);
    float val = eval_val(vx, t, i, sem);
    if ((used + 1) * 2 > cap) { /* grow */
      size_t nc = cap * 2;
      gslot *nt = (gslot *)calloc(nc, sizeof(gslot));
      for (size_t s = 0; s < cap; s++)
        if (tab[s].used) {
          size_t h = ((uint32_t)tab[s].key * 2654435761u) & (nc - 1);
          while (nt[h].used) h = (h + 1) & (nc - 1);
          nt[h] = tab[s];
        }
      free(tab);
      tab = nt;
      cap = nc;
    }
    size_t h = ((uint32_t)key * 2654435761u) & (cap - 1);
    while (tab[h].used && tab[h].key != key) h = (h + 1) & (cap - 1);
    if (!tab[h].used) { tab[h].used = 1; tab[h].key = key; tab[h].mn = tab[h].mx = NAN; used++; }
    tab[h].sum += (double)val;
    tab[h].cnt += 1;
    mm_fold(val, &tab[h].have_mm, &tab[h].mn, &tab[h].mx);
  }
  /* compact + ascending key order */
  size_t g = 0;
  for (size_t s = 0; s < cap; s++)
    if (tab[s].used) tab[g++] = tab[s];
  qsort(tab, g, sizeof(gslot), cmp_gslot);
  if ((int64_t)g > capacity) {
    seterr(&e, "group capacity %lld exceeded (%zu groups)", (long long)capacity, g);
  } else {
    for (size_t s = 0; s < g; s++) {
      if (out_keys) out_keys[s] = tab[s].key;
      if (out_sums) out_sums[s] = tab[s].sum;
      if (out_counts) out_counts[s] = tab[s].cnt;
      if (out_mins) out_mins[s] = tab[s].mn;
      if (out_maxs) out_maxs[s] = tab[s].mx;
    }
  }
  *out_groups = (int64_t)g;
  free(tab);
  freenode(vx);
  freenode(kx);
  freenode(cx);
  return e.failed ? -1 : 0;
}

int ora_group_sum(const ora_table *t, const char *val_expr, const char *key_expr, const char *cond,
                  int sem, int64_t capacity, int32_t *out_keys, double *out_sums,
                  int64_t *out_counts, int64_t *out_groups, char *err, size_t errlen) {
  return ora_group_agg(t, val_expr, key_expr, cond, sem, capacity, out_keys, out_sums, out_counts, NULL, NULL,
                       out_groups, err, errlen);
}

/* total order used by top-K: key (desc or asc), then row index ascending.
 * NaN keys order after every number in either direction. */
static inline int topk_better(float ka, int64_t ia, float kb, int64_t ib, int desc) {
  int na = isnan(ka), nb = isnan(kb);
  if (na || nb) {
    if (na && nb) return ia < ib;
    return nb;
  }
  if (ka != kb) return desc ? ka > kb : ka < kb;
  return ia < ib;
}

int ora_topk(const ora_table *t, const char *order_expr, const char *cond, const char *select_expr,
             int64_t k, int descending, int sem, float *out_keys, int64_t *out_idx,
             float *out_vals, int64_t *out_count, char *err, size_t errlen) {
  errctx e = {err, errlen, 0};
  node *ox = prep(order_expr, t, &e, 0);
  if (e.failed) return -1;
  node *cx = prep(cond, t, &e, 1);
  node *sx = e.failed ? NULL : prep(select_expr, t, &e, 1);
  if (e.failed) { freenode(ox); freenode(cx); return -1; }
  float *kk = (float *)malloc(sizeof(float) * (size_t)(k > 0 ? k : 1));
  int64_t *ki = (int64_t *)malloc(sizeof(int64_t) * (size_t)(k > 0 ? k : 1));
  int64_t n = 0;
  for (int64_t i = 0; i < t->n_rows && k > 0; i++) {
    if (!eval_cond(cx, t, i, sem)) continue;
    float key = eval_val(ox, t, i, sem);
    if (n == k && !topk_better(key, i, kk[n - 1], ki[n - 1], descending)) continue;
    int64_t p = n < k ? n : k - 1;
    if (n < k) n++;
    while (p > 0 && topk_better(key, i, kk[p - 1], ki[p - 1], descending)) {
      kk[p] = kk[p - 1];
      ki[p] = ki[p - 1];
      p--;
    }
    kk[p] = key;
    ki[p] = i;
  }
  for (int64_t j = 0; j < n; j++) {
    if (out_keys) out_keys[j] = kk[j];
    if (out_idx) out_idx[j] = ki[j];
    if (out_vals) out_vals[j] = sx ? eval_val(sx, t, ki[j], sem) : kk[j];
  }
  *out_count = n;
  free(kk);
  free(ki);
  freenode(ox);
  freenode(cx);
  freenode(sx);
  return 0;
}

/* --------------------------------------------------- CPU baseline timing */
/* Faithful to the reference's cost structure (src/warpdb.cpp:111-155): per
 * row, per node: get_column() name lookup, std::stof of the constant text and
 * string comparison of the operator. */
static float eval_faithful(const node *x, const ora_table *t, int64_t i) {
  if (x->kind == N_CONST) return strtof(x->text, NULL);
  if (x->kind == N_VAR) {
    for (int c = 0; c < t->n_cols; c++)
      if (strcmp(t->cols[c].name, x->text) == 0) return col_as_float(&t->cols[c], i);
    return 0.0f;
  }
  if (x->kind == N_CALL) return eval_faithful(x->args[0], t, i) * eval_faithful(x->args[1], t, i);
  float l = eval_faithful(x->l, t, i), r = eval_faithful(x->r, t, i);
  const char *op = x->text;
  if (strcmp(op, "+") == 0) return l + r;
  if (strcmp(op, "-") == 0) return l - r;
  if (strcmp(op, "*") == 0) return l * r;
  if (strcmp(op, "/") == 0) return l / r;
  if (strcmp(op, ">") == 0) return l > r;
  if (strcmp(op, "<") == 0) return l < r;
  if (strcmp(op, ">=") == 0) return l >= r;
  if (strcmp(op, "<=") == 0) return l <= r;
  if (strcmp(op, "==") == 0) return l == r;
  if (strcmp(op, "!=") == 0) return l != r;
  if (strcmp(op, "&&") == 0) return l != 0.0f && r != 0.0f;
  if (strcmp(op, "||") == 0) return l != 0.0f || r != 0.0f;
  return 0.0f;
}

int64_t ora_scan_baseline(const ora_table *t, const char *query, float *out_vals, int64_t *out_idx) {
  char ebuf[1024], cbuf[1024], err[256];
  ora_split_where(query, ebuf, sizeof(ebuf), cbuf, sizeof(cbuf));
  errctx e = {err, sizeof(err), 0};
  node *ex = prep(ebuf, t, &e, 0);
  node *cx = e.failed ? NULL : prep(cbuf, t, &e, 1);
  if (e.failed) { freenode(ex); freenode(cx); return -1; }
  int64_t k = 0;
  for (int64_t i = 0; i < t->n_rows; i++) {
    if (cx && !(eval_faithful(cx, t, i) != 0.0f)) continue;
    out_vals[k] = eval_faithful(ex, t, i);
    out_idx[k] = i;
    k++;
  }
  freenode(ex);
  freenode(cx);
  return k;
}
