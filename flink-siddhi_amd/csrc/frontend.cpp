#include <algorithm>
// SiddhiQL subset -> CompiledApp.  See frontend.h.
//
// Grammar (the part of Siddhi 4.2.40 that the hot path uses — SURVEY.md §7.1):
//   app        := { define | query | partition | ';' }
//   define     := 'define' 'stream' ID '(' ID type {',' ID type} ')'
//                  — the exact DDL emitted by SiddhiStreamSchema.java:36,63-71
//   query      := 'from' input ['select' ('*' | item {',' item})]
//                 ['group' 'by' attr {',' attr}] ['having' expr]
//                 'insert' [('all'|'current'|'expired') 'events'] 'into' ID
//   input      := ID {'[' expr ']'} ['as' ID]
//               | state ('->' state)* ['within' time]          (patterns)
//   state      := ['every'] ID '=' ID ['[' expr ']']
//   partition  := 'partition' 'with' '(' ID 'of' ID {',' ...} ')' 'begin' {query ';'} 'end'
// Expressions: or/and/not, == != < <= > >=, + - * / %, unary -, literals
// (int, long L, float f, double, 'string', true/false), attribute refs
// (x, s.x, s[0].x, s[last].x), aggregates sum/count/avg/min/max.
#include "frontend.h"

#include <cctype>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <set>
#include <stdexcept>

#include "../../include/cep.h"

namespace cep {

const char* type_name(int t) {
  switch (t) {
    case T_INT: return "int";
    case T_LONG: return "long";
    case T_FLOAT: return "float";
    case T_DOUBLE: return "double";
    case T_BOOL: return "bool";
    case T_STRING: return "string";
    default: return "object";
  }
}

namespace {

struct CepError : std::runtime_error {
  int code;
  CepError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

[[noreturn]] void fail(int code, const std::string& m) { throw CepError(code, m); }

// ------------------------------------------------------------------ lexer --
enum TK { TK_ID, TK_KW, TK_NUM, TK_STR, TK_OP, TK_EOF };
struct Token {
  TK k;
  std::string v;
  size_t pos;
};

const std::set<std::string>& keywords() {
  static const std::set<std::string> kw = {
      "define", "stream", "from", "select", "insert", "into", "every",
      "within", "and", "or", "not", "as", "partition", "with", "of",
      "begin", "end", "group", "by", "having", "true", "false", "last",
      "all", "events", "current", "expired", "is", "null", "join", "table",
      "window", "trigger", "function", "aggregation", "on", "unidirectional"};
  return kw;
}

std::string lower(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

std::vector<Token> tokenize(const std::string& s) {
  std::vector<Token> out;
  size_t i = 0, n = s.size();
  while (i < n) {
    char c = s[i];
    if (std::isspace((unsigned char)c)) { ++i; continue; }
    if (c == '-' && i + 1 < n && s[i + 1] == '-') {
      while (i < n && s[i] != '\n') ++i;
      continue;
    }
    if (c == '/' && i + 1 < n && s[i + 1] == '*') {
      size_t e = s.find("*/", i + 2);
      if (e == std::string::npos) fail(CEP_E_PARSE, "unterminated comment");
      i = e + 2;
      continue;
    }
    size_t st = i;
    if (c == '\'' || c == '"') {
      std::string v;
      ++i;
      while (i < n && s[i] != c) {
        if (s[i] == '\\' && i + 1 < n) {
          char e = s[i + 1];
          v += e == 'n' ? '\n' : e == 't' ? '\t' : e;
          i += 2;
        } else {
          v += s[i++];
        }
      }
      if (i >= n) fail(CEP_E_PARSE, "unterminated string literal");
      ++i;
      out.push_back({TK_STR, v, st});
      continue;
    }
    if (std::isdigit((unsigned char)c) ||
        (c == '.' && i + 1 < n && std::isdigit((unsigned char)s[i + 1]))) {
      while (i < n && std::isdigit((unsigned char)s[i])) ++i;
      if (i < n && s[i] == '.') {
        ++i;
        while (i < n && std::isdigit((unsigned char)s[i])) ++i;
      }
      if (i < n && (s[i] == 'e' || s[i] == 'E')) {
        size_t j = i + 1;
        if (j < n && (s[j] == '+' || s[j] == '-')) ++j;
        if (j < n && std::isdigit((unsigned char)s[j])) {
          i = j;
          while (i < n && std::isdigit((unsigned char)s[i])) ++i;
        }
      }
      if (i < n && std::strchr("lLfFdD", s[i]) &&
          !(i + 1 < n && (std::isalnum((unsigned char)s[i + 1]) || s[i + 1] == '_')))
        ++i;
      out.push_back({TK_NUM, s.substr(st, i - st), st});
      continue;
    }
    if (std::isalpha((unsigned char)c) || c == '_') {
      while (i < n && (std::isalnum((unsigned char)s[i]) || s[i] == '_')) ++i;
      std::string v = s.substr(st, i - st);
      std::string lv = lower(v);
      if (keywords().count(lv))
        out.push_back({TK_KW, lv, st});
      else
        out.push_back({TK_ID, v, st});
      continue;
    }
    static const char* two[] = {"->", "==", "!=", "<=", ">="};
    bool matched = false;
    for (const char* t : two) {
      if (s.compare(i, 2, t) == 0) {
        out.push_back({TK_OP, t, st});
        i += 2;
        matched = true;
        break;
      }
    }
    if (matched) continue;
    if (std::strchr("<>+-*/%()[],;=.#:@?", c)) {
      out.push_back({TK_OP, std::string(1, c), st});
      ++i;
      continue;
    }
    fail(CEP_E_PARSE, std::string("unexpected character '") + c + "' at " +
                          std::to_string(i));
  }
  out.push_back({TK_EOF, "", n});
  return out;
}

// -------------------------------------------------------------------- AST --
struct Expr;
using ExprP = std::shared_ptr<Expr>;
struct Expr {
  enum K { CONST, ATTR, BIN, NOT, NEG, CALL } k;
  std::string op;            // BIN operator / CALL name
  std::vector<ExprP> args;
  int vtype = -1;            // CONST type
  uint64_t bits = 0;         // CONST value bits
  std::string sval;          // CONST string
  std::string ref;           // ATTR stream/alias qualifier ("" = none)
  int idx = -1;              // ATTR s[i] index; -2 = last
  std::string name;          // ATTR attribute name
  int t = -1;                // bound type
  // binding
  int state = -1;            // pattern state index of ATTR
  int col = -1;              // raw column index of ATTR
  int out = -1;              // output attribute index (HAVING)
  int agg = -1;              // aggregate slot (CALL)
};

struct State {
  bool every = false;
  std::string alias, stream;
  ExprP cond;
  int min_count = 1, max_count = 1;
};

struct SelItem {
  ExprP e;
  std::string name;
};

struct QueryAst {
  bool single = true;
  bool sequence = false;
  std::string stream, alias;
  std::vector<ExprP> filters;
  std::vector<State> states;
  int64_t within = -1;
  bool select_all = true;
  std::vector<SelItem> select;
  std::vector<ExprP> group_by;
  ExprP having;
  std::string out;
  bool partitioned = false;
  std::map<std::string, std::string> partition;  // stream -> key attr
};

int64_t time_unit_ms(const std::string& u) {
  static const std::map<std::string, int64_t> m = {
      {"millisec", 1}, {"millisecond", 1}, {"milliseconds", 1},
      {"millisecs", 1}, {"ms", 1}, {"sec", 1000}, {"secs", 1000},
      {"second", 1000}, {"seconds", 1000}, {"min", 60000}, {"mins", 60000},
      {"minute", 60000}, {"minutes", 60000}, {"hour", 3600000},
      {"hours", 3600000}, {"day", 86400000}, {"days", 86400000},
      {"week", 604800000}, {"weeks", 604800000}, {"month", 2630000000LL},
      {"months", 2630000000LL}, {"year", 31556900000LL},
      {"years", 31556900000LL}};
  auto it = m.find(lower(u));
  return it == m.end() ? -1 : it->second;
}

class Parser {
 public:
  explicit Parser(const std::string& text) : toks_(tokenize(text)) {}

  void parse(std::vector<StreamSchema>* streams, std::vector<QueryAst>* qs) {
    while (peek().k != TK_EOF) {
      if (accept(TK_OP, ";")) continue;
      while (peek().k == TK_OP && peek().v == "@") skip_annotation();
      const Token& t = peek();
      if (t.k == TK_KW && t.v == "define") {
        next();
        if (!(peek().k == TK_KW && peek().v == "stream"))
          fail(CEP_E_UNSUPPORTED, "only 'define stream' is supported (got define " +
                                      peek().v + ")");
        next();
        StreamSchema sd;
        sd.id = ident();
        expect(TK_OP, "(");
        while (true) {
          AttrDef a;
          Token nt = next();
          if (nt.k != TK_ID && nt.k != TK_KW) fail(CEP_E_PARSE, "attribute name expected");
          a.name = nt.v;
          Token tt = next();
          std::string tn = lower(tt.v);
          if (tn == "int") a.type = T_INT;
          else if (tn == "long") a.type = T_LONG;
          else if (tn == "float") a.type = T_FLOAT;
          else if (tn == "double") a.type = T_DOUBLE;
          else if (tn == "bool" || tn == "boolean") a.type = T_BOOL;
          else if (tn == "string") a.type = T_STRING;
          else if (tn == "object") a.type = T_OBJECT;
          else fail(CEP_E_PARSE, "unknown attribute type '" + tt.v + "'");
          if (sd.index(a.name) >= 0) fail(CEP_E_PARSE, "duplicate attribute " + a.name);
          sd.attrs.push_back(a);
          if (accept(TK_OP, ")")) break;
          expect(TK_OP, ",");
        }
        for (auto& s : *streams)
          if (s.id == sd.id)
            fail(CEP_E_DUPLICATED_STREAM, "stream " + sd.id + " already defined");
        streams->push_back(sd);
      } else if (t.k == TK_KW && t.v == "from") {
        qs->push_back(query());
      } else if (t.k == TK_KW && t.v == "partition") {
        partition(qs);
      } else if (t.k == TK_KW && (t.v == "define" || t.v == "table" ||
                                  t.v == "trigger" || t.v == "function" ||
                                  t.v == "aggregation" || t.v == "window")) {
        fail(CEP_E_UNSUPPORTED, "unsupported definition: " + t.v);
      } else {
        fail(CEP_E_PARSE, "unexpected '" + t.v + "' at " + std::to_string(t.pos));
      }
    }
  }

 private:
  std::vector<Token> toks_;
  size_t i_ = 0;

  const Token& peek(size_t k = 0) const {
    return toks_[std::min(i_ + k, toks_.size() - 1)];
  }
  Token next() { return toks_[i_ < toks_.size() - 1 ? i_++ : i_]; }
  bool accept(TK k, const char* v = nullptr) {
    const Token& t = peek();
    if (t.k == k && (!v || t.v == v)) {
      ++i_;
      return true;
    }
    return false;
  }
  void expect(TK k, const char* v) {
    if (!accept(k, v))
      fail(CEP_E_PARSE, std::string("expected '") + (v ? v : "?") + "' at " +
                            std::to_string(peek().pos) + ", got '" + peek().v + "'");
  }
  std::string ident() {
    const Token& t = peek();
    if (t.k != TK_ID)
      fail(CEP_E_PARSE, "identifier expected at " + std::to_string(t.pos) +
                            ", got '" + t.v + "'");
    ++i_;
    return t.v;
  }
  void skip_annotation() {
    expect(TK_OP, "@");
    next();
    if (accept(TK_OP, ":")) next();
    if (accept(TK_OP, "(")) {
      int depth = 1;
      while (depth) {
        Token t = next();
        if (t.k == TK_EOF) fail(CEP_E_PARSE, "unterminated annotation");
        if (t.k == TK_OP && t.v == "(") ++depth;
        if (t.k == TK_OP && t.v == ")") --depth;
      }
    }
  }

  void partition(std::vector<QueryAst>* qs) {
    expect(TK_KW, "partition");
    expect(TK_KW, "with");
    expect(TK_OP, "(");
    std::map<std::string, std::string> keys;
    while (true) {
      std::string attr = ident();
      if (peek().k == TK_OP && (peek().v == "<" || peek().v == ">" || peek().v == "=="))
        fail(CEP_E_UNSUPPORTED, "range partitions are not supported");
      expect(TK_KW, "of");
      std::string sid = ident();
      keys[sid] = attr;
      if (accept(TK_OP, ")")) break;
      expect(TK_OP, ",");
    }
    expect(TK_KW, "begin");
    while (!accept(TK_KW, "end")) {
      if (accept(TK_OP, ";")) continue;
      if (peek().k == TK_EOF) fail(CEP_E_PARSE, "partition without 'end'");
      QueryAst q = query();
      q.partitioned = true;
      q.partition = keys;
      qs->push_back(q);
    }
  }

  bool is_state_start() const {
    if (peek().k == TK_KW && peek().v == "every") return true;
    return peek().k == TK_ID && peek(1).k == TK_OP && peek(1).v == "=";
  }

  QueryAst query() {
    expect(TK_KW, "from");
    QueryAst q;
    if (!is_state_start()) {
      q.single = true;
      q.stream = ident();
      while (true) {
        if (accept(TK_OP, "[")) {
          q.filters.push_back(expr());
          expect(TK_OP, "]");
        } else if (peek().k == TK_OP && peek().v == "#") {
          fail(CEP_E_UNSUPPORTED, "windows / stream functions are not supported");
        } else {
          break;
        }
      }
      if (accept(TK_KW, "as")) q.alias = ident();
      if ((peek().k == TK_KW && (peek().v == "join" || peek().v == "unidirectional")) ||
          (peek().k == TK_ID && (lower(peek().v) == "left" || lower(peek().v) == "right" ||
                                 lower(peek().v) == "full" || lower(peek().v) == "inner" ||
                                 lower(peek().v) == "outer")))
        fail(CEP_E_UNSUPPORTED, "joins are not supported");
    } else {
      q.single = false;
      q.states.push_back(state());
      std::string sep;
      while (peek().k == TK_OP && (peek().v == "->" || peek().v == ",")) {
        std::string s = next().v;
        if (sep.empty()) sep = s;
        else if (sep != s) fail(CEP_E_UNSUPPORTED, "mixed '->' and ',' is not supported");
        q.states.push_back(state());
      }
      q.sequence = (sep == ",");
      if (accept(TK_KW, "within")) q.within = time_const();
    }
    if (accept(TK_KW, "select")) {
      if (accept(TK_OP, "*")) {
        q.select_all = true;
      } else {
        q.select_all = false;
        while (true) {
          SelItem it;
          it.e = expr();
          if (accept(TK_KW, "as")) {
            it.name = ident();
          } else if (it.e->k == Expr::ATTR) {
            it.name = it.e->name;
          } else {
            fail(CEP_E_PARSE, "select expression requires an 'as' name");
          }
          q.select.push_back(it);
          if (!accept(TK_OP, ",")) break;
        }
      }
    }
    if (accept(TK_KW, "group")) {
      expect(TK_KW, "by");
      while (true) {
        q.group_by.push_back(primary());
        if (!accept(TK_OP, ",")) break;
      }
    }
    if (accept(TK_KW, "having")) q.having = expr();
    expect(TK_KW, "insert");
    if (peek().k == TK_KW &&
        (peek().v == "all" || peek().v == "current" || peek().v == "expired")) {
      next();
      expect(TK_KW, "events");
    }
    expect(TK_KW, "into");
    q.out = ident();
    return q;
  }

  int64_t time_const() {
    int64_t total = 0;
    bool got = false;
    while (peek().k == TK_NUM) {
      std::string n = next().v;
      while (!n.empty() && (n.back() == 'l' || n.back() == 'L')) n.pop_back();
      if (peek().k != TK_ID) fail(CEP_E_PARSE, "time unit expected");
      int64_t u = time_unit_ms(next().v);
      if (u < 0) fail(CEP_E_PARSE, "unknown time unit");
      total += (int64_t)(std::stod(n) * (double)u);
      got = true;
    }
    if (!got) fail(CEP_E_PARSE, "time constant expected after 'within'");
    return total;
  }

  State state() {
    State s;
    s.every = accept(TK_KW, "every");
    s.alias = ident();
    expect(TK_OP, "=");
    s.stream = ident();
    if (accept(TK_OP, "[")) {
      s.cond = expr();
      expect(TK_OP, "]");
    }
    if (accept(TK_OP, "+")) { s.min_count = 1; s.max_count = -1; }
    else if (accept(TK_OP, "*")) { s.min_count = 0; s.max_count = -1; }
    else if (accept(TK_OP, "?")) { s.min_count = 0; s.max_count = 1; }
    else if (peek().k == TK_OP && peek().v == "<" && peek(1).k == TK_NUM) {
      next();
      s.min_count = std::stoi(next().v);
      s.max_count = s.min_count;
      if (accept(TK_OP, ":")) {
        s.max_count = -1;
        if (peek().k == TK_NUM) s.max_count = std::stoi(next().v);
      }
      expect(TK_OP, ">");
    }
    return s;
  }

  ExprP mk(Expr::K k) {
    auto e = std::make_shared<Expr>();
    e->k = k;
    return e;
  }
  ExprP bin(const std::string& op, ExprP a, ExprP b) {
    auto e = mk(Expr::BIN);
    e->op = op;
    e->args = {a, b};
    return e;
  }
  ExprP expr() {
    ExprP e = and_expr();
    while (accept(TK_KW, "or")) e = bin("or", e, and_expr());
    return e;
  }
  ExprP and_expr() {
    ExprP e = not_expr();
    while (accept(TK_KW, "and")) e = bin("and", e, not_expr());
    return e;
  }
  ExprP not_expr() {
    if (accept(TK_KW, "not")) {
      auto e = mk(Expr::NOT);
      e->args = {not_expr()};
      return e;
    }
    return cmp_expr();
  }
  ExprP cmp_expr() {
    ExprP e = add_expr();
    const Token& t = peek();
    if (t.k == TK_OP && (t.v == "==" || t.v == "!=" || t.v == "<" || t.v == "<=" ||
                         t.v == ">" || t.v == ">=")) {
      std::string op = next().v;
      e = bin(op, e, add_expr());
    }
    return e;
  }
  ExprP add_expr() {
    ExprP e = mul_expr();
    while (peek().k == TK_OP && (peek().v == "+" || peek().v == "-")) {
      std::string op = next().v;
      e = bin(op, e, mul_expr());
    }
    return e;
  }
  ExprP mul_expr() {
    ExprP e = unary();
    while (peek().k == TK_OP && (peek().v == "*" || peek().v == "/" || peek().v == "%")) {
      std::string op = next().v;
      e = bin(op, e, unary());
    }
    return e;
  }
  ExprP unary() {
    if (accept(TK_OP, "-")) {
      ExprP in = unary();
      if (in->k == Expr::CONST && (in->vtype == T_INT || in->vtype == T_LONG)) {
        int64_t v = -(int64_t)in->bits;
        if (in->vtype == T_INT) v = (int32_t)(uint32_t)v;
        in->bits = (uint64_t)v;
        return in;
      }
      if (in->k == Expr::CONST && in->vtype == T_DOUBLE) {
        double d;
        std::memcpy(&d, &in->bits, 8);
        d = -d;
        std::memcpy(&in->bits, &d, 8);
        return in;
      }
      if (in->k == Expr::CONST && in->vtype == T_FLOAT) {
        float f;
        uint32_t u = (uint32_t)in->bits;
        std::memcpy(&f, &u, 4);
        f = -f;
        std::memcpy(&u, &f, 4);
        in->bits = u;
        return in;
      }
      auto e = mk(Expr::NEG);
      e->args = {in};
      return e;
    }
    return primary();
  }
  ExprP number(const std::string& s) {
    auto e = mk(Expr::CONST);
    char suf = (char)std::tolower((unsigned char)s.back());
    bool fp = s.find_first_of(".eE") != std::string::npos && suf != 'l';
    if (suf == 'l') {
      e->vtype = T_LONG;
      e->bits = (uint64_t)std::stoll(s.substr(0, s.size() - 1));
    } else if (suf == 'f') {
      e->vtype = T_FLOAT;
      float f = std::stof(s.substr(0, s.size() - 1));
      uint32_t u;
      std::memcpy(&u, &f, 4);
      e->bits = u;
    } else if (suf == 'd' || fp) {
      e->vtype = T_DOUBLE;
      double d = std::stod(suf == 'd' ? s.substr(0, s.size() - 1) : s);
      std::memcpy(&e->bits, &d, 8);
    } else {
      long long v = std::stoll(s);
      if (v > 0x7fffffffLL) fail(CEP_E_PARSE, "int literal out of range: " + s);
      e->vtype = T_INT;
      e->bits = (uint64_t)(int64_t)(int32_t)v;
    }
    return e;
  }
  ExprP primary() {
    const Token& t = peek();
    if (accept(TK_OP, "(")) {
      ExprP e = expr();
      expect(TK_OP, ")");
      return e;
    }
    if (t.k == TK_NUM) return number(next().v);
    if (t.k == TK_STR) {
      auto e = mk(Expr::CONST);
      e->vtype = T_STRING;
      e->sval = next().v;
      return e;
    }
    if (t.k == TK_KW && (t.v == "true" || t.v == "false")) {
      auto e = mk(Expr::CONST);
      e->vtype = T_BOOL;
      e->bits = next().v == "true";
      return e;
    }
    if (t.k == TK_ID) {
      std::string name = next().v;
      if (peek().k == TK_OP && peek().v == ":")
        fail(CEP_E_UNSUPPORTED, "extension functions are not supported (" + name + ")");
      if (accept(TK_OP, "(")) {
        auto e = mk(Expr::CALL);
        e->op = lower(name);
        if (!accept(TK_OP, ")")) {
          while (true) {
            e->args.push_back(expr());
            if (accept(TK_OP, ")")) break;
            expect(TK_OP, ",");
          }
        }
        return e;
      }
      auto e = mk(Expr::ATTR);
      if (peek().k == TK_OP && peek().v == "[") {
        next();
        if (accept(TK_KW, "last")) {
          e->idx = -2;
        } else {
          if (peek().k != TK_NUM) fail(CEP_E_PARSE, "index expected");
          e->idx = std::stoi(next().v);
        }
        expect(TK_OP, "]");
        if (!(peek().k == TK_OP && peek().v == "."))
          fail(CEP_E_PARSE, "indexed reference needs an attribute");
      }
      if (accept(TK_OP, ".")) {
        e->ref = name;
        Token at = next();
        if (at.k != TK_ID && at.k != TK_KW) fail(CEP_E_PARSE, "attribute expected");
        e->name = at.v;
      } else {
        e->name = name;
      }
      return e;
    }
    fail(CEP_E_PARSE, "unexpected '" + t.v + "' at " + std::to_string(t.pos));
  }
};

// ------------------------------------------------------------ binding -----
bool numeric(int t) { return t == T_INT || t == T_LONG || t == T_FLOAT || t == T_DOUBLE; }
int rank(int t) { return t == T_INT ? 0 : t == T_LONG ? 1 : t == T_FLOAT ? 2 : 3; }
int promote(int a, int b) {
  if (!numeric(a) || !numeric(b))
    fail(CEP_E_PARSE, std::string("arithmetic on non-numeric types ") + type_name(a) +
                          ", " + type_name(b));
  return rank(a) >= rank(b) ? a : b;
}

// Resolution context for attribute references.
struct Ctx {
  enum Mode { SINGLE, PATTERN, HAVING } mode = SINGLE;
  const StreamSchema* single = nullptr;
  std::string single_id, single_alias;
  std::vector<const StreamSchema*> states;   // pattern: schema per state
  std::vector<std::string> aliases;
  int cur_state = -1;                         // condition being compiled (-1 select)
  const std::vector<OutItem>* outs = nullptr; // HAVING: output attributes
  bool allow_aggs = false;
  std::vector<ExprP>* agg_calls = nullptr;
};

void bind_expr(const ExprP& e, Ctx& c, CompiledApp* app) {
  switch (e->k) {
    case Expr::CONST:
      e->t = e->vtype;
      if (e->vtype == T_STRING) {
        int id = -1;
        for (size_t i = 0; i < app->strings.size(); ++i)
          if (app->strings[i] == e->sval) id = (int)i;
        if (id < 0) {
          id = (int)app->strings.size();
          app->strings.push_back(e->sval);
        }
        e->bits = (uint64_t)(uint32_t)id;
      }
      return;
    case Expr::ATTR: {
      if (c.mode == Ctx::HAVING && e->ref.empty() && c.outs) {
        for (size_t i = 0; i < c.outs->size(); ++i)
          if ((*c.outs)[i].name == e->name) {
            e->out = (int)i;
            e->t = (*c.outs)[i].type;
            return;
          }
      }
      if (c.mode == Ctx::SINGLE || (c.mode == Ctx::HAVING && c.single)) {
        if (!e->ref.empty() && e->ref != c.single_id && e->ref != c.single_alias)
          fail(CEP_E_PARSE, "unknown stream reference " + e->ref);
        int i = c.single->index(e->name);
        if (i < 0) fail(CEP_E_PARSE, "attribute " + e->name + " not in stream " + c.single->id);
        e->col = i;
        e->t = c.single->attrs[i].type;
        return;
      }
      // pattern
      int st = -1;
      if (e->ref.empty()) {
        if (c.cur_state < 0)
          fail(CEP_E_PARSE, "unqualified attribute " + e->name + " in pattern select");
        st = c.cur_state;
      } else {
        for (size_t k = 0; k < c.aliases.size(); ++k)
          if (c.aliases[k] == e->ref) st = (int)k;
        if (st < 0) fail(CEP_E_PARSE, "unknown reference " + e->ref);
        if (c.cur_state >= 0 && st > c.cur_state)
          fail(CEP_E_PARSE, "reference to a later state " + e->ref);
      }
      int i = c.states[st]->index(e->name);
      if (i < 0) fail(CEP_E_PARSE, "attribute " + e->name + " not in stream " + c.states[st]->id);
      e->state = st;
      e->col = i;
      e->t = c.states[st]->attrs[i].type;
      return;
    }
    case Expr::NOT:
      bind_expr(e->args[0], c, app);
      if (e->args[0]->t != T_BOOL) fail(CEP_E_PARSE, "'not' requires a bool operand");
      e->t = T_BOOL;
      return;
    case Expr::NEG:
      bind_expr(e->args[0], c, app);
      if (!numeric(e->args[0]->t)) fail(CEP_E_PARSE, "negation of a non-numeric value");
      e->t = e->args[0]->t;
      return;
    case Expr::BIN: {
      bind_expr(e->args[0], c, app);
      bind_expr(e->args[1], c, app);
      int a = e->args[0]->t, b = e->args[1]->t;
      const std::string& op = e->op;
      if (op == "and" || op == "or") {
        if (a != T_BOOL || b != T_BOOL) fail(CEP_E_PARSE, "'" + op + "' requires bool operands");
        e->t = T_BOOL;
      } else if (op == "==" || op == "!=") {
        if (!(numeric(a) && numeric(b)) && a != b)
          fail(CEP_E_PARSE, std::string("cannot compare ") + type_name(a) + " with " + type_name(b));
        if (a == T_OBJECT) fail(CEP_E_UNSUPPORTED, "object comparison");
        e->t = T_BOOL;
      } else if (op == "<" || op == "<=" || op == ">" || op == ">=") {
        if (!numeric(a) || !numeric(b)) fail(CEP_E_PARSE, "ordering comparison of non-numeric values");
        e->t = T_BOOL;
      } else {
        e->t = promote(a, b);
      }
      return;
    }
    case Expr::CALL: {
      const std::string& f = e->op;
      if (f != "sum" && f != "count" && f != "avg" && f != "min" && f != "max")
        fail(CEP_E_UNSUPPORTED, "function " + f + " is not supported");
      if (!c.allow_aggs) fail(CEP_E_PARSE, "aggregate " + f + " outside select");
      if (f == "count") {
        e->t = T_LONG;
      } else {
        if (e->args.size() != 1) fail(CEP_E_PARSE, f + " takes one argument");
        bool save = c.allow_aggs;
        c.allow_aggs = false;
        bind_expr(e->args[0], c, app);
        c.allow_aggs = save;
        int at = e->args[0]->t;
        if (!numeric(at)) fail(CEP_E_PARSE, f + " of a non-numeric value");
        if (f == "sum") e->t = (at == T_INT || at == T_LONG) ? T_LONG : T_DOUBLE;
        else if (f == "avg") e->t = T_DOUBLE;
        else e->t = at;
      }
      if (c.agg_calls) {
        e->agg = (int)c.agg_calls->size();
        c.agg_calls->push_back(e);
      }
      return;
    }
  }
}

bool has_call(const ExprP& e) {
  if (e->k == Expr::CALL) return true;
  for (auto& a : e->args)
    if (has_call(a)) return true;
  return false;
}

void collect_refs(const ExprP& e, std::vector<std::pair<int, int>>* refs) {
  if (e->k == Expr::ATTR && e->state >= 0) refs->push_back({e->state, e->col});
  for (auto& a : e->args) collect_refs(a, refs);
}

// ----------------------------------------------------------- code gen -----
// Attribute load strategy during code generation.
struct Loader {
  // returns (op, imm) to load the attribute e
  std::function<std::pair<uint8_t, uint32_t>(const Expr&)> load;
};

class CodeGen {
 public:
  CodeGen(CompiledApp* app, const Loader& ld) : app_(app), ld_(ld) {}

  Prog compile(const ExprP& e) {
    Prog p;
    p.off = (int)app_->code.size();
    gen(e, 0);
    app_->code.push_back({OP_END, 0, 0, 0, 0});
    p.len = (int)app_->code.size() - p.off;
    p.res = 0;
    p.type = e->t;
    if (p.len > kMaxProgLen) fail(CEP_E_UNSUPPORTED, "expression too long");
    return p;
  }

 private:
  CompiledApp* app_;
  const Loader& ld_;

  void emit(uint8_t op, int dst, int a, int b, uint32_t imm) {
    app_->code.push_back({op, (uint8_t)dst, (uint8_t)a, (uint8_t)b, imm});
  }
  uint32_t konst(uint64_t v) {
    for (size_t i = 0; i < app_->konst.size(); ++i)
      if (app_->konst[i] == v) return (uint32_t)i;
    app_->konst.push_back(v);
    return (uint32_t)(app_->konst.size() - 1);
  }
  void cvt(int r, int from, int to) {
    if (from != to) emit(OP_CVT, r, r, 0, (uint32_t)((from << 8) | to));
  }
  void gen(const ExprP& e, int r) {
    if (r >= kMaxRegs) fail(CEP_E_UNSUPPORTED, "expression nests too deeply");
    switch (e->k) {
      case Expr::CONST:
        emit(OP_LDK, r, 0, 0, konst(e->bits));
        return;
      case Expr::ATTR: {
        auto [op, imm] = ld_.load(*e);
        emit(op, r, 0, (uint8_t)e->t, imm);
        return;
      }
      case Expr::CALL: {
        if (e->agg < 0) fail(CEP_E_PARSE, "unexpected aggregate");
        emit(OP_LDAGG, r, 0, (uint8_t)e->t, (uint32_t)e->agg);
        return;
      }
      case Expr::NOT:
        gen(e->args[0], r);
        emit(OP_NOT, r, r, 0, 0);
        return;
      case Expr::NEG:
        gen(e->args[0], r);
        emit(OP_NEG, r, r, 0, (uint32_t)e->t);
        return;
      case Expr::BIN: {
        const std::string& op = e->op;
        gen(e->args[0], r);
        gen(e->args[1], r + 1);
        int a = e->args[0]->t, b = e->args[1]->t;
        if (op == "and") { emit(OP_AND, r, r, r + 1, 0); return; }
        if (op == "or") { emit(OP_OR, r, r, r + 1, 0); return; }
        int ct;
        if (numeric(a) && numeric(b)) {
          ct = promote(a, b);
          cvt(r, a, ct);
          cvt(r + 1, b, ct);
        } else {
          ct = (a == T_BOOL || a == T_STRING) ? T_INT : a;   // ids / 0-1 compare as int
        }
        uint8_t o;
        if (op == "==") o = OP_EQ;
        else if (op == "!=") o = OP_NE;
        else if (op == "<") o = OP_LT;
        else if (op == "<=") o = OP_LE;
        else if (op == ">") o = OP_GT;
        else if (op == ">=") o = OP_GE;
        else if (op == "+") o = OP_ADD;
        else if (op == "-") o = OP_SUB;
        else if (op == "*") o = OP_MUL;
        else if (op == "/") o = OP_DIV;
        else o = OP_MOD;
        emit(o, r, r, r + 1, (uint32_t)ct);
        return;
      }
    }
  }
};

// ---- interpreter-free predicate lowering (plan.h TermList) ----------------
uint64_t host_convert(uint64_t v, int from, int to) {
  if (from == to || to == T_LONG) return v;
  if (to == T_FLOAT) {
    float f = from == T_INT ? (float)(int32_t)v : from == T_LONG ? (float)(int64_t)v : 0.f;
    if (from == T_FLOAT) return v;
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
  }
  if (to == T_DOUBLE) {
    double d;
    if (from == T_INT) d = (double)(int32_t)v;
    else if (from == T_LONG) d = (double)(int64_t)v;
    else if (from == T_FLOAT) {
      float f;
      uint32_t u = (uint32_t)v;
      std::memcpy(&f, &u, 4);
      d = f;
    } else return v;
    uint64_t r;
    std::memcpy(&r, &d, 8);
    return r;
  }
  return v;
}

uint8_t cmp_op(const std::string& op, bool flip) {
  if (op == "==") return OP_EQ;
  if (op == "!=") return OP_NE;
  if (op == "<") return flip ? OP_GT : OP_LT;
  if (op == "<=") return flip ? OP_GE : OP_LE;
  if (op == ">") return flip ? OP_LT : OP_GT;
  return flip ? OP_LE : OP_GE;
}

uint8_t arith_op(const std::string& op) {
  if (op == "+") return OP_ADD;
  if (op == "-") return OP_SUB;
  if (op == "*") return OP_MUL;
  if (op == "/") return OP_DIV;
  if (op == "%") return OP_MOD;
  return 0;
}

bool is_col(const ExprP& e) { return e->k == Expr::ATTR && e->col >= 0 && e->out < 0; }

bool lower_atom(const ExprP& e, Term* t) {
  ExprP lhs, rhs;
  bool flip = false;
  if (e->k == Expr::ATTR && e->t == T_BOOL && is_col(e)) {   // `[flag]`
    t->col = e->col; t->coltype = T_BOOL; t->aop = 0; t->atype = T_BOOL; t->aconst = 0;
    t->cop = OP_EQ; t->ctype = T_INT; t->cconst = 1;
    return true;
  }
  if (e->k != Expr::BIN) return false;
  const std::string& op = e->op;
  if (!(op == "==" || op == "!=" || op == "<" || op == "<=" || op == ">" || op == ">=")) return false;
  if (e->args[1]->k == Expr::CONST) { lhs = e->args[0]; rhs = e->args[1]; }
  else if (e->args[0]->k == Expr::CONST) { lhs = e->args[1]; rhs = e->args[0]; flip = true; }
  else return false;
  ExprP col;
  int aop = 0;
  ExprP ak;
  if (is_col(lhs)) col = lhs;
  else if (lhs->k == Expr::BIN && arith_op(lhs->op) && is_col(lhs->args[0]) &&
           lhs->args[1]->k == Expr::CONST) {
    col = lhs->args[0];
    aop = arith_op(lhs->op);
    ak = lhs->args[1];
  } else return false;
  t->col = col->col;
  t->coltype = col->t;
  t->aop = aop;
  if (aop) {
    t->atype = promote(col->t, ak->t);
    t->aconst = host_convert(ak->bits, ak->t, t->atype);
  } else {
    t->atype = col->t;
    t->aconst = 0;
  }
  const int at = aop ? t->atype : col->t;
  if (numeric(at) && numeric(rhs->t)) {
    t->ctype = promote(at, rhs->t);
  } else if (at == rhs->t && (at == T_STRING || at == T_BOOL)) {
    t->ctype = T_INT;
  } else {
    return false;
  }
  t->cconst = numeric(rhs->t) ? host_convert(rhs->bits, rhs->t, t->ctype) : rhs->bits;
  t->cop = cmp_op(op, flip);
  return true;
}

void flatten(const ExprP& e, const std::string& op, std::vector<ExprP>* out) {
  if (e->k == Expr::BIN && e->op == op) {
    flatten(e->args[0], op, out);
    flatten(e->args[1], op, out);
  } else {
    out->push_back(e);
  }
}

TermList lower_terms(const std::vector<ExprP>& conj) {
  TermList tl;
  if (conj.empty()) return tl;
  std::vector<ExprP> atoms;
  for (auto& c : conj) flatten(c, "and", &atoms);
  bool any = false;
  if (atoms.size() == 1 && atoms[0]->k == Expr::BIN && atoms[0]->op == "or") {
    std::vector<ExprP> ors;
    flatten(atoms[0], "or", &ors);
    atoms = ors;
    any = true;
  }
  if ((int)atoms.size() > kMaxTerms) return tl;
  TermList r;
  r.any = any ? 1 : 0;
  r.n = 0;
  for (auto& a : atoms) {
    if (!lower_atom(a, &r.t[r.n])) return tl;
    ++r.n;
  }
  return r;
}

// Plain attribute copies bypass the VM in the output projection.
int32_t direct_source(const CompiledApp* app, const Prog& p) {
  if (p.len != 2) return SRC_VM;
  const Ins& in = app->code[p.off];
  if (app->code[p.off + 1].op != OP_END || in.dst != 0) return SRC_VM;
  if (in.op == OP_LDCAP) return SRC_CAP + (int32_t)in.imm;
  if (in.op == OP_LDCOL) return SRC_REC + (int32_t)in.imm;
  return SRC_VM;
}

Prog compile_and(CompiledApp* app, const std::vector<ExprP>& es, const Loader& ld) {
  if (es.empty()) return Prog{};
  ExprP acc = es[0];
  for (size_t i = 1; i < es.size(); ++i) {
    auto b = std::make_shared<Expr>();
    b->k = Expr::BIN;
    b->op = "and";
    b->args = {acc, es[i]};
    b->t = T_BOOL;
    acc = b;
  }
  CodeGen cg(app, ld);
  return cg.compile(acc);
}

void add_output(CompiledApp* app, const std::string& id, const std::vector<OutItem>& items) {
  StreamSchema od;
  od.id = id;
  for (auto& it : items) od.attrs.push_back({it.name, it.type});
  if (app->input_index(id) >= 0)
    fail(CEP_E_UNSUPPORTED, "inserting into an input stream (query chaining) is not supported");
  int k = app->output_index(id);
  if (k >= 0) {
    const auto& prev = app->outputs[k];
    bool same = prev.attrs.size() == od.attrs.size();
    for (size_t i = 0; same && i < od.attrs.size(); ++i)
      same = prev.attrs[i].name == od.attrs[i].name && prev.attrs[i].type == od.attrs[i].type;
    if (!same) fail(CEP_E_PARSE, "incompatible definitions for output stream " + id);
    return;
  }
  app->outputs.push_back(od);
}

int key_column(const StreamSchema& s, const std::string& attr) {
  int i = s.index(attr);
  if (i < 0) fail(CEP_E_PARSE, "partition attribute " + attr + " not in stream " + s.id);
  int t = s.attrs[i].type;
  if (t != T_INT && t != T_LONG && t != T_STRING)
    fail(CEP_E_UNSUPPORTED, "partition key must be int, long or string");
  return i;
}

// Having over a group-by query: output-attribute references become the
// select expressions they name (same value, recomputed).
ExprP inline_outputs(const ExprP& e, const std::vector<SelItem>& sel) {
  if (e->k == Expr::ATTR && e->out >= 0) return sel[e->out].e;
  auto c = std::make_shared<Expr>(*e);
  for (auto& a : c->args) a = inline_outputs(a, sel);
  return c;
}

// Copy of program p with every OP_LDCOL column index mapped through `word`.
Prog remap_cols(CompiledApp* app, const Prog& p, const std::vector<int>& cols) {
  if (!p.valid()) return p;
  Prog r = p;
  r.off = (int)app->code.size();
  for (int i = 0; i < p.len; ++i) {
    Ins in = app->code[p.off + i];
    if (in.op == OP_LDCOL) {
      int w = -1;
      for (size_t j = 0; j < cols.size(); ++j)
        if (cols[j] == (int)in.imm) w = (int)j;
      in.imm = (uint32_t)w;
    }
    app->code.push_back(in);
  }
  return r;
}

void collect_cols(const CompiledApp* app, const Prog& p, std::vector<int>* cols) {
  if (!p.valid()) return;
  for (int i = 0; i < p.len; ++i) {
    const Ins& in = app->code[p.off + i];
    if (in.op == OP_LDCOL && std::find(cols->begin(), cols->end(), (int)in.imm) == cols->end())
      cols->push_back((int)in.imm);
  }
}

// Device form of a group-by query: the partition pass keeps rows passing the
// filter as records keyed by the group attribute, carrying every column the
// select items, aggregate arguments and having read; the walk runs one lane
// per group over its records in arrival order (running aggregates, having,
// emission).  Programs are remapped so LDCOL c reads carried word c.
void lower_aggregation(CompiledApp* app, Query& q) {
  if ((int)q.aggs.size() > kMaxAggs) fail(CEP_E_UNSUPPORTED, "more than 8 aggregates");
  std::vector<int> cols;
  for (auto& a : q.aggs) {
    if (!a.arg.valid()) continue;
    const Ins& in = app->code[a.arg.off];
    if (a.arg.len != 2 || in.op != OP_LDCOL)
      fail(CEP_E_UNSUPPORTED, "aggregate arguments must be plain attributes on the device");
    collect_cols(app, a.arg, &cols);
  }
  for (auto& it : q.select) collect_cols(app, it.prog, &cols);
  collect_cols(app, q.having, &cols);
  if ((int)cols.size() > kMaxCaps) fail(CEP_E_UNSUPPORTED, "group-by query reads too many attributes");
  q.a_stream = q.in_stream;
  q.b_stream = -1;
  q.f = q.filter;
  q.f_terms = q.filter_terms;
  q.every = true;
  q.key_col_a = q.key_col_b = q.key_col;
  q.rec_cols_a = cols;
  for (auto& a : q.aggs) {
    a.word = a.arg.valid() ? (int)(std::find(cols.begin(), cols.end(), (int)app->code[a.arg.off].imm) -
                                   cols.begin())
                           : -1;
    a.arg_type = a.arg.valid() ? app->code[a.arg.off].b : T_LONG;
  }
  for (auto& it : q.select) {
    const Ins& in = app->code[it.prog.off];
    const bool single = it.prog.len == 2 && in.dst == 0;
    it.prog = remap_cols(app, it.prog, cols);
    it.src = SRC_VM;
    if (single && in.op == OP_LDAGG) it.src = SRC_AGG + (int32_t)in.imm;
    else if (single && in.op == OP_LDCOL && (int)in.imm == q.key_col) it.src = SRC_KEY;
    else if (single && in.op == OP_LDCOL) it.src = SRC_REC + (int32_t)app->code[it.prog.off].imm;
  }
  q.having = remap_cols(app, q.having, cols);
}

void compile_single(CompiledApp* app, QueryAst& q) {
  int si = app->input_index(q.stream);
  if (si < 0) fail(CEP_E_UNDEFINED_STREAM, "stream " + q.stream + " is not defined");
  const StreamSchema& sd = app->inputs[si];
  Query out;
  out.in_stream = si;
  out.out_stream = q.out;
  Ctx c;
  c.mode = Ctx::SINGLE;
  c.single = &sd;
  c.single_id = q.stream;
  c.single_alias = q.alias;
  for (auto& f : q.filters) {
    bind_expr(f, c, app);
    if (f->t != T_BOOL) fail(CEP_E_PARSE, "filter condition must be bool");
  }
  Loader raw{[](const Expr& e) { return std::make_pair((uint8_t)OP_LDCOL, (uint32_t)e.col); }};
  out.filter = compile_and(app, q.filters, raw);
  out.filter_terms = lower_terms(q.filters);
  if (q.select_all) {
    q.select.clear();
    for (auto& a : sd.attrs) {
      SelItem it;
      it.e = std::make_shared<Expr>();
      it.e->k = Expr::ATTR;
      it.e->name = a.name;
      it.name = a.name;
      q.select.push_back(it);
    }
  }
  std::vector<ExprP> calls;
  c.allow_aggs = true;
  c.agg_calls = &calls;
  std::set<std::string> names;
  for (auto& it : q.select) {
    bind_expr(it.e, c, app);
    if (!names.insert(it.name).second) fail(CEP_E_PARSE, "duplicate output attribute " + it.name);
  }
  c.allow_aggs = false;
  c.agg_calls = nullptr;
  for (auto& it : q.select) {
    CodeGen cg(app, raw);
    OutItem oi;
    oi.name = it.name;
    oi.type = it.e->t;
    if (oi.type == T_OBJECT) fail(CEP_E_UNSUPPORTED, "object attributes in select");
    oi.prog = cg.compile(it.e);
    oi.src = direct_source(app, oi.prog);   // SRC_REC + c = input column c
    out.select.push_back(oi);
  }
  for (auto& call : calls) {
    AggSpec a;
    const std::string& f = call->op;
    a.fn = f == "sum" ? AGG_SUM : f == "count" ? AGG_COUNT : f == "avg" ? AGG_AVG
         : f == "min" ? AGG_MIN : AGG_MAX;
    a.out_type = call->t;
    a.arg_type = call->args.empty() ? T_LONG : call->args[0]->t;
    if (!call->args.empty()) {
      CodeGen cg(app, raw);
      a.arg = cg.compile(call->args[0]);
    }
    out.aggs.push_back(a);
  }
  if (q.partitioned) {
    auto it = q.partition.find(q.stream);
    if (it == q.partition.end())
      fail(CEP_E_PARSE, "stream " + q.stream + " is not partitioned in the enclosing partition");
    out.part_col = key_column(sd, it->second);
  }
  for (auto& g : q.group_by) {
    if (g->k != Expr::ATTR) fail(CEP_E_PARSE, "group by takes attributes");
    bind_expr(g, c, app);
    CodeGen cg(app, raw);
    out.group_progs.push_back(cg.compile(g));
    out.group_cols.push_back(g->col);
  }
  bool agg = !out.aggs.empty();
  // group by without aggregates: Siddhi's selector evaluates each event's
  // projection as it comes (no group state), so it is a plain projection; the
  // attributes still name the plan's routing keys (cep_plan_partition_keys)
  if (!agg) out.group_progs.clear();
  if (agg) {
    out.kind = Q_AGG;
    if (q.group_by.size() > 1)
      fail(CEP_E_UNSUPPORTED, "group by over more than one attribute");
    if (q.group_by.size() == 1) {
      out.key_col = q.group_by[0]->col;
      int kt = sd.attrs[out.key_col].type;
      if (kt != T_INT && kt != T_LONG && kt != T_STRING)
        fail(CEP_E_UNSUPPORTED, "group by key must be int, long or string");
      if (out.part_col >= 0 && out.part_col != out.key_col)
        fail(CEP_E_UNSUPPORTED, "group by a different attribute than the partition key");
    } else {
      out.key_col = out.part_col;   // one group per partition key (or global)
    }
  }
  if (q.having) {
    Ctx h;
    h.mode = Ctx::HAVING;
    h.single = &sd;
    h.single_id = q.stream;
    h.single_alias = q.alias;
    h.outs = &out.select;
    bind_expr(q.having, h, app);
    if (q.having->t != T_BOOL) fail(CEP_E_PARSE, "having condition must be bool");
    // `<output attribute> op constant` (either order): the multi-query walk
    // compares the item's value without the interpreter
    out.having_simple = false;
    {
      const ExprP& hx = q.having;
      if (hx->k == Expr::BIN && hx->args.size() == 2) {
        const std::string& op = hx->op;
        const bool cmp = op == "==" || op == "!=" || op == "<" || op == "<=" || op == ">" || op == ">=";
        ExprP item, k;
        bool flip = false;
        if (hx->args[1]->k == Expr::CONST) { item = hx->args[0]; k = hx->args[1]; }
        else if (hx->args[0]->k == Expr::CONST) { item = hx->args[1]; k = hx->args[0]; flip = true; }
        if (cmp && item && item->k == Expr::ATTR && item->out >= 0 && numeric(item->t) && numeric(k->t)) {
          out.having_simple = true;
          out.having_item = item->out;
          out.having_ctype = promote(item->t, k->t);
          out.having_cconst = host_convert(k->bits, k->t, out.having_ctype);
          out.having_cop = cmp_op(op, flip);
        }
      }
    }
    if (agg) {
      // output attributes inline as their select expressions, so the device
      // evaluates having over aggregates and event columns only
      ExprP hx = inline_outputs(q.having, q.select);
      CodeGen cg(app, raw);
      out.having = cg.compile(hx);
    } else {
      Loader hl{[](const Expr& e) {
        if (e.out >= 0) return std::make_pair((uint8_t)OP_LDOUT, (uint32_t)e.out);
        return std::make_pair((uint8_t)OP_LDCOL, (uint32_t)e.col);
      }};
      CodeGen cg(app, hl);
      out.having = cg.compile(q.having);
    }
  }
  if (agg) lower_aggregation(app, out);
  add_output(app, q.out, out.select);
  app->queries.push_back(out);
}

int index_of(std::vector<int>& v, int x, bool add) {
  for (size_t i = 0; i < v.size(); ++i)
    if (v[i] == x) return (int)i;
  if (!add) return -1;
  v.push_back(x);
  return (int)v.size() - 1;
}

// N-state patterns and sequences (with count states in sequences): one NFA
// lane per key in the walk.  Semantics follow oracle/siddhi_oracle.py
// (_pattern_event / _sequence_event).
void compile_nfa(CompiledApp* app, QueryAst& q) {
  const int n = (int)q.states.size();
  if (n < 1 || n > kMaxStates) fail(CEP_E_UNSUPPORTED, "patterns / sequences of more than 6 states");
  for (int j = 0; j < n; ++j) {
    auto& st = q.states[j];
    if (app->input_index(st.stream) < 0)
      fail(CEP_E_UNDEFINED_STREAM, "stream " + st.stream + " is not defined");
    if (j > 0 && st.every) fail(CEP_E_UNSUPPORTED, "'every' on a non-start state");
    if (!q.sequence && (st.min_count != 1 || st.max_count != 1))
      fail(CEP_E_UNSUPPORTED, "count states in patterns are not supported");
    for (int k = 0; k < j; ++k)
      if (q.states[k].alias == st.alias && !st.alias.empty()) fail(CEP_E_PARSE, "duplicate state alias");
  }
  if (!q.group_by.empty() || q.having) fail(CEP_E_UNSUPPORTED, "group by / having on patterns");
  if (q.select_all) fail(CEP_E_PARSE, "pattern query needs an explicit select");
  Query out;
  out.kind = Q_PATTERN;
  out.nfa = true;
  out.sequence = q.sequence;
  out.out_stream = q.out;
  out.every = q.states[0].every;
  out.within = q.within;
  out.a_stream = app->input_index(q.states[0].stream);
  Ctx c;
  c.mode = Ctx::PATTERN;
  for (auto& st : q.states) {
    c.states.push_back(&app->inputs[app->input_index(st.stream)]);
    c.aliases.push_back(st.alias);
  }
  // bind conditions and select
  for (int j = 0; j < n; ++j) {
    if (!q.states[j].cond) continue;
    c.cur_state = j;
    bind_expr(q.states[j].cond, c, app);
    if (q.states[j].cond->t != T_BOOL) fail(CEP_E_PARSE, "condition must be bool");
  }
  c.cur_state = -1;
  std::set<std::string> names;
  for (auto& it : q.select) {
    if (has_call(it.e)) fail(CEP_E_UNSUPPORTED, "aggregates in pattern select");
    bind_expr(it.e, c, app);
    if (it.e->t == T_OBJECT) fail(CEP_E_UNSUPPORTED, "object attributes in select");
    if (!names.insert(it.name).second) fail(CEP_E_PARSE, "duplicate output attribute " + it.name);
  }
  // partition keys per input stream
  out.key_col_s.assign(app->inputs.size(), -1);
  if (q.partitioned) {
    for (auto& st : q.states) {
      auto it = q.partition.find(st.stream);
      if (it == q.partition.end())
        fail(CEP_E_PARSE, "pattern stream not covered by the enclosing partition");
      const int si = app->input_index(st.stream);
      out.key_col_s[si] = key_column(app->inputs[si], it->second);
    }
  }
  out.key_col_a = out.key_col_b = q.partitioned ? out.key_col_s[out.a_stream] : -1;
  // records carry one column list for every stream (batches mixing streams
  // require identical definitions)
  auto rec_word = [&](int col) { return index_of(out.rec_cols_a, col, true); };
  // captures: (state, index, column); "cur" (-1) in a select means the first event
  auto cap_of = [&](int state, int idx, int col) {
    const int index = idx == -2 ? -1 : (idx < 0 ? 0 : idx);
    const int w = rec_word(col);
    for (size_t i = 0; i < out.ncaps.size(); ++i)
      if (out.ncaps[i].state == state && out.ncaps[i].index == index && out.ncaps[i].word == w)
        return (int)i;
    out.ncaps.push_back({state, index, w});
    return (int)out.ncaps.size() - 1;
  };
  auto key_ref = [&](const ExprP& e) {
    return q.partitioned && e->k == Expr::ATTR && e->state >= 0 &&
           e->col == out.key_col_s[app->input_index(q.states[e->state].stream)];
  };
  std::function<bool(const ExprP&, int)> self_only = [&](const ExprP& e, int j) -> bool {
    if (e->k == Expr::ATTR && (e->state != j || e->idx != -1)) return false;
    for (auto& a : e->args)
      if (!self_only(a, j)) return false;
    return true;
  };
  Loader raw{[](const Expr& e) { return std::make_pair((uint8_t)OP_LDCOL, (uint32_t)e.col); }};
  for (int j = 0; j < n; ++j) {
    Query::NState ns;
    ns.stream = app->input_index(q.states[j].stream);
    ns.min_count = q.states[j].min_count;
    ns.max_count = q.states[j].max_count;
    ns.terms.n = 0;   // no condition: always true
    if (q.states[j].cond) {
      ns.terms.n = -1;
      if (self_only(q.states[j].cond, j)) {
        CodeGen cg(app, raw);
        ns.raw = cg.compile(q.states[j].cond);
        ns.terms = lower_terms({q.states[j].cond});
      } else {
        const int jj = j;
        Loader wl{[&, jj](const Expr& e) {
          if (e.state == jj && e.idx == -1)
            return std::make_pair((uint8_t)OP_LDCOL, (uint32_t)rec_word(e.col));
          return std::make_pair((uint8_t)OP_LDCAP, (uint32_t)cap_of(e.state, e.idx, e.col));
        }};
        CodeGen cg(app, wl);
        ns.walk = cg.compile(q.states[j].cond);
      }
    }
    out.nstates.push_back(ns);
  }
  Loader sl{[&](const Expr& e) {
    return std::make_pair((uint8_t)OP_LDCAP, (uint32_t)cap_of(e.state, e.idx, e.col));
  }};
  for (auto& it : q.select) {
    OutItem oi;
    oi.name = it.name;
    oi.type = it.e->t;
    if (key_ref(it.e)) {
      oi.prog = Prog{};
      oi.src = SRC_KEY;
    } else {
      CodeGen cg(app, sl);
      oi.prog = cg.compile(it.e);
      oi.src = direct_source(app, oi.prog);   // SRC_CAP + i
    }
    out.select.push_back(oi);
  }
  if ((int)out.ncaps.size() > kMaxCaps || (int)out.rec_cols_a.size() > kMaxCaps)
    fail(CEP_E_UNSUPPORTED, "too many captured attributes");
  out.rec_cols_b = out.rec_cols_a;
  add_output(app, q.out, out.select);
  app->queries.push_back(out);
}

// Whether e reads an attribute qualified by `alias` (before binding).
bool refs_alias(const ExprP& e, const std::string& alias) {
  if (!e) return false;
  if (e->k == Expr::ATTR && e->ref == alias) return true;
  for (auto& a : e->args)
    if (refs_alias(a, alias)) return true;
  return false;
}

void compile_pattern(CompiledApp* app, QueryAst& q) {
  bool counts = false;
  for (auto& s : q.states) counts |= s.min_count != 1 || s.max_count != 1;
  if (q.sequence || q.states.size() != 2 || counts) return compile_nfa(app, q);
  // s2's condition reads s1: the N-state walk (its pending lists continue in
  // the pending pool, so no key runs out of slots); CEP_PAIR_WALK=1 keeps the
  // two-state walk (lists of pending_slots)
  static const bool pair_walk = std::getenv("CEP_PAIR_WALK") != nullptr;
  if (!pair_walk && !q.states[0].alias.empty() && refs_alias(q.states[1].cond, q.states[0].alias))
    return compile_nfa(app, q);
  for (auto& s : q.states) {
    if (app->input_index(s.stream) < 0)
      fail(CEP_E_UNDEFINED_STREAM, "stream " + s.stream + " is not defined");
    if (s.min_count != 1 || s.max_count != 1)
      fail(CEP_E_UNSUPPORTED, "count states in patterns are not supported");
  }
  if (q.states[1].every) fail(CEP_E_UNSUPPORTED, "'every' on a non-start state");
  if (q.states[0].alias == q.states[1].alias) fail(CEP_E_PARSE, "duplicate state alias");
  if (!q.group_by.empty() || q.having)
    fail(CEP_E_UNSUPPORTED, "group by / having on patterns");
  if (q.select_all) fail(CEP_E_PARSE, "pattern query needs an explicit select");
  Query out;
  out.kind = Q_PATTERN;
  out.out_stream = q.out;
  out.a_stream = app->input_index(q.states[0].stream);
  out.b_stream = app->input_index(q.states[1].stream);
  out.every = q.states[0].every;
  out.within = q.within;
  const StreamSchema& A = app->inputs[out.a_stream];
  const StreamSchema& B = app->inputs[out.b_stream];
  Ctx c;
  c.mode = Ctx::PATTERN;
  c.states = {&A, &B};
  c.aliases = {q.states[0].alias, q.states[1].alias};
  if (q.states[0].cond) {
    c.cur_state = 0;
    bind_expr(q.states[0].cond, c, app);
    if (q.states[0].cond->t != T_BOOL) fail(CEP_E_PARSE, "condition must be bool");
  }
  std::vector<std::pair<int, int>> grefs;
  if (q.states[1].cond) {
    c.cur_state = 1;
    bind_expr(q.states[1].cond, c, app);
    if (q.states[1].cond->t != T_BOOL) fail(CEP_E_PARSE, "condition must be bool");
    collect_refs(q.states[1].cond, &grefs);
  }
  c.cur_state = -1;
  std::set<std::string> names;
  std::vector<std::pair<int, int>> srefs;
  for (auto& it : q.select) {
    if (has_call(it.e)) fail(CEP_E_UNSUPPORTED, "aggregates in pattern select");
    bind_expr(it.e, c, app);
    if (it.e->t == T_OBJECT) fail(CEP_E_UNSUPPORTED, "object attributes in select");
    if (!names.insert(it.name).second) fail(CEP_E_PARSE, "duplicate output attribute " + it.name);
    collect_refs(it.e, &srefs);
  }
  for (auto& r : grefs)
    if (r.first == 0) out.g_in_walk = true;
  if (q.partitioned) {
    auto ia = q.partition.find(q.states[0].stream);
    auto ib = q.partition.find(q.states[1].stream);
    if (ia == q.partition.end() || ib == q.partition.end())
      fail(CEP_E_PARSE, "pattern stream not covered by the enclosing partition");
    out.key_col_a = key_column(A, ia->second);
    out.key_col_b = key_column(B, ib->second);
  }
  // a select item that is just the partition key of s1 or s2 is emitted from
  // the key itself (both states share it) and is not carried in records
  auto is_key_ref = [&](const ExprP& e) {
    return q.partitioned && e->k == Expr::ATTR && e->state >= 0 &&
           e->col == (e->state == 0 ? out.key_col_a : out.key_col_b);
  };
  // captured columns
  std::vector<int> cap_a, cap_b;
  if (out.g_in_walk)
    for (auto& r : grefs) index_of(r.first == 0 ? cap_a : cap_b, r.second, true);
  for (auto& it : q.select) {
    if (is_key_ref(it.e)) continue;
    std::vector<std::pair<int, int>> refs;
    collect_refs(it.e, &refs);
    for (auto& r : refs) index_of(r.first == 0 ? cap_a : cap_b, r.second, true);
  }
  if ((int)cap_a.size() > kMaxCaps || (int)cap_b.size() > kMaxCaps)
    fail(CEP_E_UNSUPPORTED, "too many captured attributes");
  if (out.a_stream != out.b_stream) {
    out.rec_cols_a = cap_a;
    out.rec_cols_b = cap_b;
    for (size_t i = 0; i < cap_a.size(); ++i) out.cap_from_rec.push_back((int)i);
  } else {
    std::vector<int> uni = cap_a;
    for (int x : cap_b) index_of(uni, x, true);
    if ((int)uni.size() > kMaxCaps) fail(CEP_E_UNSUPPORTED, "too many captured attributes");
    out.rec_cols_a = uni;
    out.rec_cols_b = uni;
    for (int x : cap_a) out.cap_from_rec.push_back(index_of(uni, x, false));
  }
  // programs
  Loader raw{[](const Expr& e) { return std::make_pair((uint8_t)OP_LDCOL, (uint32_t)e.col); }};
  if (q.states[0].cond) {
    CodeGen cg(app, raw);
    out.f = cg.compile(q.states[0].cond);
    out.f_terms = lower_terms({q.states[0].cond});
  }
  Query* op = &out;
  Loader walk{[op, &cap_a](const Expr& e) {
    if (e.state == 0) {
      int i = -1;
      for (size_t k = 0; k < cap_a.size(); ++k)
        if (cap_a[k] == e.col) i = (int)k;
      return std::make_pair((uint8_t)OP_LDCAP, (uint32_t)i);
    }
    int i = -1;
    for (size_t k = 0; k < op->rec_cols_b.size(); ++k)
      if (op->rec_cols_b[k] == e.col) i = (int)k;
    return std::make_pair((uint8_t)OP_LDCOL, (uint32_t)i);
  }};
  if (q.states[1].cond) {
    CodeGen cg(app, out.g_in_walk ? walk : raw);
    if (out.g_in_walk) {
      out.g_walk = cg.compile(q.states[1].cond);
    } else {
      out.g_raw = cg.compile(q.states[1].cond);
      out.g_terms = lower_terms({q.states[1].cond});
    }
  }
  for (auto& it : q.select) {
    OutItem oi;
    oi.name = it.name;
    oi.type = it.e->t;
    if (is_key_ref(it.e)) {
      oi.prog = Prog{};
      oi.src = SRC_KEY;
    } else {
      CodeGen cg(app, walk);
      oi.prog = cg.compile(it.e);
      oi.src = direct_source(app, oi.prog);   // SRC_CAP + i = s1 capture, SRC_REC + i = s2 word
    }
    out.select.push_back(oi);
  }
  add_output(app, q.out, out.select);
  app->queries.push_back(out);
}

}  // namespace

std::vector<int> read_inputs(const CompiledApp& app) {
  std::vector<char> used(app.inputs.size(), 0);
  auto mark = [&](int s) {
    if (s >= 0 && s < (int)used.size()) used[s] = 1;
  };
  for (auto& q : app.queries) {
    mark(q.in_stream);
    mark(q.a_stream);
    mark(q.b_stream);
    for (auto& st : q.nstates) mark(st.stream);
  }
  std::vector<int> out;
  for (size_t i = 0; i < used.size(); ++i)
    if (used[i]) out.push_back((int)i);
  return out;
}

int compile_app(const std::string& text, CompiledApp* out, std::string* err,
                const std::vector<std::string>* dict_seed) {
  try {
    CompiledApp app;
    if (dict_seed) app.strings = *dict_seed;
    std::vector<QueryAst> qs;
    Parser(text).parse(&app.inputs, &qs);
    for (auto& q : qs) {
      if (q.single) compile_single(&app, q);
      else compile_pattern(&app, q);
    }
    *out = std::move(app);
    return CEP_OK;
  } catch (const CepError& e) {
    if (err) *err = e.what();
    return e.code;
  } catch (const std::exception& e) {
    if (err) *err = std::string("parse error: ") + e.what();
    return CEP_E_PARSE;
  }
}

}  // namespace cep
