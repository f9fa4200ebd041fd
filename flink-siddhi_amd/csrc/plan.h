// Compiled-plan representation shared by the host front end and the gfx950
// kernels.  A SiddhiQL app (the "enriched execution plan" built by
// SiddhiExecutionPlanner.java:51-60 / SiddhiOperatorContext.java:105-115:
// `define stream ...;` + queries) compiles into:
//   * typed columnar stream schemas (SiddhiTypeFactory.java:42-54 type map),
//   * predicate / projection programs for a small register VM (Siddhi's
//     expression executors, Java value semantics — SURVEY.md App. A.2),
//   * per-query descriptors: filter/projection, 2-state keyed pattern
//     (`[every] s1=A[f] -> s2=B[g] [within W]`, optionally under
//     `partition with`), running group-by aggregation.
#pragma once
#include <cstdint>

namespace cep {

// Attribute types; values match cep_type in include/cep.h.
enum Type : int32_t {
  T_INT = 0, T_LONG = 1, T_FLOAT = 2, T_DOUBLE = 3, T_BOOL = 4, T_STRING = 5,
  T_OBJECT = 6
};

// Column element width in bytes (bool = 1 byte, string = int32 dictionary id).
inline constexpr int type_width(int t) {
  return t == T_LONG || t == T_DOUBLE ? 8 : (t == T_BOOL ? 1 : 4);
}

// ---------------------------------------------------------------- VM ISA --
// Register machine over 64-bit words.  int/float values live in the low 32
// bits (int sign-extended), long/double use all 64, bool is 0/1.  A per-
// register null bit models Siddhi's null results (int div/mod by zero).
enum Op : uint8_t {
  OP_END = 0,
  OP_LDCOL,      // dst <- column[imm] of the current event (type in b)
  OP_LDTS,       // dst <- event timestamp
  OP_LDK,        // dst <- konst[imm]
  OP_LDCAP,      // dst <- captured word imm of the earlier state (s1.x)
  OP_LDOUT,      // dst <- output attribute imm (HAVING over select items)
  OP_CVT,        // dst <- convert a from type imm>>8 to type imm&0xff
  OP_ADD, OP_SUB, OP_MUL, OP_DIV, OP_MOD,   // type in imm
  OP_NEG,
  OP_EQ, OP_NE, OP_LT, OP_LE, OP_GT, OP_GE, // operand type in imm
  OP_AND, OP_OR, OP_NOT,
  OP_MOV,
  OP_LDAGG,      // dst <- aggregate slot imm (running value)
};

struct Ins {
  uint8_t op, dst, a, b;
  uint32_t imm;
};
static_assert(sizeof(Ins) == 8, "Ins must be 8 bytes");

constexpr int kMaxRegs = 8;
constexpr int kMaxCols = 16;
constexpr int kMaxCaps = 8;
constexpr int kMaxOut = 16;
constexpr int kMaxProgLen = 64;

// A program is a slice [off, off+len) of the plan's instruction array; the
// result is register `res`.
struct Prog {
  int32_t off = -1, len = 0;
  int32_t res = 0;
  int32_t type = T_BOOL;
  bool valid() const { return off >= 0; }
};

// Interpreter-free predicate form: a flat AND (or OR) of up to kMaxTerms
// atoms `(column [aop aconst]) cop cconst`, with Siddhi's numeric promotion
// applied at compile time (atype = promote(column, aconst), ctype =
// promote(atype, cconst); constants stored already converted).  Covers the
// filters of every BASELINE config; anything else runs on the VM.
constexpr int kMaxTerms = 4;
struct Term {
  int32_t col, coltype;
  int32_t aop, atype;      // aop = 0: no arithmetic
  uint64_t aconst;
  int32_t cop, ctype;
  uint64_t cconst;
};
struct TermList {
  int32_t n = -1;          // -1: not expressible, use the VM program
  int32_t any = 0;         // 0: all terms (AND), 1: any term (OR)
  Term t[kMaxTerms];
};

// Output attribute sources that bypass the VM (plain attribute copies).
enum : int32_t {
  SRC_VM = -1,
  SRC_CAP = 0,      // + i: captured word i of s1 (pattern) / column i (filter)
  SRC_REC = 64,     // + i: record word i of the completing event (pattern)
  SRC_TS = 128,     // event timestamp of the completing / current event
  SRC_KEY = 129,    // the partition key (pattern under `partition with`)
  SRC_AGG = 160,    // + i: running value of aggregate i (group-by query)
};

constexpr int kMaxAggs = 8;
constexpr int kMaxStates = 6;     // states of an N-state pattern / sequence
enum AggFn { AGG_SUM = 0, AGG_COUNT = 1, AGG_AVG = 2, AGG_MIN = 3, AGG_MAX = 4 };

// Role bits carried in partition records (pattern path).
enum : uint32_t {
  ROLE_A = 1u,        // event passes the start state's filter f
  ROLE_B = 2u,        // event is a candidate for the second state
  ROLE_G = 4u,        // g(B) already evaluated true in the partition pass
};

}  // namespace cep
