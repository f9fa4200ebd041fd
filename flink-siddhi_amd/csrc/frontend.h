// SiddhiQL-subset front end: parse + bind + compile.
//
// Replaces the plan-side uses of Siddhi that flink-siddhi makes:
//   SiddhiManager.validateSiddhiApp      (AbstractSiddhiOperator.java:292-299)
//   SiddhiCompiler.parse                 (SiddhiExecutionPlanner.java:76)
//   SiddhiAppRuntime.getStreamDefinitionMap for output-type inference
//                                         (SiddhiTypeFactory.java:64-112)
// Unsupported-but-valid SiddhiQL (joins, windows, tables, extensions) fails
// with CEP_E_UNSUPPORTED so the Java shim can fall back to real Siddhi.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "plan.h"

namespace cep {

struct AttrDef {
  std::string name;
  int type;
};

struct StreamSchema {
  std::string id;
  std::vector<AttrDef> attrs;
  int index(const std::string& n) const {
    for (size_t i = 0; i < attrs.size(); ++i)
      if (attrs[i].name == n) return (int)i;
    return -1;
  }
};

enum QueryKind { Q_FILTER = 0, Q_PATTERN = 1, Q_AGG = 2 };


struct AggSpec {
  int fn;
  int arg_type;         // input type (after evaluation of arg program)
  int out_type;
  Prog arg;             // argument program over the current event (unused for count)
  int word = -1;        // device: carried record word holding the argument (-1: count)
};

struct OutItem {
  std::string name;
  int type;
  Prog prog;
  int32_t src = SRC_VM;          // direct copy source when the item is a plain attribute
};

struct Query {
  int kind = Q_FILTER;
  std::string out_stream;
  std::vector<OutItem> select;   // output attributes in definition order
  Prog having;                   // over LDOUT / LDCOL / LDAGG
  // interpreter-free having (multi-query walk): `<select item> cop constant`;
  // having_item -1 with having_simple = true: no having
  bool having_simple = true;
  int having_item = -1;
  int having_cop = 0, having_ctype = 0;
  uint64_t having_cconst = 0;

  // ---- filter / aggregation (single input stream)
  int in_stream = -1;
  Prog filter;                   // conjunction of all [..] filters, invalid = true
  TermList filter_terms;
  int key_col = -1;              // partition / group key column (-1: none)
  int part_col = -1;             // `partition with` column (-1: none)
  std::vector<Prog> group_progs; // group-by expressions (host path when not a column)
  std::vector<int> group_cols;   // group-by attribute columns (routing keys)
  std::vector<AggSpec> aggs;

  // ---- 2-state pattern `[every] s1=A[f] -> s2=B[g] [within W]`
  int a_stream = -1, b_stream = -1;
  Prog f;                        // over A's columns (LDCOL = raw column)
  Prog g_raw;                    // g over B's raw columns (valid iff !g_in_walk)
  TermList f_terms, g_terms;     // interpreter-free forms of f / g_raw
  Prog g_walk;                   // g in the walk: LDCOL = record word, LDCAP = s1 capture
  bool g_in_walk = false;
  bool every = false;
  int64_t within = -1;           // ms, -1 = none
  int key_col_a = -1, key_col_b = -1;  // partition key columns (-1: unpartitioned)
  std::vector<int> rec_cols_a;   // raw columns carried in A-stream records
  std::vector<int> rec_cols_b;   // raw columns carried in B-stream records
  std::vector<int> cap_from_rec; // pending capture word i <- A-record word cap_from_rec[i]

  // ---- N-state pattern / sequence (general NFA walk): `nfa` queries keep
  // every event of the states' streams (sequences) or every event some
  // state's own condition accepts (patterns) as records carrying rec_cols_a
  struct NState {
    int stream = -1;
    int min_count = 1, max_count = 1;   // max -1: unbounded
    Prog raw;      // condition over the event's own columns (partition pass)
    Prog walk;     // condition reading earlier states (walk: LDCOL word, LDCAP capture)
    TermList terms;   // interpreter-free form of raw (n = 0: no condition, -1: not expressible)
  };
  struct NCap {
    int state, index, word;           // index: k-th event of the state (0 = first), -1 = last
  };
  bool nfa = false;
  bool sequence = false;
  std::vector<NState> nstates;
  std::vector<NCap> ncaps;
  std::vector<int> key_col_s;    // per input stream handle: partition key column (-1)
};

struct CompiledApp {
  std::vector<StreamSchema> inputs;     // defined input streams
  std::vector<StreamSchema> outputs;    // output streams (inferred)
  std::vector<Query> queries;
  std::vector<Ins> code;
  std::vector<uint64_t> konst;
  std::vector<std::string> strings;     // string literals (dictionary order)

  int input_index(const std::string& id) const {
    for (size_t i = 0; i < inputs.size(); ++i)
      if (inputs[i].id == id) return (int)i;
    return -1;
  }
  int output_index(const std::string& id) const {
    for (size_t i = 0; i < outputs.size(); ++i)
      if (outputs[i].id == id) return (int)i;
    return -1;
  }
};

// Status codes mirror include/cep.h.
// dict_seed: strings that take dictionary ids 0..n-1 before the plan's own
// literals (plans of one operator share their ids, operator.cpp).
int compile_app(const std::string& text, CompiledApp* out, std::string* err,
                const std::vector<std::string>* dict_seed = nullptr);

}  // namespace cep

struct cep_app;
struct cep_options;
namespace cep {
// cep_create with a dictionary seed (engine.cpp).
cep_app* create_app(const char* plan, const cep_options* opt, const std::vector<std::string>* dict_seed,
                    char* err, size_t errlen);

const char* type_name(int t);

// Input streams some query reads (InputStream.getUniqueStreamIds over the
// plan's queries), in definition order.
std::vector<int> read_inputs(const CompiledApp& app);

}  // namespace cep
