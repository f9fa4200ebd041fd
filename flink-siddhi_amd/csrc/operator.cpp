// Dynamic plans behind one operator: the QueryRuntimeHandler map of
// AbstractSiddhiOperator (operator/AbstractSiddhiOperator.java:114-176) and
// its control-event handling (onEventReceived, :400-467), over libcep apps.
//
//   MetadataControlEvent  added plan   -> cep_operator_add_plan     (new runtime)
//                         updated plan -> cep_operator_update_plan  (new runtime
//                                         replaces the old one; the old one's state
//                                         is dropped, as the reference shuts it down)
//                         deleted plan -> cep_operator_remove_plan
//   OperationControlEvent ENABLE_QUERY / DISABLE_QUERY -> cep_operator_enable
//   data record of stream S -> every enabled plan that reads S
//                              (router/AddRouteOperator.java:65-96)
//
// Plans are independent runtimes, so adding, updating or removing one leaves
// every other plan's state untouched.  Partition keys for the dynamic path's
// routing (AddRouteOperator.java:83-92) come from cep_partition_channels
// (kernels in keymap.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/cep.h"
#include "frontend.h"
#include "kernels.h"

using namespace cep;

struct cep_operator {
  cep_options opt{};
  struct Plan {
    cep_app* app = nullptr;
    bool enabled = true;
    std::vector<std::string> inputs;
  };
  std::map<std::string, Plan> plans;   // plan id -> runtime (ordered: deterministic fan-out)
  // Shared string dictionary: every plan's dictionary equals `dict`, so a
  // STRING column's ids mean the same in every plan the batch reaches.
  std::vector<std::string> dict;
  std::map<std::string, int32_t> dict_index;
  std::string last_error;
};

namespace {

int op_fail(cep_operator* o, int code, const std::string& m) {
  if (o) o->last_error = m;
  return code;
}

void dict_add(cep_operator* o, const std::string& s, cep_app* except) {
  o->dict_index.emplace(s, (int32_t)o->dict.size());
  o->dict.push_back(s);
  for (auto& kv : o->plans)
    if (kv.second.app != except) cep_dict_intern(kv.second.app, s.c_str());
}

int make_plan(cep_operator* o, const char* plan, cep_operator::Plan* out) {
  char err[1024];
  cep_app* a = create_app(plan, &o->opt, &o->dict, err, sizeof(err));
  if (!a) {
    const int rc = cep_validate(plan, nullptr, 0);
    int code = rc ? rc : CEP_E_DEVICE;
    if (!rc && std::strstr(err, "not supported")) code = CEP_E_UNSUPPORTED;
    else if (!rc && std::strstr(err, "capacity")) code = CEP_E_CAPACITY;
    return op_fail(o, code, err);
  }
  // the plan's own string literals follow the shared ids: every other plan
  // learns them in the same order
  for (int32_t i = (int32_t)o->dict.size();; ++i) {
    const char* s = cep_dict_lookup(a, i);
    if (!s) break;
    dict_add(o, s, a);
  }
  out->app = a;
  out->enabled = true;
  out->inputs.clear();
  CompiledApp app;
  std::string m;
  if (compile_app(plan, &app, &m) == CEP_OK)
    for (int i : read_inputs(app)) out->inputs.push_back(app.inputs[i].id);
  return CEP_OK;
}

}  // namespace

extern "C" {

cep_operator* cep_operator_create(const cep_options* opt, char* err, size_t errlen) {
  auto* o = new cep_operator();
  if (opt) o->opt = *opt;
  else cep_default_options(&o->opt);
  if (err && errlen) err[0] = 0;
  return o;
}

void cep_operator_destroy(cep_operator* o) {
  if (!o) return;
  for (auto& kv : o->plans) cep_destroy(kv.second.app);
  delete o;
}

int cep_operator_add_plan(cep_operator* o, const char* plan_id, const char* plan) {
  if (!o || !plan_id || !plan) return CEP_E_ARG;
  if (o->plans.count(plan_id)) return op_fail(o, CEP_E_ARG, std::string("Execution plan ") + plan_id + " already exists!");
  cep_operator::Plan p;
  const int rc = make_plan(o, plan, &p);
  if (rc) return rc;
  o->plans[plan_id] = p;
  return CEP_OK;
}

int cep_operator_update_plan(cep_operator* o, const char* plan_id, const char* plan) {
  if (!o || !plan_id || !plan) return CEP_E_ARG;
  cep_operator::Plan p;
  if (!o->plans.count(plan_id))   // AddRouteOperator.java:128-133
    return op_fail(o, CEP_E_ARG, std::string("Execution plan ") + plan_id + " does not exist!");
  const int rc = make_plan(o, plan, &p);   // the old runtime keeps serving if this fails
  if (rc) return rc;
  auto it = o->plans.find(plan_id);
  cep_flush(it->second.app);
  cep_destroy(it->second.app);
  p.enabled = it->second.enabled;
  it->second = p;
  return CEP_OK;
}

int cep_operator_remove_plan(cep_operator* o, const char* plan_id) {
  if (!o || !plan_id) return CEP_E_ARG;
  auto it = o->plans.find(plan_id);
  if (it == o->plans.end()) return CEP_OK;   // the reference ignores unknown ids
  cep_flush(it->second.app);
  cep_destroy(it->second.app);
  o->plans.erase(it);
  return CEP_OK;
}

int cep_operator_enable(cep_operator* o, const char* plan_id, int enabled) {
  if (!o || !plan_id) return CEP_E_ARG;
  auto it = o->plans.find(plan_id);
  if (it == o->plans.end()) return CEP_OK;   // handler == null: ignored (:452-463)
  it->second.enabled = enabled != 0;
  return cep_set_enabled(it->second.app, enabled);
}

cep_app* cep_operator_plan(cep_operator* o, const char* plan_id) {
  if (!o || !plan_id) return nullptr;
  auto it = o->plans.find(plan_id);
  return it == o->plans.end() ? nullptr : it->second.app;
}

int cep_operator_send(cep_operator* o, const char* stream_id, const cep_batch* b, int* plans_sent) {
  if (!o || !stream_id || !b) return CEP_E_ARG;
  if (b->stream) return op_fail(o, CEP_E_ARG, "cep_operator_send takes single-stream batches (stream == NULL)");
  // Every enabled plan gets the batch on its own, as AddRouteOperator sends
  // to each plan (router/AddRouteOperator.java:54-175): a plan that fails
  // does not keep the later ones from their input; the first failure (with
  // its plan id) is returned after the loop.
  int sent = 0, first_rc = CEP_OK;
  std::string first_msg;
  for (auto& kv : o->plans) {
    auto& p = kv.second;
    if (!p.enabled) continue;
    if (std::find(p.inputs.begin(), p.inputs.end(), stream_id) == p.inputs.end()) continue;
    cep_batch bb = *b;
    bb.input = cep_input(p.app, stream_id);
    if (bb.input < 0) continue;
    const int rc = cep_send_batch(p.app, &bb);
    if (rc) {
      if (first_rc == CEP_OK) {
        first_rc = rc;
        first_msg = kv.first + ": " + cep_last_error(p.app);
      }
      continue;
    }
    ++sent;
  }
  if (plans_sent) *plans_sent = sent;
  if (first_rc != CEP_OK) return op_fail(o, first_rc, first_msg);
  return CEP_OK;
}

int cep_operator_flush(cep_operator* o) {
  if (!o) return CEP_E_ARG;
  for (auto& kv : o->plans) {
    const int rc = cep_flush(kv.second.app);
    if (rc) return op_fail(o, rc, kv.first + ": " + cep_last_error(kv.second.app));
  }
  return CEP_OK;
}

int cep_operator_plan_ids(cep_operator* o, char* buf, size_t len) {
  if (!o || !buf || !len) return CEP_E_ARG;
  std::string s;
  for (auto& kv : o->plans) {
    if (!s.empty()) s += '\n';
    s += kv.first;
  }
  std::snprintf(buf, len, "%s", s.c_str());
  return s.size() < len ? CEP_OK : CEP_E_CAPACITY;
}

int32_t cep_operator_intern(cep_operator* o, const char* s) {
  if (!o || !s) return -CEP_E_ARG;
  auto it = o->dict_index.find(s);
  if (it != o->dict_index.end()) return it->second;
  dict_add(o, s, nullptr);
  return (int32_t)o->dict.size() - 1;
}

const char* cep_operator_lookup(cep_operator* o, int32_t id) {
  if (!o || id < 0 || id >= (int32_t)o->dict.size()) return nullptr;
  return o->dict[id].c_str();
}

int cep_plan_input_streams(const char* plan, char* buf, size_t len) {
  if (!plan || !buf || !len) return CEP_E_ARG;
  CompiledApp app;
  std::string m;
  const int rc = compile_app(plan, &app, &m);
  if (rc) {
    std::snprintf(buf, len, "%s", m.c_str());
    return rc;
  }
  std::string s;
  for (int i : read_inputs(app)) {
    if (!s.empty()) s += '\n';
    s += app.inputs[i].id;
  }
  std::snprintf(buf, len, "%s", s.c_str());
  return s.size() < len ? CEP_OK : CEP_E_CAPACITY;
}

const char* cep_operator_last_error(cep_operator* o) { return o ? o->last_error.c_str() : "null operator"; }

}  // extern "C"
