// libcep runtime: the C ABI of include/cep.h over the gfx950 kernels.
//
// One cep_app = one Siddhi app runtime (AbstractSiddhiOperator.java:114-176
// QueryRuntimeHandler).  Device layout (HBM, sized for 288 GB/GPU):
//   * plan: VM instruction array + constant pool (tiny, read-only),
//   * per output stream: typed columns + ts + seq + a device row cursor,
//     capacity = the host-known bound on rows since the last flush (no
//     device->host sync is ever needed to size a launch),
//   * per keyed pattern: dense per-key state [key][S][2+ncap] words plus a
//     pending count and `started` byte per key, and a chunk-sized record
//     arena [tiles][2048 rows][rec_words] + tile offset table.
// All work for a batch is enqueued on the app's HIP stream; cep_flush
// synchronises, checks the device error word and delivers rows to callbacks.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/cep.h"
#include "frontend.h"
#include "kernels.h"

using namespace cep;

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

bool dev_ensure(DevBuf* b, size_t bytes, hipStream_t s, bool keep) {
  if (b->bytes >= bytes && b->p) return true;
  size_t nb = std::max(bytes, b->bytes * 2);
  void* p = nullptr;
  if (hipMalloc(&p, nb) != hipSuccess) return false;
  if (keep && b->p && b->bytes) hipMemcpyAsync(p, b->p, b->bytes, hipMemcpyDeviceToDevice, s);
  if (b->p) {
    hipStreamSynchronize(s);
    hipFree(b->p);
  }
  b->p = p;
  b->bytes = nb;
  return true;
}

void dev_free(DevBuf* b) {
  if (b->p) hipFree(b->p);
  b->p = nullptr;
  b->bytes = 0;
}

// Pinned (page-locked) host memory: DMA at PCIe speed, no driver bounce.
struct HostBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

bool host_ensure(HostBuf* b, size_t bytes) {
  if (b->bytes >= bytes && b->p) return true;
  // pinning hundreds of MB takes ~100 ms: grow with headroom, so a delivery
  // buffer sized by one flush's rows is not re-pinned when the next flush
  // brings a few more
  const size_t nb = std::max(bytes + bytes / 2, b->bytes * 2);
  if (b->p) hipHostFree(b->p);
  b->p = nullptr;
  b->bytes = 0;
  if (hipHostMalloc(&b->p, nb, hipHostMallocDefault) != hipSuccess) return false;
  b->bytes = nb;
  return true;
}

void host_free(HostBuf* b) {
  if (b->p) hipHostFree(b->p);
  b->p = nullptr;
  b->bytes = 0;
}

bool is_pinned(const void* p) {
  hipPointerAttribute_t at;
  if (!p || hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();   // pageable memory: clear the sticky lookup error
    return false;
  }
  return at.type == hipMemoryTypeHost;
}

struct OutStream {
  std::string id;
  std::vector<int> types;
  std::vector<DevBuf> cols;
  DevBuf ts, seq;
  unsigned long long* count = nullptr;   // device cursor
  int64_t cap = 0;                       // allocated rows
  int64_t bound = 0;                     // upper bound of rows since last flush
  bool write_seq = true;                 // the kernels store arrival numbers (someone reads them)
  cep_emit_fn fn = nullptr;
  void* user = nullptr;
  // pinned host copies for callback delivery (D2H at PCIe speed)
  std::vector<HostBuf> hcols;
  HostBuf hts, hseq;
  // ordered_output: the rows permuted into Siddhi's emission order on the
  // device (stable sort on seq) before the D2H
  std::vector<DevBuf> scols;
  DevBuf sts, sseq;
};

struct PatternRT {
  int q = -1;
  PatternArgs pa{};
  DevBuf khdr, kslot;        // per-key state, SoA over the bucket-major key index
  int64_t kstride = 0;       // keys_per_bucket * buckets
  // double-buffered chunk arenas: partition(c+1) runs on the side stream
  // while walk(c) runs on the main stream
  DevBuf recs[2], tile_off[2], chunk_base[2];
  hipEvent_t part_done[2] = {nullptr, nullptr}, walk_done[2] = {nullptr, nullptr};
  PrefPlan pref;               // fast partition path (n < 0: generic)
  bool used[2] = {false, false};
  int cur = 0;                 // arena of the next chunk
  int64_t chunk = 0;
  int64_t chunk_tol = 0;       // chunk of the order-tolerant form (walked by the VM build: up to 16 Mi rows)
  int64_t extra_bound = 0;   // pending partials that may still complete
  bool part_vm = true;       // partition pass needs the interpreter
  bool walk_vm = true;       // walk needs the interpreter (g on s1, computed select items)
  // closed-form fast path (cf_kernels.hip): its own, larger chunk arenas
  bool cf = false;
  int64_t cf_chunk = 0;
  DevBuf cf_recs[2], cf_toff[2];
  // pending lists longer than S (closed-form path): per-key count + run
  // offset, and two pools of overflow slots swapped per walk launch
  DevBuf kext, pool[2], pool_cur;
  int pool_side = 0;           // pool[pool_side] holds the current runs
  int64_t pool_cap = 0;        // slots per pool
  // sparse partition keys (cep_options.sparse_keys): value -> dense slot map
  bool sparse = false;
  uint64_t table_cap = 0;
  DevBuf tkey, tval, krev, kcount, dense;
  // hot keys (hot.hip): keys that would make their bucket a straggler are
  // matched by grid-wide scans; the walk reports candidates, diversion starts
  // (sticky) once the device has put a key into a hot slot
  bool hot = false;            // candidate collection on (closed-form path, P + kCfHotMax buckets fit)
  bool hot_on = false;         // diversion active: hot arenas allocated
  bool hot_probed = false;     // the first (short) chunk ran and its candidates were read back
  uint32_t hot_thresh = 0;     // records per key per launch that make a key hot
  int hot_blocks = 0;
  DevBuf hot_id, hot_key, hot_m, hot_gbase, hoff, cand, ncand, harr, hrow, hnb, bsum, bcnt, boff, hcm, hobase,
      hot_active, htmn, htmx, hflag, btol;   // (the last four: order-tolerant runs)
  HostBuf hot_active_host;     // pinned: slots in use (read without a sync)
  hipEvent_t hot_fork = nullptr, hot_join = nullptr;   // hot kernels on the side stream, beside the walk
  // a pattern whose result depends on event-time order (`within`, not a
  // sequence): with cep_options.ts_order = 0 it runs the order-tolerant path
  bool order_sensitive = false;
};

// Multi-query group (mq_kernels.hip): keyed queries of one app sharing a
// key column, run by one partition pass + one walk per chunk.
struct MqRT {
  std::vector<int> qs;                   // query indices, plan order
  std::vector<MqQuery> hq;               // host copy of the device descriptors
  DevBuf dq, dconds;
  std::vector<MqCond> conds;             // [8][kMqMaxCond]
  int32_t ncond[8] = {0};
  uint32_t stream_mask = 0;
  int key_col = -1;
  std::vector<int> carry;                // logical carried columns
  std::vector<int> cond_cols;            // columns the conditions read
  bool check_order = false;
  int64_t key_capacity = 0, kstride = 0;
  int lg = 0, kpb = 0;
  int key_stride = 1, key_offset = 0;
  DevBuf state;
  int64_t words = 0;                     // state words per key (all queries)
  int64_t chunk = 0;
  DevBuf recs[2], toff[2], chunk_base[2];
  hipEvent_t part_done[2] = {nullptr, nullptr}, walk_done[2] = {nullptr, nullptr};
  bool used[2] = {false, false};
  int cur = 0;
  bool dq_dirty = true;
  std::vector<int> classes_kind, classes_n;   // shape classes in descriptor order (MqUnit kinds, sizes)
  std::vector<MqUnit> units;
  DevBuf du;
};

struct TimedLaunch {
  int kind;
  hipEvent_t a, b;
};

}  // namespace

struct cep_app {
  CompiledApp app;
  cep_options opt{};
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;    // partition pass of the next chunk
  hipEvent_t in_ready = nullptr;
  hipEvent_t ext_ready = nullptr;   // cep_stream_wait: producer stream of device inputs
  hipEvent_t out_ready = nullptr;   // cep_stream_signal: the engine's work so far
  // Shuffle sender (cep_route_batch of device batches) runs on its own stream:
  // routing step s+1 overlaps the walk of step s (it touches no walk state)
  hipStream_t rstream = nullptr;
  hipEvent_t r_ready = nullptr;
  hipEvent_t r_host = nullptr;     // a host batch's route (engine stream) joined into the route stream
  bool enabled = true;
  std::string last_error;
  std::vector<std::string> dict;
  std::unordered_map<std::string, int32_t> dict_index;
  DevBuf code, konst;
  std::vector<OutStream> outs;
  std::vector<PatternRT> pats;
  std::vector<MqRT> mqs;          // multi-query groups
  std::vector<char> in_mq;        // per query: served by a multi-query group
  DevBuf tile_state, ticket, err;
  DevBuf route_arena, route_tcount, route_toffs, route_dcount;   // key shuffle (sender)
  DevBuf rerr;                 // error word of the route kernels (route stream; the walk's is `err`)
  DevBuf stamps;               // CEP_STAMPS=1: walk phase stamps (diagnostics)
  DevBuf str_hash;             // Java String.hashCode per dictionary id (dynamic routing)
  HostBuf flush_words;         // cep_flush: error word + output cursors + seq stats (pinned)
  DevBuf out_counts;           // every output's row cursor (OutStream::count points here)
  DevBuf ostats;               // cep_flush: per output {~min seq, max seq, descents} (k_seq_stats)
  DevBuf okeys[2], oidx[2], otemp;   // cep_flush: emission-order sort scratch (shared by the outputs)
  DevBuf rr_col[kMaxCols], rr_ts, rr_stream, rr_seq;   // cep_send_rows: unpacked rows
  // host batches: two staging slots (pinned host arena + device arena); a
  // batch's H2D copy runs on the copy stream while the previous batch's
  // kernels run on the main stream
  struct HostSlot {
    HostBuf pinned;
    DevBuf dev;
    hipEvent_t dma_done = nullptr, free = nullptr;
    bool used = false;
  } hs[2];
  int hs_next = 0;
  hipStream_t copy = nullptr;
  // event-time reorder buffer (cep_buffer_batch / cep_watermark): rows of
  // one input layout since the last watermark, SoA in arrival order
  struct Reorder {
    int input = -1;            // layout owner (-1: empty)
    bool has_stream = false;
    int64_t n = 0, cap = 0;
    int64_t released_max = INT64_MIN;   // latest ts handed to the engine
    DevBuf col[kMaxCols], ts, stream;  // buffered rows
    DevBuf out[kMaxCols], ots, ostream;   // sorted released rows (a device batch)
    DevBuf keys, idx_in, idx_out, temp, bound;
  } ro;
  int64_t events_in = 0, matches_out = 0, batches = 0, late_events = 0;
  int64_t last_ts = INT64_MIN;
  DevBuf last_ts_dev;          // last ts of the previous batch (RowsArgs::prev_ts_dev)
  bool force_tolerant = false; // this batch holds late rows (cep_watermark, late_policy 2)
  int64_t launches[16] = {0};
  double kernel_ms[16] = {0};
  int64_t kernel_timed[16] = {0};
  std::vector<TimedLaunch> timed;
  std::vector<hipEvent_t> event_pool;
  std::vector<std::unique_ptr<char[]>> name_store;
};

namespace {

void set_err(char* err, size_t errlen, const std::string& m) {
  if (err && errlen) {
    std::snprintf(err, errlen, "%s", m.c_str());
  }
}

int fail(cep_app* a, int code, const std::string& m) {
  if (a) a->last_error = m;
  return code;
}

hipEvent_t pool_event(cep_app* a) {
  if (!a->event_pool.empty()) {
    hipEvent_t e = a->event_pool.back();
    a->event_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  hipEventCreate(&e);
  return e;
}

struct LaunchTimer {
  cep_app* a;
  int kind;
  hipStream_t st;
  hipEvent_t s = nullptr;
  // profile = k: HIP events around every k-th launch of each kernel kind
  // (each event between two kernels widens the gap between them by ~5 us)
  LaunchTimer(cep_app* app, int k, hipStream_t on = nullptr)
      : a(app), kind(k), st(on ? on : app->stream) {
    const bool timed = a->opt.profile > 0 && a->launches[k] % a->opt.profile == 0;
    a->launches[k]++;
    if (timed) {
      s = pool_event(a);
      hipEventRecord(s, st);
    }
  }
  ~LaunchTimer() {
    if (s) {
      hipEvent_t e = pool_event(a);
      hipEventRecord(e, st);
      a->timed.push_back({kind, s, e});
    }
  }
};

void harvest_timers(cep_app* a) {
  for (auto& t : a->timed) {
    float ms = 0;
    hipEventElapsedTime(&ms, t.a, t.b);
    a->kernel_ms[t.kind] += ms;
    a->kernel_timed[t.kind]++;
    a->event_pool.push_back(t.a);
    a->event_pool.push_back(t.b);
  }
  a->timed.clear();
}

int ensure_out_cap(cep_app* a, OutStream& o, int64_t need) {
  if (need <= o.cap) return CEP_OK;
  int64_t nc = std::max<int64_t>(need, std::max<int64_t>(o.cap * 2, 1 << 16));
  for (size_t c = 0; c < o.cols.size(); ++c)
    if (!dev_ensure(&o.cols[c], (size_t)nc * type_width(o.types[c]), a->stream, true))
      return fail(a, CEP_E_DEVICE, "out of device memory (output columns)");
  if (!dev_ensure(&o.ts, (size_t)nc * 8, a->stream, true) ||
      !dev_ensure(&o.seq, (size_t)nc * 8, a->stream, true))
    return fail(a, CEP_E_DEVICE, "out of device memory (output ts/seq)");
  o.cap = nc;
  return CEP_OK;
}

OutArgs out_args(OutStream& o, const Query& q) {
  OutArgs oa{};
  oa.ncols = (int32_t)o.cols.size();
  for (int c = 0; c < oa.ncols; ++c) {
    oa.col[c] = o.cols[c].p;
    oa.type[c] = o.types[c];
    oa.prog[c] = q.select[c].prog.off;
    oa.src[c] = q.select[c].src;
  }
  oa.ts = (int64_t*)o.ts.p;
  oa.seq = (int64_t*)o.seq.p;
  oa.count = o.count;
  oa.cap = o.cap;
  oa.write_seq = o.write_seq ? 1 : 0;
  return oa;
}

// ---- multi-query groups (mq_kernels.hip) ------------------------------------
// A query joins a group when its per-event work is interpreter-free and keyed
// on the group's key column: group-by aggregations (term-list filter, plain
// column arguments, select items key / aggregate / column, having on one
// output item) and sequences of the one-live-partial shape (a single start
// event on a stream no later state reads) with own-column term-list
// conditions and first / last captures.  Queries of one group share the
// partition pass (one read of the batch, each distinct condition evaluated
// once per row) and the walk (AbstractSiddhiOperator.java:283-287: every
// event goes to every query).  CEP_NO_MQ=1: no groups (general path).
bool same_layout(const CompiledApp& app, int s, int t) {
  const auto& x = app.inputs[s].attrs;
  const auto& y = app.inputs[t].attrs;
  if (x.size() != y.size()) return false;
  for (size_t c = 0; c < x.size(); ++c)
    if (x[c].type != y[c].type) return false;
  return true;
}

bool same_terms(const TermList& x, const TermList& y) {
  if (x.n != y.n || x.any != y.any) return false;
  for (int i = 0; i < x.n; ++i) {
    const Term &u = x.t[i], &v = y.t[i];
    if (u.col != v.col || u.coltype != v.coltype || u.aop != v.aop || u.atype != v.atype || u.aconst != v.aconst ||
        u.cop != v.cop || u.ctype != v.ctype || u.cconst != v.cconst)
      return false;
  }
  return true;
}

// What one query adds to a group: its conditions per stream, carried columns.
struct MqNeeds {
  int key_col = -1, layout = -1;
  std::vector<std::pair<int, TermList>> conds;   // (stream, condition), n == 0: always true
  std::vector<int> carry;                        // columns carried in records
  std::vector<int> cols;                         // columns conditions read
};

bool mq_candidate(const cep_app* a, const Query& q, MqNeeds* nd) {
  const CompiledApp& app = a->app;
  if (a->opt.sparse_keys) return false;
  auto key_ok = [&](int s, int col) {
    if (s < 0 || col < 0) return false;
    const int t = app.inputs[s].attrs[col].type;
    return t == T_INT || t == T_LONG;
  };
  auto add_cols = [&](const TermList& tl) {
    for (int i = 0; i < tl.n; ++i)
      if (std::find(nd->cols.begin(), nd->cols.end(), tl.t[i].col) == nd->cols.end()) nd->cols.push_back(tl.t[i].col);
  };
  auto carry = [&](int col) {
    if (col == nd->key_col) return;
    if (std::find(nd->carry.begin(), nd->carry.end(), col) == nd->carry.end()) nd->carry.push_back(col);
  };
  if (q.kind == Q_AGG) {
    if (q.in_stream < 0 || !key_ok(q.in_stream, q.key_col)) return false;
    if ((int)q.aggs.size() > kMqMaxAggs || !q.having_simple || (int)q.select.size() > kMqMaxSel) return false;
    if (q.f.valid() && q.f_terms.n < 0) return false;
    nd->key_col = q.key_col;
    nd->layout = q.in_stream;
    TermList f;
    f.n = 0;
    if (q.f.valid()) f = q.f_terms;
    nd->conds.push_back({q.in_stream, f});
    add_cols(f);
    for (auto& ag : q.aggs) {
      if (ag.arg.valid() && ag.word < 0) return false;
      if (ag.word >= 0) carry(q.rec_cols_a[ag.word]);
    }
    for (auto& it : q.select) {
      if (it.src == SRC_KEY || (it.src >= SRC_AGG && it.src < SRC_AGG + (int)q.aggs.size())) continue;
      if (it.src >= SRC_REC && it.src < SRC_REC + (int)q.rec_cols_a.size()) {
        carry(q.rec_cols_a[it.src - SRC_REC]);
        continue;
      }
      return false;
    }
    return true;
  }
  if (q.kind != Q_PATTERN || !q.nfa || !q.sequence) return false;
  const int n = (int)q.nstates.size();
  if (n < 1 || n > kMaxStates || q.nstates[0].min_count != 1 || q.nstates[0].max_count != 1) return false;
  if ((int)q.ncaps.size() > kMqMaxCaps || (int)q.select.size() > kMqMaxSel) return false;
  for (int j = 0; j < n; ++j) {
    const auto& st = q.nstates[j];
    if (j > 0 && st.stream == q.nstates[0].stream) return false;   // one live partial per key
    if (st.walk.valid() || st.terms.n < 0 || st.min_count > 254 || st.max_count > 254) return false;
    const int col = st.stream < (int)q.key_col_s.size() ? q.key_col_s[st.stream] : -1;
    if (!key_ok(st.stream, col) || (nd->key_col >= 0 && col != nd->key_col)) return false;
    if (!same_layout(app, st.stream, q.nstates[0].stream)) return false;
    nd->key_col = col;
  }
  nd->layout = q.nstates[0].stream;
  for (int j = 0; j < n; ++j) {
    nd->conds.push_back({q.nstates[j].stream, q.nstates[j].terms});
    add_cols(q.nstates[j].terms);
  }
  for (auto& cp : q.ncaps) {
    if (cp.index != 0 && cp.index != -1) return false;
    carry(q.rec_cols_a[cp.word]);
  }
  for (auto& it : q.select)
    if (!(it.src == SRC_KEY || (it.src >= SRC_CAP && it.src < SRC_CAP + (int)q.ncaps.size()))) return false;
  return true;
}

int mq_index(std::vector<int>& v, int x) {
  for (size_t i = 0; i < v.size(); ++i)
    if (v[i] == x) return (int)i;
  v.push_back(x);
  return (int)v.size() - 1;
}

// Condition bit of `tl` on stream s in group g (added when new); -1: full.
int mq_cond_bit(MqRT& g, int s, const TermList& tl, bool add) {
  if (tl.n == 0) return kMqTrueBit;
  for (int c = 0; c < g.ncond[s]; ++c)
    if (same_terms(g.conds[s * kMqMaxCond + c].tl, tl)) return c;
  if (g.ncond[s] >= kMqMaxCond) return -1;
  if (!add) return g.ncond[s];
  MqCond& mc = g.conds[s * kMqMaxCond + g.ncond[s]];
  std::memset(&mc, 0, sizeof(mc));
  mc.tl = tl;
  return g.ncond[s]++;
}

// Prefetched columns of a group: the key first, then condition and carried
// columns (k_mqpart loads each once per row).
std::vector<int> mq_pref_cols(const MqRT& g) {
  std::vector<int> v{g.key_col};
  for (int c : g.cond_cols) mq_index(v, c);
  for (int c : g.carry) mq_index(v, c);
  return v;
}

// A shape class of one group's queries (walk unit kinds, kernels.h MqUnit).
struct MqClassB {
  int kind = MQU_SEQ;
  std::string sig;
  int key_col = -1, layout = -1;
  std::vector<int> qs;
  std::vector<MqNeeds> nds;
};

// Shape signature: queries with equal signatures run as one walk unit
// (sequence classes advance bit-parallel, aggregations share the decode).
std::string mq_signature(const cep_app* a, const Query& q, const MqNeeds& nd, int* kind) {
  const CompiledApp& app = a->app;
  std::string sg = std::to_string(nd.key_col) + "/" + std::to_string(nd.layout) + "|";
  auto add = [&](int64_t v) { sg += std::to_string(v) + ","; };
  const auto& od = app.outputs[app.output_index(q.out_stream)];
  for (auto& at : od.attrs) add(at.type);
  sg += "|";
  for (auto& it : q.select) add(it.src >= SRC_REC && it.src < SRC_REC + (int)q.rec_cols_a.size()
                                    ? 1000 + q.rec_cols_a[it.src - SRC_REC] : it.src);
  sg += "|";
  if (q.kind == Q_AGG) {
    *kind = MQU_AGG;
    add(q.in_stream);
    for (auto& ag : q.aggs) {
      add(ag.fn);
      add(ag.word >= 0 ? q.rec_cols_a[ag.word] : -1);
      add(ag.arg_type);
      add(ag.out_type);
    }
    sg += "|";
    add(q.having_item);
    if (q.having_item >= 0) {
      add(q.having_cop);
      add(q.having_ctype);
    }
    return "A" + sg;
  }
  // sequences: bit-parallel when every state reads its own stream and counts
  // "one" or "one or more" (optional states allowed)
  bool bp = true;
  const int n = (int)q.nstates.size();
  for (int j = 0; j < n; ++j) {
    const auto& st = q.nstates[j];
    for (int k = 0; k < j; ++k) bp = bp && q.nstates[k].stream != st.stream;
    bp = bp && st.min_count <= 1 && (st.max_count == 1 || st.max_count < 0);
  }
  *kind = bp ? MQU_SEQ_BP : MQU_SEQ;
  add(q.every ? 1 : 0);
  add(q.within);
  for (auto& st : q.nstates) {
    add(st.stream);
    add(st.min_count);
    add(st.max_count);
  }
  sg += "|";
  for (auto& cp : q.ncaps) {
    add(cp.state);
    add(cp.index);
    add(q.rec_cols_a[cp.word]);
  }
  return "S" + sg;
}

// Record bit of a run of conditions on stream s (query order), sharing an
// identical run already placed; -1 when the stream's bits are used up.
int mq_cond_run(MqRT& g, int s, const std::vector<TermList>& run, bool add) {
  const int n = (int)run.size();
  for (int i = 0; i + n <= g.ncond[s]; ++i) {
    bool same = true;
    for (int j = 0; j < n && same; ++j) same = same_terms(g.conds[s * kMqMaxCond + i + j].tl, run[j]);
    if (same) return i;
  }
  if (g.ncond[s] + n > kMqMaxCond) return -1;
  if (!add) return g.ncond[s];
  const int at = g.ncond[s];
  for (int j = 0; j < n; ++j) {
    MqCond& mc = g.conds[s * kMqMaxCond + at + j];
    std::memset(&mc, 0, sizeof(mc));
    mc.tl = run[j];
  }
  g.ncond[s] += n;
  return at;
}

// Place a class's conditions into group g (bit-parallel classes: one run per
// state; others: one bit per distinct condition).  false: no room.
bool mq_place_conds(const cep_app* a, MqRT& g, const MqClassB& c) {
  const CompiledApp& app = a->app;
  if (c.kind == MQU_SEQ_BP) {
    const Query& q0 = app.queries[c.qs[0]];
    for (size_t j = 0; j < q0.nstates.size(); ++j) {
      std::vector<TermList> run;
      bool any = false;
      for (int qi : c.qs) {
        run.push_back(app.queries[qi].nstates[j].terms);
        any = any || app.queries[qi].nstates[j].terms.n > 0;
      }
      if (any && mq_cond_run(g, q0.nstates[j].stream, run, true) < 0) return false;
    }
    return true;
  }
  for (auto& nd : c.nds)
    for (auto& cd : nd.conds)
      if (cd.second.n > 0 && mq_cond_run(g, cd.first, {cd.second}, true) < 0) return false;
  return true;
}

int build_mq_groups(cep_app* a) {
  const CompiledApp& app = a->app;
  a->in_mq.assign(app.queries.size(), 0);
  if (std::getenv("CEP_NO_MQ") || app.inputs.size() > 8) return CEP_OK;
  // shape classes of the candidates, in plan order of their first query
  std::vector<MqClassB> classes;
  for (size_t qi = 0; qi < app.queries.size(); ++qi) {
    MqNeeds nd;
    if (!mq_candidate(a, app.queries[qi], &nd)) continue;
    int kind;
    const std::string sig = mq_signature(a, app.queries[qi], nd, &kind);
    MqClassB* c = nullptr;
    for (auto& x : classes)
      if (x.sig == sig && x.kind != MQU_SEQ && (int)x.qs.size() < (x.kind == MQU_SEQ_BP ? kMqMaxCond : kMqMaxQ))
        c = &x;
    if (!c) {
      classes.push_back(MqClassB());
      c = &classes.back();
      c->kind = kind;
      c->sig = sig;
      c->key_col = nd.key_col;
      c->layout = nd.layout;
    }
    c->qs.push_back((int)qi);
    c->nds.push_back(nd);
  }
  // classes into groups: a class joins the first group with room (queries,
  // carried / prefetched columns, condition bits); a class too large for an
  // empty group is halved
  std::vector<int> layouts;   // per group: a stream of its layout
  std::vector<std::vector<MqClassB>> gclasses;
  for (size_t ci = 0; ci < classes.size(); ++ci) {
    MqClassB c = classes[ci];
    auto fits = [&](MqRT& g) {
      MqRT t;
      t.key_col = g.key_col;
      t.cond_cols = g.cond_cols;
      t.carry = g.carry;
      t.conds = g.conds;
      std::copy(g.ncond, g.ncond + 8, t.ncond);
      for (auto& nd : c.nds) {
        for (int x : nd.cols) mq_index(t.cond_cols, x);
        for (int x : nd.carry) mq_index(t.carry, x);
      }
      if ((int)t.carry.size() > kMqMaxCarry || (int)mq_pref_cols(t).size() > kPref) return false;
      if ((int)(g.qs.size() + c.qs.size()) > kMqMaxQ) return false;
      if (!mq_place_conds(a, t, c)) return false;
      g.cond_cols = t.cond_cols;
      g.carry = t.carry;
      g.conds = t.conds;
      std::copy(t.ncond, t.ncond + 8, g.ncond);
      return true;
    };
    int gi = -1;
    for (size_t i = 0; i < a->mqs.size() && gi < 0; ++i)
      if (a->mqs[i].key_col == c.key_col && same_layout(app, layouts[i], c.layout) && fits(a->mqs[i])) gi = (int)i;
    if (gi < 0) {
      MqRT g;
      g.key_col = c.key_col;
      g.conds.resize(8 * kMqMaxCond);
      if (!fits(g)) {
        if (c.qs.size() > 1) {   // halve the class and place both halves
          MqClassB h = c;
          const size_t m = c.qs.size() / 2;
          c.qs.resize(m);
          c.nds.resize(m);
          h.qs.erase(h.qs.begin(), h.qs.begin() + m);
          h.nds.erase(h.nds.begin(), h.nds.begin() + m);
          classes[ci] = c;
          classes.insert(classes.begin() + ci + 1, h);
          --ci;
        }
        continue;   // a single query that fits no group: general path
      }
      a->mqs.push_back(std::move(g));
      layouts.push_back(c.layout);
      gclasses.emplace_back();
      gi = (int)a->mqs.size() - 1;
    }
    MqRT& g = a->mqs[gi];
    for (int qi : c.qs) {
      g.qs.push_back(qi);
      a->in_mq[qi] = 1;
    }
    gclasses[gi].push_back(c);
  }
  // a group of one query stays on its own PatternRT: the key shuffle entry
  // points (cep_route_batch / cep_send_records) and v2-v4 snapshots of such
  // apps address that runtime
  for (size_t gi = a->mqs.size(); gi-- > 0;) {
    if (a->mqs[gi].qs.size() >= 2) continue;
    for (int qi : a->mqs[gi].qs) a->in_mq[qi] = 0;
    a->mqs.erase(a->mqs.begin() + gi);
    gclasses.erase(gclasses.begin() + gi);
    layouts.erase(layouts.begin() + gi);
  }
  for (size_t gi = 0; gi < a->mqs.size(); ++gi)
    for (auto& c : gclasses[gi]) {
      a->mqs[gi].classes_kind.push_back(c.kind);
      a->mqs[gi].classes_n.push_back((int)c.qs.size());
    }
  // device descriptors, state and arenas per group
  for (auto& g : a->mqs) {
    const int64_t K = a->opt.key_capacity;
    g.key_capacity = K;
    g.key_stride = std::max(1, a->opt.key_stride);
    g.key_offset = a->opt.key_offset;
    int64_t chunk = std::max<int64_t>(a->opt.chunk_events, kMqTile);
    chunk = std::min<int64_t>(chunk, (int64_t)kMqMaxTiles * kMqTile);
    g.chunk = (chunk / kMqTile) * kMqTile;
    const int nphys_max = std::min<int>((int)g.carry.size(), kMqMaxPhys);
    const int W = mq_window(nphys_max);
    // keys per bucket: about half a window of records per bucket per chunk
    int64_t kpb = 64;
    while (kpb * 2 <= kMqMaxKpb && (double)g.chunk * (double)(kpb * 2) / (double)K <= W / 2) kpb *= 2;
    int lg = 0;
    while (((K + (1 << lg) - 1) >> lg) > kpb) ++lg;
    while (lg > 0 && (1 << lg) > kMqMaxBuckets) --lg;
    kpb = (K + (1 << lg) - 1) >> lg;
    if (kpb > kMqMaxKpb) return fail(a, CEP_E_CAPACITY, "key_capacity too large for a multi-query group");
    g.lg = lg;
    g.kpb = (int)kpb;
    g.kstride = kpb << lg;
    // descriptors (class order), then the walk units
    int64_t off = 0;
    std::vector<int> qkind;   // per descriptor: its class's unit kind
    for (size_t ci = 0; ci < g.classes_kind.size(); ++ci)
      for (int i = 0; i < g.classes_n[ci]; ++i) qkind.push_back(g.classes_kind[ci]);
    for (int qi : g.qs) {
      const Query& q = app.queries[qi];
      MqQuery d;
      std::memset(&d, 0, sizeof(d));
      d.st_off = off;
      const int oi = app.output_index(q.out_stream);
      const auto& od = app.outputs[oi];
      d.nsel = (int)q.select.size();
      for (int i = 0; i < d.nsel; ++i) d.sel_type[i] = od.attrs[i].type;
      d.hav_item = -1;
      auto lword = [&](int col) { return col == g.key_col ? (int)MQ_SRC_KEY : mq_index(g.carry, col); };
      if (q.kind == Q_AGG) {
        d.kind = MQ_AGG;
        d.in_stream = q.in_stream;
        d.stream_mask = 1u << q.in_stream;
        TermList f;
        f.n = 0;
        if (q.f.valid()) f = q.f_terms;
        d.filter_bit = mq_cond_bit(g, q.in_stream, f, false);
        d.nagg = (int)q.aggs.size();
        for (int i = 0; i < d.nagg; ++i) {
          d.agg_fn[i] = q.aggs[i].fn;
          d.agg_arg_type[i] = q.aggs[i].arg_type;
          d.agg_out_type[i] = q.aggs[i].out_type;
          d.agg_src[i] = q.aggs[i].word >= 0 ? lword(q.rec_cols_a[q.aggs[i].word]) : (int)MQ_SRC_KEY;
        }
        for (int i = 0; i < d.nsel; ++i) {
          const int src = q.select[i].src;
          d.sel_src[i] = (src >= SRC_REC && src < SRC_REC + (int)q.rec_cols_a.size())
                             ? SRC_REC + lword(q.rec_cols_a[src - SRC_REC])
                             : src;
        }
        if (q.having_item >= 0) {
          d.hav_item = q.having_item;
          d.hav_cop = q.having_cop;
          d.hav_ctype = q.having_ctype;
          d.hav_cconst = q.having_cconst;
        }
        d.nwords = 1 + d.nagg;
      } else {
        d.kind = MQ_SEQ;
        d.nstates = (int)q.nstates.size();
        d.every = q.every ? 1 : 0;
        d.within = q.within;
        for (int j = 0; j < d.nstates; ++j) {
          const auto& st = q.nstates[j];
          d.stream_mask |= 1u << st.stream;
          d.st_stream |= (uint32_t)st.stream << (3 * j);
          d.st_bit |= (uint64_t)mq_cond_bit(g, st.stream, st.terms, false) << (6 * j);
          d.st_min |= (uint64_t)st.min_count << (8 * j);
          d.st_max |= (uint64_t)(st.max_count < 0 ? 0xff : st.max_count) << (8 * j);
          bool opt = true;
          for (int k = j + 1; k < d.nstates; ++k) opt = opt && q.nstates[k].min_count == 0;
          if (opt) d.tail_opt |= 1u << j;
        }
        d.ncap = (int)q.ncaps.size();
        for (int i = 0; i < d.ncap; ++i) {
          d.cap_state[i] = q.ncaps[i].state;
          d.cap_last[i] = q.ncaps[i].index < 0 ? 1 : 0;
          d.cap_src[i] = lword(q.rec_cols_a[q.ncaps[i].word]);
        }
        for (int i = 0; i < d.nsel; ++i) d.sel_src[i] = q.select[i].src;
        d.nwords = 2 + d.ncap;
      }
      for (int i = 0; i < d.nsel; ++i) {
        const int src = d.sel_src[i];
        d.sel_vi[i] = (src >= SRC_CAP && src < SRC_CAP + kMqMaxCaps) ? 1 + (src - SRC_CAP)
                      : (src >= SRC_AGG && src < SRC_AGG + kMqMaxAggs) ? 1 + (src - SRC_AGG)
                      : (src >= SRC_REC && src < SRC_REC + kMqMaxCarry) ? 5 + (src - SRC_REC)
                                                                         : 0;
        d.sel_w[i] = type_width(d.sel_type[i]);
      }
      d.hav_vi = d.hav_item >= 0 ? d.sel_vi[d.hav_item] : 0;
      g.stream_mask |= d.stream_mask;
      g.check_order = g.check_order || (d.kind == MQ_SEQ && d.within >= 0);
      if (qkind[g.hq.size()] == MQU_SEQ_BP) d.nwords = 0;   // class state (unit)
      off += d.nwords;
      g.hq.push_back(d);
    }
    g.units.clear();
    for (size_t ci = 0, q0 = 0; ci < g.classes_kind.size(); q0 += g.classes_n[ci], ++ci) {
      const int n = g.classes_n[ci];
      MqUnit u;
      std::memset(&u, 0, sizeof(u));
      u.kind = g.classes_kind[ci];
      u.q0 = (int)q0;
      if (u.kind == MQU_SEQ) {
        for (int i = 0; i < n; ++i) {
          u.q0 = (int)q0 + i;
          u.nq = 1;
          g.units.push_back(u);
        }
      } else if (u.kind == MQU_SEQ_BP) {
        const Query& q = app.queries[g.qs[q0]];
        const int N = (int)q.nstates.size();
        u.nq = n;
        u.st_off = off;
        off += 4 + (int64_t)q.ncaps.size();   // live mask, started mask, state, start ts, captures
        u.keep_last = q.nstates[N - 1].max_count < 0 ? 1 : 0;
        for (int j = 0; j < N; ++j) {
          const auto& st = q.nstates[j];
          u.st_of_stream |= (uint32_t)(j + 1) << (4 * st.stream);
          for (int t = 0; t < N; ++t) {
            bool ok = (t == j && st.max_count < 0);
            if (t > j) {
              ok = true;
              for (int k = j + 1; k < t; ++k) ok = ok && q.nstates[k].min_count == 0;
            }
            if (ok) u.allow |= 1ull << (j * 8 + t);
          }
          std::vector<TermList> run;
          bool any = false;
          for (int i = 0; i < n; ++i) {
            run.push_back(app.queries[g.qs[q0 + i]].nstates[j].terms);
            any = any || run.back().n > 0;
          }
          const uint64_t cb = any ? (uint64_t)mq_cond_run(g, st.stream, run, false) : 0xffull;
          u.cbase |= cb << (8 * j);
        }
        for (int j = N; j < 8; ++j) u.cbase |= 0xffull << (8 * j);
        g.units.push_back(u);
      } else {
        const Query& q = app.queries[g.qs[q0]];
        int na = 0;
        for (auto& ag : q.aggs) na += ag.fn != AGG_COUNT ? 1 : 0;
        int nu = na <= 1 ? 8 : na == 2 ? 4 : 2;   // k_mqwalk's mq_agg_unit widths
        static const int nu_cap = std::getenv("CEP_MQ_NU") ? std::atoi(std::getenv("CEP_MQ_NU")) : 8;
        if (nu_cap == 4 || nu_cap == 2) nu = std::min(nu, nu_cap);   // diagnostics: narrower units
        // mq_agg_fast: at most one non-count accumulator, having compared as
        // a double or an integer (not a float)
        const MqQuery& d0 = g.hq[q0];
        int fast = 0;
        if (na <= 1 && (d0.hav_item < 0 || d0.hav_ctype == T_DOUBLE || d0.hav_ctype == T_LONG ||
                        d0.hav_ctype == T_INT)) {
          fast = 9;
          for (int y = 0; y < d0.nagg; ++y) {
            const int fn = d0.agg_fn[y], t = d0.agg_arg_type[y];
            if (fn == AGG_COUNT) continue;
            const int acmp = (t == T_LONG || t == T_INT) ? 0 : t == T_FLOAT ? 1 : 2;
            (void)acmp;   // min / max: generic mq_agg_unit (fast shapes 3-8 are not built)
            fast = (fn == AGG_MIN || fn == AGG_MAX) ? 0 : (fn == AGG_SUM && d0.agg_out_type[y] == T_LONG) ? 2 : 1;
          }
        }
        static const bool no_fast = std::getenv("CEP_MQ_GENERIC") != nullptr;   // diagnostics
        if (fast && !no_fast) nu = std::min(nu, 4);   // mq_agg_fast is built 4 queries wide
        for (int i = 0; i < n; i += nu) {
          u.q0 = (int)q0 + i;
          u.nq = std::min(nu, n - i);
          u.nu = nu;
          u.fast = no_fast ? 0 : fast;
          g.units.push_back(u);
        }
      }
    }
    g.words = off;
    const int ntiles = (int)(g.chunk / kMqTile);
    bool ok = dev_ensure(&g.dq, g.hq.size() * sizeof(MqQuery), a->stream, false) &&
              dev_ensure(&g.du, g.units.size() * sizeof(MqUnit), a->stream, false) &&
              dev_ensure(&g.dconds, g.conds.size() * sizeof(MqCond), a->stream, false) &&
              dev_ensure(&g.state, (size_t)g.words * g.kstride * 8, a->stream, false);
    for (int b = 0; b < 2 && ok; ++b)
      ok = dev_ensure(&g.recs[b], (size_t)g.chunk * (2 + nphys_max) * 8 + 16, a->stream, false) &&
           dev_ensure(&g.toff[b], (size_t)((1 << lg) + 1) * ntiles * 2 + 16, a->stream, false) &&
           dev_ensure(&g.chunk_base[b], 64, a->stream, false) &&
           hipEventCreateWithFlags(&g.part_done[b], hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&g.walk_done[b], hipEventDisableTiming) == hipSuccess;
    if (!ok) return fail(a, CEP_E_DEVICE, "out of device memory (multi-query group)");
    hipMemset(g.state.p, 0, (size_t)g.words * g.kstride * 8);
    // condition slots: the prefetch slot of each term's column
    const std::vector<int> pc = mq_pref_cols(g);
    for (auto& mc : g.conds)
      for (int i = 0; i < mc.tl.n && i < kMaxTerms; ++i)
        for (size_t sl = 0; sl < pc.size(); ++sl)
          if (pc[sl] == mc.tl.t[i].col) mc.slot[i] = (int32_t)sl;
    hipMemcpy(g.dconds.p, g.conds.data(), g.conds.size() * sizeof(MqCond), hipMemcpyHostToDevice);
    hipMemcpy(g.du.p, g.units.data(), g.units.size() * sizeof(MqUnit), hipMemcpyHostToDevice);
  }
  return CEP_OK;
}

int create_runtime(cep_app* a) {
  const CompiledApp& app = a->app;
  if (hipSetDevice(a->opt.device) != hipSuccess)
    return fail(a, CEP_E_DEVICE, "no HIP device " + std::to_string(a->opt.device));
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, a->opt.device) != hipSuccess)
    return fail(a, CEP_E_DEVICE, "hipGetDeviceProperties failed");
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
    return fail(a, CEP_E_DEVICE, std::string("libcep is built for gfx950, device is ") +
                                     prop.gcnArchName);
  if (hipStreamCreateWithFlags(&a->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&a->side, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&a->in_ready, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&a->ext_ready, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&a->out_ready, hipEventDisableTiming) != hipSuccess ||
      hipStreamCreateWithFlags(&a->copy, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&a->rstream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&a->r_ready, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&a->r_host, hipEventDisableTiming) != hipSuccess)
    return fail(a, CEP_E_DEVICE, "hipStreamCreate failed");
  size_t cb = std::max<size_t>(app.code.size(), 1) * sizeof(Ins);
  size_t kb = std::max<size_t>(app.konst.size(), 1) * 8;
  if (!dev_ensure(&a->code, cb, a->stream, false) || !dev_ensure(&a->konst, kb, a->stream, false) ||
      !dev_ensure(&a->err, 64, a->stream, false) || !dev_ensure(&a->rerr, 64, a->stream, false) ||
      !dev_ensure(&a->ticket, 64, a->stream, false))
    return fail(a, CEP_E_DEVICE, "out of device memory (plan)");
  if (!app.code.empty())
    hipMemcpy(a->code.p, app.code.data(), app.code.size() * sizeof(Ins), hipMemcpyHostToDevice);
  if (!app.konst.empty())
    hipMemcpy(a->konst.p, app.konst.data(), app.konst.size() * 8, hipMemcpyHostToDevice);
  hipMemset(a->err.p, 0, 64);
  hipMemset(a->rerr.p, 0, 64);
  // every output's row cursor in one device array: the flush reads them with
  // one copy and resets them with one memset (64 outputs at config 5)
  if (!dev_ensure(&a->out_counts, std::max<size_t>(app.outputs.size(), 1) * 8, a->stream, false))
    return fail(a, CEP_E_DEVICE, "out of device memory");
  hipMemset(a->out_counts.p, 0, std::max<size_t>(app.outputs.size(), 1) * 8);
  for (auto& sd : app.outputs) {
    OutStream o;
    o.id = sd.id;
    for (auto& at : sd.attrs) o.types.push_back(at.type);
    o.cols.resize(sd.attrs.size());
    o.count = (unsigned long long*)a->out_counts.p + a->outs.size();
    // arrival numbers: read by the ordered flush and by consumers that asked
    // for them (cep_output_device returns seq = NULL otherwise)
    o.write_seq = !(a->opt.omit_seq && !a->opt.ordered_output);
    a->outs.push_back(std::move(o));
  }
  {
    const int rc = build_mq_groups(a);
    if (rc) return rc;
  }
  for (size_t qi = 0; qi < app.queries.size(); ++qi) {
    const Query& q = app.queries[qi];
    if (q.kind != Q_PATTERN && q.kind != Q_AGG) continue;
    if (a->in_mq[qi]) continue;   // served by a multi-query group
    const bool agg = q.kind == Q_AGG;
    // group-by state: one slot of (accumulator, count) pairs per group
    const int S = agg ? 1 : a->opt.pending_slots;
    PatternRT rt;
    rt.q = (int)qi;
    PatternArgs& p = rt.pa;
    p.a_stream = q.a_stream;
    p.b_stream = q.b_stream;
    p.f_prog = q.f.off;
    p.g_raw_prog = q.g_raw.off;
    p.g_walk_prog = q.g_walk.off;
    p.f_terms = q.f_terms;
    p.g_terms = q.g_terms;
    p.every = q.every ? 1 : 0;
    p.within = q.within;
    p.key_col_a = q.key_col_a;
    p.key_col_b = q.key_col_b;
    p.nrec_a = (int)q.rec_cols_a.size();
    p.nrec_b = (int)q.rec_cols_b.size();
    for (int i = 0; i < p.nrec_a; ++i) p.rec_a[i] = q.rec_cols_a[i];
    for (int i = 0; i < p.nrec_b; ++i) p.rec_b[i] = q.rec_cols_b[i];
    p.ncap = (int)q.cap_from_rec.size();
    for (int i = 0; i < p.ncap; ++i) p.cap_from_rec[i] = q.cap_from_rec[i];
    p.rec_words = 2 + std::max(p.nrec_a, p.nrec_b);
    p.slot_words = agg ? 2 * (int)q.aggs.size() : 2 + p.ncap;
    p.key_words = 1 + S * p.slot_words;
    p.pending_slots = S;
    // closed form keeps each record's carried words in LDS (kWalkCapLds)
    p.closed_form = (!agg && q.every && !q.g_in_walk && p.rec_words <= 2 + kWalkCapLds) ? 1 : 0;
    p.agg_mode = agg ? 1 : 0;
    p.nagg = agg ? (int)q.aggs.size() : 0;
    for (int i = 0; i < p.nagg; ++i) {
      p.agg_fn[i] = q.aggs[i].fn;
      p.agg_arg_type[i] = q.aggs[i].arg_type;
      p.agg_out_type[i] = q.aggs[i].out_type;
      p.agg_word[i] = q.aggs[i].word;
    }
    p.having_prog = agg ? q.having.off : -1;
    if (q.nfa) {
      if (app.inputs.size() > 8)
        return fail(a, CEP_E_UNSUPPORTED, "patterns / sequences over apps with more than 8 input streams");
      p.nfa_mode = 1;
      p.nfa_seq = q.sequence ? 1 : 0;
      p.nstates = (int)q.nstates.size();
      p.closed_form = 0;
      p.ncap = (int)q.ncaps.size();
      p.slot_words = 2 + p.ncap;
      p.key_words = 1 + S * p.slot_words;
      p.stream_mask = 0;
      for (int j = 0; j < p.nstates; ++j) {
        const auto& st = q.nstates[j];
        p.st_stream[j] = st.stream;
        p.st_min[j] = st.min_count;
        p.st_max[j] = st.max_count;
        p.st_raw[j] = st.raw.off;
        p.st_walk[j] = st.walk.off;
        p.stream_mask |= 1 << st.stream;
      }
      for (int j = 0; j < p.nstates; ++j) {
        bool opt = true;
        for (int k = j + 1; k < p.nstates; ++k) opt = opt && q.nstates[k].min_count == 0;
        p.st_tail_opt[j] = opt ? 1 : 0;
      }
      for (int i = 0; i < 8; ++i) p.key_col_s[i] = i < (int)q.key_col_s.size() ? q.key_col_s[i] : -1;
      for (int i = 0; i < p.ncap; ++i) {
        p.cap_state[i] = q.ncaps[i].state;
        p.cap_index[i] = q.ncaps[i].index;
        p.cap_word[i] = q.ncaps[i].word;
        // Siddhi reads an unmatched (optional) state's attribute as null: for
        // a STRING the engine writes dictionary id -1, which no string has
        const int st = q.nstates[q.ncaps[i].state].stream;
        const int col = q.ncaps[i].word < (int)q.rec_cols_a.size() ? q.rec_cols_a[q.ncaps[i].word] : -1;
        const bool str = st >= 0 && st < (int)app.inputs.size() && col >= 0 &&
                         col < (int)app.inputs[st].attrs.size() && app.inputs[st].attrs[col].type == T_STRING;
        p.cap_null[i] = str ? ~0ull : 0ull;
      }
    }
    // NFA patterns stage advanced partials in a second bank of S slots (so do
    // the order-tolerant runs of a 2-state pattern with `within`: nfa_pair)
    const int bank = (q.nfa || (q.within >= 0 && !agg)) ? 2 : 1;
    const bool keyed = q.key_col_a >= 0;
    int64_t kcap = keyed ? a->opt.key_capacity : 1;
    p.key_capacity = kcap;
    p.key_stride = keyed ? std::max(1, a->opt.key_stride) : 1;
    p.key_offset = keyed ? a->opt.key_offset : 0;
    if (!keyed && (a->opt.key_stride > 1))
      return fail(a, CEP_E_UNSUPPORTED, "an unpartitioned query cannot be sharded");
    int lg = std::max(0, std::min(12, a->opt.buckets_log2));
    while ((kcap >> lg) > kWalkMaxKeys && lg < 12) ++lg;
    if ((kcap + (1 << lg) - 1) >> lg > kWalkMaxKeys)
      return fail(a, CEP_E_CAPACITY, "key_capacity exceeds 1024 * 4096 keys");
    if (!keyed) lg = 0;
    p.buckets_log2 = lg;
    const int64_t kc = kcap;
    const int64_t kpb = (kc + (1 << lg) - 1) >> lg;
    rt.kstride = kpb << lg;
    if (!dev_ensure(&rt.khdr, (size_t)rt.kstride * 4, a->stream, false) ||
        !dev_ensure(&rt.kslot, (size_t)rt.kstride * bank * S * p.slot_words * 8, a->stream, false) ||
        !dev_ensure(&rt.chunk_base[0], 64, a->stream, false) ||
        !dev_ensure(&rt.chunk_base[1], 64, a->stream, false))
      return fail(a, CEP_E_DEVICE, "out of device memory (pattern state)");
    hipMemset(rt.khdr.p, 0, (size_t)rt.kstride * 4);
    // the walk build decides the chunk cap (its LDS segment tables)
    bool walk_vm = q.g_in_walk || agg || q.nfa;
    for (auto& it : q.select) walk_vm |= it.src == SRC_VM;
    int64_t chunk = a->opt.chunk_events;
    chunk = std::max<int64_t>(chunk, kPartThreads * kPartItems);
    chunk = std::min<int64_t>(chunk, (int64_t)(walk_vm ? kWalkMaxTiles : kWalkMaxTiles / 4) *
                                         kPartThreads * kPartItems);
    chunk = (chunk / (kPartThreads * kPartItems)) * (kPartThreads * kPartItems);
    rt.chunk = chunk;
    // the order-tolerant form of a `within` pattern (ts_order 0, released
    // late rows) runs on the VM walk, whose segment tables hold 4x the tiles:
    // its chunks may be that long, so per-key state is loaded and committed
    // a quarter as often
    int64_t chunk_tol = chunk;
    if (!walk_vm && q.within >= 0) {
      chunk_tol = std::max<int64_t>(a->opt.chunk_events, kPartThreads * kPartItems);
      chunk_tol = std::min<int64_t>(chunk_tol, (int64_t)kWalkMaxTiles * kPartThreads * kPartItems);
      chunk_tol = (chunk_tol / (kPartThreads * kPartItems)) * (kPartThreads * kPartItems);
    }
    rt.chunk_tol = chunk_tol;
    const int64_t ntiles = std::max(chunk, chunk_tol) / (kPartThreads * kPartItems);
    for (int b = 0; b < 2; ++b) {
      if (!dev_ensure(&rt.recs[b], (size_t)std::max(chunk, chunk_tol) * p.rec_words * 8 + 16, a->stream, false) ||
          !dev_ensure(&rt.tile_off[b], (size_t)ntiles * ((1 << lg) + 1) * 2, a->stream, false))
        return fail(a, CEP_E_DEVICE, "out of device memory (record arena)");
      if (hipEventCreateWithFlags(&rt.part_done[b], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&rt.walk_done[b], hipEventDisableTiming) != hipSuccess)
        return fail(a, CEP_E_DEVICE, "hipEventCreate failed");
    }
    rt.extra_bound = (int64_t)S * kc;
    rt.part_vm = (q.f.off >= 0 && q.f_terms.n < 0) || (q.g_raw.off >= 0 && q.g_terms.n < 0) || q.nfa;
    // fast partition path: all columns the pass reads fit kPref registers
    if (!rt.part_vm && q.key_col_a == q.key_col_b && p.nrec_a <= kPfRec && p.nrec_b <= kPfRec) {
      PrefPlan& pf = rt.pref;
      std::vector<int> cols;
      auto slot = [&](int c) {
        for (size_t i = 0; i < cols.size(); ++i)
          if (cols[i] == c) return (int)i;
        cols.push_back(c);
        return (int)cols.size() - 1;
      };
      pf.key_slot = q.key_col_a >= 0 ? slot(q.key_col_a) : -1;   // slot 0: k_cfpart reads it there
      if (q.f.off >= 0)
        for (int i = 0; i < q.f_terms.n; ++i) pf.f_slot[i] = slot(q.f_terms.t[i].col);
      if (q.g_raw.off >= 0)
        for (int i = 0; i < q.g_terms.n; ++i) pf.g_slot[i] = slot(q.g_terms.t[i].col);
      for (int i = 0; i < p.nrec_a; ++i) pf.reca_slot[i] = slot(p.rec_a[i]);
      for (int i = 0; i < p.nrec_b; ++i) pf.recb_slot[i] = slot(p.rec_b[i]);
      if (!cols.empty() && (int)cols.size() <= kPref) {
        pf.n = (int)cols.size();
        for (int i = 0; i < kPref; ++i) pf.col[i] = i < pf.n ? cols[i] : cols[0];
      } else {
        pf.n = -1;
      }
    }
    // group-by and N-state / sequence walks live in the VM build of k_walk
    rt.walk_vm = walk_vm;
    // N-state patterns / sequences: partial lists longer than pending_slots
    // continue in the pending pool (nfa_key), as on the closed-form path
    if (q.nfa) {
      const int plg = a->opt.pending_pool_log2 > 0 ? std::min(a->opt.pending_pool_log2, 30) : 20;
      rt.pool_cap = (int64_t)1 << plg;
      const bool ok = dev_ensure(&rt.kext, (size_t)rt.kstride * 8, a->stream, false) &&
                      dev_ensure(&rt.pool[0], (size_t)rt.pool_cap * p.slot_words * 8, a->stream, false) &&
                      dev_ensure(&rt.pool[1], (size_t)rt.pool_cap * p.slot_words * 8, a->stream, false) &&
                      dev_ensure(&rt.pool_cur, 64, a->stream, false);
      if (!ok) return fail(a, CEP_E_DEVICE, "out of device memory (pending pool)");
      hipMemset(rt.kext.p, 0, (size_t)rt.kstride * 8);
      rt.extra_bound += rt.pool_cap;   // pool partials may complete too
    }
    // closed-form fast path: `every A -> B` with f / g as term lists on the
    // events' own columns, plain-copy select items, <= 2 captures, <= 512
    // keys per bucket (CEP_NO_CF=1 forces the general path)
    {
      bool ok = p.closed_form && !q.nfa && !agg && !rt.part_vm && !rt.walk_vm && rt.pref.n >= 0 &&
                p.ncap <= kCfMaxCaps && p.nrec_a <= kPfRec && p.nrec_b <= kPfRec &&
                kpb <= kCfMaxKeys && (1 << lg) <= kCfMaxBuckets && !std::getenv("CEP_NO_CF") && S >= 2 &&
                (double)rt.kstride * S * p.slot_words * 8 < 4294967296.0;   // 32-bit slot offsets
      ok = ok && (int)q.select.size() <= kCfMaxOut;
      for (auto& it : q.select)
        ok = ok && (it.src == SRC_KEY || (it.src >= SRC_CAP && it.src < SRC_CAP + kCfMaxCaps) ||
                    (it.src >= SRC_REC && it.src < SRC_REC + kPfRec));
      if (ok) {
        int64_t cc = std::max<int64_t>(a->opt.chunk_events, kCfTile);
        cc = std::min<int64_t>(cc, (int64_t)kCfMaxTiles * kCfTile);
        cc = (cc / kCfTile) * kCfTile;
        const int64_t nt = cc / kCfTile;
        const int rw = 1 + std::max(p.nrec_a, p.nrec_b);
        for (int b = 0; b < 2 && ok; ++b)
          ok = dev_ensure(&rt.cf_recs[b], (size_t)cc * rw * 8 + 16, a->stream, false) &&
               dev_ensure(&rt.cf_toff[b], (size_t)nt * ((1 << lg) + kCfHotMax + 1) * 2 + 16, a->stream, false);
        if (!ok) return fail(a, CEP_E_DEVICE, "out of device memory (record arena)");
        const int plg = a->opt.pending_pool_log2 > 0 ? std::min(a->opt.pending_pool_log2, 30) : 20;
        rt.pool_cap = (int64_t)1 << plg;
        ok = dev_ensure(&rt.kext, (size_t)rt.kstride * 8, a->stream, false) &&
             dev_ensure(&rt.pool[0], (size_t)rt.pool_cap * p.slot_words * 8, a->stream, false) &&
             dev_ensure(&rt.pool[1], (size_t)rt.pool_cap * p.slot_words * 8, a->stream, false) &&
             dev_ensure(&rt.pool_cur, 64, a->stream, false);
        if (!ok) return fail(a, CEP_E_DEVICE, "out of device memory (pending pool)");
        hipMemset(rt.kext.p, 0, (size_t)rt.kstride * 8);
        rt.extra_bound += rt.pool_cap;   // pool partials may complete too
        rt.cf = true;
        rt.cf_chunk = cc;
        // hot keys: candidate lists now, the match arenas when first needed
        if ((1 << lg) + kCfHotMax <= kCfMaxBuckets && !std::getenv("CEP_NO_HOT")) {
          rt.hot_thresh = (uint32_t)std::max<int64_t>(256, cc >> 16);
          if (const char* e = std::getenv("CEP_HOT_THRESH")) rt.hot_thresh = (uint32_t)std::max(16, std::atoi(e));
          ok = dev_ensure(&rt.hot_id, (size_t)kc * 2 + 16, a->stream, false) &&
               dev_ensure(&rt.hot_key, kCfHotMax * 4, a->stream, false) &&
               dev_ensure(&rt.hot_m, kCfHotMax * 4, a->stream, false) &&
               dev_ensure(&rt.cand, kCfHotMax * 4 * 8, a->stream, false) &&
               dev_ensure(&rt.ncand, 64, a->stream, false) && dev_ensure(&rt.hot_active, 64, a->stream, false) &&
               host_ensure(&rt.hot_active_host, 64);
          ok = ok && hipEventCreateWithFlags(&rt.hot_fork, hipEventDisableTiming) == hipSuccess &&
               hipEventCreateWithFlags(&rt.hot_join, hipEventDisableTiming) == hipSuccess;
          if (!ok) return fail(a, CEP_E_DEVICE, "out of device memory (hot keys)");
          hipMemset(rt.hot_id.p, 0xff, (size_t)kc * 2 + 16);
          hipMemset(rt.hot_key.p, 0xff, kCfHotMax * 4);
          hipMemset(rt.hot_m.p, 0, kCfHotMax * 4);
          hipMemset(rt.ncand.p, 0, 64);
          hipMemset(rt.hot_active.p, 0, 64);
          std::memset(rt.hot_active_host.p, 0, 64);
          rt.hot = true;
        }
      }
    }
    if (a->opt.sparse_keys && keyed) {
      // the map feeds the closed-form path's key column: the key may appear
      // in the plan only as the partition key (and `select s1.k`)
      const PrefPlan& pf = rt.pref;
      bool ok = rt.cf && a->opt.key_stride <= 1 && pf.key_slot == 0;
      for (int i = 0; ok && i < q.f_terms.n; ++i) ok = pf.f_slot[i] != 0;
      for (int i = 0; ok && i < q.g_terms.n; ++i) ok = pf.g_slot[i] != 0;
      for (int i = 0; ok && i < p.nrec_a; ++i) ok = pf.reca_slot[i] != 0;
      for (int i = 0; ok && i < p.nrec_b; ++i) ok = pf.recb_slot[i] != 0;
      const int kt = app.inputs[q.a_stream].attrs[q.key_col_a].type;
      ok = ok && (kt == T_INT || kt == T_LONG);
      if (!ok)
        return fail(a, CEP_E_UNSUPPORTED, "not supported: sparse_keys needs a closed-form `every A -> B` pattern whose int / long "
                                          "partition key is used only as the key, on one shard");
      uint64_t tc = 1;
      while (tc < 2 * (uint64_t)kc) tc <<= 1;
      rt.sparse = true;
      rt.table_cap = tc;
      if (!dev_ensure(&rt.tkey, tc * 8, a->stream, false) || !dev_ensure(&rt.tval, tc * 4, a->stream, false) ||
          !dev_ensure(&rt.krev, (size_t)kc * 8, a->stream, false) || !dev_ensure(&rt.kcount, 64, a->stream, false))
        return fail(a, CEP_E_DEVICE, "out of device memory (key map)");
      hipMemset(rt.tkey.p, 0, tc * 8);
      hipMemset(rt.tval.p, 0xff, tc * 4);
      hipMemset(rt.kcount.p, 0, 4);
      hipMemset((char*)rt.kcount.p + 4, 0xff, 4);
    }
    // `within` makes a pattern's result depend on event-time order (App. A.3
    // prunes on every event of the waiting state's stream); a sequence keeps
    // every row of its streams and prunes by |ts - ts(s1)| in any order, an
    // aggregation has no window: neither needs the re-run
    rt.order_sensitive = p.within >= 0 && !agg && !(q.nfa && q.sequence);
    a->pats.push_back(rt);
  }
  {
    const int64_t none = INT64_MIN;
    if (!dev_ensure(&a->last_ts_dev, 64, a->stream, false) ||
        hipMemcpy(a->last_ts_dev.p, &none, 8, hipMemcpyHostToDevice) != hipSuccess)
      return fail(a, CEP_E_DEVICE, "out of device memory");
  }
  if (std::getenv("CEP_STAMPS") && !dev_ensure(&a->stamps, (size_t)2 * 4096 * 16 * 8, a->stream, false))
    return fail(a, CEP_E_DEVICE, "out of device memory (stamps)");
  hipStreamSynchronize(a->stream);
  return CEP_OK;
}

const StreamSchema* find_schema(cep_app* a, const char* id) {
  if (!id) return nullptr;
  int i = a->app.input_index(id);
  if (i >= 0) return &a->app.inputs[i];
  i = a->app.output_index(id);
  if (i >= 0) return &a->app.outputs[i];
  return nullptr;
}

int fill_attrs(const StreamSchema* s, cep_attr* out, int cap, int* n) {
  if (n) *n = (int)s->attrs.size();
  for (int i = 0; i < (int)s->attrs.size() && i < cap; ++i) {
    std::snprintf(out[i].name, sizeof(out[i].name), "%s", s->attrs[i].name.c_str());
    out[i].type = s->attrs[i].type;
  }
  return CEP_OK;
}

// Run one filter query over a device batch.
int run_filter(cep_app* a, const Query& q, const RowsArgs& rows) {
  OutStream& o = a->outs[a->app.output_index(q.out_stream)];
  o.bound += rows.n;
  int rc = ensure_out_cap(a, o, o.bound);
  if (rc) return rc;
  constexpr int64_t kTile = kFilterThreads * kFilterItems;
  const int64_t ntiles = (rows.n + kTile - 1) / kTile;
  if (ntiles == 0) return CEP_OK;
  // look-back words for k_filter's or k_filterc's (smaller) tiles
  const int64_t fcr = filterc_rows_per_tile();
  const int64_t nflags = std::max<int64_t>(ntiles, (rows.n + fcr - 1) / fcr);
  if (!dev_ensure(&a->tile_state, (size_t)nflags * 8, a->stream, false))
    return fail(a, CEP_E_DEVICE, "out of device memory (tile state)");
  hipMemsetAsync(a->tile_state.p, 0, (size_t)nflags * 8, a->stream);
  hipMemsetAsync(a->ticket.p, 0, 16, a->stream);
  FilterArgs fa{};
  fa.rows = rows;
  fa.vm = {(const Ins*)a->code.p, (const uint64_t*)a->konst.p};
  fa.in_stream = q.in_stream;
  fa.filter_prog = q.filter.off;
  fa.filter_terms = q.filter_terms;
  fa.out = out_args(o, q);
  fa.tile_state = (unsigned long long*)a->tile_state.p;
  fa.ticket = (unsigned int*)a->ticket.p;
  fa.err = (unsigned int*)a->err.p;
  bool vm = q.filter.off >= 0 && q.filter_terms.n < 0;
  for (auto& it : q.select) vm |= it.src < SRC_REC || it.src >= SRC_TS;
  // k_filterc (filter.hip): term-list predicate over at most 3 distinct
  // columns, plain projection, pair loads aligned (8-byte columns at 16
  // bytes, 4-byte at 8, 1-byte at 2 from the slice's first row, which is
  // even).  CEP_NO_FILTERC=1 keeps k_filter.
  static const bool no_fc = std::getenv("CEP_NO_FILTERC") != nullptr;
  bool fc = !vm && !no_fc && (rows.row0 & 1) == 0;
  if (fc) {
    fa.npref = 0;
    for (int i = 0; fc && i < std::max(0, q.filter_terms.n); ++i) {
      const int c = q.filter_terms.t[i].col;
      int slot = -1;
      for (int k = 0; k < fa.npref; ++k)
        if (fa.pcol[k] == c) slot = k;
      if (slot < 0) {
        if (fa.npref == 3) {
          fc = false;
          break;
        }
        slot = fa.npref;
        fa.pcol[fa.npref++] = c;
      }
      fa.fslot[i] = slot;
    }
    if (fa.npref == 0) fa.pcol[fa.npref++] = 0;   // no predicate: one (unused) column
    auto al = [&](const void* ptr, int w) {
      return (((uintptr_t)ptr + (uintptr_t)(rows.row0 * w)) & (uintptr_t)(2 * w - 1)) == 0;
    };
    for (int k = 0; fc && k < fa.npref; ++k)
      fc = al(rows.cols.p[fa.pcol[k]], type_width(rows.cols.t[fa.pcol[k]]));
    if (fc && rows.stream) fc = al(rows.stream, 1);
  }
  LaunchTimer t(a, CEP_K_FILTER);
  if (fc) {
    const int64_t tr = filterc_rows_per_tile();
    const int64_t nt = (rows.n + tr - 1) / tr;
    launch_filterc(fa, nt, a->stream);
  } else {
    launch_filter(fa, ntiles, vm, a->stream);
  }
  return CEP_OK;
}

// 16-byte loads need every prefetched column (and ts) 16-byte aligned at
// each lane's first row (lanes start at multiples of 8 rows; 1-byte columns:
// 8-byte aligned, the hardware takes dword-aligned x4 loads)
bool pref_aligned(const PrefPlan& pf, const RowsArgs& rows) {
  auto al = [&](const void* ptr, int w) {
    const uintptr_t need = w == 1 ? 7u : 15u;
    return (((uintptr_t)ptr + (uintptr_t)(rows.row0 * w)) & need) == 0;
  };
  bool ok = al(rows.ts, 8) && (!rows.stream || al(rows.stream, 1));
  for (int i = 0; i < pf.n; ++i) {
    const int c = pf.col[i];
    ok = ok && al(rows.cols.p[c], type_width(rows.cols.t[c]));
  }
  return ok;
}

// Per-batch layout of the closed-form fast path's records: carried columns
// whose buffer is the batch's event-ts buffer are rebuilt from the record ts.
bool cf_plan(const PatternRT& rt, const RowsArgs& rows, CfPlan* cf, bool from_records = false) {
  const PatternArgs& p = rt.pa;
  std::memset(cf, 0, sizeof(*cf));
  int a_phys[kMaxCaps], b_phys[kMaxCaps];
  int na = 0, nb = 0;
  auto alias = [&](int col) {
    return !from_records && rows.cols.p[col] == (const void*)rows.ts && rows.cols.t[col] == T_LONG;
  };
  for (int c = 0; c < p.nrec_a; ++c) {
    a_phys[c] = alias(p.rec_a[c]) ? -1 : na;
    if (a_phys[c] >= 0) {
      cf->a_log[na] = c;
      cf->a_slot[na++] = rt.pref.reca_slot[c];
    }
  }
  for (int c = 0; c < p.nrec_b; ++c) {
    b_phys[c] = alias(p.rec_b[c]) ? -1 : nb;
    if (b_phys[c] >= 0) {
      cf->b_log[nb] = c;
      cf->b_slot[nb++] = rt.pref.recb_slot[c];
    }
  }
  cf->nw = std::max(na, nb);
  if (cf->nw > 2) return false;
  for (int w = na; w < 2; ++w) cf->a_slot[w] = 0;
  for (int w = nb; w < 2; ++w) cf->b_slot[w] = 0;
  for (int i = 0; i < kMaxCaps; ++i) cf->cap_phys[i] = i < p.ncap ? a_phys[p.cap_from_rec[i]] : 0;
  for (int c = 0; c < kMaxCaps; ++c) cf->bcol_phys[c] = c < p.nrec_b ? b_phys[c] : 0;
  return true;
}

// Closed-form fast path: k_cfpart(c) then k_cfwalk(c) per chunk (double-
// buffered arenas; CEP_OVERLAP=1 runs the partitions on the side stream).
// tol: the order-tolerant closed form (ts in any order: g-failing B rows kept
// as expiry-only records, no pruning at A arrivals; hot keys through the
// hot kernels' order-tolerant scans).
int run_pattern_cf(cep_app* a, PatternRT& rt, const Query& q, OutStream& o,
                   const RowsArgs& rows_all, const CfPlan& cf,
                   const uint64_t* in_recs = nullptr, int in_rec_words = 0, bool tol = false) {
  const int P = 1 << rt.pa.buckets_log2;
  const bool hot_ok = rt.hot;
  // Both passes on the main stream by default: k_cfpart and k_cfwalk cannot
  // share a CU (each fills its register file), so the side stream only
  // time-slices them (measured: no throughput gain, inflated kernel times).
  // CEP_OVERLAP=1 puts the partition on the side stream.  Serial mode issues
  // no cross-stream events: every event between two kernels of one stream
  // costs a gap (rocprofv3 trace: ~15 us between k_cfpart and k_cfwalk).
  static const bool overlap = std::getenv("CEP_OVERLAP") != nullptr;
  hipStream_t side = overlap ? a->side : a->stream;
  if (overlap) {
    hipEventRecord(a->in_ready, a->stream);
    hipStreamWaitEvent(a->side, a->in_ready, 0);
  }
  // Hot-key probe: until diversion has been decided once, the first chunk is
  // short (kHotProbeRows) and followed by one stream sync, so a skewed
  // stream's hottest keys are diverted from the second chunk on instead of
  // one workgroup walking a hot key's whole run of a full chunk (seconds at
  // Zipf s = 1.1).  Uniform streams pay one short chunk and one sync per
  // runtime.
  constexpr int64_t kHotProbeRows = 1 << 20;
  for (int64_t r0 = 0, step = 0; r0 < rows_all.n; r0 += step) {
    const int b = rt.cur;
    rt.cur ^= 1;
    const bool probe = hot_ok && !rt.hot_on && !rt.hot_probed;
    step = std::min<int64_t>(probe ? std::min<int64_t>(kHotProbeRows, rt.cf_chunk) : rt.cf_chunk, rows_all.n - r0);
    RowsArgs rows = rows_all;
    rows.row0 = rows_all.row0 + r0;
    rows.n = step;
    if (r0 > 0) rows.prev_ts = INT64_MIN;   // checked inside the kernel via ts[row-1]
    const int64_t ntiles = (rows.n + kCfTile - 1) / kCfTile;
    CfPartArgs pa{};
    pa.rows = rows;
    pa.pref = rt.pref;
    pa.ts_slot = -1;
    pa.in_recs = in_recs;
    pa.in_rec_words = in_rec_words;
    for (int i = 0; i < rt.pref.n && !in_recs; ++i)
      if (rows.cols.p[rt.pref.col[i]] == (const void*)rows.ts && rows.cols.t[rt.pref.col[i]] == T_LONG)
        pa.ts_slot = i;
    pa.pat = rt.pa;
    pa.pat.tolerant = tol ? 1 : 0;
    pa.cf = cf;
    pa.chunk_base = (int64_t*)rt.chunk_base[b].p;
    pa.recs = (uint64_t*)rt.cf_recs[b].p;
    pa.tile_off = (uint16_t*)rt.cf_toff[b].p;
    pa.ntiles = (int32_t)ntiles;
    pa.err = (unsigned int*)a->err.p;
    if (a->stamps.p) pa.stamps = (uint64_t*)a->stamps.p + 4096 * 16;
    // hot keys: diversion starts once the device reported a slot in use (the
    // pinned word is refreshed asynchronously after every walk)
    const bool hot = hot_ok;
    if (hot && !rt.hot_on && *(volatile uint32_t*)rt.hot_active_host.p > 0) {
      const int rw = 1 + cf.nw;
      const int64_t cc = rt.cf_chunk, ntmax = cc / kCfTile;
      rt.hot_blocks = (int)((cc + kHotBlock - 1) / kHotBlock);
      const bool ok = dev_ensure(&rt.hot_gbase, (kCfHotMax + 1) * 4, a->stream, false) &&
                      dev_ensure(&rt.hoff, (size_t)kCfHotMax * ntmax * 4, a->stream, false) &&
                      dev_ensure(&rt.harr, (size_t)cc * rw * 8, a->stream, false) &&
                      dev_ensure(&rt.hrow, (size_t)cc * 4, a->stream, false) &&
                      dev_ensure(&rt.hnb, (size_t)cc * 4, a->stream, false) &&
                      dev_ensure(&rt.bsum, (size_t)rt.hot_blocks * 16, a->stream, false) &&
                      dev_ensure(&rt.bcnt, (size_t)rt.hot_blocks * 4, a->stream, false) &&
                      dev_ensure(&rt.boff, (size_t)rt.hot_blocks * 4, a->stream, false) &&
                      dev_ensure(&rt.hcm, kCfHotMax * 3 * 4, a->stream, false) &&
                      dev_ensure(&rt.hobase, 64, a->stream, false) &&
                      dev_ensure(&rt.htmn, (size_t)cc * 4, a->stream, false) &&
                      dev_ensure(&rt.htmx, (size_t)cc * 4, a->stream, false) &&
                      dev_ensure(&rt.hflag, (size_t)cc, a->stream, false) &&
                      dev_ensure(&rt.btol, (size_t)rt.hot_blocks * 12, a->stream, false);
      if (!ok) return fail(a, CEP_E_DEVICE, "out of device memory (hot-key arenas)");
      rt.hot_on = true;
    }
    const bool divert = hot && rt.hot_on;
    pa.hot_id = divert ? (const uint16_t*)rt.hot_id.p : nullptr;
    pa.nhot = divert ? kCfHotMax : 0;
    if (overlap && rt.used[b]) hipStreamWaitEvent(side, rt.walk_done[b], 0);   // arena b is free
    // hot keys: k_cfpart reads hot_id, which the previous chunk's
    // k_hot_update rewrites on the main stream (walk_done is recorded after
    // it), so with diversion candidates the partition waits for that chunk
    if (overlap && hot && rt.used[b ^ 1]) hipStreamWaitEvent(side, rt.walk_done[b ^ 1], 0);
    {
      LaunchTimer t(a, CEP_K_CF_PARTITION, side);
      launch_cf_partition(pa, ntiles, side);
    }
    if (overlap) {
      hipEventRecord(rt.part_done[b], side);
      hipStreamWaitEvent(a->stream, rt.part_done[b], 0);
    }
    CfWalkArgs wa{};
    wa.pat = pa.pat;
    wa.cf = cf;
    wa.recs = pa.recs;
    wa.tile_off = pa.tile_off;
    wa.ntiles = (int32_t)ntiles;
    wa.chunk_base = (const int64_t*)rt.chunk_base[b].p;
    wa.khdr = (uint32_t*)rt.khdr.p;
    wa.kslot = (uint64_t*)rt.kslot.p;
    wa.kstride = rt.kstride;
    wa.kext = (uint64_t*)rt.kext.p;
    wa.pool_rd = (const uint64_t*)rt.pool[rt.pool_side].p;
    wa.pool_wr = (uint64_t*)rt.pool[rt.pool_side ^ 1].p;
    wa.pool_cursor = (unsigned long long*)rt.pool_cur.p;
    wa.pool_cap = (uint64_t)rt.pool_cap;
    wa.key_rev = rt.sparse ? (const uint64_t*)rt.krev.p : nullptr;
    hipMemsetAsync(rt.pool_cur.p, 0, 8, a->stream);
    wa.out = out_args(o, q);
    wa.err = pa.err;
    HotArgs ha{};
    if (hot) {
      ha.pat = pa.pat;   // (tolerant flag included)
      ha.cf = cf;
      ha.recs = pa.recs;
      ha.tile_off = pa.tile_off;
      ha.ntiles = (int32_t)ntiles;
      ha.chunk_base = (const int64_t*)rt.chunk_base[b].p;
      ha.hot_id = (uint16_t*)rt.hot_id.p;
      ha.hot_key = (int32_t*)rt.hot_key.p;
      ha.hot_m = (uint32_t*)rt.hot_m.p;
      ha.hot_gbase = (uint32_t*)rt.hot_gbase.p;
      ha.hoff = (uint32_t*)rt.hoff.p;
      ha.cand = (uint64_t*)rt.cand.p;
      ha.ncand = (uint32_t*)rt.ncand.p;
      ha.cand_cap = kCfHotMax * 4;
      ha.thresh = rt.hot_thresh;
      ha.harr = (uint64_t*)rt.harr.p;
      ha.hrow = (uint32_t*)rt.hrow.p;
      ha.hnb = (uint32_t*)rt.hnb.p;
      ha.bsum = (uint32_t*)rt.bsum.p;
      ha.bcnt = (uint32_t*)rt.bcnt.p;
      ha.boff = (uint32_t*)rt.boff.p;
      ha.hcm = (uint32_t*)rt.hcm.p;
      ha.obase = (unsigned long long*)rt.hobase.p;
      ha.htmn = (uint32_t*)rt.htmn.p;
      ha.htmx = (uint32_t*)rt.htmx.p;
      ha.hflag = (uint8_t*)rt.hflag.p;
      ha.btol = (uint32_t*)rt.btol.p;
      ha.max_blocks = rt.hot_blocks;
      ha.khdr = wa.khdr;
      ha.kslot = wa.kslot;
      ha.kstride = wa.kstride;
      ha.kext = wa.kext;
      ha.pool_rd = wa.pool_rd;
      ha.pool_wr = wa.pool_wr;
      ha.pool_cursor = wa.pool_cursor;
      ha.pool_cap = wa.pool_cap;
      ha.key_rev = wa.key_rev;
      ha.out = wa.out;
      ha.active = (uint32_t*)rt.hot_active.p;
      ha.in_seq = in_recs ? in_recs + rows.row0 * in_rec_words + 1 : nullptr;
      ha.in_rec_words = in_rec_words;
      static const int hot_ablate = std::getenv("CEP_HOT_ABLATE") ? std::atoi(std::getenv("CEP_HOT_ABLATE")) : 0;
      ha.ablate = hot_ablate;
      ha.err = pa.err;
      wa.hot_cand = ha.cand;
      wa.hot_ncand = ha.ncand;
      wa.hot_thresh = rt.hot_thresh;
      wa.hot_id = divert ? ha.hot_id : nullptr;
    }
    // the hot kernels run on the side stream beside the walk: disjoint keys,
    // shared output / pool cursors are atomics (CEP_HOT_SERIAL=1: main stream)
    static const bool hot_serial = std::getenv("CEP_HOT_SERIAL") != nullptr;
    hipStream_t hs = hot_serial ? a->stream : a->side;
    if (divert) {
      if (!hot_serial) {
        hipEventRecord(rt.hot_fork, a->stream);
        hipStreamWaitEvent(hs, rt.hot_fork, 0);
      }
      {
        LaunchTimer t(a, CEP_K_HOT, hs);
        launch_hot_match(ha, hs);
      }
      if (!hot_serial) hipEventRecord(rt.hot_join, hs);
    }
    wa.in_seq = in_recs ? in_recs + rows.row0 * in_rec_words + 1 : nullptr;
    wa.in_rec_words = in_rec_words;
    static const int ablate = std::getenv("CEP_ABLATE") ? std::atoi(std::getenv("CEP_ABLATE")) : 0;
    wa.ablate = ablate;
    if (a->stamps.p) {
      wa.stamps = (uint64_t*)a->stamps.p;
      hipMemsetAsync(wa.stamps, 0, (size_t)4096 * 16 * 8, a->stream);
    }
    {
      LaunchTimer t(a, CEP_K_CF_WALK);
      launch_cf_walk(wa, P, a->stream);
    }
    if (hot) {
      if (divert && !hot_serial) hipStreamWaitEvent(a->stream, rt.hot_join, 0);
      launch_hot_update(ha, divert ? 1 : 0, a->stream);
      // slots in use, for the next batch's diversion check and cep_stats:
      // once per batch (and after the probe), not per chunk — each copy is
      // a blit on the engine stream between two walks
      if (probe || r0 + step >= rows_all.n)
        hipMemcpyAsync(rt.hot_active_host.p, rt.hot_active.p, 4, hipMemcpyDeviceToHost, a->stream);
      if (probe) {   // the probe's verdict decides the next chunk's diversion
        hipStreamSynchronize(a->stream);
        rt.hot_probed = true;
      }
    }
    rt.pool_side ^= 1;   // this launch's write pool holds every run now
    if (overlap) hipEventRecord(rt.walk_done[b], a->stream);
    rt.used[b] = true;
  }
  return CEP_OK;
}

// The order-tolerant form of a pattern (rows whose ts may go backwards).
// Every row of the waiting state's stream may expire partials, so the
// partition keeps them all; the walk's closed form (event-time order, only
// g-passing B's) is off.  A 2-state pattern is walked by the N-state walk on
// its own record roles and state layout (nfa_pair): that walk keeps lists
// longer than pending_slots in the pending pool, as the closed-form path does.
PatternArgs tolerant_args(const PatternRT& rt, const Query& q) {
  PatternArgs p = rt.pa;
  p.tolerant = 1;
  p.closed_form = 0;
  if (!p.nfa_mode && !p.agg_mode) {
    p.nfa_mode = 1;
    p.nfa_pair = 1;
    p.nfa_seq = 0;
    p.nstates = 2;
    p.st_stream[0] = q.a_stream;
    p.st_stream[1] = q.b_stream;
    for (int j = 0; j < 2; ++j) {
      p.st_min[j] = p.st_max[j] = 1;
      p.st_raw[j] = -1;
      p.st_walk[j] = -1;
    }
    p.st_tail_opt[0] = 0;
    p.st_tail_opt[1] = 1;
    p.stream_mask = (1 << q.a_stream) | (1 << q.b_stream);
    for (int i = 0; i < 8; ++i) p.key_col_s[i] = -1;
    p.key_col_s[q.a_stream] = q.key_col_a;
    p.key_col_s[q.b_stream] = q.key_col_b;
    for (int i = 0; i < p.ncap; ++i) {   // s1's captures, from the A record
      p.cap_state[i] = 0;
      p.cap_index[i] = -1;
      p.cap_word[i] = p.cap_from_rec[i];
      p.cap_null[i] = 0;
    }
  }
  return p;
}

// tolerant: run on the order-tolerant path (rows whose ts may go backwards:
// a watermark release holding late rows, or the re-run after a descent).
int run_pattern(cep_app* a, PatternRT& rt, const RowsArgs& rows_in,
                const uint64_t* in_recs = nullptr, int in_rec_words = 0, bool tolerant = false) {
  const Query& q = a->app.queries[rt.q];
  OutStream& o = a->outs[a->app.output_index(q.out_stream)];
  if (o.bound == 0) o.bound = rt.extra_bound;
  o.bound += rows_in.n;
  int rc = ensure_out_cap(a, o, o.bound);
  if (rc) return rc;
  // Timestamps in any order (cep_options.ts_order = 0): a pattern with
  // `within` runs the order-tolerant path, whose state is exactly the
  // oracle's (App. A.3: partials pruned only by |ts - ts(s1)| > W on events
  // of the stream they wait on); the event-time fast paths (closed form,
  // push-down of g-failing B's, pruning at A arrivals) need ts_order = 1.
  // A sequence prunes by |ts - ts(s1)| on every row of its streams in any
  // order: tolerant only drops its order check.  The multi-GPU record / row
  // shuffles always take the event-time paths.
  if (!tolerant && a->opt.ts_order == 0 && rt.pa.within >= 0 && (rt.order_sensitive || rt.pa.nfa_seq) &&
      !in_recs && !rows_in.seq)
    tolerant = true;
  const RowsArgs& rows_all = rows_in;
  if (rt.sparse && tolerant)
    return fail(a, CEP_E_UNSUPPORTED, "sparse_keys with out-of-order timestamps under `within`");
  if (rt.sparse) {
    // partition values -> dense slots (keymap.hip); the pattern then reads
    // the dense column in place of the key column
    if (in_recs || rows_all.seq) return fail(a, CEP_E_UNSUPPORTED, "sparse_keys with the multi-GPU key shuffle");
    const int kcol = rows_all.input == q.b_stream ? q.key_col_b : q.key_col_a;
    if (!dev_ensure(&rt.dense, (size_t)std::max<int64_t>(rows_all.n, 1) * 4 + 16, a->stream, false))
      return fail(a, CEP_E_DEVICE, "out of device memory (dense keys)");
    KeyMapArgs ka{};
    ka.key = rows_all.cols.p[kcol];
    ka.key_is_long = rows_all.cols.t[kcol] == T_LONG ? 1 : 0;
    ka.stream = rows_all.stream;
    ka.input = rows_all.input;
    ka.a_stream = q.a_stream;
    ka.b_stream = q.b_stream;
    ka.row0 = rows_all.row0;
    ka.n = rows_all.n;
    ka.tkey = (unsigned long long*)rt.tkey.p;
    ka.tval = (uint32_t*)rt.tval.p;
    ka.table_cap = rt.table_cap;
    ka.rev = (uint64_t*)rt.krev.p;
    ka.count = (unsigned int*)rt.kcount.p;
    ka.minus_one = (unsigned int*)rt.kcount.p + 1;
    ka.cap = (uint32_t)rt.pa.key_capacity;
    ka.out = (int32_t*)rt.dense.p;
    ka.err = (unsigned int*)a->err.p;
    {
      LaunchTimer t(a, CEP_K_OTHER);
      launch_keymap(ka, a->stream);
    }
    RowsArgs rows = rows_all;
    // the dense column is indexed from the slice's first row
    rows.cols.p[kcol] = (const int32_t*)rt.dense.p - rows_all.row0;
    rows.cols.t[kcol] = T_INT;
    CfPlan cf;
    if (!pref_aligned(rt.pref, rows) || !cf_plan(rt, rows, &cf, false))
      return fail(a, CEP_E_ARG, "sparse_keys needs 16-byte aligned columns");
    return run_pattern_cf(a, rt, q, o, rows, cf);
  }
  if (rt.cf && !tolerant && !rows_all.seq && (in_recs || pref_aligned(rt.pref, rows_all))) {
    CfPlan cf;
    if (cf_plan(rt, rows_all, &cf, in_recs != nullptr))
      return run_pattern_cf(a, rt, q, o, rows_all, cf, in_recs, in_rec_words);
  }
  // ts in any order on the closed form (k_cfpart / k_cfwalk TOL builds);
  // CEP_TOL_GENERAL=1 keeps the N-state walk (nfa_pair) for these runs
  static const bool tol_general = std::getenv("CEP_TOL_GENERAL") != nullptr;
  if (rt.cf && tolerant && !tol_general && !in_recs && !rows_all.seq && pref_aligned(rt.pref, rows_all)) {
    CfPlan cf;
    if (cf_plan(rt, rows_all, &cf, false))
      return run_pattern_cf(a, rt, q, o, rows_all, cf, nullptr, 0, true);
  }
  const int P = 1 << rt.pa.buckets_log2;
  // the side stream starts after everything already queued on the main stream
  // (host-batch staging copies, earlier queries)
  hipEventRecord(a->in_ready, a->stream);
  hipStreamWaitEvent(a->side, a->in_ready, 0);
  // CEP_NO_OVERLAP=1 (diagnostics): both passes on the main stream
  static const bool no_overlap = std::getenv("CEP_NO_OVERLAP") != nullptr;
  hipStream_t side = no_overlap ? a->stream : a->side;
  const int64_t cstep = tolerant ? rt.chunk_tol : rt.chunk;
  for (int64_t r0 = 0; r0 < rows_all.n; r0 += cstep) {
    const int b = rt.cur;
    rt.cur ^= 1;
    RowsArgs rows = rows_all;
    rows.row0 = rows_all.row0 + r0;
    rows.n = std::min<int64_t>(cstep, rows_all.n - r0);
    if (r0 > 0) rows.prev_ts = INT64_MIN;   // checked inside the kernel via ts[row-1]
    const int64_t ntiles = (rows.n + kPartThreads * kPartItems - 1) / (kPartThreads * kPartItems);
    PartArgs pa{};
    pa.rows = rows;
    pa.pref = rt.pref;
    if (in_recs) {   // received shuffle records (cep_send_records)
      pa.from_records = 1;
      pa.in_recs = in_recs;
      pa.in_rec_words = in_rec_words;
      pa.pref.n = -1;
    }
    if (pa.pref.n >= 0 && !pref_aligned(pa.pref, rows)) pa.pref.n = -1;
    if (r0 > 0) pa.rows.prev_ts = INT64_MIN;
    pa.vm = {(const Ins*)a->code.p, (const uint64_t*)a->konst.p};
    pa.pat = tolerant ? tolerant_args(rt, q) : rt.pa;
    pa.tile_rows = kPartThreads * kPartItems;
    pa.recs = (uint64_t*)rt.recs[b].p;
    pa.tile_off = (uint16_t*)rt.tile_off[b].p;
    pa.chunk_base = (int64_t*)rt.chunk_base[b].p;
    pa.err = (unsigned int*)a->err.p;
    if (a->stamps.p) pa.stamps = (uint64_t*)a->stamps.p + 4096 * 16;
    if (rt.used[b]) hipStreamWaitEvent(side, rt.walk_done[b], 0);   // arena b is free
    {
      LaunchTimer t(a, CEP_K_PARTITION, side);
      launch_partition(pa, ntiles, rt.part_vm, side);
    }
    hipEventRecord(rt.part_done[b], side);
    hipStreamWaitEvent(a->stream, rt.part_done[b], 0);
    WalkArgs wa{};
    wa.vm = pa.vm;
    wa.pat = pa.pat;
    wa.recs = pa.recs;
    wa.tile_off = pa.tile_off;
    wa.ntiles = (int)ntiles;
    wa.tile_rows = pa.tile_rows;
    wa.chunk_base = (const int64_t*)rt.chunk_base[b].p;
    if (a->stamps.p) {
      // keep the last chunk's stamps (diagnostics only)
      wa.stamps = (uint64_t*)a->stamps.p;
    }
    wa.khdr = (uint32_t*)rt.khdr.p;
    wa.kslot = (uint64_t*)rt.kslot.p;
    wa.kstride = rt.kstride;
    wa.out = out_args(o, q);
    wa.err = pa.err;
    const bool pool = (q.nfa || pa.pat.nfa_pair) && rt.kext.p;
    if (pool) {
      wa.kext = (uint64_t*)rt.kext.p;
      wa.pool_rd = (const uint64_t*)rt.pool[rt.pool_side].p;
      wa.pool_wr = (uint64_t*)rt.pool[rt.pool_side ^ 1].p;
      wa.pool_cursor = (unsigned long long*)rt.pool_cur.p;
      wa.pool_cap = (uint64_t)rt.pool_cap;
      hipMemsetAsync(rt.pool_cur.p, 0, 8, a->stream);
    }
    {
      LaunchTimer t(a, CEP_K_WALK);
      launch_walk(wa, P, rt.walk_vm || pa.pat.nfa_pair, a->stream);
    }
    if (pool) rt.pool_side ^= 1;   // this launch's write pool holds every run now
    hipEventRecord(rt.walk_done[b], a->stream);
    rt.used[b] = true;
  }
  return CEP_OK;
}

// One batch through a multi-query group: per chunk, k_mqpart on the side
// stream (double-buffered arenas: the partition of chunk c+1 overlaps the
// walk of chunk c) and k_mqwalk on the main stream.
int run_mq(cep_app* a, MqRT& g, const RowsArgs& rows_all) {
  const CompiledApp& app = a->app;
  // output capacity: at most one row per query per input row
  for (size_t i = 0; i < g.qs.size(); ++i) {
    const Query& q = app.queries[g.qs[i]];
    OutStream& o = a->outs[app.output_index(q.out_stream)];
    o.bound += rows_all.n;
    const int rc = ensure_out_cap(a, o, o.bound);
    if (rc) return rc;
    MqQuery& d = g.hq[i];
    int64_t* oseq = o.write_seq ? (int64_t*)o.seq.p : nullptr;   // not read: not stored
    bool same = d.out_ts == (int64_t*)o.ts.p && d.out_seq == oseq && d.out_count == o.count &&
                d.out_cap == o.cap;
    for (int c = 0; c < d.nsel; ++c) same = same && d.out_col[c] == o.cols[c].p;
    if (!same) {
      for (int c = 0; c < d.nsel; ++c) d.out_col[c] = o.cols[c].p;
      d.out_ts = (int64_t*)o.ts.p;
      d.out_seq = oseq;
      d.out_count = o.count;
      d.out_cap = o.cap;
      g.dq_dirty = true;
    }
  }
  if (g.dq_dirty) {   // rare (output growth): the walks in flight read the old table
    hipStreamSynchronize(a->stream);
    hipMemcpy(g.dq.p, g.hq.data(), g.hq.size() * sizeof(MqQuery), hipMemcpyHostToDevice);
    g.dq_dirty = false;
  }
  // this batch's column layout: a carried column whose buffer IS the event-ts
  // buffer is not carried (its value is the record's ts)
  const std::vector<int> pc = mq_pref_cols(g);
  MqPartArgs pa{};
  pa.pref.n = (int)pc.size();
  for (int i = 0; i < kPref; ++i) pa.pref.col[i] = i < pa.pref.n ? pc[i] : pc[0];
  pa.ts_slot = -1;
  for (int i = 0; i < pa.pref.n; ++i)
    if (rows_all.cols.p[pc[i]] == (const void*)rows_all.ts && rows_all.cols.t[pc[i]] == T_LONG) pa.ts_slot = i;
  MqWalkArgs wa{};
  int nphys = 0;
  for (size_t w = 0; w < g.carry.size(); ++w) {
    const int col = g.carry[w];
    if (rows_all.cols.p[col] == (const void*)rows_all.ts && rows_all.cols.t[col] == T_LONG) {
      wa.lmap[w] = -1;
      continue;
    }
    if (nphys >= kMqMaxPhys)
      return fail(a, CEP_E_UNSUPPORTED, "multi-query group carries more than " + std::to_string(kMqMaxPhys) + " columns");
    wa.lmap[w] = nphys;
    for (int i = 0; i < pa.pref.n; ++i)
      if (pc[i] == col) pa.phys_slot[nphys] = i;
    ++nphys;
  }
  if (nphys > std::min<int>((int)g.carry.size(), kMqMaxPhys)) return fail(a, CEP_E_DEVICE, "record arena too small");
  pa.stream_mask = g.stream_mask;
  pa.key_slot = 0;
  for (int s = 0; s < 8; ++s) pa.ncond[s] = g.ncond[s];
  pa.conds = (const MqCond*)g.dconds.p;
  pa.nphys = nphys;
  // the group's sequences prune by |ts - ts(s1)| on every row of their
  // streams (any order); the check stays for callers that asked for it
  pa.check_order = (g.check_order && a->opt.ts_order == 1 && !a->force_tolerant) ? 1 : 0;
  pa.key_capacity = g.key_capacity;
  pa.key_stride = g.key_stride;
  pa.key_offset = g.key_offset;
  pa.buckets_log2 = g.lg;
  pa.err = (unsigned int*)a->err.p;
  wa.q = (const MqQuery*)g.dq.p;
  wa.nq = (int)g.qs.size();
  wa.units = (const MqUnit*)g.du.p;
  wa.nunits = (int)g.units.size();
  wa.nphys = nphys;
  wa.buckets_log2 = g.lg;
  wa.kpb = g.kpb;
  wa.key_stride = g.key_stride;
  wa.key_offset = g.key_offset;
  wa.state = (uint64_t*)g.state.p;
  wa.kstride = g.kstride;
  wa.words = g.words;
  static const int mq_ablate = std::getenv("CEP_MQ_ABLATE") ? std::atoi(std::getenv("CEP_MQ_ABLATE")) : 0;
  wa.ablate = mq_ablate;
  wa.err = pa.err;
  if (a->stamps.p && (1 << g.lg) * 16 <= 2 * 4096 * 16) {
    wa.stamps = (uint64_t*)a->stamps.p;
    hipMemsetAsync(wa.stamps, 0, (size_t)(1 << g.lg) * 16 * 8, a->stream);
  }
  // the side stream starts after everything already queued on the main one
  hipEventRecord(a->in_ready, a->stream);
  hipStreamWaitEvent(a->side, a->in_ready, 0);
  static const bool no_overlap = std::getenv("CEP_NO_OVERLAP") != nullptr;
  hipStream_t side = no_overlap ? a->stream : a->side;
  for (int64_t r0 = 0; r0 < rows_all.n; r0 += g.chunk) {
    const int b = g.cur;
    g.cur ^= 1;
    RowsArgs rows = rows_all;
    rows.row0 = rows_all.row0 + r0;
    rows.n = std::min<int64_t>(g.chunk, rows_all.n - r0);
    const int ntiles = (int)((rows.n + kMqTile - 1) / kMqTile);
    pa.rows = rows;
    pa.ntiles = ntiles;
    pa.chunk_base = (int64_t*)g.chunk_base[b].p;
    pa.recs = (uint64_t*)g.recs[b].p;
    pa.tile_off = (uint16_t*)g.toff[b].p;
    if (g.used[b]) hipStreamWaitEvent(side, g.walk_done[b], 0);   // arena b is free
    {
      LaunchTimer t(a, CEP_K_MQ_PARTITION, side);
      launch_mq_partition(pa, side);
    }
    hipEventRecord(g.part_done[b], side);
    hipStreamWaitEvent(a->stream, g.part_done[b], 0);
    wa.recs = pa.recs;
    wa.tile_off = pa.tile_off;
    wa.ntiles = ntiles;
    wa.chunk_base = pa.chunk_base;
    wa.in_seq = rows.seq ? rows.seq + rows.row0 : nullptr;
    {
      LaunchTimer t(a, CEP_K_MQ_WALK);
      launch_mq_walk(wa, 1 << g.lg, a->stream);
    }
    hipEventRecord(g.walk_done[b], a->stream);
    g.used[b] = true;
  }
  return CEP_OK;
}

int send_device_rows(cep_app* a, const RowsArgs& rows) {
  for (auto& g : a->mqs) {
    const int rc = run_mq(a, g, rows);
    if (rc) return rc;
  }
  for (size_t qi = 0; qi < a->app.queries.size(); ++qi) {
    const Query& q = a->app.queries[qi];
    if (a->in_mq[qi]) continue;
    int rc = CEP_OK;
    if (q.kind == Q_FILTER) {
      rc = run_filter(a, q, rows);
    } else if (q.kind == Q_PATTERN || q.kind == Q_AGG) {
      for (auto& rt : a->pats)
        if (rt.q == (int)qi) rc = run_pattern(a, rt, rows, nullptr, 0, a->force_tolerant);
    }
    if (rc) return rc;
  }
  // the batch's last ts: the next batch's first-row order check (device
  // batches; the host does not see their ts)
  if (rows.n > 0 && rows.prev_ts_dev)
    hipMemcpyAsync(a->last_ts_dev.p, rows.ts + rows.row0 + rows.n - 1, 8, hipMemcpyDeviceToDevice, a->stream);
  return CEP_OK;
}


int device_error(cep_app* a, unsigned int e);

int check_device_error(cep_app* a) {
  unsigned int e = 0;
  hipMemcpy(&e, a->err.p, sizeof(e), hipMemcpyDeviceToHost);
  return device_error(a, e);
}

int error_status(cep_app* a, unsigned int e);

// Error flags read back -> status (the flags are cleared).
int device_error(cep_app* a, unsigned int e) {
  if (!e) return CEP_OK;
  hipMemset(a->err.p, 0, 64);
  return error_status(a, e);
}

// Status of device error flags (the flags are not touched).
int error_status(cep_app* a, unsigned int e) {
  if (!e) return CEP_OK;
  if (e & ERR_ORDER)   // root cause first: out-of-order input also defeats `within` pruning
    return fail(a, CEP_E_ARG, "events not in event-time order: `within` requires non-decreasing timestamps");
  if (e & ERR_PENDING)
    return fail(a, CEP_E_CAPACITY, "per-key pending partial capacity exceeded (raise pending_slots)");
  if (e & ERR_POOL)
    return fail(a, CEP_E_CAPACITY, "pending overflow pool exhausted (raise pending_pool_log2)");
  if (e & ERR_KEYMAP)
    return fail(a, CEP_E_CAPACITY, "more distinct partition values than key_capacity (sparse_keys)");
  if (e & ERR_KEY_RANGE)
    return fail(a, CEP_E_CAPACITY, "partition key outside [0, key_capacity) or not owned by this shard");
  if (e & ERR_SHUFFLE_CAP)
    return fail(a, CEP_E_CAPACITY,
                "padded key shuffle: an owner segment overflowed seg_cap (its excess records were dropped; "
                "raise seg_cap or use the two-phase exchange)");
  if (e & ERR_TS_SPAN)
    return fail(a, CEP_E_ARG, "timestamps of one chunk lie more than 2^31 ms apart (lower chunk_events)");
  if (e & ERR_OUT_CAP) return fail(a, CEP_E_DEVICE, "output capacity exceeded");
  return fail(a, CEP_E_DEVICE, "device error flags " + std::to_string(e));
}

}  // namespace

// ======================================================================= C ABI
extern "C" {

void cep_default_options(cep_options* o) {
  std::memset(o, 0, sizeof(*o));
  o->device = 0;
  o->pending_slots = 16;
  o->key_capacity = 1 << 20;
  o->chunk_events = 1 << 22;
  o->buckets_log2 = 10;
  o->profile = 0;
  o->ordered_output = 1;
  o->key_stride = 1;
  o->key_offset = 0;
  o->pending_pool_log2 = 20;
  o->late_policy = 2;
  o->ts_order = 0;
}

int cep_validate(const char* plan, char* err, size_t errlen) {
  if (!plan) {
    set_err(err, errlen, "plan is null");
    return CEP_E_ARG;
  }
  CompiledApp app;
  std::string m;
  int rc = compile_app(plan, &app, &m);
  if (rc) set_err(err, errlen, m);
  else set_err(err, errlen, "");
  return rc;
}

int cep_plan_schema(const char* plan, const char* stream_id, cep_attr* out, int cap, int* n,
                    char* err, size_t errlen) {
  if (!plan || !stream_id) {
    set_err(err, errlen, "null argument");
    return CEP_E_ARG;
  }
  CompiledApp app;
  std::string m;
  int rc = compile_app(plan, &app, &m);
  if (rc) {
    set_err(err, errlen, m);
    return rc;
  }
  const StreamSchema* s = nullptr;
  int i = app.input_index(stream_id);
  if (i >= 0) s = &app.inputs[i];
  i = app.output_index(stream_id);
  if (!s && i >= 0) s = &app.outputs[i];
  if (!s) {
    set_err(err, errlen, std::string("Unknown stream id ") + stream_id);
    return CEP_E_UNDEFINED_STREAM;
  }
  return fill_attrs(s, out, cap, n);
}

cep_app* cep_create(const char* plan, const cep_options* opt, char* err, size_t errlen) {
  return cep::create_app(plan, opt, nullptr, err, errlen);
}

}  // extern "C"

cep_app* cep::create_app(const char* plan, const cep_options* opt, const std::vector<std::string>* dict_seed,
                         char* err, size_t errlen) {
  if (!plan) {
    set_err(err, errlen, "plan is null");
    return nullptr;
  }
  auto* a = new cep_app();
  if (opt) a->opt = *opt;
  else cep_default_options(&a->opt);
  if (a->opt.pending_slots <= 0 || a->opt.pending_slots > kMaxPending) {
    set_err(err, errlen, "pending_slots must be in [1, " + std::to_string(kMaxPending) + "]");
    delete a;
    return nullptr;
  }
  if (a->opt.key_stride <= 0) a->opt.key_stride = 1;
  std::string m;
  int rc = compile_app(plan, &a->app, &m, dict_seed);
  if (rc) {
    set_err(err, errlen, m);
    delete a;
    return nullptr;
  }
  for (auto& s : a->app.strings) cep_dict_intern(a, s.c_str());
  rc = create_runtime(a);
  if (rc) {
    set_err(err, errlen, a->last_error);
    cep_destroy(a);
    return nullptr;
  }
  set_err(err, errlen, "");
  return a;
}

extern "C" {

void cep_destroy(cep_app* a) {
  if (!a) return;
  if (a->stream) hipStreamSynchronize(a->stream);
  if (a->stamps.p && !a->pats.empty()) {
    // diagnostics: mean duration of each k_walk phase over the last launch's blocks
    const int nb = 1 << a->pats[0].pa.buckets_log2;
    std::vector<uint64_t> st((size_t)4096 * 16);
    hipMemcpy(st.data(), a->stamps.p, st.size() * 8, hipMemcpyDeviceToHost);
    // phases 1..7 of window 0, then phases 2..7 of window 1 (stamps 10..15,
    // relative to window 0's last stamp); blocks with one window have zeros
    double sum[16] = {0};
    int n1 = 0;
    for (int b = 0; b < nb; ++b) {
      const uint64_t* t = &st[(size_t)b * 16];
      for (int i = 1; i < 8; ++i)
        if (t[i] && t[i - 1]) sum[i] += (double)(t[i] - t[i - 1]);
      if (t[10] && t[7]) {
        ++n1;
        sum[10] += (double)(t[10] - t[7]);
        for (int i = 11; i < 16; ++i)
          if (t[i] && t[i - 1]) sum[i] += (double)(t[i] - t[i - 1]);
      }
    }
    {   // slowest blocks (stragglers): first stamp to the last one written
      std::vector<std::pair<uint64_t, int>> dur;
      for (int b = 0; b < nb; ++b) {
        const uint64_t* t = &st[(size_t)b * 16];
        uint64_t hi = 0;
        for (int i = 0; i < 16; ++i) hi = std::max(hi, t[i]);
        if (t[0] && hi > t[0]) dur.push_back({hi - t[0], b});
      }
      std::sort(dur.rbegin(), dur.rend());
      std::fprintf(stderr, "[cep stamps] slowest walk blocks (ticks):");
      for (size_t i = 0; i < dur.size() && i < 6; ++i) std::fprintf(stderr, " b%d=%llu", dur[i].second,
                                                                   (unsigned long long)dur[i].first);
      if (!dur.empty()) std::fprintf(stderr, " median=%llu", (unsigned long long)dur[dur.size() / 2].first);
      std::fprintf(stderr, "\n");
    }
    {   // every stamp against the previous one (both kernels' layouts)
      double dsum[16] = {0};
      int dn[16] = {0};
      for (int b = 0; b < nb; ++b) {
        const uint64_t* t = &st[(size_t)b * 16];
        for (int i = 1; i < 16; ++i)
          if (t[i] && t[i - 1]) {
            dsum[i] += (double)(t[i] - t[i - 1]);
            ++dn[i];
          }
      }
      std::fprintf(stderr, "[cep stamps] walk deltas ticks/block:");
      for (int i = 1; i < 16; ++i) std::fprintf(stderr, " d%d=%.0f(%d)", i, dn[i] ? dsum[i] / dn[i] : 0.0, dn[i]);
      std::fprintf(stderr, "\n");
    }
    if (std::getenv("CEP_WAVESTAMP")) {   // -DCF_WAVESTAMP build: per-wave ends vs slot 0
      double m[16] = {0};
      int c[16] = {0};
      for (int b = 0; b < nb; ++b) {
        const uint64_t* t = &st[(size_t)b * 16];
        if (!t[0]) continue;
        for (int i = 1; i < 16; ++i)
          if (t[i]) {
            m[i] += (double)(int64_t)(t[i] - t[0]);
            ++c[i];
          }
      }
      std::fprintf(stderr, "[cep wavestamps] commit end per wave:");
      for (int i = 1; i <= 8; ++i) std::fprintf(stderr, " w%d=%.0f", i - 1, c[i] ? m[i] / c[i] : 0.0);
      std::fprintf(stderr, "\n[cep wavestamps] emission end per wave:");
      for (int i = 9; i < 16; ++i) std::fprintf(stderr, " w%d=%.0f", i - 9, c[i] ? m[i] / c[i] : 0.0);
      std::fprintf(stderr, "\n");
    }
    std::fprintf(stderr, "[cep stamps] walk window0 ticks/block:");
    for (int i = 1; i < 8; ++i) std::fprintf(stderr, " p%d=%.0f", i, sum[i] / nb);
    std::fprintf(stderr, "\n[cep stamps] walk window1 (%d blocks):", n1);
    for (int i = 10; i < 16; ++i) std::fprintf(stderr, " p%d=%.0f", i - 8, n1 ? sum[i] / n1 : 0.0);
    std::fprintf(stderr, "\n");
    const uint64_t* c = &st[(size_t)4095 * 16];
    if (nb <= 4095 && c[0] && !c[5 + 8])
      std::fprintf(stderr, "[cep counters] walk2 active keys=%llu n>2=%llu n>4=%llu n>6=%llu n>8=%llu | waves: n>2=%llu n>4=%llu of %llu\n",
                   (unsigned long long)c[0], (unsigned long long)c[1], (unsigned long long)c[2],
                   (unsigned long long)c[3], (unsigned long long)c[4], (unsigned long long)c[5],
                   (unsigned long long)c[6], (unsigned long long)c[7]);
    if (nb <= 4095 && (c[5] || c[7]))
      std::fprintf(stderr, "[cep counters] walk: carried=%llu all=%llu keylanes_n>2=%llu drop_n>2=%llu "
                   "slot_st>=2=%llu windows=%llu keylanes=%llu\n",
                   (unsigned long long)c[0], (unsigned long long)c[1], (unsigned long long)c[2],
                   (unsigned long long)c[3], (unsigned long long)c[4], (unsigned long long)c[5],
                   (unsigned long long)c[7]);
    const bool cf = a->pats[0].cf;
    const int nt = (int)std::min<int64_t>(4096, cf ? a->pats[0].cf_chunk / kCfTile
                                                   : a->pats[0].chunk / (kPartThreads * kPartItems));
    std::vector<uint64_t> pt((size_t)nt * 16);
    hipMemcpy(pt.data(), (uint64_t*)a->stamps.p + 4096 * 16, pt.size() * 8, hipMemcpyDeviceToHost);
    double ps[16] = {0};
    uint64_t plo = UINT64_MAX, phi = 0;
    for (int b = 0; b < nt; ++b) {
      for (int i = 1; i < 8; ++i)
        if (pt[b * 16 + i] && pt[b * 16 + i - 1]) ps[i] += (double)(pt[b * 16 + i] - pt[b * 16 + i - 1]);
      if (pt[b * 16]) plo = std::min(plo, pt[b * 16]);
      for (int i = 0; i < 8; ++i) phi = std::max(phi, pt[b * 16 + i]);
    }
    std::fprintf(stderr, "[cep stamps] partition phase ticks/block:");
    for (int i = 1; i < 8; ++i) std::fprintf(stderr, " p%d=%.0f", i, ps[i] / nt);
    std::fprintf(stderr, " span=%.0f\n", (double)(phi - plo));
  }
  if (a->stamps.p && !a->mqs.empty()) {
    // diagnostics: mean ticks per multi-query walk phase over the last launch's buckets
    const int nb = 1 << a->mqs[0].lg;
    std::vector<uint64_t> st((size_t)nb * 16);
    hipMemcpy(st.data(), a->stamps.p, st.size() * 8, hipMemcpyDeviceToHost);
    double sum[8] = {0}, ut[8] = {0}, p1 = 0, rs = 0;
    for (int b = 0; b < nb; ++b) {
      const uint64_t* x = &st[(size_t)b * 16];
      for (int i = 1; i < 5; ++i)
        if (x[i] && x[i - 1]) sum[i] += (double)(x[i] - x[i - 1]);
      if (x[5] && x[2]) p1 += (double)(x[5] - x[2]);
      if (x[3] && x[5]) rs += (double)(x[3] - x[5]);
      for (int i = 0; i < 8; ++i) ut[i] += (double)x[8 + i];
    }
    std::fprintf(stderr, "[cep stamps] mq walk ticks/bucket: gather=%.0f sort=%.0f count=%.0f (pass1 %.0f, "
                 "reserve %.0f) emit=%.0f\n", sum[1] / nb, sum[2] / nb, sum[3] / nb, p1 / nb, rs / nb, sum[4] / nb);
    std::fprintf(stderr, "[cep stamps] mq unit ticks/bucket (units 0-3) pass1: %.0f %.0f %.0f %.0f pass2: %.0f %.0f "
                 "%.0f %.0f\n", ut[0] / nb, ut[1] / nb, ut[2] / nb, ut[3] / nb, ut[4] / nb, ut[5] / nb,
                 ut[6] / nb, ut[7] / nb);
  }
  harvest_timers(a);
  for (auto e : a->event_pool) hipEventDestroy(e);
  for (auto& o : a->outs) {
    for (auto& c : o.cols) dev_free(&c);
    dev_free(&o.ts);
    dev_free(&o.seq);
    for (auto& c : o.scols) dev_free(&c);
    dev_free(&o.sts);
    dev_free(&o.sseq);
  }
  for (DevBuf* b : {&a->ostats, &a->okeys[0], &a->okeys[1], &a->oidx[0], &a->oidx[1], &a->otemp, &a->out_counts})
    dev_free(b);
  for (auto& p : a->pats) {
    dev_free(&p.khdr);
    dev_free(&p.kslot);
    dev_free(&p.kext);
    dev_free(&p.pool[0]);
    dev_free(&p.pool[1]);
    dev_free(&p.pool_cur);
    for (DevBuf* b : {&p.tkey, &p.tval, &p.krev, &p.kcount, &p.dense}) dev_free(b);
    for (DevBuf* b : {&p.hot_id, &p.hot_key, &p.hot_m, &p.hot_gbase, &p.hoff, &p.cand, &p.ncand, &p.harr, &p.hrow,
                      &p.hnb, &p.bsum, &p.bcnt, &p.boff, &p.hcm, &p.hobase, &p.hot_active, &p.htmn,
                      &p.htmx, &p.hflag, &p.btol})
      dev_free(b);
    host_free(&p.hot_active_host);
    if (p.hot_fork) hipEventDestroy(p.hot_fork);
    if (p.hot_join) hipEventDestroy(p.hot_join);
    for (int b = 0; b < 2; ++b) {
      dev_free(&p.recs[b]);
      dev_free(&p.tile_off[b]);
      dev_free(&p.cf_recs[b]);
      dev_free(&p.cf_toff[b]);
      dev_free(&p.chunk_base[b]);
    }
  }
  for (auto& g : a->mqs) {
    for (DevBuf* b : {&g.dq, &g.du, &g.dconds, &g.state}) dev_free(b);
    for (int b = 0; b < 2; ++b) {
      dev_free(&g.recs[b]);
      dev_free(&g.toff[b]);
      dev_free(&g.chunk_base[b]);
    }
  }
  if (a->copy) hipStreamSynchronize(a->copy);
  for (auto& h : a->hs) {
    host_free(&h.pinned);
    dev_free(&h.dev);
    if (h.dma_done) hipEventDestroy(h.dma_done);
    if (h.free) hipEventDestroy(h.free);
  }
  for (auto& o : a->outs) {
    for (auto& h : o.hcols) host_free(&h);
    host_free(&o.hts);
    host_free(&o.hseq);
  }
  for (int c = 0; c < kMaxCols; ++c) {
    dev_free(&a->ro.col[c]);
    dev_free(&a->ro.out[c]);
  }
  for (DevBuf* b : {&a->ro.ts, &a->ro.stream, &a->ro.ots, &a->ro.ostream, &a->ro.keys, &a->ro.idx_in,
                    &a->ro.idx_out, &a->ro.temp, &a->ro.bound})
    dev_free(b);
  dev_free(&a->code);
  dev_free(&a->konst);
  dev_free(&a->last_ts_dev);
  dev_free(&a->tile_state);
  dev_free(&a->route_arena);
  dev_free(&a->route_tcount);
  dev_free(&a->route_toffs);
  dev_free(&a->route_dcount);
  dev_free(&a->ticket);
  dev_free(&a->err);
  dev_free(&a->rerr);
  dev_free(&a->str_hash);
  host_free(&a->flush_words);
  for (auto& d : a->rr_col) dev_free(&d);
  dev_free(&a->rr_ts);
  dev_free(&a->rr_stream);
  dev_free(&a->rr_seq);
  if (a->stream) hipStreamSynchronize(a->stream);
  if (a->side) hipStreamSynchronize(a->side);
  for (auto& p : a->pats)
    for (int b = 0; b < 2; ++b) {
      if (p.part_done[b]) hipEventDestroy(p.part_done[b]);
      if (p.walk_done[b]) hipEventDestroy(p.walk_done[b]);
    }
  for (auto& g : a->mqs)
    for (int b = 0; b < 2; ++b) {
      if (g.part_done[b]) hipEventDestroy(g.part_done[b]);
      if (g.walk_done[b]) hipEventDestroy(g.walk_done[b]);
    }
  if (a->in_ready) hipEventDestroy(a->in_ready);
  if (a->ext_ready) hipEventDestroy(a->ext_ready);
  if (a->out_ready) hipEventDestroy(a->out_ready);
  if (a->r_ready) hipEventDestroy(a->r_ready);
  if (a->r_host) hipEventDestroy(a->r_host);
  if (a->rstream) {
    hipStreamSynchronize(a->rstream);
    hipStreamDestroy(a->rstream);
  }
  if (a->side) hipStreamDestroy(a->side);
  if (a->copy) hipStreamDestroy(a->copy);
  if (a->stream) hipStreamDestroy(a->stream);
  delete a;
}

int cep_stream_schema(cep_app* a, const char* stream_id, cep_attr* out, int cap, int* n) {
  if (!a) return CEP_E_ARG;
  const StreamSchema* s = find_schema(a, stream_id);
  if (!s) return fail(a, CEP_E_UNDEFINED_STREAM, std::string("Stream ") + (stream_id ? stream_id : "(null)") + " not defined");
  return fill_attrs(s, out, cap, n);
}

int cep_input(cep_app* a, const char* stream_id) {
  if (!a || !stream_id) return -CEP_E_ARG;
  int i = a->app.input_index(stream_id);
  if (i < 0) {
    fail(a, CEP_E_UNDEFINED_STREAM, std::string("Stream ") + stream_id + " not defined");
    return -CEP_E_UNDEFINED_STREAM;
  }
  return i;
}

int cep_set_callback(cep_app* a, const char* out_id, cep_emit_fn fn, void* user) {
  if (!a || !out_id) return CEP_E_ARG;
  int i = a->app.output_index(out_id);
  if (i < 0) return fail(a, CEP_E_UNDEFINED_STREAM, std::string("Stream ") + out_id + " not defined");
  a->outs[i].fn = fn;
  a->outs[i].user = user;
  return CEP_OK;
}

namespace {

// Batch -> device rows (host batches are staged into device memory: the
// PCIe-inclusive path).  Validates the handle and the column count.
// *slot: the host staging slot the batch went to (-1: device batch);
// *direct: its columns are DMA'd straight from pinned caller memory.
int batch_rows(cep_app* a, const cep_batch* b, RowsArgs* out, int* slot, bool* direct) {
  *slot = -1;
  *direct = false;
  if (b->n < 0 || (b->n > 0 && !b->ts)) return fail(a, CEP_E_ARG, "bad batch");
  if (b->input < 0 || b->input >= (int)a->app.inputs.size())
    return fail(a, CEP_E_UNDEFINED_STREAM, "undefined input handle");
  const StreamSchema& sd = a->app.inputs[b->input];
  if (b->ncols != (int)sd.attrs.size() || b->ncols > kMaxCols)
    return fail(a, CEP_E_ARG, "batch has " + std::to_string(b->ncols) + " columns, stream " +
                                  sd.id + " defines " + std::to_string(sd.attrs.size()));
  RowsArgs rows{};
  rows.cols.n = b->ncols;
  for (int c = 0; c < b->ncols; ++c) rows.cols.t[c] = sd.attrs[c].type;
  rows.input = b->input;
  rows.row0 = 0;
  rows.n = b->n;
  rows.seq0 = a->events_in;
  rows.prev_ts = a->last_ts;
  rows.prev_ts_dev = (const int64_t*)a->last_ts_dev.p;
  if (b->on_device) {
    for (int c = 0; c < b->ncols; ++c) rows.cols.p[c] = b->cols[c];
    rows.ts = b->ts;
    rows.stream = b->stream;
    // cross-batch order checks would need a sync to read the last ts; the
    // in-batch check covers the hot path
    a->last_ts = INT64_MIN;
  } else {
    // One staging slot holds the whole batch (columns, ts, stream; 256-B
    // aligned pieces).  Pinned caller buffers are DMA'd directly; pageable
    // ones are first copied by the CPU into the slot's pinned arena (that
    // copy is the batch's consumption: the call returns without waiting for
    // the device).  The DMA waits for the kernels that last read the slot.
    auto& h = a->hs[a->hs_next];
    *slot = a->hs_next;
    a->hs_next ^= 1;
    if (!h.dma_done && (hipEventCreateWithFlags(&h.dma_done, hipEventDisableTiming) != hipSuccess ||
                        hipEventCreateWithFlags(&h.free, hipEventDisableTiming) != hipSuccess))
      return fail(a, CEP_E_DEVICE, "hipEventCreate failed");
    const int nc = b->ncols;
    size_t off[kMaxCols + 2], len[kMaxCols + 2];
    const void* src[kMaxCols + 2];
    size_t total = 0;
    auto piece = [&](int i, const void* p, size_t bytes) {
      off[i] = total;
      len[i] = bytes;
      src[i] = p;
      total += (bytes + 255) & ~(size_t)255;
    };
    for (int c = 0; c < nc; ++c) piece(c, b->cols[c], (size_t)b->n * type_width(sd.attrs[c].type));
    piece(nc, b->ts, (size_t)b->n * 8);
    piece(nc + 1, b->stream, b->stream ? (size_t)b->n : 0);
    bool pinned = true;
    for (int i = 0; i < nc + 2 && pinned; ++i) pinned = !len[i] || is_pinned(src[i]);
    // the slot's previous DMA (two batches ago) must be done before its
    // pinned arena or device arena is rewritten
    if (h.used) hipEventSynchronize(h.dma_done);
    if (h.dev.bytes < total) {
      if (h.used) hipStreamSynchronize(a->stream);   // the old arena may still be read
      if (!dev_ensure(&h.dev, total, a->stream, false))
        return fail(a, CEP_E_DEVICE, "out of device memory (staging)");
    }
    if (!pinned) {
      if (!host_ensure(&h.pinned, total)) return fail(a, CEP_E_DEVICE, "out of pinned host memory");
      for (int i = 0; i < nc + 2; ++i)
        if (len[i]) std::memcpy((char*)h.pinned.p + off[i], src[i], len[i]);
    }
    if (h.used) hipStreamWaitEvent(a->copy, h.free, 0);   // kernels done with the device arena
    if (!pinned) {
      hipMemcpyAsync(h.dev.p, h.pinned.p, total, hipMemcpyHostToDevice, a->copy);
    } else {
      for (int i = 0; i < nc + 2; ++i)
        if (len[i]) hipMemcpyAsync((char*)h.dev.p + off[i], src[i], len[i], hipMemcpyHostToDevice, a->copy);
    }
    hipEventRecord(h.dma_done, a->copy);
    hipStreamWaitEvent(a->stream, h.dma_done, 0);
    h.used = true;
    *direct = pinned;
    for (int c = 0; c < nc; ++c) rows.cols.p[c] = (char*)h.dev.p + off[c];
    rows.ts = (const int64_t*)((char*)h.dev.p + off[nc]);
    rows.stream = b->stream ? (const uint8_t*)((char*)h.dev.p + off[nc + 1]) : nullptr;
    a->last_ts = b->ts[b->n - 1];
  }
  *out = rows;
  return CEP_OK;
}

}  // namespace

int cep_send_batch(cep_app* a, const cep_batch* b) {
  if (!a || !b) return CEP_E_ARG;
  if (!a->enabled) return CEP_OK;   // AbstractSiddhiOperator.java:128
  if (b->n == 0) return CEP_OK;
  RowsArgs rows{};
  int slot;
  bool direct;
  int rc = batch_rows(a, b, &rows, &slot, &direct);
  if (rc) return rc;
  a->events_in += b->n;
  a->batches++;
  rc = send_device_rows(a, rows);
  if (slot >= 0) {
    hipEventRecord(a->hs[slot].free, a->stream);
    // caller's pinned buffers: consumed once their DMA is done (the kernels
    // keep running); pageable buffers were consumed by the staging memcpy
    if (direct) hipEventSynchronize(a->hs[slot].dma_done);
  }
  return rc;
}

// ---- event-time reorder (AbstractSiddhiOperator.java:222-231 processElement
// offers to the PriorityQueue; :238-247 processWatermark drains ts <= mark)
int cep_buffer_batch(cep_app* a, const cep_batch* b) {
  if (!a || !b || b->n < 0) return CEP_E_ARG;
  if (b->n == 0) return CEP_OK;
  if (b->input < 0 || b->input >= (int)a->app.inputs.size())
    return fail(a, CEP_E_UNDEFINED_STREAM, "undefined input handle");
  const StreamSchema& sd = a->app.inputs[b->input];
  if (b->ncols != (int)sd.attrs.size() || b->ncols > kMaxCols)
    return fail(a, CEP_E_ARG, "batch has " + std::to_string(b->ncols) + " columns, stream " + sd.id +
                                  " defines " + std::to_string(sd.attrs.size()));
  auto& r = a->ro;
  if (r.n > 0 && (r.input != b->input || r.has_stream != (b->stream != nullptr)))
    return fail(a, CEP_E_ARG, "the reorder buffer holds rows of another input layout: call cep_watermark first");
  if (r.n + b->n > (int64_t)INT32_MAX) return fail(a, CEP_E_CAPACITY, "reorder buffer holds at most 2^31-1 rows");
  r.input = b->input;
  r.has_stream = b->stream != nullptr;
  const int64_t need = r.n + b->n;
  const hipMemcpyKind kind = b->on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  bool ok = true;
  for (int c = 0; c < b->ncols && ok; ++c) {
    const int w = type_width(sd.attrs[c].type);
    ok = dev_ensure(&r.col[c], (size_t)need * w, a->stream, true);
    if (ok) hipMemcpyAsync((char*)r.col[c].p + r.n * w, b->cols[c], (size_t)b->n * w, kind, a->stream);
  }
  ok = ok && dev_ensure(&r.ts, (size_t)need * 8, a->stream, true);
  if (ok) hipMemcpyAsync((char*)r.ts.p + r.n * 8, b->ts, (size_t)b->n * 8, kind, a->stream);
  if (ok && b->stream) {
    ok = dev_ensure(&r.stream, (size_t)need, a->stream, true);
    if (ok) hipMemcpyAsync((char*)r.stream.p + r.n, b->stream, (size_t)b->n, kind, a->stream);
  }
  if (!ok) return fail(a, CEP_E_DEVICE, "out of device memory (reorder buffer)");
  r.n = need;
  if (!b->on_device) hipStreamSynchronize(a->stream);   // host buffers may be reused
  return CEP_OK;
}

int64_t cep_buffered(cep_app* a) { return a ? a->ro.n : -1; }

int cep_watermark(cep_app* a, int64_t mark) {
  if (!a) return CEP_E_ARG;
  auto& r = a->ro;
  if (r.n == 0) return CEP_OK;
  const StreamSchema& sd = a->app.inputs[r.input];
  const int nc = (int)sd.attrs.size();
  const int64_t n = r.n;
  const size_t tb = reorder_temp_bytes(n);
  if (!dev_ensure(&r.keys, (size_t)n * 8, a->stream, false) ||
      !dev_ensure(&r.idx_in, (size_t)n * 4, a->stream, false) ||
      !dev_ensure(&r.idx_out, (size_t)n * 4, a->stream, false) || !dev_ensure(&r.temp, tb + 16, a->stream, false) ||
      !dev_ensure(&r.bound, 64, a->stream, false))
    return fail(a, CEP_E_DEVICE, "out of device memory (reorder sort)");
  if (reorder_sort(r.temp.p, r.temp.bytes, (const int64_t*)r.ts.p, (int64_t*)r.keys.p, (int32_t*)r.idx_in.p,
                   (int32_t*)r.idx_out.p, n, a->stream))
    return fail(a, CEP_E_DEVICE, "reorder sort failed");
  launch_upper_bound((const int64_t*)r.keys.p, n, mark, (int64_t*)r.bound.p, a->stream);
  // rows older than one already released (late events) sort first: count them
  const bool any_released = r.released_max != INT64_MIN;
  if (any_released)
    launch_upper_bound((const int64_t*)r.keys.p, n, r.released_max - 1, (int64_t*)r.bound.p + 3, a->stream);
  int64_t hb[6] = {0, 0, 0, 0, 0, 0};
  if (hipMemcpyAsync(hb, r.bound.p, sizeof(hb), hipMemcpyDeviceToHost, a->stream) != hipSuccess ||
      hipStreamSynchronize(a->stream) != hipSuccess)
    return fail(a, CEP_E_DEVICE, "device failure during processing");
  const int64_t rel = hb[0];
  if (rel == 0) return CEP_OK;
  // A row older than an earlier watermark's release arrived late.  The
  // reference offers it to its PriorityQueue like any row, and this
  // watermark's drain hands it to Siddhi first (smallest ts), behind rows it
  // has already processed (AbstractSiddhiOperator.java:222-231, 238-245).
  // late_policy 2 (default) does the same: the released prefix, late rows
  // included, in (ts, arrival) order, on the order-tolerant path.  Policies
  // 0 / 1 drop them (counted in cep_stats.late_events).
  const int64_t late_n = any_released ? std::min(hb[3], rel) : 0;
  a->late_events += late_n;
  const bool deliver_late = a->opt.late_policy == 2;
  const int64_t late = deliver_late ? 0 : late_n;   // rows dropped from the release
  const int32_t* perm = (const int32_t*)r.idx_out.p;
  bool ok = true;
  for (int c = 0; c < nc && ok; ++c) {
    const int w = type_width(sd.attrs[c].type);
    ok = dev_ensure(&r.out[c], (size_t)n * w, a->stream, false);
    if (ok) launch_gather(r.col[c].p, r.out[c].p, perm, 0, n, w, a->stream);
  }
  ok = ok && dev_ensure(&r.ots, (size_t)n * 8, a->stream, false);
  if (ok) hipMemcpyAsync(r.ots.p, r.keys.p, (size_t)n * 8, hipMemcpyDeviceToDevice, a->stream);
  if (ok && r.has_stream) {
    ok = dev_ensure(&r.ostream, (size_t)n, a->stream, false);
    if (ok) launch_gather(r.stream.p, r.ostream.p, perm, 0, n, 1, a->stream);
  }
  if (!ok) return fail(a, CEP_E_DEVICE, "out of device memory (reorder gather)");
  // the held-back rows stay buffered, now in (ts, arrival) order
  const int64_t keep = n - rel;
  for (int c = 0; c < nc; ++c) {
    const int w = type_width(sd.attrs[c].type);
    hipMemcpyAsync(r.col[c].p, (char*)r.out[c].p + rel * w, (size_t)keep * w, hipMemcpyDeviceToDevice, a->stream);
  }
  hipMemcpyAsync(r.ts.p, (char*)r.ots.p + rel * 8, (size_t)keep * 8, hipMemcpyDeviceToDevice, a->stream);
  if (r.has_stream)
    hipMemcpyAsync(r.stream.p, (char*)r.ostream.p + rel, (size_t)keep, hipMemcpyDeviceToDevice, a->stream);
  r.n = keep;
  const int input = r.input;
  if (keep == 0) r.input = -1;
  // the released prefix minus the late rows is a device batch in event-time order
  const void* cols[kMaxCols];
  for (int c = 0; c < nc; ++c) cols[c] = (const char*)r.out[c].p + late * type_width(sd.attrs[c].type);
  cep_batch bb{};
  bb.n = rel - late;
  bb.ts = (const int64_t*)r.ots.p + late;
  bb.stream = r.has_stream ? (const uint8_t*)r.ostream.p + late : nullptr;
  bb.input = input;
  bb.ncols = nc;
  bb.cols = cols;
  bb.on_device = 1;
  a->last_ts = r.released_max;   // the kernel's order check spans the watermark
  const int64_t rmax = hb[2];
  a->force_tolerant = deliver_late && late_n > 0;
  int rc = cep_send_batch(a, &bb);
  a->force_tolerant = false;
  if (rc == CEP_OK) r.released_max = std::max(r.released_max, rmax);
  // the sorted batch buffers are reused by the next watermark: finish first
  hipStreamSynchronize(a->stream);
  if (rc == CEP_OK && late > 0 && a->opt.late_policy == 1)
    return fail(a, CEP_E_ARG, std::to_string(late) + " late event(s) dropped (older than rows an earlier watermark "
                              "released; the reference would hand them to Siddhi out of order)");
  return rc;
}

int cep_flush(cep_app* a) {
  if (!a) return CEP_E_ARG;
  // the error word, every output cursor and (ordered_output) every delivered
  // output's seq range / descents in one pinned readback, one sync
  const size_t no = a->outs.size();
  const bool order = a->opt.ordered_output != 0;
  if (!host_ensure(&a->flush_words, (no * 4 + 1) * 8)) return fail(a, CEP_E_DEVICE, "out of pinned host memory");
  uint64_t* fw = (uint64_t*)a->flush_words.p;
  uint64_t* fst = fw + 1 + no;   // 3 words per output
  fw[0] = 0;
  if (order) {
    if (!dev_ensure(&a->ostats, no * 3 * 8, a->stream, false)) return fail(a, CEP_E_DEVICE, "out of device memory");
    hipMemsetAsync(a->ostats.p, 0, no * 3 * 8, a->stream);
    for (size_t i = 0; i < no; ++i)
      if (a->outs[i].fn)
        launch_seq_stats((const int64_t*)a->outs[i].seq.p, a->outs[i].count, a->outs[i].cap,
                         (unsigned long long*)a->ostats.p + 3 * i, a->stream);
  }
  hipMemcpyAsync(fw, a->err.p, 4, hipMemcpyDeviceToHost, a->stream);
  if (no) hipMemcpyAsync(fw + 1, a->out_counts.p, no * 8, hipMemcpyDeviceToHost, a->stream);
  if (order) hipMemcpyAsync(fst, a->ostats.p, no * 3 * 8, hipMemcpyDeviceToHost, a->stream);
  if (hipStreamSynchronize(a->stream) != hipSuccess)
    return fail(a, CEP_E_DEVICE, "device failure during processing");
  harvest_timers(a);
  int rc = device_error(a, (unsigned int)fw[0]);
  // an output cursor past its capacity is a hard failure before any count
  // is used (the rows beyond cap were never written)
  for (size_t i = 0; i < no; ++i) {
    auto& o = a->outs[i];
    const unsigned long long cnt = fw[1 + i];
    if (cnt > (unsigned long long)o.cap && rc == CEP_OK)
      rc = fail(a, CEP_E_DEVICE, "output capacity exceeded on " + o.id + ": " + std::to_string(cnt) +
                                     " rows > " + std::to_string(o.cap));
  }
  // Rows of every output are consumed by this flush, delivered or not: a
  // failure part-way stops delivery, records the first error and still resets
  // every cursor below, so a later flush never hands the same rows out again.
  const bool want_seq = !a->opt.omit_seq;
  auto deliver = [&](OutStream& o, size_t i, size_t n) -> int {
    const void* src_ts = o.ts.p;
    const void* src_seq = o.seq.p;
    std::vector<const void*> src(o.cols.size());
    for (size_t c = 0; c < o.cols.size(); ++c) src[c] = o.cols[c].p;
    if (order && fst[3 * i + 2] > 0) {
      // Siddhi's emission order (StreamOutputHandler.java:63-92 receives
      // each completing event's matches in turn): by completing event, then
      // pending order, which the walk already keeps contiguous per key — a
      // stable sort on seq over the window's seq range, then one gather
      // per column, all on the device.
      if (n > (size_t)INT32_MAX) return fail(a, CEP_E_DEVICE, "too many rows to order in one flush");
      const uint64_t bias = 0x8000000000000000ull;
      const int64_t lo = (int64_t)(~fst[3 * i] ^ bias), hi = (int64_t)(fst[3 * i + 1] ^ bias);
      const uint64_t range = (uint64_t)hi - (uint64_t)lo;
      const int bits = range ? 64 - __builtin_clzll(range) : 1;
      const size_t tb = order_temp_bytes((int64_t)n);
      bool ok = dev_ensure(&a->okeys[0], n * 8, a->stream, false) && dev_ensure(&a->okeys[1], n * 8, a->stream, false) &&
                dev_ensure(&a->oidx[0], n * 4, a->stream, false) && dev_ensure(&a->oidx[1], n * 4, a->stream, false) &&
                dev_ensure(&a->otemp, tb, a->stream, false) && dev_ensure(&o.sts, n * 8, a->stream, false) &&
                (!want_seq || dev_ensure(&o.sseq, n * 8, a->stream, false));
      o.scols.resize(o.cols.size());
      for (size_t c = 0; c < o.cols.size() && ok; ++c)
        ok = dev_ensure(&o.scols[c], n * type_width(o.types[c]), a->stream, false);
      if (!ok) return fail(a, CEP_E_DEVICE, "out of device memory (output ordering)");
      if (order_sort(a->otemp.p, a->otemp.bytes, (const int64_t*)o.seq.p, (int64_t)n, lo, bits, a->okeys[0].p,
                     a->okeys[1].p, (int32_t*)a->oidx[0].p, (int32_t*)a->oidx[1].p, a->stream) != 0)
        return fail(a, CEP_E_DEVICE, "output ordering sort failed");
      const int32_t* perm = (const int32_t*)a->oidx[1].p;
      for (size_t c = 0; c < o.cols.size(); ++c) {
        launch_gather(o.cols[c].p, o.scols[c].p, perm, 0, (int64_t)n, type_width(o.types[c]), a->stream);
        src[c] = o.scols[c].p;
      }
      launch_gather(o.ts.p, o.sts.p, perm, 0, (int64_t)n, 8, a->stream);
      src_ts = o.sts.p;
      if (want_seq) {
        launch_gather(o.seq.p, o.sseq.p, perm, 0, (int64_t)n, 8, a->stream);
        src_seq = o.sseq.p;
      }
    }
    // one async D2H per column into pinned buffers, one sync; the seq column
    // only when the consumer reads it (cep_options.omit_seq)
    o.hcols.resize(o.cols.size());
    bool ok = host_ensure(&o.hts, n * 8) && (!want_seq || host_ensure(&o.hseq, n * 8));
    for (size_t c = 0; c < o.cols.size() && ok; ++c) ok = host_ensure(&o.hcols[c], n * type_width(o.types[c]));
    if (!ok) return fail(a, CEP_E_DEVICE, "out of pinned host memory (output delivery)");
    hipMemcpyAsync(o.hts.p, src_ts, n * 8, hipMemcpyDeviceToHost, a->stream);
    if (want_seq) hipMemcpyAsync(o.hseq.p, src_seq, n * 8, hipMemcpyDeviceToHost, a->stream);
    for (size_t c = 0; c < o.cols.size(); ++c)
      hipMemcpyAsync(o.hcols[c].p, src[c], n * type_width(o.types[c]), hipMemcpyDeviceToHost, a->stream);
    if (hipStreamSynchronize(a->stream) != hipSuccess) return fail(a, CEP_E_DEVICE, "output delivery failed");
    std::vector<const void*> ptrs(o.cols.size());
    for (size_t c = 0; c < o.cols.size(); ++c) ptrs[c] = o.hcols[c].p;
    cep_rows rows{};
    rows.stream_id = o.id.c_str();
    rows.n = (int64_t)n;
    rows.ncols = (int32_t)o.cols.size();
    rows.ts = (const int64_t*)o.hts.p;
    rows.seq = want_seq ? (const int64_t*)o.hseq.p : nullptr;
    rows.cols = ptrs.data();
    o.fn(o.user, &rows);
    return CEP_OK;
  };
  for (size_t i = 0; i < no; ++i) {
    auto& o = a->outs[i];
    const unsigned long long cnt = rc == CEP_OK ? fw[1 + i] : 0ull;
    a->matches_out += (int64_t)cnt;
    if (o.fn && cnt > 0 && rc == CEP_OK) rc = deliver(o, i, (size_t)cnt);
    o.bound = 0;
  }
  if (no) hipMemsetAsync(a->out_counts.p, 0, no * 8, a->stream);
  return rc;
}

int cep_output_device(cep_app* a, const char* out_id, cep_rows* rows) {
  if (!a || !out_id || !rows) return CEP_E_ARG;
  int i = a->app.output_index(out_id);
  if (i < 0) return fail(a, CEP_E_UNDEFINED_STREAM, std::string("Stream ") + out_id + " not defined");
  if (hipStreamSynchronize(a->stream) != hipSuccess) return fail(a, CEP_E_DEVICE, "device failure");
  harvest_timers(a);
  int rc = check_device_error(a);
  if (rc) return rc;
  OutStream& o = a->outs[i];
  unsigned long long cnt = 0;
  hipMemcpy(&cnt, o.count, sizeof(cnt), hipMemcpyDeviceToHost);
  if (cnt > (unsigned long long)o.cap)
    return fail(a, CEP_E_DEVICE, "output capacity exceeded on " + o.id);
  static thread_local std::vector<const void*> ptrs;
  ptrs.assign(o.cols.size(), nullptr);
  for (size_t c = 0; c < o.cols.size(); ++c) ptrs[c] = o.cols[c].p;
  rows->stream_id = o.id.c_str();
  rows->n = (int64_t)cnt;
  rows->ncols = (int32_t)o.cols.size();
  rows->ts = (const int64_t*)o.ts.p;
  // omit_seq with unordered output: the kernels need not write them
  rows->seq = (a->opt.omit_seq && !a->opt.ordered_output) ? nullptr : (const int64_t*)o.seq.p;
  rows->cols = ptrs.data();
  return CEP_OK;
}

int cep_reset_output(cep_app* a) {
  if (!a) return CEP_E_ARG;
  for (auto& o : a->outs) {
    hipMemsetAsync(o.count, 0, sizeof(unsigned long long), a->stream);
    o.bound = 0;
  }
  return CEP_OK;
}

int cep_stream_wait(cep_app* a, void* hip_stream) {
  if (!a) return CEP_E_ARG;
  if (hipEventRecord(a->ext_ready, (hipStream_t)hip_stream) != hipSuccess ||
      hipStreamWaitEvent(a->stream, a->ext_ready, 0) != hipSuccess ||
      hipStreamWaitEvent(a->rstream, a->ext_ready, 0) != hipSuccess)
    return fail(a, CEP_E_DEVICE, "cep_stream_wait: invalid stream");
  return CEP_OK;
}

int cep_stream_signal(cep_app* a, void* hip_stream) {
  if (!a) return CEP_E_ARG;
  if (hipEventRecord(a->out_ready, a->stream) != hipSuccess ||
      hipStreamWaitEvent((hipStream_t)hip_stream, a->out_ready, 0) != hipSuccess ||
      hipEventRecord(a->r_ready, a->rstream) != hipSuccess ||
      hipStreamWaitEvent((hipStream_t)hip_stream, a->r_ready, 0) != hipSuccess)
    return fail(a, CEP_E_DEVICE, "cep_stream_signal: invalid stream");
  return CEP_OK;
}

int cep_route_signal(cep_app* a, void* hip_stream) {
  if (!a) return CEP_E_ARG;
  if (hipEventRecord(a->r_ready, a->rstream) != hipSuccess ||
      hipStreamWaitEvent((hipStream_t)hip_stream, a->r_ready, 0) != hipSuccess)
    return fail(a, CEP_E_DEVICE, "cep_route_signal: invalid stream");
  return CEP_OK;
}

int cep_set_enabled(cep_app* a, int enabled) {
  if (!a) return CEP_E_ARG;
  a->enabled = enabled != 0;
  return CEP_OK;
}

int32_t cep_dict_intern(cep_app* a, const char* s) {
  if (!a || !s) return -1;
  auto it = a->dict_index.find(s);
  if (it != a->dict_index.end()) return it->second;
  int32_t id = (int32_t)a->dict.size();
  a->dict.push_back(s);
  a->dict_index.emplace(s, id);
  return id;
}

const char* cep_dict_lookup(cep_app* a, int32_t id) {
  if (!a || id < 0 || id >= (int32_t)a->dict.size()) return nullptr;
  return a->dict[id].c_str();
}

int cep_stats(cep_app* a, cep_stats_t* s) {
  if (!a || !s) return CEP_E_ARG;
  hipStreamSynchronize(a->stream);
  harvest_timers(a);
  std::memset(s, 0, sizeof(*s));
  s->events_in = a->events_in;
  s->matches_out = a->matches_out;
  s->batches = a->batches;
  s->late_events = a->late_events;
  for (auto& p : a->pats)
    if (p.hot) s->hot_keys += *(volatile uint32_t*)p.hot_active_host.p;
  for (int i = 0; i < 16; ++i) {
    s->kernel_launches[i] = a->launches[i];
    s->kernel_ms[i] = a->kernel_ms[i];
    s->kernel_timed[i] = a->kernel_timed[i];
  }
  return CEP_OK;
}

const char* cep_last_error(cep_app* a) { return a ? a->last_error.c_str() : "null app"; }

void cep_free(void* p) { std::free(p); }

// Snapshot format (little endian), version 4:
//   "CEPS" u32 version, u64 plan_hash, i64 events_in, u32 n_patterns,
//   per pattern: i64 key_capacity, u32 S, u32 slot_words, u32 n_live,
//                n_live x { u32 key, u64 header, u32 n, n * slot_words u64 }
//                (n = pending partials, inline slots then the overflow run;
//                versions 2 / 3 have no n: n = header & 0xff)
//   (version >= 3) the event-time reorder buffer ("queuedRecordsState",
//   AbstractSiddhiOperator.java:98): i32 input (-1: empty), u8 has_stream,
//   i64 n, i64 released_max, then n rows: every column of the input's
//   definition (type width each), n x i64 ts, n x u8 stream if has_stream;
//   (version 4) per pattern: u8 sparse keys, if set u32 count, u32 id of
//   the value -1 (0xffffffff: none), count x i64 partition value per dense slot.
//   (version 5) u32 n_groups, per multi-query group: i64 key_capacity,
//   u32 words per key, u32 n_live, n_live x { u32 key, words x u64 }.
// Versions 2 (no reorder section), 3 and 4 are still restored (apps without
// multi-query groups).
static uint64_t plan_hash(const CompiledApp& app) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  };
  mix(app.code.data(), app.code.size() * sizeof(Ins));
  mix(app.konst.data(), app.konst.size() * 8);
  return h;
}

int cep_snapshot(cep_app* a, uint8_t** buf, size_t* len) {
  if (!a || !buf || !len) return CEP_E_ARG;
  if (hipStreamSynchronize(a->stream) != hipSuccess) return fail(a, CEP_E_DEVICE, "device failure");
  std::vector<uint8_t> out;
  auto put = [&](const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    out.insert(out.end(), b, b + n);
  };
  const char magic[4] = {'C', 'E', 'P', 'S'};
  put(magic, 4);
  uint32_t ver = 5;   // 3: + the event-time reorder buffer; 4: + pending counts (overflow runs); 5: + groups
  put(&ver, 4);
  uint64_t h = plan_hash(a->app);
  put(&h, 8);
  put(&a->events_in, 8);
  uint32_t np = (uint32_t)a->pats.size();
  put(&np, 4);
  for (auto& rt : a->pats) {
    const int64_t kc = rt.pa.key_capacity, ks = rt.kstride;
    const uint32_t S = rt.pa.pending_slots, sw = rt.pa.slot_words;
    const int lg = rt.pa.buckets_log2;
    const int64_t kpb = ks >> lg;
    std::vector<uint32_t> hdr(ks);
    std::vector<uint64_t> slots((size_t)ks * S * sw), ext, pool;
    hipMemcpy(hdr.data(), rt.khdr.p, hdr.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(slots.data(), rt.kslot.p, slots.size() * 8, hipMemcpyDeviceToHost);
    if (rt.kext.p) {
      ext.resize(ks);
      pool.resize((size_t)rt.pool_cap * sw);
      hipMemcpy(ext.data(), rt.kext.p, ext.size() * 8, hipMemcpyDeviceToHost);
      hipMemcpy(pool.data(), rt.pool[rt.pool_side].p, pool.size() * 8, hipMemcpyDeviceToHost);
    }
    uint32_t live = 0;
    for (int64_t i = 0; i < ks; ++i) live += hdr[i] ? 1 : 0;
    put(&kc, 8);
    put(&S, 4);
    put(&sw, 4);
    put(&live, 4);
    for (int64_t i = 0; i < ks; ++i) {
      if (!hdr[i]) continue;
      const uint32_t key = (uint32_t)(((i % kpb) << lg) | (i / kpb));   // dense key
      const bool ovf = (hdr[i] & kHdrOvf) && !ext.empty();
      const uint64_t h64 = hdr[i] & ~(uint64_t)kHdrOvf;
      const uint32_t n = ovf ? (uint32_t)ext[i] : (hdr[i] & 0xff);
      const uint64_t off = ovf ? ext[i] >> 32 : 0;
      put(&key, 4);
      put(&h64, 8);
      put(&n, 4);
      for (uint32_t j = 0; j < n; ++j)
        for (uint32_t w = 0; w < sw; ++w)
          put(j < S ? &slots[((size_t)j * sw + w) * ks + i] : &pool[(off + j - S) * sw + w], 8);
    }
  }
  // rows waiting for a watermark (the operator checkpoints its PriorityQueue
  // as "queuedRecordsState": AbstractSiddhiOperator.java:98, 396-404)
  {
    const auto& r = a->ro;
    const int32_t in = r.n > 0 ? r.input : -1;
    const uint8_t hs = r.has_stream ? 1 : 0;
    put(&in, 4);
    put(&hs, 1);
    put(&r.n, 8);
    put(&r.released_max, 8);
    if (r.n > 0) {
      const StreamSchema& sd = a->app.inputs[r.input];
      std::vector<uint8_t> tmp;
      auto pull = [&](const DevBuf& b, size_t bytes) {
        tmp.resize(bytes);
        hipMemcpy(tmp.data(), b.p, bytes, hipMemcpyDeviceToHost);
        put(tmp.data(), bytes);
      };
      for (size_t c = 0; c < sd.attrs.size(); ++c) pull(r.col[c], (size_t)r.n * type_width(sd.attrs[c].type));
      pull(r.ts, (size_t)r.n * 8);
      if (r.has_stream) pull(r.stream, (size_t)r.n);
    }
  }
  // (version 4) per pattern: the sparse-key map, dense slot -> value
  for (auto& rt : a->pats) {
    const uint8_t sp = rt.sparse ? 1 : 0;
    put(&sp, 1);
    if (!sp) continue;
    uint32_t cnt[2];
    hipMemcpy(cnt, rt.kcount.p, 8, hipMemcpyDeviceToHost);
    cnt[0] = std::min<uint32_t>(cnt[0], (uint32_t)rt.pa.key_capacity);
    put(cnt, 8);
    std::vector<uint64_t> rev(cnt[0]);
    if (cnt[0]) hipMemcpy(rev.data(), rt.krev.p, rev.size() * 8, hipMemcpyDeviceToHost);
    put(rev.data(), rev.size() * 8);
  }
  // (version 5) multi-query groups: per group every key whose state is not
  // all zero, with the group's state words (query by query, plan order)
  {
    const uint32_t ng = (uint32_t)a->mqs.size();
    put(&ng, 4);
    for (auto& g : a->mqs) {
      const int64_t ks = g.kstride, kpb = g.kpb;
      const uint32_t nw = (uint32_t)g.words;
      std::vector<uint64_t> st((size_t)g.words * ks);
      hipMemcpy(st.data(), g.state.p, st.size() * 8, hipMemcpyDeviceToHost);
      std::vector<uint32_t> live;
      // state word w of bucket-major key index i = b * kpb + k lives at
      // (b * words + w) * kpb + k (each bucket's state is one contiguous block)
      auto sidx = [&](int64_t i, uint32_t w) { return (size_t)(((i / kpb) * nw + w) * kpb + i % kpb); };
      for (int64_t i = 0; i < ks; ++i) {
        bool any = false;
        for (uint32_t w = 0; w < nw && !any; ++w) any = st[sidx(i, w)] != 0;
        if (any) live.push_back((uint32_t)i);
      }
      const uint32_t nl = (uint32_t)live.size();
      put(&g.key_capacity, 8);
      put(&nw, 4);
      put(&nl, 4);
      for (uint32_t i : live) {
        const uint32_t key = (uint32_t)(((i % kpb) << g.lg) | (i / kpb));   // dense key
        put(&key, 4);
        for (uint32_t w = 0; w < nw; ++w) put(&st[sidx(i, w)], 8);
      }
    }
  }
  *buf = (uint8_t*)std::malloc(out.size());
  if (!*buf) return fail(a, CEP_E_DEVICE, "out of host memory");
  std::memcpy(*buf, out.data(), out.size());
  *len = out.size();
  return CEP_OK;
}

int cep_restore(cep_app* a, const uint8_t* buf, size_t len) {
  if (!a || (!buf && len)) return CEP_E_ARG;
  size_t off = 0;
  auto get = [&](void* p, size_t n) -> bool {
    if (n > len - off) return false;
    std::memcpy(p, buf + off, n);
    off += n;
    return true;
  };
  char magic[4];
  uint32_t ver;
  uint64_t h;
  int64_t ev;
  uint32_t np;
  if (!get(magic, 4) || std::memcmp(magic, "CEPS", 4) || !get(&ver, 4) || ver < 2 || ver > 5 || !get(&h, 8) ||
      !get(&ev, 8) || !get(&np, 4))
    return fail(a, CEP_E_STATE, "not a libcep snapshot");
  if (h != plan_hash(a->app) || np != a->pats.size())
    return fail(a, CEP_E_STATE, "snapshot was taken with a different plan (or a build that compiled it "
                                "differently: 2-state patterns with s1-dependent conditions need CEP_PAIR_WALK=1 "
                                "to restore snapshots of builds before round 4)");
  // Phase 1: parse and validate everything into host buffers; nothing on the
  // device changes until the whole snapshot is known to be good.
  struct PatState {
    std::vector<uint32_t> hdr;
    std::vector<uint64_t> slots, ext, pool;
    uint64_t pool_used = 0;
  };
  std::vector<PatState> ps(a->pats.size());
  for (size_t pi = 0; pi < a->pats.size(); ++pi) {
    const PatternRT& rt = a->pats[pi];
    int64_t kc;
    uint32_t S, sw, live;
    if (!get(&kc, 8) || !get(&S, 4) || !get(&sw, 4) || !get(&live, 4))
      return fail(a, CEP_E_STATE, "truncated snapshot");
    if (kc != rt.pa.key_capacity || S != (uint32_t)rt.pa.pending_slots ||
        sw != (uint32_t)rt.pa.slot_words)
      return fail(a, CEP_E_STATE, "snapshot geometry differs from this runtime");
    if ((uint64_t)live > (uint64_t)kc) return fail(a, CEP_E_STATE, "corrupt snapshot (live keys)");
    const int64_t ks = rt.kstride;
    const int lg = rt.pa.buckets_log2;
    const int64_t kpb = ks >> lg;
    ps[pi].hdr.assign(ks, 0);
    ps[pi].slots.assign((size_t)ks * S * sw, 0);
    if (rt.kext.p) ps[pi].ext.assign(ks, 0);
    for (uint32_t i = 0; i < live; ++i) {
      uint32_t key, nk;
      uint64_t h64;
      if (!get(&key, 4) || !get(&h64, 8) || key >= kc || (h64 & kHdrOvf))
        return fail(a, CEP_E_STATE, "corrupt snapshot");
      if (ver >= 4) {
        if (!get(&nk, 4)) return fail(a, CEP_E_STATE, "truncated snapshot");
      } else {
        nk = (uint32_t)(h64 & 0xff);
      }
      if ((uint64_t)nk * sw > (len - off) / 8) return fail(a, CEP_E_STATE, "truncated snapshot");
      const int64_t idx = (int64_t)(key & ((1u << lg) - 1)) * kpb + (key >> lg);
      uint32_t hw = (uint32_t)h64;
      if (nk > S) {   // overflow run: the pending pool (closed-form runtimes only)
        if (ps[pi].ext.empty())
          return fail(a, CEP_E_CAPACITY, "snapshot holds more than pending_slots partials for a key");
        if (ps[pi].pool_used + (nk - S) > (uint64_t)rt.pool_cap)
          return fail(a, CEP_E_CAPACITY, "snapshot's overflow partials exceed the pending pool");
        ps[pi].ext[idx] = (uint64_t)nk | (ps[pi].pool_used << 32);
        ps[pi].pool.resize((ps[pi].pool_used + (nk - S)) * sw);
        hw = (hw & ~0xffu) | (uint32_t)S | kHdrOvf;
      } else {
        hw = (hw & ~0xffu) | nk;
      }
      for (uint32_t j = 0; j < nk; ++j)
        for (uint32_t w = 0; w < sw; ++w) {
          uint64_t* dst = j < S ? &ps[pi].slots[((size_t)j * sw + w) * ks + idx]
                                : &ps[pi].pool[(ps[pi].pool_used + j - S) * sw + w];
          if (!get(dst, 8)) return fail(a, CEP_E_STATE, "truncated snapshot");
        }
      if (nk > S) ps[pi].pool_used += nk - S;
      ps[pi].hdr[idx] = hw;
    }
  }
  int32_t in = -1;
  uint8_t hs = 0;
  int64_t n = 0, rmax = INT64_MIN;
  size_t rows_off = 0;
  if (ver >= 3) {
    if (!get(&in, 4) || !get(&hs, 1) || !get(&n, 8) || !get(&rmax, 8) || n < 0 || n > (int64_t)INT32_MAX ||
        (n > 0 && (in < 0 || in >= (int)a->app.inputs.size())))
      return fail(a, CEP_E_STATE, "corrupt snapshot (reorder buffer)");
    if (n > 0) {
      size_t row_bytes = 8 + (hs ? 1 : 0);
      for (auto& at : a->app.inputs[in].attrs) row_bytes += (size_t)type_width(at.type);
      if ((uint64_t)n > (len - off) / row_bytes)
        return fail(a, CEP_E_STATE, "truncated snapshot (reorder buffer)");
      rows_off = off;
      off += (size_t)n * row_bytes;
    }
  }
  // sparse-key maps: rebuilt here as device tables (same hash and probing
  // as keymap.hip; any valid placement serves lookups)
  struct KeyMap {
    std::vector<uint64_t> tkey, rev;
    std::vector<uint32_t> tval;
    uint32_t cnt[2] = {0, 0xffffffffu};
  };
  std::vector<KeyMap> km(a->pats.size());
  if (ver >= 4) {
    for (size_t pi = 0; pi < a->pats.size(); ++pi) {
      const PatternRT& rt = a->pats[pi];
      uint8_t sp;
      if (!get(&sp, 1) || (sp != 0) != rt.sparse) return fail(a, CEP_E_STATE, "snapshot key map does not match");
      if (!sp) continue;
      KeyMap& m = km[pi];
      if (!get(m.cnt, 8) || m.cnt[0] > (uint64_t)rt.pa.key_capacity || (uint64_t)m.cnt[0] > (len - off) / 8)
        return fail(a, CEP_E_STATE, "corrupt snapshot (key map)");
      m.rev.resize(m.cnt[0]);
      get(m.rev.data(), m.rev.size() * 8);
      m.tkey.assign(rt.table_cap, 0);
      m.tval.assign(rt.table_cap, 0xffffffffu);
      for (uint32_t id = 0; id < m.cnt[0]; ++id) {
        if (id == m.cnt[1]) continue;   // the value -1 has its own word
        const uint64_t v = m.rev[id];
        uint64_t z = v + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        uint64_t h = (z ^ (z >> 31)) & (rt.table_cap - 1);
        while (m.tkey[h]) h = (h + 1) & (rt.table_cap - 1);
        m.tkey[h] = v + 1;
        m.tval[h] = id;
      }
    }
  } else {
    for (auto& rt : a->pats)
      if (rt.sparse) return fail(a, CEP_E_STATE, "snapshot has no key map (version < 4)");
  }
  // (version 5) multi-query group state
  std::vector<std::vector<uint64_t>> mst(a->mqs.size());
  if (ver >= 5) {
    uint32_t ng;
    if (!get(&ng, 4) || ng != a->mqs.size()) return fail(a, CEP_E_STATE, "snapshot multi-query groups do not match");
    for (size_t gi = 0; gi < a->mqs.size(); ++gi) {
      const MqRT& g = a->mqs[gi];
      int64_t kc;
      uint32_t nw, nl;
      if (!get(&kc, 8) || !get(&nw, 4) || !get(&nl, 4)) return fail(a, CEP_E_STATE, "truncated snapshot");
      if (kc != g.key_capacity || nw != (uint32_t)g.words || nl > (uint64_t)kc)
        return fail(a, CEP_E_STATE, "snapshot geometry differs from this runtime");
      if ((uint64_t)nl * (4 + 8ull * nw) > len - off) return fail(a, CEP_E_STATE, "truncated snapshot");
      mst[gi].assign((size_t)g.words * g.kstride, 0);
      for (uint32_t i = 0; i < nl; ++i) {
        uint32_t key;
        get(&key, 4);
        if (key >= kc) return fail(a, CEP_E_STATE, "corrupt snapshot");
        const int64_t idx = (int64_t)(key & ((1u << g.lg) - 1)) * g.kpb + (key >> g.lg);
        for (uint32_t w = 0; w < nw; ++w)
          get(&mst[gi][(size_t)(((idx / g.kpb) * nw + w) * g.kpb + idx % g.kpb)], 8);
      }
    }
  } else if (!a->mqs.empty()) {
    // v2-v4 kept these queries on per-query runtimes: a runtime created with
    // CEP_NO_MQ=1 has that layout and restores the snapshot
    return fail(a, CEP_E_STATE, "snapshot has no multi-query group state (version < 5): "
                                "create the runtime with CEP_NO_MQ=1 to restore it on per-query state");
  }
  // Phase 2: commit (device allocations first, so a failure leaves the
  // runtime as it was)
  auto& r = a->ro;
  if (n > 0) {
    const StreamSchema& sd = a->app.inputs[in];
    bool ok = true;
    for (size_t c = 0; c < sd.attrs.size() && ok; ++c)
      ok = dev_ensure(&r.col[c], (size_t)n * type_width(sd.attrs[c].type), a->stream, false);
    ok = ok && dev_ensure(&r.ts, (size_t)n * 8, a->stream, false);
    if (hs) ok = ok && dev_ensure(&r.stream, (size_t)n, a->stream, false);
    if (!ok) return fail(a, CEP_E_DEVICE, "out of device memory (reorder buffer)");
  }
  hipStreamSynchronize(a->stream);
  for (size_t pi = 0; pi < a->pats.size(); ++pi) {
    PatternRT& rt = a->pats[pi];
    hipMemcpy(rt.khdr.p, ps[pi].hdr.data(), ps[pi].hdr.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(rt.kslot.p, ps[pi].slots.data(), ps[pi].slots.size() * 8, hipMemcpyHostToDevice);
    if (rt.kext.p) {
      hipMemcpy(rt.kext.p, ps[pi].ext.data(), ps[pi].ext.size() * 8, hipMemcpyHostToDevice);
      if (!ps[pi].pool.empty())
        hipMemcpy(rt.pool[rt.pool_side].p, ps[pi].pool.data(), ps[pi].pool.size() * 8, hipMemcpyHostToDevice);
    }
  }
  r.n = 0;
  r.input = -1;
  r.released_max = rmax;
  if (n > 0) {
    const StreamSchema& sd = a->app.inputs[in];
    size_t o = rows_off;
    for (size_t c = 0; c < sd.attrs.size(); ++c) {
      const size_t bytes = (size_t)n * type_width(sd.attrs[c].type);
      hipMemcpy(r.col[c].p, buf + o, bytes, hipMemcpyHostToDevice);
      o += bytes;
    }
    hipMemcpy(r.ts.p, buf + o, (size_t)n * 8, hipMemcpyHostToDevice);
    o += (size_t)n * 8;
    if (hs) hipMemcpy(r.stream.p, buf + o, (size_t)n, hipMemcpyHostToDevice);
    r.input = in;
    r.has_stream = hs != 0;
    r.n = n;
  }
  for (size_t pi = 0; pi < a->pats.size(); ++pi) {
    PatternRT& rt = a->pats[pi];
    if (!rt.sparse) continue;
    hipMemcpy(rt.tkey.p, km[pi].tkey.data(), km[pi].tkey.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(rt.tval.p, km[pi].tval.data(), km[pi].tval.size() * 4, hipMemcpyHostToDevice);
    if (!km[pi].rev.empty()) hipMemcpy(rt.krev.p, km[pi].rev.data(), km[pi].rev.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(rt.kcount.p, km[pi].cnt, 8, hipMemcpyHostToDevice);
  }
  for (size_t gi = 0; gi < a->mqs.size(); ++gi)
    hipMemcpy(a->mqs[gi].state.p, mst[gi].data(), mst[gi].size() * 8, hipMemcpyHostToDevice);
  a->events_in = ev;
  return CEP_OK;
}

int cep_record_words(cep_app* a) {
  if (!a || a->pats.size() != 1) return -CEP_E_UNSUPPORTED;
  return a->pats[0].pa.rec_words + 1;   // wide record: [hdr, seq, ts, carried...]
}

// seg_cap == 0: owner-contiguous output, counts read back (cep_route_batch);
// seg_cap > 0: padded owner segments with in-band counts, nothing read back
// (cep_route_batch_padded).
struct SpillArgs {
  void* out = nullptr;         // nullptr: records past seg_cap are dropped (and flagged)
  int64_t cap = 0;             // records the spill holds
  int64_t* counts = nullptr;   // device: spilled records per owner
};

static int route_batch(cep_app* a, const cep_batch* b, int world, int64_t seq0, void* rec_out,
                       int64_t rec_cap, int64_t* counts_host, int64_t seg_cap, const SpillArgs& sp = SpillArgs()) {
  if (!a || !b || world <= 0 || (seg_cap == 0 && !counts_host) || seg_cap < 0) return CEP_E_ARG;
  if (world > kMaxWorld) return fail(a, CEP_E_ARG, "world exceeds " + std::to_string(kMaxWorld));
  if (a->pats.size() != 1 || a->app.queries.size() != 1)
    return fail(a, CEP_E_UNSUPPORTED, "key shuffle needs an app with exactly one keyed pattern");
  PatternRT& rt = a->pats[0];
  const Query& q = a->app.queries[rt.q];
  if (q.key_col_a < 0 || q.key_col_b < 0)
    return fail(a, CEP_E_UNSUPPORTED, "key shuffle needs a partitioned pattern");
  if (seg_cap == 0) {
    for (int d = 0; d < world; ++d) counts_host[d] = 0;
    if (b->n == 0) return CEP_OK;
    // the gather writes rec_out as soon as it runs: at most n records are
    // routed, so a buffer of n records can never overrun (checked up front)
    if (!rec_out || rec_cap < b->n)
      return fail(a, CEP_E_ARG, "rec_out must hold at least n records (" + std::to_string(b->n) + ")");
  } else {
    // every rank ships world segments each step, so the null records need a
    // ts / seq of this batch (its first and last rows)
    if (b->n == 0) return fail(a, CEP_E_ARG, "padded key shuffle needs a non-empty batch");
    if (!rec_out || rec_cap < (int64_t)world * (1 + seg_cap))
      return fail(a, CEP_E_ARG, "rec_out must hold world * (1 + seg_cap) records");
  }
  RowsArgs rows{};
  int slot;
  bool direct;
  int rc = batch_rows(a, b, &rows, &slot, &direct);
  if (rc) return rc;
  // fast route (k_cfroute) when every column the pattern reads is prefetchable
  // and f / g are term lists (the k_cfpart load path); CEP_NO_CF=1 forces k_route
  static const bool no_cf = std::getenv("CEP_NO_CF") != nullptr;
  const bool fast = !no_cf && !rt.part_vm && rt.pref.n >= 0 && rt.pref.key_slot <= 0 &&
                    rt.pa.rec_words + 1 <= 5 && pref_aligned(rt.pref, rows);
  const int64_t tile_rows = fast ? kCfTile : kPartThreads * kPartItems;
  const int64_t ntiles = (b->n + tile_rows - 1) / tile_rows;
  const int wrw = rt.pa.rec_words + 1;
  // device batches route on the route stream (ordered after the producer by
  // cep_stream_wait), so the walk of the previous batch keeps running; host
  // batches were staged on the engine stream and route there
  hipStream_t rs = b->on_device ? a->rstream : a->stream;
  if (!dev_ensure(&a->route_arena, (size_t)ntiles * tile_rows * wrw * 8, rs, false) ||
      !dev_ensure(&a->route_tcount, (size_t)ntiles * world * 4, rs, false) ||
      !dev_ensure(&a->route_toffs, (size_t)ntiles * world * 4, rs, false) ||
      !dev_ensure(&a->route_dcount, (size_t)world * 8, rs, false))
    return fail(a, CEP_E_DEVICE, "out of device memory (route arena)");
  RouteArgs ra{};
  ra.rows = rows;
  ra.vm = {(const Ins*)a->code.p, (const uint64_t*)a->konst.p};
  ra.pat = rt.pa;
  ra.world = world;
  ra.wrw = wrw;
  ra.tile_rows = (int32_t)tile_rows;
  ra.seq0 = seq0;
  ra.arena = (uint64_t*)a->route_arena.p;
  ra.tcount = (uint32_t*)a->route_tcount.p;
  ra.err = (unsigned int*)a->rerr.p;
  ra.seg_cap = seg_cap;
  ra.spill = (uint64_t*)sp.out;
  ra.spill_cap = sp.cap;
  ra.spill_counts = sp.counts;
  {
    LaunchTimer t(a, CEP_K_ROUTE, rs);
    if (fast) {
      CfRouteArgs ca{};
      ca.r = ra;
      ca.pref = rt.pref;
      ca.ts_slot = -1;
      for (int i = 0; i < rt.pref.n; ++i)
        if (rows.cols.p[rt.pref.col[i]] == (const void*)rows.ts && rows.cols.t[rt.pref.col[i]] == T_LONG)
          ca.ts_slot = i;
      launch_cf_route(ca, ntiles, rs);
      launch_route_collect(ra, ntiles, (uint32_t*)a->route_toffs.p,
                           (unsigned long long*)a->route_dcount.p, (uint64_t*)rec_out, rs);
    } else {
      launch_route(ra, ntiles, rt.part_vm, (uint32_t*)a->route_toffs.p,
                   (unsigned long long*)a->route_dcount.p, (uint64_t*)rec_out, rs);
    }
    if (seg_cap > 0) launch_route_pad(ra, (const unsigned long long*)a->route_dcount.p, (uint64_t*)rec_out, rs);
  }
  if (slot >= 0) hipEventRecord(a->hs[slot].free, rs);
  if (seg_cap > 0) {
    // the route's error bits travel in the segment headers (every owner
    // reports them at its next flush); cleared behind the pad kernel
    hipMemsetAsync(a->rerr.p, 0, 64, rs);
    a->batches++;
    return hipGetLastError() == hipSuccess ? CEP_OK : fail(a, CEP_E_DEVICE, "padded route launch failed");
  }
  // the per-owner counts: W words, read back on the route stream only (the
  // all-to-all's split sizes are host values); the engine stream keeps going
  std::vector<unsigned long long> dc(world);
  unsigned int re = 0;
  hipMemcpyAsync(dc.data(), a->route_dcount.p, world * 8, hipMemcpyDeviceToHost, rs);
  hipMemcpyAsync(&re, a->rerr.p, 4, hipMemcpyDeviceToHost, rs);
  if (hipStreamSynchronize(rs) != hipSuccess) return fail(a, CEP_E_DEVICE, "route failed");
  int64_t total = 0;
  for (int d = 0; d < world; ++d) {
    counts_host[d] = (int64_t)dc[d];
    total += (int64_t)dc[d];
  }
  if (total > b->n) return fail(a, CEP_E_DEVICE, "route produced more records than rows");
  // the route kernels' own error word, read and cleared on the route stream
  // (the walk's word belongs to cep_flush)
  if (re) {
    hipMemsetAsync(a->rerr.p, 0, 64, rs);
    hipStreamSynchronize(rs);
    return error_status(a, re);
  }
  a->batches++;
  return CEP_OK;
}

int cep_route_batch(cep_app* a, const cep_batch* b, int world, int64_t seq0, void* rec_out,
                    int64_t rec_cap, int64_t* counts_host) {
  return route_batch(a, b, world, seq0, rec_out, rec_cap, counts_host, 0);
}

// A host batch is staged and routed on the engine stream; join that into the
// route stream so cep_route_signal (which records on the route stream) also
// orders a consumer after it (the padded routes read nothing back).
static int route_join_host(cep_app* a, const cep_batch* b, int rc) {
  if (rc != CEP_OK || !b || b->on_device) return rc;
  if (hipEventRecord(a->r_host, a->stream) != hipSuccess ||
      hipStreamWaitEvent(a->rstream, a->r_host, 0) != hipSuccess)
    return fail(a, CEP_E_DEVICE, "route: stream join failed");
  return rc;
}

int cep_route_batch_padded(cep_app* a, const cep_batch* b, int world, int64_t seq0, void* seg_out,
                           int64_t seg_out_cap, int64_t seg_cap) {
  if (seg_cap <= 0) return CEP_E_ARG;
  return route_join_host(a, b, route_batch(a, b, world, seq0, seg_out, seg_out_cap, nullptr, seg_cap));
}

int cep_route_batch_padded_spill(cep_app* a, const cep_batch* b, int world, int64_t seq0, void* seg_out,
                                 int64_t seg_out_cap, int64_t seg_cap, void* spill_out, int64_t spill_cap,
                                 int64_t* spill_counts) {
  if (seg_cap <= 0 || !spill_out || spill_cap < 0 || !spill_counts) return CEP_E_ARG;
  SpillArgs sp;
  sp.out = spill_out;
  sp.cap = spill_cap;
  sp.counts = spill_counts;
  return route_join_host(a, b, route_batch(a, b, world, seq0, seg_out, seg_out_cap, nullptr, seg_cap, sp));
}

// Row shuffle plan: per input handle the owner key column (-1: any owner,
// the stream feeds stateless filters only; -2: no query reads it).  Every
// query that keeps per-key state must key each stream it reads on one
// attribute, the same for all such queries; the shipped streams must share
// one column layout (the owner unpacks them into one multi-stream batch).
static int row_route_plan(cep_app* a, int32_t (&kc)[8], int* layout) {
  const CompiledApp& app = a->app;
  const int ni = (int)app.inputs.size();
  if (ni > 8) return fail(a, CEP_E_UNSUPPORTED, "row shuffle supports at most 8 input streams");
  for (int i = 0; i < 8; ++i) kc[i] = -2;
  auto need = [&](int s, int col) -> int {
    if (s < 0 || s >= ni) return CEP_OK;
    if (col < 0) return fail(a, CEP_E_UNSUPPORTED, "row shuffle: query state on stream " + app.inputs[s].id +
                                                     " is not keyed (needs `partition with` or group by)");
    if (kc[s] >= 0 && kc[s] != col)
      return fail(a, CEP_E_UNSUPPORTED, "row shuffle: stream " + app.inputs[s].id + " is keyed on two attributes");
    kc[s] = col;
    return CEP_OK;
  };
  for (auto& q : app.queries) {
    int rc = CEP_OK;
    if (q.kind == Q_FILTER) {
      if (q.in_stream >= 0 && kc[q.in_stream] == -2) kc[q.in_stream] = -1;
      continue;
    }
    if (q.kind == Q_AGG) {
      rc = need(q.in_stream, q.key_col);
    } else if (q.nfa) {
      for (auto& st : q.nstates) {
        rc = need(st.stream, st.stream >= 0 && st.stream < (int)q.key_col_s.size() ? q.key_col_s[st.stream] : -1);
        if (rc) break;
      }
    } else {
      rc = need(q.a_stream, q.key_col_a);
      if (!rc) rc = need(q.b_stream, q.key_col_b);
    }
    if (rc) return rc;
  }
  // a keyed stream also read by a filter keeps its key (filters are stateless)
  *layout = -1;
  for (int s = 0; s < ni; ++s) {
    if (kc[s] == -2) continue;
    if (*layout < 0) {
      *layout = s;
      continue;
    }
    const auto& x = app.inputs[*layout].attrs;
    const auto& y = app.inputs[s].attrs;
    bool same = x.size() == y.size();
    for (size_t c = 0; same && c < x.size(); ++c) same = x[c].type == y[c].type;
    if (!same)
      return fail(a, CEP_E_UNSUPPORTED, "row shuffle: streams " + app.inputs[*layout].id + " and " +
                                            app.inputs[s].id + " have different column types");
  }
  if (*layout < 0) return fail(a, CEP_E_UNSUPPORTED, "row shuffle: no query reads any input stream");
  return CEP_OK;
}

int cep_send_records(cep_app* a, const void* recs, int64_t n, int64_t events_represented) {
  if (!a || (n > 0 && !recs) || n < 0) return CEP_E_ARG;
  if (!a->enabled) return CEP_OK;
  if (a->pats.size() != 1 || a->app.queries.size() != 1)
    return fail(a, CEP_E_UNSUPPORTED, "records need an app with exactly one keyed pattern");
  a->events_in += events_represented;
  if (n == 0) return CEP_OK;
  PatternRT& rt = a->pats[0];
  RowsArgs rows{};
  rows.n = n;
  rows.row0 = 0;
  rows.input = rt.pa.a_stream;
  a->batches++;
  return run_pattern(a, rt, rows, (const uint64_t*)recs, rt.pa.rec_words + 1);
}

int cep_send_records_padded(cep_app* a, const void* segs, int world, int64_t seg_cap,
                            int64_t events_represented) {
  if (!a || !segs || world <= 0 || world > kMaxWorld || seg_cap <= 0) return CEP_E_ARG;
  if (!a->enabled) return CEP_OK;
  if (a->pats.size() != 1 || a->app.queries.size() != 1)
    return fail(a, CEP_E_UNSUPPORTED, "records need an app with exactly one keyed pattern");
  a->events_in += events_represented;
  PatternRT& rt = a->pats[0];
  const int wrw = rt.pa.rec_words + 1;
  // the headers' counts / error bits -> this engine's error word (reported
  // by the next flush); the null records flow through the partitions, which
  // skip role-0 records, so no count is read back here
  launch_route_check((const uint64_t*)segs, world, seg_cap, wrw, 0, (unsigned int*)a->err.p, a->stream);
  RowsArgs rows{};
  rows.n = (int64_t)world * (1 + seg_cap);
  rows.row0 = 0;
  rows.input = rt.pa.a_stream;
  a->batches++;
  return run_pattern(a, rt, rows, (const uint64_t*)segs, wrw);
}

int cep_row_words(cep_app* a) {
  if (!a) return -CEP_E_ARG;
  int32_t kc[8];
  int layout;
  const int rc = row_route_plan(a, kc, &layout);
  if (rc) return -rc;
  return 3 + (int)a->app.inputs[layout].attrs.size();
}

// seg_cap == 0: owner-contiguous rows, counts read back (cep_route_rows);
// seg_cap > 0: padded owner segments, counts in-band (cep_route_rows_padded).
static int route_rows(cep_app* a, const cep_batch* b, int world, int64_t seq0, void* rec_out, int64_t rec_cap,
                      int64_t* counts_host, int64_t seg_cap, const SpillArgs& sp = SpillArgs()) {
  if (!a || !b || world <= 0 || seg_cap < 0 || (seg_cap == 0 && !counts_host)) return CEP_E_ARG;
  if (world > kMaxWorld) return fail(a, CEP_E_ARG, "world exceeds " + std::to_string(kMaxWorld));
  int32_t kc[8];
  int layout;
  int rc = row_route_plan(a, kc, &layout);
  if (rc) return rc;
  if (seg_cap == 0) {
    for (int d = 0; d < world; ++d) counts_host[d] = 0;
    if (b->n == 0) return CEP_OK;
    if (!rec_out || rec_cap < b->n)
      return fail(a, CEP_E_ARG, "rec_out must hold at least n rows (" + std::to_string(b->n) + ")");
  } else {
    if (b->n == 0) return fail(a, CEP_E_ARG, "padded row shuffle needs a non-empty batch");
    if (!rec_out || rec_cap < (int64_t)world * (1 + seg_cap))
      return fail(a, CEP_E_ARG, "seg_out must hold world * (1 + seg_cap) rows");
  }
  if (b->stream) {
    // a multi-stream batch needs one layout for all its streams (batch_rows)
  } else if (kc[b->input] != -2) {
    const auto& x = a->app.inputs[layout].attrs;
    const auto& y = a->app.inputs[b->input].attrs;
    bool same = x.size() == y.size();
    for (size_t c = 0; same && c < x.size(); ++c) same = x[c].type == y[c].type;
    if (!same) return fail(a, CEP_E_UNSUPPORTED, "row shuffle: batch stream layout differs");
  }
  RowsArgs rows{};
  int slot;
  bool direct;
  rc = batch_rows(a, b, &rows, &slot, &direct);
  if (rc) return rc;
  const int64_t tile_rows = kPartThreads * kPartItems;
  const int64_t ntiles = (b->n + tile_rows - 1) / tile_rows;
  const int wrw = 3 + rows.cols.n;
  hipStream_t rs = b->on_device ? a->rstream : a->stream;
  if (!dev_ensure(&a->route_arena, (size_t)ntiles * tile_rows * wrw * 8, rs, false) ||
      !dev_ensure(&a->route_tcount, (size_t)ntiles * world * 4, rs, false) ||
      !dev_ensure(&a->route_toffs, (size_t)ntiles * world * 4, rs, false) ||
      !dev_ensure(&a->route_dcount, (size_t)world * 8, rs, false))
    return fail(a, CEP_E_DEVICE, "out of device memory (route arena)");
  RowRouteArgs ra{};
  ra.rows = rows;
  ra.world = world;
  ra.wrw = wrw;
  ra.tile_rows = (int32_t)tile_rows;
  ra.seq0 = seq0;
  for (int i = 0; i < 8; ++i) ra.key_col_s[i] = kc[i];
  ra.arena = (uint64_t*)a->route_arena.p;
  ra.tcount = (uint32_t*)a->route_tcount.p;
  ra.err = (unsigned int*)a->rerr.p;
  ra.seg_cap = seg_cap;
  ra.spill = (uint64_t*)sp.out;
  ra.spill_cap = sp.cap;
  ra.spill_counts = sp.counts;
  {
    LaunchTimer t(a, CEP_K_ROUTE, rs);
    launch_route_rows(ra, ntiles, (uint32_t*)a->route_toffs.p, (unsigned long long*)a->route_dcount.p,
                      (uint64_t*)rec_out, rs);
  }
  if (slot >= 0) hipEventRecord(a->hs[slot].free, rs);
  if (seg_cap > 0) {   // nothing read back: the error bits travel in the headers
    hipMemsetAsync(a->rerr.p, 0, 64, rs);
    a->batches++;
    return hipGetLastError() == hipSuccess ? CEP_OK : fail(a, CEP_E_DEVICE, "padded row route launch failed");
  }
  std::vector<unsigned long long> dc(world);
  unsigned int re = 0;
  hipMemcpyAsync(dc.data(), a->route_dcount.p, world * 8, hipMemcpyDeviceToHost, rs);
  hipMemcpyAsync(&re, a->rerr.p, 4, hipMemcpyDeviceToHost, rs);
  if (hipStreamSynchronize(rs) != hipSuccess) return fail(a, CEP_E_DEVICE, "row route failed");
  int64_t total = 0;
  for (int d = 0; d < world; ++d) {
    counts_host[d] = (int64_t)dc[d];
    total += (int64_t)dc[d];
  }
  if (total > b->n) return fail(a, CEP_E_DEVICE, "route produced more rows than the batch");
  if (re) {   // the route kernels' own error word (route stream)
    hipMemsetAsync(a->rerr.p, 0, 64, rs);
    hipStreamSynchronize(rs);
    return error_status(a, re);
  }
  a->batches++;
  return CEP_OK;
}

int cep_route_rows(cep_app* a, const cep_batch* b, int world, int64_t seq0, void* rec_out, int64_t rec_cap,
                   int64_t* counts_host) {
  return route_rows(a, b, world, seq0, rec_out, rec_cap, counts_host, 0);
}

int cep_route_rows_padded(cep_app* a, const cep_batch* b, int world, int64_t seq0, void* seg_out,
                          int64_t seg_out_cap, int64_t seg_cap) {
  if (seg_cap <= 0) return CEP_E_ARG;
  return route_join_host(a, b, route_rows(a, b, world, seq0, seg_out, seg_out_cap, nullptr, seg_cap));
}

int cep_route_rows_padded_spill(cep_app* a, const cep_batch* b, int world, int64_t seq0, void* seg_out,
                                int64_t seg_out_cap, int64_t seg_cap, void* spill_out, int64_t spill_cap,
                                int64_t* spill_counts) {
  if (seg_cap <= 0 || !spill_out || spill_cap < 0 || !spill_counts) return CEP_E_ARG;
  SpillArgs sp;
  sp.out = spill_out;
  sp.cap = spill_cap;
  sp.counts = spill_counts;
  return route_join_host(a, b, route_rows(a, b, world, seq0, seg_out, seg_out_cap, nullptr, seg_cap, sp));
}

int cep_send_rows_padded(cep_app* a, const void* segs, int world, int64_t seg_cap, int64_t events_represented) {
  if (!a || !segs || world <= 0 || world > kMaxWorld || seg_cap <= 0) return CEP_E_ARG;
  if (!a->enabled) return CEP_OK;
  const int w = cep_row_words(a);
  if (w < 0) return -w;
  // headers -> this engine's error word; header and null rows carry stream
  // handle kRowNullStream, which no query reads
  launch_route_check((const uint64_t*)segs, world, seg_cap, w, 1, (unsigned int*)a->err.p, a->stream);
  return cep_send_rows(a, segs, (int64_t)world * (1 + seg_cap), events_represented);
}

int cep_send_rows(cep_app* a, const void* recs, int64_t n, int64_t events_represented) {
  if (!a || (n > 0 && !recs) || n < 0) return CEP_E_ARG;
  if (!a->enabled) return CEP_OK;
  int32_t kc[8];
  int layout;
  int rc = row_route_plan(a, kc, &layout);
  if (rc) return rc;
  a->events_in += events_represented;
  if (n == 0) return CEP_OK;
  const StreamSchema& sd = a->app.inputs[layout];
  const int nc = (int)sd.attrs.size();
  RowUnpackArgs ua{};
  ua.recs = (const uint64_t*)recs;
  ua.n = n;
  ua.wrw = 3 + nc;
  ua.ncols = nc;
  bool ok = true;
  for (int c = 0; c < nc && ok; ++c) {
    ok = dev_ensure(&a->rr_col[c], (size_t)n * type_width(sd.attrs[c].type) + 16, a->stream, false);
    ua.col[c] = a->rr_col[c].p;
    ua.type[c] = sd.attrs[c].type;
  }
  ok = ok && dev_ensure(&a->rr_ts, (size_t)n * 8, a->stream, false) &&
       dev_ensure(&a->rr_stream, (size_t)n + 16, a->stream, false) &&
       dev_ensure(&a->rr_seq, (size_t)n * 8, a->stream, false);
  if (!ok) return fail(a, CEP_E_DEVICE, "out of device memory (received rows)");
  ua.ts = (int64_t*)a->rr_ts.p;
  ua.stream = (uint8_t*)a->rr_stream.p;
  ua.seq = (int64_t*)a->rr_seq.p;
  {
    LaunchTimer t(a, CEP_K_OTHER);
    launch_unpack_rows(ua, a->stream);
  }
  RowsArgs rows{};
  rows.cols.n = nc;
  for (int c = 0; c < nc; ++c) {
    rows.cols.p[c] = ua.col[c];
    rows.cols.t[c] = sd.attrs[c].type;
  }
  rows.ts = ua.ts;
  rows.stream = ua.stream;
  rows.input = layout;
  rows.row0 = 0;
  rows.n = n;
  rows.seq0 = 0;
  rows.seq = ua.seq;
  rows.prev_ts = INT64_MIN;
  a->last_ts = INT64_MIN;
  a->batches++;
  return send_device_rows(a, rows);
}

int cep_plan_partition_keys(const char* plan, const char* stream_id, char* buf, size_t len) {
  if (!plan || !stream_id || !buf || !len) return CEP_E_ARG;
  CompiledApp app;
  std::string m;
  const int rc = compile_app(plan, &app, &m);
  if (rc) return rc;
  const int in = app.input_index(stream_id);
  if (in < 0) return CEP_E_UNDEFINED_STREAM;
  // SiddhiExecutionPlanner.parse (utils/SiddhiExecutionPlanner.java:76-140,
  // retrievePartition :172-189): each query reading the stream names its
  // group-by attributes; queries that name different non-empty lists are
  // incompatible partitions.  Extension: the reference's planner rejects
  // `partition with` blocks; here a partitioned query names its partition
  // attribute of the stream.
  const auto& attrs = app.inputs[in].attrs;
  std::vector<int> keys;
  for (auto& q : app.queries) {
    std::vector<int> k;
    if (q.in_stream == in) {
      k = q.group_cols;
      if (k.empty() && q.part_col >= 0) k.push_back(q.part_col);
    } else if (q.nfa) {
      if (in < (int)q.key_col_s.size() && q.key_col_s[in] >= 0) k.push_back(q.key_col_s[in]);
    } else if (q.a_stream == in || q.b_stream == in) {
      const int c = q.a_stream == in ? q.key_col_a : q.key_col_b;
      if (c >= 0) k.push_back(c);
    }
    if (k.empty()) continue;
    if (!keys.empty() && keys != k) {
      std::snprintf(buf, len, "incompatible partitions on stream %s: [%s] vs [%s]", stream_id,
                    attrs[keys[0]].name.c_str(), attrs[k[0]].name.c_str());
      return CEP_E_PARSE;
    }
    keys = k;
  }
  std::string s;
  for (int c : keys) {
    if (!s.empty()) s += '\n';
    s += attrs[c].name;
  }
  std::snprintf(buf, len, "%s", s.c_str());
  return s.size() < len ? CEP_OK : CEP_E_CAPACITY;
}

int cep_partition_channels(cep_app* a, const cep_batch* b, const char* key_field, int nchan, int64_t seq0,
                           int32_t* chan_dev, int64_t* keys_dev) {
  if (!a || !b || nchan <= 0 || !chan_dev || !b->on_device || b->stream) return CEP_E_ARG;
  if (b->input < 0 || b->input >= (int)a->app.inputs.size()) return fail(a, CEP_E_UNDEFINED_STREAM, "undefined input handle");
  const StreamSchema& sd = a->app.inputs[b->input];
  RouteKeyArgs ra{};
  ra.n = b->n;
  ra.nchan = nchan;
  ra.seq0 = seq0;
  ra.keys = keys_dev;
  ra.chan = chan_dev;
  if (key_field && *key_field) {
    int c = -1;
    for (size_t i = 0; i < sd.attrs.size(); ++i)
      if (sd.attrs[i].name == key_field) c = (int)i;
    if (c >= b->ncols) return fail(a, CEP_E_ARG, "batch has fewer columns than the stream definition");
    if (c < 0) {
      // AddRouteOperator.java:84-91: a key the stream lacks sums no field -> key 0
      hipMemsetAsync(chan_dev, 0, (size_t)b->n * 4, a->stream);
      if (keys_dev) hipMemsetAsync(keys_dev, 0, (size_t)b->n * 8, a->stream);
      return hipGetLastError() == hipSuccess ? CEP_OK : fail(a, CEP_E_DEVICE, "memset failed");
    }
    ra.col = b->cols[c];
    ra.type = sd.attrs[c].type;
    if (ra.type == T_STRING) {
      // String.hashCode over UTF-16 code units of each dictionary entry
      std::vector<int32_t> h(a->dict.size());
      for (size_t i = 0; i < a->dict.size(); ++i) {
        const std::string& u = a->dict[i];
        uint32_t x = 0;
        for (size_t j = 0; j < u.size();) {
          uint32_t cp = (uint8_t)u[j];
          int extra = cp >= 0xf0 ? 3 : cp >= 0xe0 ? 2 : cp >= 0xc0 ? 1 : 0;
          cp = extra == 3 ? (cp & 7) : extra == 2 ? (cp & 15) : extra == 1 ? (cp & 31) : cp;
          for (int k = 1; k <= extra && j + k < u.size(); ++k) cp = (cp << 6) | ((uint8_t)u[j + k] & 63);
          j += 1 + extra;
          if (cp >= 0x10000) {   // surrogate pair
            cp -= 0x10000;
            x = x * 31u + (0xd800u + (cp >> 10));
            x = x * 31u + (0xdc00u + (cp & 0x3ff));
          } else {
            x = x * 31u + cp;
          }
        }
        h[i] = (int32_t)x;
      }
      if (!dev_ensure(&a->str_hash, std::max<size_t>(h.size(), 1) * 4, a->stream, false))
        return fail(a, CEP_E_DEVICE, "out of device memory");
      if (!h.empty()) hipMemcpyAsync(a->str_hash.p, h.data(), h.size() * 4, hipMemcpyHostToDevice, a->stream);
      hipStreamSynchronize(a->stream);
      ra.str_hash = (const int32_t*)a->str_hash.p;
      ra.nstr = (int32_t)h.size();
    }
  }
  launch_route_keys(ra, a->stream);
  return hipGetLastError() == hipSuccess ? CEP_OK : fail(a, CEP_E_DEVICE, "route key kernel failed");
}

int cep_generate(int64_t first, int64_t n, uint64_t seed, int64_t keys, int64_t rate, int64_t t0,
                 int single_stream, int32_t* key, int64_t* ts, uint8_t* stream, int32_t* id,
                 double* price, void* hip_stream) {
  if (n < 0 || keys <= 0 || rate <= 0) return CEP_E_ARG;
  launch_generate(first, n, seed, keys, rate, t0, single_stream, key, ts, stream, id, price,
                  (hipStream_t)hip_stream);
  return hipGetLastError() == hipSuccess ? CEP_OK : CEP_E_DEVICE;
}

}  // extern "C"
