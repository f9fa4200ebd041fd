/*
 * CPU ORACLE (C) — TEST INFRASTRUCTURE ONLY.
 *
 * Scalar restatement of Siddhi 4.2.40's per-event processing for apps of
 * many keyed queries over one merged, multi-stream event sequence — the
 * BASELINE config-5 family: N-state sequences (`,`: strict contiguity, count
 * states `+ * ? <n:m>`, `[0]` / `[last]` captures, `within`) and patterns
 * (`->`), and `group by <key>` aggregations (sum / count / avg / min / max)
 * with `having` on one output attribute.  Used by tests/ and bench.py as the
 * checker at sizes the Python oracle cannot reach (and as the config-5 CPU
 * baseline, kind "port").  Nothing in flink-siddhi_amd/ links or loads it.
 *
 * It follows oracle/siddhi_oracle.py line for line where that restates
 * Siddhi, reference call site
 * AbstractSiddhiOperator.java:130 (InputHandler.send per event) and
 * :283-287 (one event fans out to every query of the app):
 *   - sequences  (_sequence_event / _seq_advance / _settle, siddhi_oracle.py
 *     :1128-1188): every partial expired by `within` (|ts - start| > W) is
 *     dropped; each survivor either stays in its count state, moves to a later
 *     state (skipping optional ones), or is discarded; a start event then
 *     opens a new partial; a partial whose state count is satisfied and whose
 *     later states are all optional emits;
 *   - patterns   (_pattern_event :1094-1125);
 *   - group-by aggregation (_SingleInstance.on_event :971-1006, _Agg
 *     :914-945): running values per key in arrival order, fp64 sums in
 *     arrival order, having evaluated after the update.
 * Conditions are conjunctions of cep_oracle.c terms over the event's own
 * columns; captures are the first or last event of a state.  Keys are the
 * partition / group-by column in [0, nkeys); queries are independent per key,
 * so the work shards by key over host threads.
 */
#define _POSIX_C_SOURCE 199309L
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

enum { OP_EQ = 0, OP_NE, OP_LT, OP_LE, OP_GT, OP_GE };
enum { COL_ID = 0, COL_PRICE = 1, COL_KEY = 2, COL_TS = 3 };
enum { MQ_SEQ = 0, MQ_PAT = 1, MQ_AGG = 2 };
enum { AGG_SUM = 0, AGG_COUNT = 1, AGG_AVG = 2, AGG_MIN = 3, AGG_MAX = 4 };
enum { MQ_MAXS = 6, MQ_MAXSEL = 8, MQ_MAXAGG = 4 };

typedef struct {
  int32_t col, mod, op;
  double k;
} mq_term_t;

typedef struct {
  int32_t nterms;
  mq_term_t t[4];
} mq_cond_t;   /* layout of cep_oracle.c cond_t */

typedef struct {
  int32_t kind;
  /* sequences / patterns */
  int32_t nstates, every;
  int64_t within;                       /* -1: none */
  int32_t st_stream[MQ_MAXS], st_min[MQ_MAXS], st_max[MQ_MAXS];   /* max -1: unbounded */
  mq_cond_t st_cond[MQ_MAXS];
  /* select items.  NFA: (state, idx 0 = first / -1 = last, column).
     AGG: sel_src -1 = the key column, >= 0 = aggregate i, -2 - c = column c
     of the current event */
  int32_t nsel;
  int32_t sel_state[MQ_MAXSEL], sel_idx[MQ_MAXSEL], sel_col[MQ_MAXSEL], sel_src[MQ_MAXSEL];
  /* aggregation */
  int32_t in_stream;
  mq_cond_t filter;
  int32_t nagg;
  int32_t agg_fn[MQ_MAXAGG], agg_col[MQ_MAXAGG];   /* column COL_ID / COL_PRICE, -1: count() */
  int32_t has_having, hav_item, hav_op;
  double hav_k;
} mq_query_t;

/* One emitted row (single-threaded run with explicit rows). */
typedef struct {
  int32_t query, key;
  int64_t seq, ts;
  uint64_t w[MQ_MAXSEL];
} mq_row_t;

static int cmp_d(double a, int op, double b) {
  switch (op) {
    case OP_EQ: return a == b;
    case OP_NE: return a != b;
    case OP_LT: return a < b;
    case OP_LE: return a <= b;
    case OP_GT: return a > b;
    default: return a >= b;
  }
}

static int cmp_l(int64_t a, int op, int64_t b) {
  switch (op) {
    case OP_EQ: return a == b;
    case OP_NE: return a != b;
    case OP_LT: return a < b;
    case OP_LE: return a <= b;
    case OP_GT: return a > b;
    default: return a >= b;
  }
}

static int eval(const mq_cond_t* c, int32_t key, int32_t id, double price) {
  for (int i = 0; i < c->nterms; ++i) {
    const mq_term_t* t = &c->t[i];
    int ok;
    if (t->col == COL_PRICE) {
      ok = cmp_d(price, t->op, t->k);
    } else {
      int32_t v = t->col == COL_ID ? id : key;
      if (t->mod) v = v % t->mod;   /* C99 remainder == Java remainder */
      ok = cmp_l((int64_t)v, t->op, (int64_t)t->k);
    }
    if (!ok) return 0;
  }
  return 1;
}

static inline uint64_t smix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static inline uint64_t dbits(double d) {
  uint64_t u;
  memcpy(&u, &d, 8);
  return u;
}

/* Order-sensitive digest of one output row: key, the row's rank among its
 * key's rows in that output stream, every select word (int sign-extended to
 * 64 bits, long as is, double as its bits), the row's ts and the completing
 * event's arrival number.  Restated in torch by flink_siddhi/workload.py
 * rows_digest_words. */
uint64_t mq_row_digest(int32_t key, int64_t rank, const uint64_t* w, int nw, int64_t ts, int64_t seq) {
  uint64_t x = smix((uint64_t)(uint32_t)key | ((uint64_t)rank << 32));
  for (int i = 0; i < nw; ++i) x = smix(x ^ w[i]);
  x = smix(x ^ (uint64_t)ts);
  return smix(x ^ (uint64_t)seq);
}

/* ---- events ------------------------------------------------------------- */
typedef struct {
  const int32_t* key;
  const uint8_t* stream;
  const int32_t* id;
  const double* price;
  const int64_t* ts;
  int64_t idx0;   /* arrival number of row 0 */
} mq_events_t;

static uint64_t col_word(int col, int32_t key, int32_t id, double price, int64_t ts) {
  switch (col) {
    case COL_ID: return (uint64_t)(int64_t)id;
    case COL_PRICE: return dbits(price);
    case COL_KEY: return (uint64_t)(int64_t)key;
    default: return (uint64_t)ts;
  }
}

/* ---- NFA partials ------------------------------------------------------- */
typedef struct {
  int32_t j, count;
  int64_t start_ts;
  uint64_t cap[MQ_MAXSEL];   /* select captures, filled as their state collects */
} partial_t;

typedef struct {
  partial_t* v;
  int32_t n, cap;
  int32_t started;
} plist_t;

static void plist_push(plist_t* L, const partial_t* p) {
  if (L->n == L->cap) {
    L->cap = L->cap ? 2 * L->cap : 2;
    L->v = (partial_t*)realloc(L->v, (size_t)L->cap * sizeof(partial_t));
  }
  L->v[L->n++] = *p;
}

/* The event joins state j of partial p (as its count-th event there). */
static void collect(const mq_query_t* q, partial_t* p, int j, int first, int32_t key, int32_t id,
                    double price, int64_t ts) {
  for (int i = 0; i < q->nsel; ++i) {
    if (q->sel_state[i] != j) continue;
    if (q->sel_idx[i] == 0 && !first) continue;
    p->cap[i] = col_word(q->sel_col[i], key, id, price, ts);
  }
}

/* Output sink: per (query) count + digest with per-(query, key) ranks, and
 * optional explicit rows. */
typedef struct {
  int64_t* count;       /* [nq] */
  uint64_t* digest;     /* [nq] */
  int64_t* rank;        /* [nq * lk] */
  int64_t lk;
  mq_row_t* rows;
  int64_t nrows, rows_cap;
} sink_t;

static void emit(sink_t* s, const mq_query_t* q, int qi, int64_t lkey, int32_t key, const uint64_t* w,
                 int64_t ts, int64_t seq) {
  const int64_t r = s->rank[(int64_t)qi * s->lk + lkey]++;
  s->count[qi]++;
  s->digest[qi] += mq_row_digest(key, r, w, q->nsel, ts, seq);
  if (s->rows) {
    if (s->nrows < s->rows_cap) {
      mq_row_t* o = &s->rows[s->nrows];
      o->query = qi;
      o->key = key;
      o->seq = seq;
      o->ts = ts;
      memcpy(o->w, w, sizeof(o->w));
    }
    s->nrows++;
  }
}

/* _settle: emit when the count is satisfied and every later state is
 * optional; returns 1 if the partial stays alive. */
static int settle(const mq_query_t* q, int qi, const partial_t* p, sink_t* s, int64_t lkey, int32_t key,
                  int64_t ts, int64_t seq) {
  const int n = q->nstates;
  const int j = p->j;
  int done = p->count >= q->st_min[j];
  for (int k = j + 1; k < n && done; ++k) done = q->st_min[k] == 0;
  if (!done) return 1;
  emit(s, q, qi, lkey, key, p->cap, ts, seq);
  return j == n - 1 && (q->st_max[j] == -1 || p->count < q->st_max[j]);
}

static void sequence_event(const mq_query_t* q, int qi, plist_t* L, sink_t* s, int64_t lkey, int32_t key,
                           int st, int32_t id, double price, int64_t ts, int64_t seq) {
  const int n = q->nstates;
  int32_t w = 0;
  partial_t np;
  /* survivors are compacted in place (each partial yields at most one) */
  for (int32_t i = 0; i < L->n; ++i) {
    partial_t p = L->v[i];
    if (q->within >= 0) {
      int64_t d = ts - p.start_ts;
      if (d < 0) d = -d;
      if (d > q->within) continue;
    }
    const int j = p.j;
    int adv = 0;
    /* option 1: stay in the current count state */
    if (q->st_stream[j] == st && (q->st_max[j] == -1 || p.count < q->st_max[j]) &&
        eval(&q->st_cond[j], key, id, price)) {
      np = p;
      collect(q, &np, j, 0, key, id, price, ts);
      np.count = p.count + 1;
      if (settle(q, qi, &np, s, lkey, key, ts, seq)) L->v[w++] = np;
      adv = 1;
    }
    /* option 2: a later state (optional ones skipped) */
    if (!adv && p.count >= q->st_min[j]) {
      for (int k = j + 1; k < n; ++k) {
        if (q->st_stream[k] == st && eval(&q->st_cond[k], key, id, price)) {
          np = p;
          np.j = k;
          np.count = 1;
          collect(q, &np, k, 1, key, id, price, ts);
          if (settle(q, qi, &np, s, lkey, key, ts, seq)) L->v[w++] = np;
          break;
        }
        if (q->st_min[k] > 0) break;
      }
    }
    /* not advanced: strict contiguity discards it */
  }
  L->n = w;
  if (q->st_stream[0] == st && (q->every || !L->started) && eval(&q->st_cond[0], key, id, price)) {
    L->started = 1;
    memset(&np, 0, sizeof(np));
    np.j = 0;
    np.count = 1;
    np.start_ts = ts;
    collect(q, &np, 0, 1, key, id, price, ts);
    if (settle(q, qi, &np, s, lkey, key, ts, seq)) plist_push(L, &np);
  }
}

static void pattern_event(const mq_query_t* q, int qi, plist_t* L, sink_t* s, int64_t lkey, int32_t key,
                          int st, int32_t id, double price, int64_t ts, int64_t seq) {
  const int n = q->nstates;
  const int32_t n0 = L->n;
  /* keep (in order) then fresh (in order): advanced partials go behind the
     untouched ones, as siddhi_oracle.py _pattern_event keeps `keep + fresh` */
  partial_t* fresh = NULL;
  int32_t nf = 0, w = 0;
  if (n0) fresh = (partial_t*)malloc((size_t)(n0 + 1) * sizeof(partial_t));
  for (int32_t i = 0; i < n0; ++i) {
    partial_t p = L->v[i];
    const int j = p.j;
    if (q->st_stream[j] != st) {
      L->v[w++] = p;
      continue;
    }
    if (q->within >= 0) {
      int64_t d = ts - p.start_ts;
      if (d < 0) d = -d;
      if (d > q->within) continue;
    }
    if (!eval(&q->st_cond[j], key, id, price)) {
      L->v[w++] = p;
      continue;
    }
    collect(q, &p, j, 1, key, id, price, ts);
    if (j + 1 == n) {
      emit(s, q, qi, lkey, key, p.cap, ts, seq);
    } else {
      p.j = j + 1;
      fresh[nf++] = p;
    }
  }
  L->n = w;
  for (int32_t i = 0; i < nf; ++i) plist_push(L, &fresh[i]);
  free(fresh);
  if (q->st_stream[0] == st && (q->every || !L->started) && eval(&q->st_cond[0], key, id, price)) {
    L->started = 1;
    partial_t np;
    memset(&np, 0, sizeof(np));
    np.start_ts = ts;
    collect(q, &np, 0, 1, key, id, price, ts);
    if (n == 1) {
      emit(s, q, qi, lkey, key, np.cap, ts, seq);
    } else {
      np.j = 1;
      plist_push(L, &np);
    }
  }
}

/* ---- aggregation -------------------------------------------------------- */
typedef struct {
  double s;       /* sum / avg accumulator (double args) */
  int64_t l;      /* sum (int / long args) */
  int64_t n;      /* values seen */
  double md;      /* min / max (double) */
  int64_t ml;     /* min / max (int) */
} agg_t;

static void agg_event(const mq_query_t* q, int qi, agg_t* A, sink_t* s, int64_t lkey, int32_t key, int32_t id,
                      double price, int64_t ts, int64_t seq) {
  if (!eval(&q->filter, key, id, price)) return;
  uint64_t val[MQ_MAXAGG];
  for (int a = 0; a < q->nagg; ++a) {
    agg_t* g = &A[a];
    const int dbl = q->agg_col[a] == COL_PRICE;
    const double dv = price;
    const int64_t lv = (int64_t)id;
    switch (q->agg_fn[a]) {
      case AGG_COUNT:
        g->n++;
        val[a] = (uint64_t)g->n;
        break;
      case AGG_SUM:
        g->n++;
        if (dbl) {
          g->s += dv;
          val[a] = dbits(g->s);
        } else {
          g->l = (int64_t)((uint64_t)g->l + (uint64_t)lv);
          val[a] = (uint64_t)g->l;
        }
        break;
      case AGG_AVG:
        g->n++;
        g->s += dbl ? dv : (double)lv;
        val[a] = dbits(g->s / (double)g->n);
        break;
      default: {
        const int mx = q->agg_fn[a] == AGG_MAX;
        if (dbl) {
          if (g->n == 0 || (mx ? dv > g->md : dv < g->md)) g->md = dv;
          val[a] = dbits(g->md);
        } else {
          if (g->n == 0 || (mx ? lv > g->ml : lv < g->ml)) g->ml = lv;
          val[a] = (uint64_t)g->ml;
        }
        g->n++;
      }
    }
  }
  uint64_t w[MQ_MAXSEL];
  for (int i = 0; i < q->nsel; ++i) {
    const int src = q->sel_src[i];
    if (src == -1) w[i] = (uint64_t)(int64_t)key;
    else if (src >= 0) w[i] = val[src];
    else w[i] = col_word(-2 - src, key, id, price, ts);
  }
  if (q->has_having) {
    /* having `<item> op const`: the item's Siddhi type decides the compare */
    const int it = q->hav_item;
    const int src = q->sel_src[it];
    int isd;
    if (src >= 0) {
      const int fn = q->agg_fn[src];
      isd = fn == AGG_AVG || ((fn == AGG_SUM || fn == AGG_MIN || fn == AGG_MAX) && q->agg_col[src] == COL_PRICE);
    } else {
      isd = src < -1 && (-2 - src) == COL_PRICE;
    }
    int ok;
    if (isd) {
      double d;
      memcpy(&d, &w[it], 8);
      ok = cmp_d(d, q->hav_op, q->hav_k);
    } else {
      ok = cmp_d((double)(int64_t)w[it], q->hav_op, q->hav_k);
    }
    if (!ok) return;
  }
  emit(s, q, qi, lkey, key, w, ts, seq);
}

/* ---- one shard ---------------------------------------------------------- */
typedef struct {
  const mq_query_t* q;
  int nq;
  const mq_events_t* ev;
  int64_t n, nkeys;
  int t, T;
  sink_t sink;
  plist_t** pl;   /* [nq] -> [lk] (NFA queries) */
  agg_t** ag;     /* [nq] -> [lk * nagg] (aggregations) */
} shard_t;

static void shard_init(shard_t* j) {
  const int64_t lk = (j->nkeys + j->T - 1) / j->T;
  j->sink.lk = lk;
  j->sink.count = (int64_t*)calloc((size_t)j->nq, 8);
  j->sink.digest = (uint64_t*)calloc((size_t)j->nq, 8);
  j->sink.rank = (int64_t*)calloc((size_t)j->nq * (size_t)lk, 8);
  j->pl = (plist_t**)calloc((size_t)j->nq, sizeof(plist_t*));
  j->ag = (agg_t**)calloc((size_t)j->nq, sizeof(agg_t*));
  for (int qi = 0; qi < j->nq; ++qi) {
    if (j->q[qi].kind == MQ_AGG)
      j->ag[qi] = (agg_t*)calloc((size_t)lk * (size_t)(j->q[qi].nagg ? j->q[qi].nagg : 1), sizeof(agg_t));
    else
      j->pl[qi] = (plist_t*)calloc((size_t)lk, sizeof(plist_t));
  }
}

static void shard_free(shard_t* j) {
  const int64_t lk = j->sink.lk;
  for (int qi = 0; qi < j->nq; ++qi) {
    if (j->pl[qi]) {
      for (int64_t k = 0; k < lk; ++k) free(j->pl[qi][k].v);
      free(j->pl[qi]);
    }
    free(j->ag[qi]);
  }
  free(j->pl);
  free(j->ag);
  free(j->sink.rank);
}

static void* shard_run(void* arg) {
  shard_t* j = (shard_t*)arg;
  const mq_events_t* e = j->ev;
  for (int64_t i = 0; i < j->n; ++i) {
    const int32_t key = e->key[i];
    if (key < 0 || key >= j->nkeys || key % j->T != j->t) continue;
    const int64_t lkey = key / j->T;
    const int st = e->stream[i];
    const int32_t id = e->id[i];
    const double price = e->price[i];
    const int64_t ts = e->ts[i];
    const int64_t seq = e->idx0 + i;
    /* AbstractSiddhiOperator.java:283-287: the event goes to every query */
    for (int qi = 0; qi < j->nq; ++qi) {
      const mq_query_t* q = &j->q[qi];
      if (q->kind == MQ_AGG) {
        if (q->in_stream == st)
          agg_event(q, qi, &j->ag[qi][lkey * (q->nagg ? q->nagg : 1)], &j->sink, lkey, key, id, price, ts, seq);
        continue;
      }
      int reads = 0;
      for (int k = 0; k < q->nstates; ++k) reads |= q->st_stream[k] == st;
      if (!reads) continue;
      if (q->kind == MQ_SEQ)
        sequence_event(q, qi, &j->pl[qi][lkey], &j->sink, lkey, key, st, id, price, ts, seq);
      else
        pattern_event(q, qi, &j->pl[qi][lkey], &j->sink, lkey, key, st, id, price, ts, seq);
    }
  }
  return NULL;
}

/* Single-threaded run with explicit rows (small cross-checks): rows in
 * emission order (event by event, queries in plan order).  Returns the row
 * count (rows beyond rows_cap are counted, not stored). */
int64_t mq_run_rows(const mq_query_t* q, int nq, int64_t n, int64_t idx0, const int32_t* key, const uint8_t* stream,
                    const int32_t* id, const double* price, const int64_t* ts, int64_t nkeys, mq_row_t* rows,
                    int64_t rows_cap) {
  mq_events_t ev = {key, stream, id, price, ts, idx0};
  shard_t j;
  memset(&j, 0, sizeof(j));
  j.q = q; j.nq = nq; j.ev = &ev; j.n = n; j.nkeys = nkeys; j.t = 0; j.T = 1;
  shard_init(&j);
  j.sink.rows = rows;
  j.sink.rows_cap = rows_cap;
  shard_run(&j);
  const int64_t m = j.sink.nrows;
  shard_free(&j);
  free(j.sink.count);
  free(j.sink.digest);
  return m;
}

/* Sharded by key (k % threads) over host threads: per query the row count
 * and the order-sensitive digest; *seconds = wall time of the processing. */
void mq_run_mt(const mq_query_t* q, int nq, int64_t n, int64_t idx0, const int32_t* key, const uint8_t* stream,
               const int32_t* id, const double* price, const int64_t* ts, int64_t nkeys, int threads,
               int64_t* count, uint64_t* digest, double* seconds) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  mq_events_t ev = {key, stream, id, price, ts, idx0};
  shard_t* jobs = (shard_t*)calloc((size_t)threads, sizeof(shard_t));
  pthread_t th[256];
  for (int t = 0; t < threads; ++t) {
    shard_t* j = &jobs[t];
    j->q = q; j->nq = nq; j->ev = &ev; j->n = n; j->nkeys = nkeys; j->t = t; j->T = threads;
    shard_init(j);
  }
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, shard_run, &jobs[t]);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &b);
  if (seconds) *seconds = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
  for (int qi = 0; qi < nq; ++qi) {
    count[qi] = 0;
    digest[qi] = 0;
  }
  for (int t = 0; t < threads; ++t) {
    shard_t* j = &jobs[t];
    for (int qi = 0; qi < nq; ++qi) {
      count[qi] += j->sink.count[qi];
      digest[qi] += j->sink.digest[qi];
    }
    shard_free(j);
    free(j->sink.count);
    free(j->sink.digest);
  }
  free(jobs);
}
