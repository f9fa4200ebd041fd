/*
 * CPU ORACLE (C) — TEST INFRASTRUCTURE ONLY.
 *
 * Scalar, event-at-a-time restatement of Siddhi 4.2.40's processing for the
 * two hot-path shapes of BASELINE.json (configs 2 and 3/4), used
 *   - by tests/ as the checker at sizes the Python oracle cannot reach, and
 *   - by bench.py's cpu_baseline leg (kind "port": this is NOT the Java
 *     reference, which cannot run in this image — SURVEY.md F5).
 * Nothing in flink-siddhi_amd/ links or loads this file.
 *
 * Semantics followed (reference call site
 * AbstractSiddhiOperator.java:130 InputHandler.send(ts, row)):
 *   filter  `from S[f] select *`              — emit row iff f (A.2)
 *   pattern `[every] s1=A[f] -> s2=B[g] within W` under `partition with (k ..)`
 *     per key, in arrival order (A.3):
 *       on every B-stream event: walk pendings in creation order; drop a
 *       pending whose |ts - ts(s1)| > W; else if g: emit (s1, s2) and remove;
 *       then, on an A-stream event passing f (and `every` or not yet
 *       started): append a new pending.
 * Conditions are conjunctions of terms (column [% m]) OP constant, which
 * covers configs 2-5; the general expression language is checked by the
 * Python oracle (oracle/siddhi_oracle.py).
 */
#define _POSIX_C_SOURCE 199309L
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>

enum { OP_EQ = 0, OP_NE, OP_LT, OP_LE, OP_GT, OP_GE };
enum { COL_ID = 0, COL_PRICE = 1, COL_KEY = 2 };

typedef struct {
  int32_t col;     /* COL_ID (int32) or COL_PRICE (double) or COL_KEY (int32) */
  int32_t mod;     /* int columns: compare (v % mod) when mod != 0 (Java remainder) */
  int32_t op;
  double k;        /* constant (ints compare as long) */
} term_t;

typedef struct {
  int32_t nterms;
  term_t t[4];
} cond_t;

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

static int eval_cond(const cond_t* c, int32_t key, int32_t id, double price) {
  for (int i = 0; i < c->nterms; ++i) {
    const term_t* t = &c->t[i];
    int ok;
    if (t->col == COL_PRICE) {
      ok = cmp_d(price, t->op, t->k);
    } else {
      int32_t v = t->col == COL_ID ? id : key;
      if (t->mod) {
        if (t->mod == -1) v = 0;
        else v = v % t->mod;           /* C99 remainder == Java remainder */
      }
      ok = cmp_l((int64_t)v, t->op, (int64_t)t->k);
    }
    if (!ok) return 0;
  }
  return 1;
}

/* Config 2: returns the number of selected rows; their indices go to `sel`
 * (capacity n) in arrival order. */
int64_t oracle_filter(int64_t n, const int32_t* id, const double* price, const cond_t* f,
                      int64_t* sel) {
  int64_t m = 0;
  for (int64_t i = 0; i < n; ++i)
    if (eval_cond(f, 0, id[i], price[i])) sel[m++] = i;
  return m;
}

typedef struct {
  int64_t ts;
  int64_t idx;     /* arrival index of s1 */
  double price;    /* s1.price (captured attribute) */
} pend_t;

typedef struct {
  pend_t* v;
  int32_t n, cap;
  int32_t started;
} plist_t;

/* Config 3: keyed 2-state pattern.  keys in [0, nkeys) (nkeys = 1 and key
 * == NULL: unpartitioned).  stream[i]: 0 = A, 1 = B.  Matches are written in
 * Siddhi emission order as (s1 index, s2 index) pairs into out_a / out_b
 * (capacity out_cap); returns the match count (may exceed out_cap: only the
 * first out_cap pairs are stored).  `state` (optional, nkeys entries) keeps
 * pendings across calls; pass NULL for a one-shot run. */
typedef struct {
  plist_t* lists;
  int64_t nkeys;
} pstate_t;

pstate_t* oracle_pattern_state(int64_t nkeys) {
  pstate_t* s = (pstate_t*)calloc(1, sizeof(pstate_t));
  s->lists = (plist_t*)calloc((size_t)nkeys, sizeof(plist_t));
  s->nkeys = nkeys;
  return s;
}

void oracle_pattern_state_free(pstate_t* s) {
  if (!s) return;
  for (int64_t k = 0; k < s->nkeys; ++k) free(s->lists[k].v);
  free(s->lists);
  free(s);
}

/* Order-sensitive digest of one output row of the config-3 query
 * (`select s1.k, s1.price as p1, s2.price as p2, s2.ts as t`, completing
 * event ts and arrival number `seq`), `rank` = the row's position among its
 * key's rows.  The sum over rows is independent of the interleaving of
 * different keys and sensitive to the order inside each key (the parity
 * contract of SURVEY.md §8a a2).  Restated in torch by
 * flink_siddhi/workload.py:rows_digest. */
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

uint64_t oracle_row_digest(int32_t k, int64_t rank, double p1, double p2, int64_t t, int64_t seq) {
  uint64_t x = smix((uint64_t)(uint32_t)k | ((uint64_t)rank << 32));
  x = smix(x ^ dbits(p1));
  x = smix(x ^ dbits(p2));
  x = smix(x ^ (uint64_t)t);
  return smix(x ^ (uint64_t)seq);
}

/* Core of the pattern restatement.  Matches go to out_a / out_b (pairs) when
 * out_a != NULL, and/or into *digest (with per-key ranks kept in `rank`,
 * indexed by the state's key; gkey maps it back to the global key). */
static int64_t pattern_core(pstate_t* st, int64_t n, int64_t idx0, const int32_t* key,
                            const uint8_t* stream, const int32_t* id, const double* price,
                            const int64_t* ts, const cond_t* f, const cond_t* g, int every,
                            int64_t within, int64_t* out_a, int64_t* out_b, int64_t out_cap,
                            const int64_t* gidx, const int32_t* gkey, int64_t* rank,
                            uint64_t* digest) {
  int64_t m = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t k = key ? key[i] : 0;
    plist_t* L = &st->lists[k];
    const int64_t t = ts[i];
    const int64_t me = gidx ? gidx[i] : idx0 + i;
    if (stream[i] == 1) {
      const int gok = eval_cond(g, gkey ? gkey[i] : k, id[i], price[i]);
      int32_t w = 0;
      for (int32_t j = 0; j < L->n; ++j) {
        pend_t p = L->v[j];
        if (within >= 0) {
          int64_t d = t - p.ts;
          if (d < 0) d = -d;
          if (d > within) continue;            /* expired: dropped */
        }
        if (gok) {
          if (out_a && m < out_cap) {
            out_a[m] = p.idx;
            out_b[m] = me;
          }
          if (digest)
            *digest += oracle_row_digest(gkey ? gkey[i] : k, rank[k]++, p.price, price[i], t, me);
          ++m;
          continue;                            /* consumed */
        }
        L->v[w++] = p;
      }
      L->n = w;
    } else if ((every || !L->started) && eval_cond(f, gkey ? gkey[i] : k, id[i], price[i])) {
      L->started = 1;
      if (L->n == L->cap) {
        L->cap = L->cap ? 2 * L->cap : 4;
        L->v = (pend_t*)realloc(L->v, (size_t)L->cap * sizeof(pend_t));
      }
      L->v[L->n].ts = t;
      L->v[L->n].idx = me;
      L->v[L->n].price = price[i];
      L->n++;
    }
  }
  return m;
}

int64_t oracle_pattern(pstate_t* st, int64_t n, int64_t idx0, const int32_t* key,
                       const uint8_t* stream, const int32_t* id, const double* price,
                       const int64_t* ts, const cond_t* f, const cond_t* g, int every,
                       int64_t within, int64_t* out_a, int64_t* out_b, int64_t out_cap) {
  return pattern_core(st, n, idx0, key, stream, id, price, ts, f, g, every, within, out_a, out_b,
                      out_cap, NULL, NULL, NULL, NULL);
}

/* ---- synthetic stream (SURVEY.md §8d generator) ---------
 * r(i,j) = splitmix64(seed ^ (i * 0x9E3779B97F4A7C15) ^ j); key = r(i,0) mod K;
 * stream = r(i,1) >> 63; id = r(i,2) mod 50; price = (r(i,3) >> 11) 2^-53;
 * ts = t0 + i / rate.  Same stream as flink_siddhi/workload.py:generate. */
typedef struct {
  int64_t first, n, keys, rate, t0, lo, hi;
  uint64_t seed;
  int single;
  int32_t* key;
  int64_t* ts;
  uint8_t* stream;
  int32_t* id;
  double* price;
} gen_job_t;

static void* gen_worker(void* p) {
  gen_job_t* j = (gen_job_t*)p;
  for (int64_t r = j->lo; r < j->hi; ++r) {
    const uint64_t i = (uint64_t)(j->first + r);
    const uint64_t b = j->seed ^ (i * 0x9E3779B97F4A7C15ull);
    j->key[r] = (int32_t)(smix(b ^ 0) % (uint64_t)j->keys);
    j->stream[r] = j->single ? 0 : (uint8_t)(smix(b ^ 1) >> 63);
    j->id[r] = (int32_t)(smix(b ^ 2) % 50u);
    j->price[r] = (double)(smix(b ^ 3) >> 11) * 0x1.0p-53;
    j->ts[r] = j->t0 + (int64_t)(i / (uint64_t)j->rate);
  }
  return NULL;
}

void oracle_generate(int64_t first, int64_t n, uint64_t seed, int64_t keys, int64_t rate, int64_t t0,
                     int single, int32_t* key, int64_t* ts, uint8_t* stream, int32_t* id,
                     double* price, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  gen_job_t jobs[256];
  for (int t = 0; t < threads; ++t) {
    gen_job_t* j = &jobs[t];
    j->first = first; j->n = n; j->keys = keys; j->rate = rate; j->t0 = t0; j->seed = seed;
    j->single = single; j->key = key; j->ts = ts; j->stream = stream; j->id = id; j->price = price;
    j->lo = n * t / threads;
    j->hi = n * (t + 1) / threads;
    pthread_create(&th[t], NULL, gen_worker, j);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
}

/* ---- the pattern sharded by key over host threads -----------------------
 * Thread t owns keys k % T == t (keys are independent under `partition
 * with`), processes them in arrival order with its own state,
 * and sums the order-sensitive row digest.  The shard split is not timed;
 * *seconds = wall time of the parallel processing (the CPU baseline). */
typedef struct {
  int t, T;
  int64_t n, idx0, nkeys;
  const int32_t* key;
  const uint8_t* stream;
  const int32_t* id;
  const double* price;
  const int64_t* ts;
  const cond_t *f, *g;
  int every;
  int64_t within;
  /* shard */
  int64_t sn;
  int32_t *skey, *sgkey, *sid;
  uint8_t* sstream;
  double* sprice;
  int64_t *sts, *sidx;
  /* results */
  int64_t matches;
  uint64_t digest;
} shard_job_t;

static void* shard_split(void* p) {
  shard_job_t* j = (shard_job_t*)p;
  int64_t c = 0;
  for (int64_t i = 0; i < j->n; ++i) c += (j->key[i] % j->T) == j->t;
  j->sn = c;
  j->skey = (int32_t*)malloc((size_t)(c + 1) * 4);
  j->sgkey = (int32_t*)malloc((size_t)(c + 1) * 4);
  j->sid = (int32_t*)malloc((size_t)(c + 1) * 4);
  j->sstream = (uint8_t*)malloc((size_t)(c + 1));
  j->sprice = (double*)malloc((size_t)(c + 1) * 8);
  j->sts = (int64_t*)malloc((size_t)(c + 1) * 8);
  j->sidx = (int64_t*)malloc((size_t)(c + 1) * 8);
  int64_t o = 0;
  for (int64_t i = 0; i < j->n; ++i) {
    const int32_t k = j->key[i];
    if (k % j->T != j->t) continue;
    j->skey[o] = k / j->T;
    j->sgkey[o] = k;
    j->sid[o] = j->id[i];
    j->sstream[o] = j->stream[i];
    j->sprice[o] = j->price[i];
    j->sts[o] = j->ts[i];
    j->sidx[o] = j->idx0 + i;
    ++o;
  }
  return NULL;
}

static void* shard_run(void* p) {
  shard_job_t* j = (shard_job_t*)p;
  const int64_t lk = (j->nkeys + j->T - 1) / j->T;
  pstate_t* st = oracle_pattern_state(lk);
  int64_t* rank = (int64_t*)calloc((size_t)lk, 8);
  j->digest = 0;
  j->matches = pattern_core(st, j->sn, 0, j->skey, j->sstream, j->sid, j->sprice, j->sts, j->f, j->g,
                            j->every, j->within, NULL, NULL, 0, j->sidx, j->sgkey, rank, &j->digest);
  free(rank);
  oracle_pattern_state_free(st);
  return NULL;
}

int64_t oracle_pattern_mt(int64_t n, int64_t idx0, const int32_t* key, const uint8_t* stream,
                          const int32_t* id, const double* price, const int64_t* ts, int64_t nkeys,
                          const cond_t* f, const cond_t* g, int every, int64_t within, int threads,
                          uint64_t* digest, double* seconds) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  shard_job_t* jobs = (shard_job_t*)calloc((size_t)threads, sizeof(shard_job_t));
  for (int t = 0; t < threads; ++t) {
    shard_job_t* j = &jobs[t];
    j->t = t; j->T = threads; j->n = n; j->idx0 = idx0; j->nkeys = nkeys;
    j->key = key; j->stream = stream; j->id = id; j->price = price; j->ts = ts;
    j->f = f; j->g = g; j->every = every; j->within = within;
    pthread_create(&th[t], NULL, shard_split, j);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, shard_run, &jobs[t]);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &b);
  if (seconds) *seconds = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
  int64_t m = 0;
  uint64_t d = 0;
  for (int t = 0; t < threads; ++t) {
    shard_job_t* j = &jobs[t];
    m += j->matches;
    d += j->digest;
    free(j->skey); free(j->sgkey); free(j->sid); free(j->sstream); free(j->sprice); free(j->sts);
    free(j->sidx);
  }
  free(jobs);
  if (digest) *digest = d;
  return m;
}
