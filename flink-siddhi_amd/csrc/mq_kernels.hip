// gfx950 kernels of multi-query groups: the keyed queries of one app that
// share a partition / group-by key, run together.  This is the Siddhi work
// behind AbstractSiddhiOperator.java:130 when one app holds many queries —
// every event fans out to every query (AbstractSiddhiOperator.java:283-287) —
// as in BASELINE config 5: 32 `every s1=A[f], s2=B[g]+, s3=C[h] within W`
// sequences under `partition with (k ...)` and 32 `group by k having ...`
// aggregations over one merged stream.  Semantics: SURVEY.md App. A.5 / A.6
// as restated by oracle/siddhi_oracle.py (_sequence_event, _SingleInstance)
// and oracle/mq_oracle.c.
//
//   k_mqpart  one 1024-lane workgroup per 4096-row tile: key, ts, stream and
//             every column a condition or capture reads loaded once per row;
//             every distinct condition of the row's stream (deduplicated over
//             the group's queries) evaluated once into a bit mask; LDS
//             histogram over the key buckets + LDS scan; records
//             [ts | row | stream, mask | key, carried...] scattered into the
//             tile's bucket-sorted region; bucket-major tile offsets.
//   k_mqwalk  one 1024-lane workgroup per key bucket: gathers the bucket's
//             records in windows of <= 4096 (LDS), counting sort by key +
//             arrival sort per key run, then every query over every key of
//             the window with lane = key and wave = query: a wave's control
//             flow, descriptors and output stream are uniform, a key's state
//             for one query is one lane's registers.  Count pass, one output
//             reservation per (window, query), emit pass whose rows of one
//             wave step are contiguous (coalesced stores), state commit.
//
// Sequences admitted here have at most one live partial per (query, key):
// the start state is a single event on a stream no later state reads, so an
// event either advances the partial or starts a new one, never both
// (engine.cpp checks the shape).
#include <hip/hip_runtime.h>

#include "dev_common.h"
#include "kernels.h"
#include "vm.h"

namespace cep {

namespace {

__device__ __forceinline__ uint32_t mq_row(uint64_t w0) { return (uint32_t)(w0 >> 32) & 0x1ffffffu; }
__device__ __forceinline__ int mq_stream(uint64_t w0) { return (int)(w0 >> 57) & 7; }
__device__ __forceinline__ uint32_t mq_key(uint64_t w1) { return (uint32_t)(w1 >> 48); }

}  // namespace

// ============================================================== k_mqpart ==
template <int NP>   // prefetched columns
__global__ __launch_bounds__(kMqPartThreads, 1) void k_mqpart(MqPartArgs a) {
  constexpr int E = kMqTile / kMqPartThreads, NT = kMqPartThreads;
  static_assert(NT * E == kMqTile, "tile geometry");
  __shared__ uint32_t scratch[NT / 64 + 1];
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];   // P + 1 (dynamic)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t tile = xcd_tile(blockIdx.x, a.ntiles);
  const int lg = a.buckets_log2;
  const int P = 1 << lg;
  const int RW = 2 + a.nphys;
  for (int i = tid; i <= P; i += NT) hist[i] = 0;
  const int64_t ts_base = a.rows.ts[a.rows.row0];
  if (tile == 0 && tid == 0) {
    a.chunk_base[0] = ts_base;
    a.chunk_base[1] = row_seq(a.rows, a.rows.row0);
  }
  // lane-interleaved rows: lane l of wave w owns chunk rows w*64*E + 64*e + l
  const int64_t r0 = tile * kMqTile + (int64_t)wave * 64 * E + lane;
  const int64_t row0 = a.rows.row0 + r0;
  uint32_t valid = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) valid |= (r0 + 64 * e < a.rows.n ? 1u : 0u) << e;
  uint64_t tsv[E], pv[NP][E], mask[E];
  uint32_t sb[E];
  uint32_t keep = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    tsv[e] = 0;
    sb[e] = 0;
    mask[e] = 1ull << kMqTrueBit;
  }
  if (valid) {
    cf_load_cols<E, NP>(a.rows, a.pref, a.ts_slot, row0, valid, tsv, sb, pv);
    if (a.check_order) {
      // event-time order (`within` relies on it): row r - 1 is held by the
      // previous lane (same e), lane 63 (e - 1), or loaded
      const int64_t before = row0 > 0 ? a.rows.ts[row0 - 1] : a.rows.prev_ts;
      bool bad = false;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const uint64_t up = __shfl_up(tsv[e], 1, 64);
        const uint64_t last = e > 0 ? __shfl(tsv[e > 0 ? e - 1 : 0], 63, 64) : 0ull;
        const int64_t prev = lane > 0 ? (int64_t)up : (e > 0 ? (int64_t)last : before);
        if ((valid >> e) & 1u) bad |= (int64_t)tsv[e] < prev;
      }
      if (bad) set_err(a.err, ERR_ORDER);
    }
    // every distinct condition of each stream, once per row (uniform loops)
    for (int s = 0; s < 8; ++s) {
      if (!((a.stream_mask >> s) & 1u)) continue;
      uint32_t is_s = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) is_s |= (((valid >> e) & 1u) && sb[e] == (uint32_t)s ? 1u : 0u) << e;
      keep |= is_s;
      const int nc = a.ncond[s];
      if (!__ballot(is_s != 0) || nc == 0) continue;
      const MqCond* cs = a.conds + s * kMqMaxCond;
      for (int c = 0; c < nc; ++c) {
        const uint32_t bits = eval_terms_regs<E, NP>(cs[c].tl, cs[c].slot, a.rows.cols, pv) & is_s;
#pragma unroll
        for (int e = 0; e < E; ++e) mask[e] |= (uint64_t)((bits >> e) & 1u) << c;
      }
    }
  }
  lds_barrier();   // hist zeroed
  // bits 0-12 rank in tile, 13-25 bucket
  uint32_t packed[E], lkey[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    packed[e] = 0xffffffffu;
    lkey[e] = 0;
    if (!((keep >> e) & 1u)) continue;
    const int64_t kfield = shard_key((int64_t)pv[0][e], a.key_stride, a.key_offset);   // key: slot 0
    if (kfield < 0 || kfield >= a.key_capacity) {
      set_err(a.err, ERR_KEY_RANGE);
      continue;
    }
    const uint32_t bucket = (uint32_t)(kfield & (P - 1));
    lkey[e] = (uint32_t)(kfield >> lg);
    const uint32_t rank = atomicAdd(&hist[bucket], 1u);
    packed[e] = (bucket << 13) | rank;
  }
  lds_barrier();
  {
    constexpr int MAXPER = kMqMaxBuckets / NT;
    const int per = (P + NT - 1) / NT;
    uint32_t c[MAXPER];
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < MAXPER; ++i) {
      const int idx = tid * per + i;
      c[i] = (i < per && idx < P) ? hist[idx] : 0u;
      sum += c[i];
    }
    uint32_t total;
    uint32_t off = bscan<NT>(sum, scratch, &total);
#pragma unroll
    for (int i = 0; i < MAXPER; ++i) {
      const int idx = tid * per + i;
      if (i < per && idx < P) {
        hist[idx] = off;
        off += c[i];
      }
    }
    if (tid == 0) hist[P] = total;
  }
  lds_barrier();
  uint64_t* trecs = a.recs + tile * (int64_t)kMqTile * RW;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if (packed[e] == 0xffffffffu) continue;
    const uint32_t b = packed[e] >> 13;
    const uint32_t slot = hist[b] + (packed[e] & 0x1fffu);
    const int64_t dts = (int64_t)tsv[e] - ts_base;
    if (dts < 0 || dts > 0xffffffffll) set_err(a.err, ERR_ORDER);
    uint64_t* g = trecs + (int64_t)slot * RW;
    g[0] = (uint64_t)(uint32_t)dts | ((uint64_t)(uint32_t)(r0 + 64 * e) << 32) | ((uint64_t)sb[e] << 57);
    g[1] = mask[e] | ((uint64_t)lkey[e] << 48);
#pragma unroll
    for (int w = 0; w < kMqMaxPhys; ++w)
      if (w < a.nphys) g[2 + w] = pick<E, NP>(pv, a.phys_slot[w], e);
  }
  for (int i = tid; i <= P; i += NT) a.tile_off[(int64_t)i * a.ntiles + tile] = (uint16_t)hist[i];
}

void launch_mq_partition(const MqPartArgs& a, hipStream_t s) {
  const int P = 1 << a.buckets_log2;
  const size_t dyn = ((size_t)(P + 1) * 4 + 15) & ~(size_t)15;
  const dim3 g((unsigned)a.ntiles), b(kMqPartThreads);
  switch (a.pref.n) {
    case 1: hipLaunchKernelGGL(k_mqpart<1>, g, b, dyn, s, a); break;
    case 2: hipLaunchKernelGGL(k_mqpart<2>, g, b, dyn, s, a); break;
    case 3: hipLaunchKernelGGL(k_mqpart<3>, g, b, dyn, s, a); break;
    default: hipLaunchKernelGGL(k_mqpart<4>, g, b, dyn, s, a); break;
  }
}

// ============================================================== k_mqwalk ==
namespace {

constexpr int mq_window(int nc) { return nc <= 1 ? kMqWindow : (nc == 2 ? 3072 : 2048); }

// A window's records in LDS (structure of arrays).
template <int NC>
struct MqLds {
  static constexpr int W = mq_window(NC);
  uint64_t w0[W], w1[W];
  uint64_t car[NC > 0 ? W * NC : 1];
  uint16_t sorted[W];                    // window slots grouped by key, arrival order
  uint32_t kstart[kMqMaxKpb + 1];
  uint32_t kcur[kMqMaxKpb];
  uint32_t bmax[kMqMaxKpb / 64];         // longest key run per 64-key block
  uint32_t qoff[kMqMaxQ * (kMqMaxKpb / 64)];   // per (query, block): rows, then first row
  unsigned long long qbase[kMqMaxQ];
  uint32_t seg[kMqMaxTiles + 1];         // exclusive prefix of the bucket's tile segments
  uint16_t lo[kMqMaxTiles];              // segment start inside each tile
  uint32_t scratch[kMqWalkThreads / 64 + 1];
  int32_t wt1;                           // window end tile (-1: a split tile)
  uint32_t nwin;                         // records of a split tile's row range
};

// Per-window view one lane needs to read its records.
template <int NC>
struct MqCtx {
  const MqLds<NC>* L;
  const MqWalkArgs* a;
  int64_t ts_base, seq_base;
  int64_t keyv;       // the lane's partition key value
  uint32_t r0, len;   // the lane's key run in `sorted`
};

// Logical carried word `src` of window record r (MQ_SRC_*: key / event ts).
template <int NC>
__device__ __forceinline__ uint64_t mq_src(const MqCtx<NC>& c, int src, int r, int64_t ts) {
  if (src == MQ_SRC_KEY) return (uint64_t)c.keyv;
  if (src == MQ_SRC_TS) return (uint64_t)ts;
  const int w = c.a->lmap[src];
  if (w < 0) return (uint64_t)ts;   // the column is the event-ts buffer
  if constexpr (NC > 0) return c.L->car[r * NC + (NC > 1 ? w : 0)];   // w < NC (host-checked)
  return 0;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// One sequence query over the 64 keys of a block (lane = key): restates
// oracle/mq_oracle.c sequence_event for the one-partial shape.  kEmit =
// false: returns the rows the wave would emit; true: stores them from `pos`
// and commits the state.
template <bool kEmit, int NC>
__device__ uint32_t mq_seq(const MqCtx<NC>& c, const MqQuery& Q, uint64_t* S, int64_t ks, uint32_t maxlen,
                           unsigned long long pos) {
  const MqLds<NC>& L = *c.L;
  const int N = Q.nstates;
  uint64_t hdr = 0, sts = 0, cap[kMqMaxCaps];
#pragma unroll
  for (int i = 0; i < kMqMaxCaps; ++i) cap[i] = 0;
  if (c.len) {
    hdr = S[0];
    if (hdr & 1u) {
      sts = S[ks];
#pragma unroll
      for (int i = 0; i < kMqMaxCaps; ++i)
        if (i < Q.ncap) cap[i] = S[(int64_t)(2 + i) * ks];
    }
  }
  bool live = (hdr & 1u) != 0, started = (hdr & 2u) != 0;
  int j = (int)((hdr >> 8) & 0xffu);
  uint32_t cnt = (uint32_t)(hdr >> 16);
  uint32_t rows = 0;
  auto stream_of = [&](int s) { return (int)((Q.st_stream >> (3 * s)) & 7u); };
  auto min_of = [&](int s) { return (uint32_t)((Q.st_min >> (8 * s)) & 0xffu); };
  auto max_of = [&](int s) { return (uint32_t)((Q.st_max >> (8 * s)) & 0xffu); };
  for (uint32_t i = 0; i < maxlen; ++i) {
    bool em = false;
    int r = 0;
    int64_t ts = 0;
    if (i < c.len) {
      r = L.sorted[c.r0 + i];
      const uint64_t w0 = L.w0[r], w1 = L.w1[r];
      const int st = mq_stream(w0);
      if ((Q.stream_mask >> st) & 1u) {
        ts = c.ts_base + (int64_t)(uint32_t)w0;
        auto cond = [&](int s) { return ((w1 >> ((Q.st_bit >> (6 * s)) & 63u)) & 1ull) != 0; };
        auto collect = [&](int s, bool first) {
#pragma unroll
          for (int x = 0; x < kMqMaxCaps; ++x)
            if (x < Q.ncap && Q.cap_state[x] == s && (Q.cap_last[x] || first)) cap[x] = mq_src(c, Q.cap_src[x], r, ts);
        };
        auto settle = [&]() {
          if (cnt >= min_of(j) && ((Q.tail_opt >> j) & 1u)) {
            em = true;
            live = j == N - 1 && (max_of(j) == 0xffu || cnt < max_of(j));
          }
        };
        if (live && Q.within >= 0) {
          const int64_t d = ts - (int64_t)sts;
          if ((d < 0 ? -d : d) > Q.within) live = false;   // expired: dropped
        }
        if (live) {
          bool adv = false;
          if (stream_of(j) == st && (max_of(j) == 0xffu || cnt < max_of(j)) && cond(j)) {
            cnt += 1;   // stay in the count state
            collect(j, false);
            adv = true;
            settle();
          } else if (cnt >= min_of(j)) {
            bool stop = false;   // move on, skipping optional states
            for (int j2 = 1; j2 < kMaxStates; ++j2) {
              if (j2 >= N) break;
              if (j2 <= j || stop) continue;
              if (stream_of(j2) == st && cond(j2)) {
                j = j2;
                cnt = 1;
                collect(j2, true);
                adv = true;
                stop = true;
                settle();
              } else if (min_of(j2) > 0) {
                stop = true;
              }
            }
          }
          if (!adv) live = false;   // strict contiguity: discarded
        }
        if (stream_of(0) == st && (Q.every || !started) && cond(0)) {
          started = true;
          live = true;
          j = 0;
          cnt = 1;
          sts = (uint64_t)ts;
#pragma unroll
          for (int x = 0; x < kMqMaxCaps; ++x) cap[x] = 0;
          collect(0, true);
          settle();
        }
      }
    }
    const uint64_t m = __ballot(em);
    if (kEmit && m) {
      if (em) {
        const unsigned long long p = pos + (unsigned long long)__popcll(m & lanemask_lt());
        if ((int64_t)p < Q.out_cap) {
          for (int x = 0; x < Q.nsel; ++x) {
            const int src = Q.sel_src[x];
            uint64_t v = (uint64_t)c.keyv;
#pragma unroll
            for (int y = 0; y < kMqMaxCaps; ++y)
              if (src == SRC_CAP + y) v = cap[y];
            store_col(Q.out_col[x], Q.sel_type[x], (int64_t)p, v);
          }
          const uint32_t row = mq_row(L.w0[r]);
          Q.out_ts[p] = ts;
          Q.out_seq[p] = c.a->in_seq ? c.a->in_seq[row] : c.seq_base + row;
        } else {
          set_err(c.a->err, ERR_OUT_CAP);
        }
      }
      pos += (unsigned long long)__popcll(m);
    }
    rows += (uint32_t)__popcll(m);
  }
  if (kEmit && c.len) {
    S[0] = (live ? 1ull : 0ull) | (started ? 2ull : 0ull) | ((uint64_t)(uint32_t)j << 8) | ((uint64_t)cnt << 16);
    if (live) {
      S[ks] = sts;
#pragma unroll
      for (int i = 0; i < kMqMaxCaps; ++i)
        if (i < Q.ncap) S[(int64_t)(2 + i) * ks] = cap[i];
    }
  }
  return rows;
}

__device__ __forceinline__ double mq_as_double(uint64_t v, int t) {
  switch (t) {
    case T_INT: return (double)(int32_t)v;
    case T_LONG: return (double)(int64_t)v;
    case T_FLOAT: return (double)as_f32(v);
    default: return as_f64(v);
  }
}

__device__ __forceinline__ bool mq_less(uint64_t a, uint64_t b, int t) {
  switch (t) {
    case T_LONG: return (int64_t)a < (int64_t)b;
    case T_FLOAT: return as_f32(a) < as_f32(b);
    case T_DOUBLE: return as_f64(a) < as_f64(b);
    default: return (int32_t)a < (int32_t)b;
  }
}

// One group-by aggregation over the 64 keys of a block (lane = group):
// running values in arrival order (oracle/mq_oracle.c agg_event; sum over
// int / long wraps in 64 bits, sum / avg over float / double accumulate in
// double, min / max compare in the argument type), having on one output item.
template <bool kEmit, int NC>
__device__ uint32_t mq_agg(const MqCtx<NC>& c, const MqQuery& Q, uint64_t* S, int64_t ks, uint32_t maxlen,
                           unsigned long long pos) {
  const MqLds<NC>& L = *c.L;
  uint64_t cnt = 0, acc[kMqMaxAggs];
#pragma unroll
  for (int i = 0; i < kMqMaxAggs; ++i) acc[i] = 0;
  if (c.len) {
    cnt = S[0];
#pragma unroll
    for (int i = 0; i < kMqMaxAggs; ++i)
      if (i < Q.nagg) acc[i] = S[(int64_t)(1 + i) * ks];
  }
  auto aggval = [&](int i) -> uint64_t {
    uint64_t x = 0;
#pragma unroll
    for (int y = 0; y < kMqMaxAggs; ++y)
      if (y == i) x = acc[y];
    const int fn = Q.agg_fn[i];
    if (fn == AGG_COUNT) return cnt;
    if (fn == AGG_AVG) return from_f64(as_f64(x) / (double)(int64_t)cnt);
    return x;
  };
  uint32_t rows = 0;
  for (uint32_t i = 0; i < maxlen; ++i) {
    bool em = false;
    int r = 0;
    int64_t ts = 0;
    if (i < c.len) {
      r = L.sorted[c.r0 + i];
      const uint64_t w0 = L.w0[r], w1 = L.w1[r];
      if (mq_stream(w0) == Q.in_stream && ((w1 >> Q.filter_bit) & 1ull)) {
        ts = c.ts_base + (int64_t)(uint32_t)w0;
        const bool first = cnt == 0;
        cnt += 1;
#pragma unroll
        for (int y = 0; y < kMqMaxAggs; ++y) {
          if (y >= Q.nagg) break;
          const int fn = Q.agg_fn[y];
          if (fn == AGG_COUNT) continue;
          const int at = Q.agg_arg_type[y];
          const uint64_t v = mq_src(c, Q.agg_src[y], r, ts);
          if (fn == AGG_SUM) {
            acc[y] = Q.agg_out_type[y] == T_LONG ? acc[y] + v : from_f64(as_f64(acc[y]) + mq_as_double(v, at));
          } else if (fn == AGG_AVG) {
            acc[y] = from_f64(as_f64(acc[y]) + mq_as_double(v, at));
          } else if (fn == AGG_MIN) {
            if (first || mq_less(v, acc[y], at)) acc[y] = v;
          } else {
            if (first || mq_less(acc[y], v, at)) acc[y] = v;
          }
        }
        em = true;
        if (Q.hav_item >= 0) {
          const int src = Q.sel_src[Q.hav_item];
          uint64_t v = (uint64_t)c.keyv;
          if (src >= SRC_AGG && src < SRC_AGG + kMaxAggs) v = aggval(src - SRC_AGG);
          else if (src >= SRC_REC && src < SRC_REC + kMqMaxCarry) v = mq_src(c, src - SRC_REC, r, ts);
          v = vm_convert(v, Q.sel_type[Q.hav_item], Q.hav_ctype);
          em = vm_compare(Q.hav_cop, Q.hav_ctype, v, Q.hav_cconst);
        }
      }
    }
    const uint64_t m = __ballot(em);
    if (kEmit && m) {
      if (em) {
        const unsigned long long p = pos + (unsigned long long)__popcll(m & lanemask_lt());
        if ((int64_t)p < Q.out_cap) {
          for (int x = 0; x < Q.nsel; ++x) {
            const int src = Q.sel_src[x];
            uint64_t v = (uint64_t)c.keyv;
            if (src >= SRC_AGG && src < SRC_AGG + kMaxAggs) v = aggval(src - SRC_AGG);
            else if (src >= SRC_REC && src < SRC_REC + kMqMaxCarry) v = mq_src(c, src - SRC_REC, r, ts);
            store_col(Q.out_col[x], Q.sel_type[x], (int64_t)p, v);
          }
          const uint32_t row = mq_row(L.w0[r]);
          Q.out_ts[p] = ts;
          Q.out_seq[p] = c.a->in_seq ? c.a->in_seq[row] : c.seq_base + row;
        } else {
          set_err(c.a->err, ERR_OUT_CAP);
        }
      }
      pos += (unsigned long long)__popcll(m);
    }
    rows += (uint32_t)__popcll(m);
  }
  if (kEmit && c.len) {
    S[0] = cnt;
#pragma unroll
    for (int i = 0; i < kMqMaxAggs; ++i)
      if (i < Q.nagg) S[(int64_t)(1 + i) * ks] = acc[i];
  }
  return rows;
}

}  // namespace

template <int NC>   // physical carried words per record
__global__ __launch_bounds__(kMqWalkThreads, 1) void k_mqwalk(MqWalkArgs a) {
  constexpr int NT = kMqWalkThreads, NWV = NT / 64;
  constexpr int W = MqLds<NC>::W;
  __shared__ MqLds<NC> L;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lg = a.buckets_log2;
  const int P = 1 << lg;
  const int bucket = xcd_bucket(blockIdx.x, P);
  const int kpb = a.kpb;
  const int nblk = (kpb + 63) >> 6;
  const int ntiles = a.ntiles;
  const int RW = 2 + NC;
  const int64_t ks = a.kstride;
  const int64_t ts_base = a.chunk_base[0], seq_base = a.chunk_base[1];
  // this bucket's segment of every tile -> exclusive prefix over tiles
  {
    constexpr int MAXPER = kMqMaxTiles / NT;
    const int per = (ntiles + NT - 1) / NT;
    uint32_t cnt[MAXPER];
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < MAXPER; ++i) {
      const int t = tid * per + i;
      cnt[i] = 0;
      if (i < per && t < ntiles) {
        const uint32_t lo = a.tile_off[(int64_t)bucket * ntiles + t];
        const uint32_t hi = a.tile_off[(int64_t)(bucket + 1) * ntiles + t];
        L.lo[t] = (uint16_t)lo;
        cnt[i] = hi - lo;
      }
      sum += cnt[i];
    }
    uint32_t total;
    uint32_t off = bscan<NT>(sum, L.scratch, &total);
#pragma unroll
    for (int i = 0; i < MAXPER; ++i) {
      const int t = tid * per + i;
      if (i < per && t < ntiles) {
        L.seg[t] = off;
        off += cnt[i];
      }
    }
    if (tid == 0) L.seg[ntiles] = total;
  }
  lds_barrier();
  // Windows are whole tiles [t0, t1) of at most W records; a tile whose
  // segment alone exceeds W is split into row ranges of W rows (a tile's
  // records are not in arrival order inside its segment, so a window never
  // ends inside a segment by position).
  int t0 = 0;
  uint32_t sub = 0;   // row range of a split tile
  while (t0 < ntiles) {
    if (tid == 0) {
      int lo = t0 + 1, hi = ntiles;
      const uint32_t lim = L.seg[t0] + (uint32_t)W;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (L.seg[mid] <= lim) lo = mid;
        else hi = mid - 1;
      }
      L.wt1 = L.seg[t0 + 1] - L.seg[t0] > (uint32_t)W ? -1 : lo;   // -1: split tile t0
      L.nwin = 0;
    }
    for (int k = tid; k <= kpb; k += NT) L.kstart[k] = 0;
    lds_barrier();
    const int t1 = L.wt1;
    const bool split = t1 < 0;
    auto load = [&](uint32_t p, int64_t ri) {
      const uint64_t* rec = a.recs + ri * RW;
      const uint64_t w0 = rec[0], w1 = rec[1];
      L.w0[p] = w0;
      L.w1[p] = w1;
#pragma unroll
      for (int w = 0; w < NC; ++w) L.car[p * NC + w] = rec[2 + w];
      atomicAdd(&L.kstart[mq_key(w1) + 1], 1u);
    };
    uint32_t nw;
    if (!split) {
      // gather: window slot p = bucket record seg[t0] + p, in tile t = last with seg[t] <= that
      const uint32_t wb = L.seg[t0];
      nw = L.seg[t1] - wb;
      for (uint32_t p = tid; p < nw; p += NT) {
        const uint32_t g = wb + p;
        int lo = t0, hi = t1 - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (L.seg[mid] <= g) lo = mid;
          else hi = mid - 1;
        }
        load(p, (int64_t)lo * kMqTile + L.lo[lo] + (g - L.seg[lo]));
      }
      lds_barrier();
    } else {
      // rows [t0 * T + sub * W, + W) of tile t0: at most W records
      const uint32_t cnt = L.seg[t0 + 1] - L.seg[t0];
      const uint32_t rlo = (uint32_t)t0 * kMqTile + sub * (uint32_t)W, rhi = rlo + (uint32_t)W;
      for (uint32_t p = tid; p < cnt; p += NT) {
        const int64_t ri = (int64_t)t0 * kMqTile + L.lo[t0] + p;
        const uint32_t row = mq_row(a.recs[ri * RW]);
        if (row >= rlo && row < rhi) load(atomicAdd(&L.nwin, 1u), ri);
      }
      lds_barrier();
      nw = L.nwin;
    }
    if (split) {
      ++sub;
      if (sub * (uint32_t)W >= (uint32_t)kMqTile) {
        sub = 0;
        ++t0;
      }
    } else {
      t0 = t1;
    }
    {
      const uint32_t c = tid < kpb ? L.kstart[tid + 1] : 0u;
      uint32_t tot;
      const uint32_t off = bscan<NT>(c, L.scratch, &tot);
      if (tid < kpb) {
        L.kstart[tid] = off;
        L.kcur[tid] = off;
      }
      if (tid == 0) L.kstart[kpb] = tot;
    }
    lds_barrier();
    for (uint32_t p = tid; p < nw; p += NT) {
      const uint32_t slot = atomicAdd(&L.kcur[mq_key(L.w1[p])], 1u);
      L.sorted[slot] = (uint16_t)p;
    }
    lds_barrier();
    // arrival order inside each key run (insertion sort on the chunk row)
    for (int k = tid; k < kpb; k += NT) {
      const uint32_t q0 = L.kstart[k], q1 = L.kstart[k + 1];
      for (uint32_t i = q0 + 1; i < q1; ++i) {
        const uint16_t v = L.sorted[i];
        const uint32_t rv = mq_row(L.w0[v]);
        uint32_t j = i;
        while (j > q0 && mq_row(L.w0[L.sorted[j - 1]]) > rv) {
          L.sorted[j] = L.sorted[j - 1];
          --j;
        }
        L.sorted[j] = v;
      }
    }
    // longest run per 64-key block (the wave loops' trip count)
    for (int b = wave; b < nblk; b += NWV) {
      const int k = b * 64 + lane;
      uint32_t len = k < kpb ? L.kstart[k + 1] - L.kstart[k] : 0u;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = __shfl_xor(len, o, 64);
        len = y > len ? y : len;
      }
      if (lane == 0) L.bmax[b] = len;
    }
    lds_barrier();
    const int nitems = a.nq * nblk;
    // pass 1: rows per (query, block)
    for (int it = wave; it < nitems; it += NWV) {
      const int q = it / nblk, b = it - q * nblk;
      const uint32_t maxlen = L.bmax[b];
      uint32_t rows = 0;
      if (maxlen) {
        const MqQuery& Q = a.q[q];
        const int k = b * 64 + lane;
        MqCtx<NC> c{&L, &a, ts_base, seq_base, 0, 0, 0};
        if (k < kpb) {
          c.r0 = L.kstart[k];
          c.len = L.kstart[k + 1] - c.r0;
        }
        uint64_t* S = a.state + Q.st_off * ks + (int64_t)bucket * kpb + (k < kpb ? k : 0);
        rows = Q.kind == MQ_SEQ ? mq_seq<false, NC>(c, Q, S, ks, maxlen, 0)
                                : mq_agg<false, NC>(c, Q, S, ks, maxlen, 0);
      }
      if (lane == 0) L.qoff[q * nblk + b] = rows;
    }
    lds_barrier();
    // one output reservation per (window, query)
    if (tid < a.nq) {
      uint32_t s = 0;
      for (int b = 0; b < nblk; ++b) {
        const uint32_t c = L.qoff[tid * nblk + b];
        L.qoff[tid * nblk + b] = s;
        s += c;
      }
      L.qbase[tid] = s ? atomicAdd(a.q[tid].out_count, (unsigned long long)s) : 0ull;
    }
    lds_barrier();
    // pass 2: rows + state commit
    for (int it = wave; it < nitems; it += NWV) {
      const int q = it / nblk, b = it - q * nblk;
      const uint32_t maxlen = L.bmax[b];
      if (!maxlen) continue;
      const MqQuery& Q = a.q[q];
      const int k = b * 64 + lane;
      MqCtx<NC> c{&L, &a, ts_base, seq_base, 0, 0, 0};
      if (k < kpb) {
        c.r0 = L.kstart[k];
        c.len = L.kstart[k + 1] - c.r0;
        const int64_t kl = ((int64_t)k << lg) | bucket;
        c.keyv = kl * a.key_stride + a.key_offset;
      }
      uint64_t* S = a.state + Q.st_off * ks + (int64_t)bucket * kpb + (k < kpb ? k : 0);
      const unsigned long long pos = L.qbase[q] + L.qoff[q * nblk + b];
      if (Q.kind == MQ_SEQ) mq_seq<true, NC>(c, Q, S, ks, maxlen, pos);
      else mq_agg<true, NC>(c, Q, S, ks, maxlen, pos);
    }
    // the next window re-reads state this one wrote and reuses the LDS arrays
    if (t0 < ntiles) __syncthreads();
  }
}

void launch_mq_walk(const MqWalkArgs& a, int nbuckets, hipStream_t s) {
  const dim3 g((unsigned)nbuckets), b(kMqWalkThreads);
  switch (a.nphys) {
    case 0: hipLaunchKernelGGL(k_mqwalk<0>, g, b, 0, s, a); break;
    case 1: hipLaunchKernelGGL(k_mqwalk<1>, g, b, 0, s, a); break;
    case 2: hipLaunchKernelGGL(k_mqwalk<2>, g, b, 0, s, a); break;
    case 3: hipLaunchKernelGGL(k_mqwalk<3>, g, b, 0, s, a); break;
    default: hipLaunchKernelGGL(k_mqwalk<4>, g, b, 0, s, a); break;
  }
}

}  // namespace cep
