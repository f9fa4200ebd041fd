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
//   k_mqpart  one 1024-lane workgroup per 16384-row tile: key, ts, stream and
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

#include <type_traits>

#include "dev_common.h"
#include "kernels.h"
#include "vm.h"

namespace cep {

namespace {

__device__ __forceinline__ uint32_t mq_row(uint64_t w0) { return (uint32_t)(w0 >> 32) & 0x1ffffffu; }
__device__ __forceinline__ int mq_stream(uint64_t w0) { return (int)(w0 >> 57) & 7; }
__device__ __forceinline__ uint32_t mq_key(uint64_t w1) { return (uint32_t)(w1 >> 48); }

}  // namespace

// Conditions are read through the constant address space: scalar loads into
// a local copy (a generic pointer makes every term field a vector load).
typedef __attribute__((address_space(4))) const MqCond CMqCond;

__device__ __forceinline__ void mq_load_cond(CMqCond& c, TermList* tl, int32_t (&slot)[kMaxTerms]) {
  tl->n = c.tl.n;
  tl->any = c.tl.any;
  // only the condition's own terms (most are one comparison): copying all
  // kMaxTerms descriptors per condition and row group was most of k_mqpart's
  // scalar work
#pragma unroll
  for (int i = 0; i < kMaxTerms; ++i) {
    if (i >= tl->n) break;
    tl->t[i].col = c.tl.t[i].col;
    tl->t[i].coltype = c.tl.t[i].coltype;
    tl->t[i].aop = c.tl.t[i].aop;
    tl->t[i].atype = c.tl.t[i].atype;
    tl->t[i].aconst = c.tl.t[i].aconst;
    tl->t[i].cop = c.tl.t[i].cop;
    tl->t[i].ctype = c.tl.t[i].ctype;
    tl->t[i].cconst = c.tl.t[i].cconst;
    slot[i] = c.slot[i];
  }
}

// ============================================================== k_mqpart ==
// Two passes over the tile's rows inside one workgroup, so a tile can be
// large (16 rows per lane) without holding every column of 16 rows in
// registers: pass A reads the key and stream of all rows (bucket + LDS rank),
// then, after the bucket scan, pass B reads the condition / carried columns
// four rows per lane at a time and writes the records.  Large tiles keep the
// bucket-major tile offset table small (P / 16384 entries per row).
template <int NP>   // prefetched columns
__global__ __launch_bounds__(kMqPartThreads, 1) void k_mqpart(MqPartArgs a) {
  constexpr int NT = kMqPartThreads, RPL = kMqTile / kMqPartThreads, EB = 4;
  static_assert(RPL % EB == 0 && RPL <= 32, "tile geometry");
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
  // lane-interleaved rows: lane l of wave w owns chunk rows w*64*RPL + 64*e + l
  const int64_t r0 = tile * kMqTile + (int64_t)wave * 64 * RPL + lane;
  const int64_t row0 = a.rows.row0 + r0;
  uint32_t valid = 0;
#pragma unroll
  for (int e = 0; e < RPL; ++e) valid |= (r0 + 64 * e < a.rows.n ? 1u : 0u) << e;
  // pass A: key and stream of every row
  const int kc = a.pref.col[0];
  const bool klong = a.rows.cols.t[kc] == T_LONG;
  uint64_t kv[RPL];
  uint32_t sv[RPL];
#pragma unroll
  for (int e = 0; e < RPL; ++e) {
    const bool ok = (valid >> e) & 1u;
    const int64_t rr = row0 + 64 * e;
    kv[e] = !ok ? 0ull : klong ? ((const uint64_t*)a.rows.cols.p[kc])[rr]
                               : from_i32(((const int32_t*)a.rows.cols.p[kc])[rr]);
    sv[e] = (ok && a.rows.stream) ? (uint32_t)a.rows.stream[rr] : (uint32_t)a.rows.input;
  }
  lds_barrier();   // hist zeroed
  // bits 0-14 rank in tile, 15-27 bucket; lkey: key within its bucket
  uint32_t packed[RPL], lkey[RPL];
#pragma unroll
  for (int e = 0; e < RPL; ++e) {
    packed[e] = 0xffffffffu;
    lkey[e] = 0;
    if (!((valid >> e) & 1u) || !((a.stream_mask >> sv[e]) & 1u)) continue;
    const int64_t kfield = shard_key((int64_t)kv[e], a.key_stride, a.key_offset);
    if (kfield < 0 || kfield >= a.key_capacity) {
      set_err(a.err, ERR_KEY_RANGE);
      continue;
    }
    const uint32_t bucket = (uint32_t)(kfield & (P - 1));
    lkey[e] = (uint32_t)(kfield >> lg);
    packed[e] = (bucket << 15) | atomicAdd(&hist[bucket], 1u);
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
  for (int i = tid; i <= P; i += NT) a.tile_off[(int64_t)i * a.ntiles + tile] = (uint16_t)hist[i];
  // pass B: conditions and carried columns, EB rows per lane at a time
  uint64_t* trecs = a.recs + tile * (int64_t)kMqTile * RW;
  // predecessor of the lane's first row (read by lanes that hold rows only:
  // row0 - 1 of a lane past the batch end would read past the ts column)
  int64_t prev_last = 0;
  if (valid & 1u) prev_last = row0 > 0 ? a.rows.ts[row0 - 1] : batch_prev_ts(a.rows);
#pragma unroll
  for (int g = 0; g < RPL / EB; ++g) {
    const uint32_t vg = (valid >> (EB * g)) & ((1u << EB) - 1u);
    uint64_t tsv[EB], pv[NP][EB], mask[EB];
    uint32_t sb[EB];
#pragma unroll
    for (int e = 0; e < EB; ++e) mask[e] = 1ull << kMqTrueBit;
    if (__ballot(vg != 0)) {
      cf_load_cols<EB, NP>(a.rows, a.pref, a.ts_slot, row0 + 64 * EB * g, vg, tsv, sb, pv);
      if (a.check_order) {
        // event-time order (`within` relies on it): row r - 1 is held by the
        // previous lane (same e) or lane 63 (e - 1, possibly of the last round)
        bool bad = false;
#pragma unroll
        for (int e = 0; e < EB; ++e) {
          const uint64_t up = __shfl_up(tsv[e], 1, 64);
          const uint64_t last = e > 0 ? __shfl(tsv[e > 0 ? e - 1 : 0], 63, 64) : 0ull;
          const int64_t pl = e > 0 ? (int64_t)last : prev_last;
          const int64_t prev = lane > 0 ? (int64_t)up : pl;
          if ((vg >> e) & 1u) bad |= (int64_t)tsv[e] < prev;
        }
        if (bad) set_err(a.err, ERR_ORDER);
        prev_last = (int64_t)__shfl(tsv[EB - 1], 63, 64);
      }
      // every distinct condition of each stream, once per row (uniform loops)
      for (int s = 0; s < 8; ++s) {
        if (!((a.stream_mask >> s) & 1u)) continue;
        uint32_t is_s = 0;
#pragma unroll
        for (int e = 0; e < EB; ++e) is_s |= (((vg >> e) & 1u) && sb[e] == (uint32_t)s ? 1u : 0u) << e;
        const int nc = a.ncond[s];
        if (!__ballot(is_s != 0) || nc == 0) continue;
        CMqCond* cs = (CMqCond*)a.conds + s * kMqMaxCond;
        for (int c = 0; c < nc; ++c) {
          TermList tl;
          int32_t slot[kMaxTerms];
          mq_load_cond(cs[c], &tl, slot);
          const uint32_t bits = eval_terms_regs<EB, NP>(tl, slot, a.rows.cols, pv) & is_s;
#pragma unroll
          for (int e = 0; e < EB; ++e) mask[e] |= (uint64_t)((bits >> e) & 1u) << c;
        }
      }
#pragma unroll
      for (int e = 0; e < EB; ++e) {
        const int ee = EB * g + e;
        if (packed[ee] == 0xffffffffu) continue;
        const uint32_t b = packed[ee] >> 15;
        const uint32_t slot = hist[b] + (packed[ee] & 0x7fffu);
        // ts relative to the chunk's first row, signed: rows before it are
        // legal unless some query has `within` (checked above)
        const int64_t dts = (int64_t)tsv[e] - ts_base;
        if (dts < INT32_MIN || dts > INT32_MAX) set_err(a.err, ERR_TS_SPAN);
        uint64_t* gp = trecs + (int64_t)slot * RW;
        gp[0] = (uint64_t)(uint32_t)dts | ((uint64_t)(uint32_t)(r0 + 64 * ee) << 32) | ((uint64_t)sb[e] << 57);
        gp[1] = mask[e] | ((uint64_t)lkey[ee] << 48);
#pragma unroll
        for (int w = 0; w < kMqMaxPhys; ++w)
          if (w < a.nphys) gp[2 + w] = pick<EB, NP>(pv, a.phys_slot[w], e);
      }
    }
  }
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


// Per-query data the step loops read, staged in LDS at kernel start: read
// where used (a scalar copy of every query's output pointers would not fit
// the scalar register file).
struct MqHot {
  uint64_t col[kMqMaxSel];
  uint64_t ts, seq, hconst;
  int64_t cap;
  uint64_t viw;                           // 8 bits per select item: value slot | width << 4
  uint32_t fbit, pad;
};

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
  uint16_t korder[kMqMaxKpb];            // keys by descending run length (lane blocks of alike runs)
  uint32_t lhist[257];                   // run-length bins (descending), then their cursors
  unsigned long long wcur[kMqWalkThreads / 64][kMqMaxQ];   // per wave: a unit's row counts / output cursors
  MqHot hot[kMqMaxQ];                    // per query: what the step loops read (outputs, filter, having constant)
  uint64_t stg[kMqWalkThreads / 64][kMqStgWords];   // per wave: output rows staged for full-width stores
  uint32_t seg[kMqMaxTiles + 1];         // exclusive prefix of the bucket's tile segments
  uint16_t lo[kMqMaxTiles];              // segment start inside each tile
  uint32_t scratch[kMqWalkThreads / 64 + 1];
  int32_t wt1;                           // window end tile (-1: a split tile)
  uint32_t nwin;                         // records of a split tile's row range
};

// Descriptors are read through the constant address space: wave-uniform
// scalar loads the compiler may keep in SGPRs across the loops (a generic
// pointer would be reloaded after every output store it might alias).
typedef __attribute__((address_space(4))) const MqQuery CMqQuery;

// Per-window view one lane needs to read its records.
template <int NC>
struct MqCtx {
  int64_t ts_base, seq_base;
  int64_t keyv;       // the lane's partition key value
  uint32_t r0, len;   // the lane's key run in `sorted`
  int32_t lmap0, lmap1, lmap2, lmap3;   // logical carried word -> physical (-1: event ts)
  const int64_t* in_seq;
  unsigned int* err;
  int ablate;
  int32_t lg, bucket, key_stride, key_offset;   // key value of a record's key in bucket
};

// Logical carried word `src` (uniform) of window record r (MQ_SRC_*: key /
// event ts).
template <int NC>
__device__ __forceinline__ uint64_t mq_src(const MqLds<NC>& L, const MqCtx<NC>& c, int src, int r, int64_t ts) {
  if (src == MQ_SRC_KEY) return (uint64_t)c.keyv;
  if (src == MQ_SRC_TS) return (uint64_t)ts;
  const int w = src == 0 ? c.lmap0 : src == 1 ? c.lmap1 : src == 2 ? c.lmap2 : c.lmap3;
  if (w < 0) return (uint64_t)ts;   // the column is the event-ts buffer
  if constexpr (NC > 0) return L.car[r * NC + (NC > 1 ? w : 0)];   // w < NC (host-checked)
  return 0;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Output row p of a query from its value slots (MqQuery::sel_vi: 0 the key,
// 1 + i capture / aggregate i, 5 + w carried word w): one uniform-indexed
// register read and one store per column, unrolled.
__device__ __forceinline__ void mq_store_row(const MqHot& H, int nsel, unsigned long long p, const uint64_t (&vals)[9],
                                             int64_t ts, int64_t seq) {
  // The column pointers come from LDS, so the compiler cannot infer their
  // address space: generic (flat) stores would count against lgkmcnt too, and
  // every later LDS read of the step loop would wait for them to reach
  // memory.  They are global buffers: store through global pointers.
  typedef __attribute__((address_space(1))) uint64_t g64;
  typedef __attribute__((address_space(1))) uint32_t g32;
  typedef __attribute__((address_space(1))) uint8_t g8;
  const uint64_t viw = H.viw;
#pragma unroll
  for (int x = 0; x < kMqMaxSel; ++x) {
    if (x >= nsel) break;
    const uint32_t f = (uint32_t)(viw >> (8 * x)) & 0xffu;
    const uint64_t v = vals[f & 15u];
    const uint32_t w = f >> 4;
    if (w == 8) ((g64*)(uintptr_t)H.col[x])[p] = v;
    else if (w == 4) ((g32*)(uintptr_t)H.col[x])[p] = (uint32_t)v;
    else ((g8*)(uintptr_t)H.col[x])[p] = (uint8_t)(v & 1u);
  }
  ((g64*)(uintptr_t)H.ts)[p] = (uint64_t)ts;
  if (H.seq) ((g64*)(uintptr_t)H.seq)[p] = (uint64_t)seq;   // 0: nobody reads them
}

// One sequence query over a block of 64 keys (lane = key): restates
// oracle/mq_oracle.c sequence_event for the one-partial shape.  The step is
// branch-free (selects): the kernel is issue-bound, and every divergent
// branch costs scalar exec-mask instructions.  kEmit = false: returns the
// rows the wave would emit; true: stores them from `pos` and commits the state.
template <bool kEmit, int NC>
__device__ __forceinline__ uint32_t mq_seq(const MqLds<NC>& L, const MqCtx<NC>& c, CMqQuery& Q, const MqHot& H,
                                           uint64_t* S, int64_t ks, uint32_t maxlen, unsigned long long pos) {
  // the descriptor, decoded once (uniform: scalar registers)
  const int N = Q.nstates, ncap = Q.ncap, nsel = Q.nsel;
  const uint32_t smask = Q.stream_mask, sstream = Q.st_stream, topt = Q.tail_opt;
  const uint64_t sbit = Q.st_bit, smin = Q.st_min, smax = Q.st_max;
  const int64_t within = Q.within;
  const bool every = Q.every != 0;
  int cst[kMqMaxCaps], clast[kMqMaxCaps], csrc[kMqMaxCaps];
#pragma unroll
  for (int x = 0; x < kMqMaxCaps; ++x) {
    cst[x] = x < ncap ? Q.cap_state[x] : -1;
    clast[x] = Q.cap_last[x];
    csrc[x] = Q.cap_src[x];
  }
  uint64_t hdr = 0, sts = 0, cap[kMqMaxCaps];
#pragma unroll
  for (int i = 0; i < kMqMaxCaps; ++i) cap[i] = 0;
  if (c.len) {
    hdr = S[0];
    if (hdr & 1u) {
      sts = S[ks];
#pragma unroll
      for (int i = 0; i < kMqMaxCaps; ++i)
        if (i < ncap) cap[i] = S[(int64_t)(2 + i) * ks];
    }
  }
  bool live = (hdr & 1u) != 0, started = (hdr & 2u) != 0;
  int j = (int)((hdr >> 8) & 0xffu);
  uint32_t cnt = (uint32_t)(hdr >> 16);
  uint32_t rows = 0;
  auto stream_of = [&](int s) { return (int)((sstream >> (3 * s)) & 7u); };
  auto min_of = [&](int s) { return (uint32_t)((smin >> (8 * s)) & 0xffu); };
  auto max_of = [&](int s) { return (uint32_t)((smax >> (8 * s)) & 0xffu); };
  const bool done0 = ((topt & 1u) != 0) && min_of(0) <= 1u;             // a start alone completes
  const bool keep0 = N == 1 && (max_of(0) == 0xffu || 1u < max_of(0));   // ... and stays open
  for (uint32_t i = 0; i < maxlen; ++i) {
    const bool valid = i < c.len;
    const int r = L.sorted[c.r0 + (valid ? i : 0u)];   // lanes past their run re-read a record
    const uint64_t w0 = L.w0[r], w1 = L.w1[r];
    const int st = mq_stream(w0);
    const int64_t ts = c.ts_base + (int64_t)(int32_t)(uint32_t)w0;
    const bool rel = valid && ((smask >> st) & 1u) != 0;
    auto cond = [&](int s) { return ((w1 >> ((sbit >> (6 * s)) & 63u)) & 1ull) != 0; };
    // the live partial: expired by `within`, else stays in its count state
    // (c1) or moves to a later state, skipping optional ones (found)
    const int64_t d = ts - (int64_t)sts;
    const bool alive = live && !(within >= 0 && (d < 0 ? -d : d) > within);
    const uint32_t mj = max_of(j);
    const bool c1 = rel && alive && stream_of(j) == st && (mj == 0xffu || cnt < mj) && cond(j);
    bool found = false, stop = !(rel && alive && !c1 && cnt >= min_of(j));
    int nj = j;
#pragma unroll
    for (int k = 1; k < kMaxStates; ++k) {
      if (k >= N) break;
      const bool inr = k > j && !stop && !found;
      const bool hit = inr && stream_of(k) == st && cond(k);
      nj = hit ? k : nj;
      found = found || hit;
      stop = stop || (inr && !hit && min_of(k) > 0u);
    }
    const bool adv = c1 || found;
    const int j2 = found ? nj : j;
    const uint32_t cnt2 = found ? 1u : cnt + (c1 ? 1u : 0u);
    const bool done2 = adv && cnt2 >= min_of(j2) && ((topt >> j2) & 1u) != 0;
    const bool live2 = adv && (!done2 || (j2 == N - 1 && (max_of(j2) == 0xffu || cnt2 < max_of(j2))));
    // a start event opens a new partial (never on an event that advanced one)
    const bool start = rel && stream_of(0) == st && (every || !started) && cond(0);
#pragma unroll
    for (int x = 0; x < kMqMaxCaps; ++x) {
      if (x >= ncap) break;
      const uint64_t v = mq_src(L, c, csrc[x], r, ts);
      const bool take = (c1 && cst[x] == j && clast[x]) || (found && cst[x] == nj);
      cap[x] = start ? (cst[x] == 0 ? v : 0ull) : (take ? v : cap[x]);
    }
    const bool em = (rel && done2) || (start && done0);
    live = start ? (!done0 || keep0) : (rel ? live2 : live);
    j = start ? 0 : (rel ? j2 : j);
    cnt = start ? 1u : (rel ? cnt2 : cnt);
    sts = start ? (uint64_t)ts : sts;
    started = started || start;
    const uint64_t m = __ballot(em);
    if (kEmit && m) {
      if (em) {
        const unsigned long long p = pos + (unsigned long long)__popcll(m & lanemask_lt());
        if ((int64_t)p < H.cap) {
          const uint32_t row = mq_row(w0);
          uint64_t vals[9];
          vals[0] = (uint64_t)c.keyv;
#pragma unroll
          for (int y = 0; y < kMqMaxCaps; ++y) vals[1 + y] = cap[y];
#pragma unroll
          for (int y = 5; y < 9; ++y) vals[y] = 0;
          mq_store_row(H, nsel, p, vals, ts, c.in_seq ? c.in_seq[row] : c.seq_base + row);
        } else {
          set_err(c.err, ERR_OUT_CAP);
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
        if (i < ncap) S[(int64_t)(2 + i) * ks] = cap[i];
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

typedef __attribute__((address_space(4))) const MqUnit CMqUnit;

// A class of sequence queries advanced bit-parallel (MQU_SEQ_BP): per key one
// live mask (bit q: query q0 + q has a partial), one state, one start ts and
// one set of captures for the whole class — every event either advances all
// of a key's partials into the state its stream names, or (condition false,
// move not allowed) drops them, or (the start stream) replaces them.  Same
// semantics as mq_seq / oracle/mq_oracle.c sequence_event for this shape.
// Per-query row counts (count pass) / output cursors (emit pass) live in the
// wave's LDS row `cur`.
template <bool kEmit, int NC>
__device__ __forceinline__ void mq_seq_bp(const MqLds<NC>& L, const MqCtx<NC>& c, CMqUnit& U, CMqQuery* qc,
                                          uint64_t* S, int64_t ks, uint32_t maxlen, unsigned long long* cur) {
  CMqQuery& Q0 = qc[U.q0];
  const int nq = U.nq, N = Q0.nstates, ncap = Q0.ncap, nsel = Q0.nsel;
  const uint64_t qmask = nq >= 64 ? ~0ull : ((1ull << nq) - 1ull);
  const uint32_t sos = U.st_of_stream, topt = Q0.tail_opt;
  const uint64_t allow = U.allow, cbase = U.cbase;
  const bool keep_last = U.keep_last != 0, every = Q0.every != 0;
  const int64_t within = Q0.within;
  const int lane = threadIdx.x & 63;
  int cst[kMqMaxCaps], clast[kMqMaxCaps], csrc[kMqMaxCaps];
#pragma unroll
  for (int x = 0; x < kMqMaxCaps; ++x) {
    cst[x] = x < ncap ? Q0.cap_state[x] : -1;
    clast[x] = Q0.cap_last[x];
    csrc[x] = Q0.cap_src[x];
  }
  uint64_t live = 0, started = 0, sts = 0, cap[kMqMaxCaps];
  int j = 0;
#pragma unroll
  for (int x = 0; x < kMqMaxCaps; ++x) cap[x] = 0;
  if (c.len) {
    live = S[0];
    started = S[ks];
    j = (int)S[2 * ks];
    sts = S[3 * ks];
    if (live) {
#pragma unroll
      for (int x = 0; x < kMqMaxCaps; ++x)
        if (x < ncap) cap[x] = S[(int64_t)(4 + x) * ks];
    }
  }
  for (uint32_t i = 0; i < maxlen; ++i) {
    const bool valid = i < c.len;
    const int r = L.sorted[c.r0 + (valid ? i : 0u)];   // lanes past their run re-read a record
    const uint64_t w0 = L.w0[r], w1 = L.w1[r];
    const int st = mq_stream(w0);
    const int64_t ts = c.ts_base + (int64_t)(int32_t)(uint32_t)w0;
    const uint32_t s1 = valid ? ((sos >> (4 * st)) & 15u) : 0u;   // target state + 1 (0: not read)
    const bool rel = s1 != 0;
    const int s = rel ? (int)s1 - 1 : 0;
    const int64_t d = ts - (int64_t)sts;
    const uint64_t lv = (within >= 0 && (d < 0 ? -d : d) > within) ? 0ull : live;   // expired: dropped
    const uint32_t cb = (uint32_t)((cbase >> (8 * s)) & 0xffu);
    const uint64_t cm = cb == 0xffu ? qmask : ((w1 >> cb) & qmask);   // the class's conditions of state s
    const bool isstart = rel && s == 0;
    const uint64_t nl = isstart ? (cm & (every ? qmask : ~started))
                                : ((((allow >> (j * 8 + s)) & 1ull) != 0) ? (lv & cm) : 0ull);
    const bool done = ((topt >> s) & 1u) != 0;   // counts here are "at least one": satisfied on arrival
    const uint64_t em = (rel && done) ? nl : 0ull;
    const uint64_t after = done ? ((s == N - 1 && keep_last) ? nl : 0ull) : nl;
    const bool first = isstart || s != j;
#pragma unroll
    for (int x = 0; x < kMqMaxCaps; ++x) {
      if (x >= ncap) break;
      const uint64_t v = mq_src(L, c, csrc[x], r, ts);
      const bool take = cst[x] == s && (clast[x] || first);
      cap[x] = !rel ? cap[x] : (take ? v : (isstart ? 0ull : cap[x]));
    }
    live = rel ? after : live;
    started = isstart ? (started | nl) : started;
    j = rel ? s : j;
    sts = isstart ? (uint64_t)ts : sts;
    if (__ballot(em != 0)) {   // rare: rows of this step, query by query
      for (int q = 0; q < nq; ++q) {
        const bool e = ((em >> q) & 1ull) != 0;
        const uint64_t m = __ballot(e);
        if (!m) continue;
        if (kEmit && e) {
          const MqHot& H = L.hot[U.q0 + q];
          const unsigned long long p = cur[q] + (unsigned long long)__popcll(m & lanemask_lt());
          if ((int64_t)p < H.cap) {
            const uint32_t row = mq_row(w0);
            uint64_t vals[9];
            vals[0] = (uint64_t)c.keyv;
#pragma unroll
            for (int y = 0; y < kMqMaxCaps; ++y) vals[1 + y] = cap[y];
#pragma unroll
            for (int y = 5; y < 9; ++y) vals[y] = 0;
            mq_store_row(H, nsel, p, vals, ts, c.in_seq ? c.in_seq[row] : c.seq_base + row);
          } else {
            set_err(c.err, ERR_OUT_CAP);
          }
        }
        if (lane == 0) cur[q] += (unsigned long long)__popcll(m);
      }
    }
  }
  if (kEmit && c.len) {
    S[0] = live;
    S[ks] = started;
    S[2 * ks] = (uint64_t)(uint32_t)j;
    S[3 * ks] = sts;
    if (live) {
#pragma unroll
      for (int x = 0; x < kMqMaxCaps; ++x)
        if (x < ncap) S[(int64_t)(4 + x) * ks] = cap[x];
    }
  }
}

// Up to NU group-by aggregations of one shape over a block of 64 keys (lane
// = group), each query's running values in registers (NA accumulators beside
// the shared count): the record and the aggregate arguments are decoded once
// per step for all of them.  Running values in arrival order as
// oracle/mq_oracle.c agg_event (sum over int / long wraps in 64 bits, sum /
// avg over float / double accumulate in double, min / max compare in the
// argument type), having on one output item.  Branch-free on lane data.
template <bool kEmit, int NC, int NU, int NA>
__device__ __forceinline__ void mq_agg_unit(const MqLds<NC>& L, const MqCtx<NC>& c, CMqUnit& U, CMqQuery* qc,
                                            uint64_t* state, int64_t kidx, int64_t ks, uint32_t maxlen,
                                            unsigned long long* cur) {
  CMqQuery& Q0 = qc[U.q0];
  const int nq = U.nq, in_st = Q0.in_stream, nagg = Q0.nagg, nsel = Q0.nsel;
  const int lane = threadIdx.x & 63;
  // accumulator a <- aggregate slot; per accumulator: op (0 sum / avg in
  // double, 1 sum in 64-bit ints, 2 min, 3 max), comparison domain (0 int64,
  // 1 float, 2 double), argument source and type
  int aslot[NA], aop[NA], acmp[NA], asrc[NA], atyp[NA];
  int slot_acc[kMqMaxAggs];
  {
    int na = 0;
#pragma unroll
    for (int y = 0; y < kMqMaxAggs; ++y) {
      slot_acc[y] = -1;
      if (y < nagg && Q0.agg_fn[y] != AGG_COUNT && na < NA) {
        const int fn = Q0.agg_fn[y], t = Q0.agg_arg_type[y];
#pragma unroll
        for (int a2 = 0; a2 < NA; ++a2)
          if (a2 == na) {
            aslot[a2] = y;
            aop[a2] = fn == AGG_MIN ? 2 : fn == AGG_MAX ? 3 : (fn == AGG_SUM && Q0.agg_out_type[y] == T_LONG) ? 1 : 0;
            acmp[a2] = (t == T_LONG || t == T_INT) ? 0 : t == T_FLOAT ? 1 : 2;
            asrc[a2] = Q0.agg_src[y];
            atyp[a2] = t;
          }
        slot_acc[y] = na++;
      }
    }
#pragma unroll
    for (int a2 = 0; a2 < NA; ++a2)
      if (a2 >= na) { aslot[a2] = 0; aop[a2] = 0; acmp[a2] = 0; asrc[a2] = MQ_SRC_KEY; atyp[a2] = T_LONG; }
  }
  // having: the item's value as a double or an int64, compared with the query's constant
  const int hitem = Q0.hav_item, hvi = Q0.hav_vi;
  const int htype = hitem >= 0 ? Q0.sel_type[hitem] : T_LONG;
  const int hcop = Q0.hav_cop, hctype = Q0.hav_ctype;
  const bool hdbl = hctype == T_DOUBLE || hctype == T_FLOAT;
  uint64_t cnt[NU], acc[NU][NA];
#pragma unroll
  for (int i = 0; i < NU; ++i) {
    cnt[i] = 0;
#pragma unroll
    for (int a2 = 0; a2 < NA; ++a2) acc[i][a2] = 0;
  }
  if (c.len) {
#pragma unroll
    for (int i = 0; i < NU; ++i) {
      if (i >= nq) break;
      const uint64_t* S = state + qc[U.q0 + i].st_off * ks + kidx;
      cnt[i] = S[0];
#pragma unroll
      for (int a2 = 0; a2 < NA; ++a2)
        if (slot_acc[aslot[a2]] == a2) acc[i][a2] = S[(int64_t)(1 + aslot[a2]) * ks];
    }
  }
  // value of aggregate slot y of query i
  auto aggval = [&](int i, int y) -> uint64_t {
    const int fn = Q0.agg_fn[y];
    uint64_t x = 0;
#pragma unroll
    for (int a2 = 0; a2 < NA; ++a2) x = slot_acc[y] == a2 ? acc[i][a2] : x;
    return fn == AGG_COUNT ? cnt[i] : fn == AGG_AVG ? from_f64(as_f64(x) / (double)(int64_t)cnt[i]) : x;
  };
  for (uint32_t s = 0; s < maxlen; ++s) {
    const bool valid = s < c.len;
    const int r = L.sorted[c.r0 + (valid ? s : 0u)];   // lanes past their run re-read a record
    const uint64_t w0 = L.w0[r], w1 = L.w1[r];
    const int64_t ts = c.ts_base + (int64_t)(int32_t)(uint32_t)w0;
    const bool pbase = valid && mq_stream(w0) == in_st;
    // the arguments, once for every query of the unit
    uint64_t av[NA];
    double ad[NA];
#pragma unroll
    for (int a2 = 0; a2 < NA; ++a2) {
      av[a2] = mq_src(L, c, asrc[a2], r, ts);
      ad[a2] = mq_as_double(av[a2], atyp[a2]);
    }
#pragma unroll
    for (int i = 0; i < NU; ++i) {
      if (i >= nq) break;
      const bool pass = pbase && ((w1 >> L.hot[U.q0 + i].fbit) & 1ull) != 0;
      const bool first = cnt[i] == 0;
      cnt[i] += pass ? 1u : 0u;
#pragma unroll
      for (int a2 = 0; a2 < NA; ++a2) {
        const uint64_t o = acc[i][a2];
        const uint64_t sumd = from_f64(as_f64(o) + ad[a2]);
        const uint64_t suml = o + av[a2];
        const bool lt = acmp[a2] == 0 ? (int64_t)av[a2] < (int64_t)o
                        : acmp[a2] == 1 ? as_f32(av[a2]) < as_f32(o) : as_f64(av[a2]) < as_f64(o);
        const bool gt = acmp[a2] == 0 ? (int64_t)o < (int64_t)av[a2]
                        : acmp[a2] == 1 ? as_f32(o) < as_f32(av[a2]) : as_f64(o) < as_f64(av[a2]);
        const uint64_t nv = aop[a2] == 0 ? sumd : aop[a2] == 1 ? suml
                            : aop[a2] == 2 ? ((first || lt) ? av[a2] : o) : ((first || gt) ? av[a2] : o);
        acc[i][a2] = pass ? nv : o;
      }
      bool em = pass;
      if (hitem >= 0) {
        uint64_t hv = (uint64_t)c.keyv;
        if (hvi >= 1 && hvi <= kMqMaxAggs) hv = aggval(i, hvi - 1);
        else if (hvi >= 5) hv = mq_src(L, c, hvi - 5, r, ts);
        const uint64_t cv = vm_convert(hv, htype, hctype);
        bool ok;
        if (hdbl) {
          const double x = hctype == T_FLOAT ? (double)as_f32(cv) : as_f64(cv);
          const uint64_t hk = L.hot[U.q0 + i].hconst;
          const double y = hctype == T_FLOAT ? (double)as_f32(hk) : as_f64(hk);
          ok = hcop == OP_EQ ? x == y : hcop == OP_NE ? x != y : hcop == OP_LT ? x < y
               : hcop == OP_LE ? x <= y : hcop == OP_GT ? x > y : x >= y;
        } else {
          const int64_t x = hctype == T_LONG ? (int64_t)cv : (int64_t)(int32_t)cv;
          const uint64_t hk = L.hot[U.q0 + i].hconst;
          const int64_t y = hctype == T_LONG ? (int64_t)hk : (int64_t)(int32_t)hk;
          ok = hcop == OP_EQ ? x == y : hcop == OP_NE ? x != y : hcop == OP_LT ? x < y
               : hcop == OP_LE ? x <= y : hcop == OP_GT ? x > y : x >= y;
        }
        em = em && ok;
      }
      const uint64_t m = __ballot(em);
      if (kEmit && m) {
        if (em) {
          const MqHot& H = L.hot[U.q0 + i];
          const unsigned long long p = cur[i] + (unsigned long long)__popcll(m & lanemask_lt());
          if ((int64_t)p < H.cap) {
            const uint32_t row = mq_row(w0);
            uint64_t vals[9];
            vals[0] = (uint64_t)c.keyv;
#pragma unroll
            for (int y = 0; y < kMqMaxAggs; ++y) vals[1 + y] = y < nagg ? aggval(i, y) : 0ull;
#pragma unroll
            for (int w = 0; w < kMqMaxCarry; ++w) vals[5 + w] = mq_src(L, c, w, r, ts);
            mq_store_row(H, nsel, p, vals, ts, c.in_seq ? c.in_seq[row] : c.seq_base + row);
          } else {
            set_err(c.err, ERR_OUT_CAP);
          }
        }
      }
      if (m && lane == 0) cur[i] += (unsigned long long)__popcll(m);
    }
  }
  if (kEmit && c.len) {
#pragma unroll
    for (int i = 0; i < NU; ++i) {
      if (i >= nq) break;
      uint64_t* S = state + qc[U.q0 + i].st_off * ks + kidx;
      S[0] = cnt[i];
#pragma unroll
      for (int a2 = 0; a2 < NA; ++a2)
        if (slot_acc[aslot[a2]] == a2) S[(int64_t)(1 + aslot[a2]) * ks] = acc[i][a2];
    }
  }
}


// Bit-pattern select without a branch (the compiler turns ternaries on
// wave-uniform values into scalar branches, each followed by waits).
__device__ __forceinline__ uint64_t msel(bool c, uint64_t a, uint64_t b) {
  const uint64_t m = 0ull - (uint64_t)c;
  return (a & m) | (b & ~m);
}

// A vmcnt(0) wait (gfx9 s_waitcnt encoding: expcnt / lgkmcnt left at max).
// Issued after a unit's state loads so the step loop starts with no loads in
// flight: the waitcnt pass then keeps vmcnt waits out of the loop, where they
// would also wait for every output store issued by earlier steps (on CDNA
// vmcnt counts stores too).
__device__ __forceinline__ void wait_vm() { __builtin_amdgcn_s_waitcnt(0x0f70); }

// LDS written by some lanes of a wave, then read by others: one wave's LDS
// operations are performed in issue order, so only the compiler must not
// reorder them (a wavefront-scope fence: no wait instruction).
// __threadfence_block would also wait for every global store in flight (on
// CDNA vmcnt counts stores).
__device__ __forceinline__ void wave_lds_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// Up to NU group-by aggregations of one shape with at most one non-count
// accumulator, its operation fixed at compile time (AOP 0: sum / avg in
// double, 1: sum in 64-bit ints, 2: min, 3: max, 4: count only; ACMP: min /
// max domain 0 int64, 1 float, 2 double).  Same running values, having and
// rows as mq_agg_unit (oracle/mq_oracle.c agg_event), with the per-step code
// free of branches on descriptor values: those are decoded once per item.
template <bool kEmit, int NC, int NU, int AOP, int ACMP>
__device__ __forceinline__ void mq_agg_fast(const MqLds<NC>& L, const MqCtx<NC>& c, CMqUnit& U, CMqQuery* qc,
                                            uint64_t* state, int64_t kidx, int64_t ks, uint32_t maxlen,
                                            unsigned long long* cur) {
  CMqQuery& Q0 = qc[U.q0];
  const int nq = U.nq, in_st = Q0.in_stream, nagg = Q0.nagg, nsel = Q0.nsel;
  const int lane = threadIdx.x & 63;
  int ys = -1;   // the accumulator's aggregate slot
#pragma unroll
  for (int y = 0; y < kMqMaxAggs; ++y)
    if (y < nagg && Q0.agg_fn[y] != AGG_COUNT) ys = y;
  const int asrc = ys >= 0 ? Q0.agg_src[ys] : (int)MQ_SRC_KEY;
  const int atyp = ys >= 0 ? Q0.agg_arg_type[ys] : (int)T_LONG;
  // value kinds (having item, select items): 0 key, 1 count, 2 accumulator,
  // 3 average, 4 + w carried word w
  auto vkind = [&](int vi) {
    if (vi >= 5) return 4 + (vi - 5);
    if (vi >= 1) {
      const int fn = Q0.agg_fn[vi - 1];
      return fn == AGG_COUNT ? 1 : fn == AGG_AVG ? 3 : 2;
    }
    return 0;
  };
  const bool hav = Q0.hav_item >= 0;
  const int hk = hav ? vkind(Q0.hav_vi) : 0;
  const int htype = hav ? Q0.sel_type[Q0.hav_item] : (int)T_LONG;
  const bool hdbl = Q0.hav_ctype == T_DOUBLE;
  const int hcop = Q0.hav_cop;
  const bool mlt = hcop == OP_LT || hcop == OP_LE || hcop == OP_NE;
  const bool meq = hcop == OP_EQ || hcop == OP_LE || hcop == OP_GE;
  const bool mgt = hcop == OP_GT || hcop == OP_GE || hcop == OP_NE;
  const bool mne = hcop == OP_NE;
  // per query: filter bit and having constant through the constant address
  // space (scalar loads where used), running values and cursor in registers
  uint64_t cnt[NU], acc[NU];
  unsigned long long curv[NU];
#pragma unroll
  for (int i = 0; i < NU; ++i) {
    curv[i] = i < nq ? cur[i] : 0ull;
    cnt[i] = 0;
    acc[i] = 0;
  }
  if (c.len) {
#pragma unroll
    for (int i = 0; i < NU; ++i) {
      if (i >= nq) break;
      const uint64_t* S = state + qc[U.q0 + i].st_off * ks + kidx;
      cnt[i] = S[0];
      if (AOP != 4) acc[i] = S[(int64_t)(1 + ys) * ks];
    }
  }
  wait_vm();
  // the unit's select layout (one shape per unit): value kind and width per
  // column, decoded once (wave-uniform, scalar registers)
  int ckind[kMqMaxSel], cw[kMqMaxSel];
#pragma unroll
  for (int x = 0; x < kMqMaxSel; ++x) {
    ckind[x] = x < nsel ? vkind(Q0.sel_vi[x]) : 0;
    cw[x] = x < nsel ? Q0.sel_w[x] : 8;
  }
  auto todouble = [](uint64_t v, int t) {
    const double di = (double)(int32_t)v, dl = (double)(int64_t)v, df = (double)as_f32(v);
    return t == T_INT ? di : t == T_LONG ? dl : t == T_FLOAT ? df : as_f64(v);
  };
  const bool need_avg = hk == 3 || [&] {
    bool any = false;
#pragma unroll
    for (int x = 0; x < kMqMaxSel; ++x) any = any || (x < nsel && ckind[x] == 3);
    return any;
  }();
  // Emit pass: each query's rows are staged in its own part of the wave's
  // LDS rows and written as contiguous runs of up to scap rows per column,
  // not as the ~10 rows a step emits per query.  A staged row is its record
  // slot, count and accumulator (3 words whatever the select list): key, ts,
  // seq, carried columns and the average are rebuilt from them at the flush.
  constexpr int kPart = kMqStgWords / NU;
  constexpr uint32_t scap = (uint32_t)(kPart / 3);
  uint64_t* stg0 = const_cast<uint64_t*>(L.stg[threadIdx.x >> 6]);
  uint32_t sc[NU];                 // staged rows per query
#pragma unroll
  for (int i = 0; i < NU; ++i) sc[i] = 0;
  auto flush = [&](int i) {
    typedef __attribute__((address_space(1))) uint64_t g64;
    typedef __attribute__((address_space(1))) uint32_t g32;
    typedef __attribute__((address_space(1))) uint8_t g8;
    CMqQuery& Q = qc[U.q0 + i];
    const uint64_t* stg = stg0 + i * kPart;
    wave_lds_sync();
    for (uint32_t j = lane; j < sc[i]; j += 64) {
      const unsigned long long p = curv[i] + j;
      if ((int64_t)p >= Q.out_cap) {
        set_err(c.err, ERR_OUT_CAP);
        continue;
      }
      if (c.ablate & 1) continue;
      const int r = (int)stg[j];
      const uint64_t rc = stg[scap + j], ra = stg[2 * scap + j];
      const uint64_t w0 = L.w0[r];
      const int64_t ts = c.ts_base + (int64_t)(int32_t)(uint32_t)w0;
      const int64_t keyv = ((((int64_t)mq_key(L.w1[r]) << c.lg) | c.bucket) * c.key_stride) + c.key_offset;
      const uint64_t ravg = need_avg ? from_f64(as_f64(ra) / (double)(int64_t)rc) : 0ull;
#pragma unroll
      for (int x = 0; x < kMqMaxSel; ++x) {
        if (x >= nsel) break;
        const int k = ckind[x];
        const uint64_t v = k == 0 ? (uint64_t)keyv : k == 1 ? rc : k == 2 ? ra : k == 3 ? ravg
                           : mq_src(L, c, k - 4, r, ts);
        if (cw[x] == 8) ((g64*)Q.out_col[x])[p] = v;
        else if (cw[x] == 4) ((g32*)Q.out_col[x])[p] = (uint32_t)v;
        else ((g8*)Q.out_col[x])[p] = (uint8_t)(v & 1u);
      }
      const uint32_t row = mq_row(w0);
      ((g64*)Q.out_ts)[p] = (uint64_t)ts;
      if (Q.out_seq) ((g64*)Q.out_seq)[p] = (uint64_t)(c.in_seq ? c.in_seq[row] : c.seq_base + row);
    }
    wave_lds_sync();
    curv[i] += sc[i];
    sc[i] = 0;
  };
  // The step loop is a chain of LDS reads (run slot -> record -> argument)
  // with few waves per SIMD to hide it: the next step's record is read one
  // step ahead and the slot after it two steps ahead.
  const int aw = (AOP == 4 || asrc == MQ_SRC_KEY || asrc == MQ_SRC_TS) ? -1
                 : (asrc == 0 ? c.lmap0 : asrc == 1 ? c.lmap1 : asrc == 2 ? c.lmap2 : c.lmap3);
  auto slot_of = [&](uint32_t st) { return (int)L.sorted[c.r0 + (st < c.len ? st : 0u)]; };
  auto car_of = [&](int r) -> uint64_t {
    if constexpr (NC > 0) return aw >= 0 ? L.car[r * NC + (NC > 1 ? aw : 0)] : 0ull;
    return 0ull;
  };
  int rn = slot_of(0);
  uint64_t nw0 = L.w0[rn], nw1 = L.w1[rn], ncar = car_of(rn);
  int rnn = slot_of(1);
  for (uint32_t st = 0; st < maxlen; ++st) {
    const bool valid = st < c.len;
    const int r = rn;   // lanes past their run re-read a record
    const uint64_t w0 = nw0, w1 = nw1, car = ncar;
    rn = rnn;
    nw0 = L.w0[rn];
    nw1 = L.w1[rn];
    ncar = car_of(rn);
    rnn = slot_of(st + 2);
    const int64_t ts = c.ts_base + (int64_t)(int32_t)(uint32_t)w0;
    const bool pbase = valid && mq_stream(w0) == in_st;
    const uint64_t av = AOP == 4 ? 0ull : asrc == MQ_SRC_KEY ? (uint64_t)c.keyv
                        : (asrc == MQ_SRC_TS || aw < 0) ? (uint64_t)ts : car;
    const double ad = AOP == 0 ? todouble(av, atyp) : 0.0;
    const uint64_t hcar = hk >= 4 ? mq_src(L, c, hk - 4, r, ts) : 0ull;
#pragma unroll
    for (int i = 0; i < NU; ++i) {
      if (i >= nq) break;
      const bool pass = pbase && ((w1 >> qc[U.q0 + i].filter_bit) & 1ull) != 0;
      const uint64_t hconst_i = qc[U.q0 + i].hav_cconst;
      const uint64_t o = acc[i];
      const bool first = cnt[i] == 0;
      cnt[i] += pass ? 1u : 0u;
      uint64_t nv = o;
      if (AOP == 0) nv = from_f64(as_f64(o) + ad);
      if (AOP == 1) nv = o + av;
      if (AOP == 2 || AOP == 3) {
        const bool lt = ACMP == 0 ? (int64_t)av < (int64_t)o : ACMP == 1 ? as_f32(av) < as_f32(o)
                                                                         : as_f64(av) < as_f64(o);
        const bool gt = ACMP == 0 ? (int64_t)o < (int64_t)av : ACMP == 1 ? as_f32(o) < as_f32(av)
                                                                         : as_f64(o) < as_f64(av);
        nv = (first || (AOP == 2 ? lt : gt)) ? av : o;
      }
      if (AOP != 4) acc[i] = pass ? nv : o;
      const uint64_t avgb = (AOP == 0 && need_avg) ? from_f64(as_f64(acc[i]) / (double)(int64_t)cnt[i]) : 0ull;
      bool em = pass;
      if (hav) {
        const uint64_t hv = msel(hk == 0, (uint64_t)c.keyv,
                                 msel(hk == 1, cnt[i], msel(hk == 2, acc[i], msel(hk == 3, avgb, hcar))));
        bool lt, eq, gt;
        if (hdbl) {
          const double x = todouble(hv, htype), y = as_f64(hconst_i);
          lt = x < y; eq = x == y; gt = x > y;
        } else {
          const int64_t x = Q0.hav_ctype == T_LONG ? (int64_t)hv : (int64_t)(int32_t)hv;
          const int64_t y = Q0.hav_ctype == T_LONG ? (int64_t)hconst_i : (int64_t)(int32_t)hconst_i;
          lt = x < y; eq = x == y; gt = x > y;
        }
        em = em && (mne ? !eq : ((lt && mlt) || (eq && meq) || (gt && mgt)));
      }
      const uint64_t m = __ballot(em);
      if (kEmit && m) {
        const uint32_t n = (uint32_t)__popcll(m);
        if (sc[i] + n > scap && !(c.ablate & 4)) flush(i);
        if (c.ablate & 4) sc[i] = 0;
        if (n > scap) {
          // more rows than the staging part holds (rare): stored directly
          typedef __attribute__((address_space(1))) uint64_t g64;
          typedef __attribute__((address_space(1))) uint32_t g32;
          typedef __attribute__((address_space(1))) uint8_t g8;
          CMqQuery& Q = qc[U.q0 + i];
          const unsigned long long p = curv[i] + (unsigned long long)__popcll(m & lanemask_lt());
          if (em && (int64_t)p >= Q.out_cap) set_err(c.err, ERR_OUT_CAP);
          if (em && (int64_t)p < Q.out_cap && !(c.ablate & 1)) {
            const uint32_t row = mq_row(w0);
#pragma unroll
            for (int x = 0; x < kMqMaxSel; ++x) {
              if (x >= nsel) break;
              const int k = ckind[x];
              const uint64_t v = k == 0 ? (uint64_t)c.keyv : k == 1 ? cnt[i] : k == 2 ? acc[i] : k == 3 ? avgb
                                 : mq_src(L, c, k - 4, r, ts);
              if (cw[x] == 8) ((g64*)Q.out_col[x])[p] = v;
              else if (cw[x] == 4) ((g32*)Q.out_col[x])[p] = (uint32_t)v;
              else ((g8*)Q.out_col[x])[p] = (uint8_t)(v & 1u);
            }
            ((g64*)Q.out_ts)[p] = (uint64_t)ts;
            if (Q.out_seq) ((g64*)Q.out_seq)[p] = (uint64_t)(c.in_seq ? c.in_seq[row] : c.seq_base + row);
          }
          curv[i] += n;
        } else if (em && !(c.ablate & 2)) {
          uint64_t* stg = stg0 + i * kPart;
          const uint32_t pos = sc[i] + (uint32_t)__popcll(m & lanemask_lt());
          stg[pos] = (uint64_t)r;
          stg[scap + pos] = cnt[i];
          stg[2 * scap + pos] = acc[i];
        }
        if (n <= scap) sc[i] += n;
      }
      if (!kEmit) curv[i] += (unsigned long long)__popcll(m);
    }
  }
  if (kEmit) {
#pragma unroll
    for (int i = 0; i < NU; ++i)
      if (i < nq && sc[i]) flush(i);
  }
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NU; ++i)
      if (i < nq) cur[i] = curv[i];
  }
  if (kEmit && c.len) {
#pragma unroll
    for (int i = 0; i < NU; ++i) {
      if (i >= nq) break;
      uint64_t* S = state + qc[U.q0 + i].st_off * ks + kidx;
      S[0] = cnt[i];
      if (AOP != 4) S[(int64_t)(1 + ys) * ks] = acc[i];
    }
  }
}

}  // namespace

#define MQ_STAMP(i)                                                                       \
  do {                                                                                    \
    if (a.stamps && threadIdx.x == 0) a.stamps[(int64_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// diagnostics: ticks of unit u (< 4) summed over its items, pass p, slot 8 + 4 p + u
#define MQ_UNIT_TICKS(p, u, t0)                                                            \
  do {                                                                                    \
    if (a.stamps && (threadIdx.x & 63) == 0 && (u) < 4)                                   \
      atomicAdd((unsigned long long*)&a.stamps[(int64_t)blockIdx.x * 16 + 8 + 4 * (p) + (u)], \
                (unsigned long long)(__builtin_amdgcn_s_memtime() - (t0)));                \
  } while (0)

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
  // this bucket's state block: word w of key k at state_b[w * kpb + k]
  const int64_t ks = kpb;
  uint64_t* const state_b = a.state + (int64_t)bucket * a.words * kpb;
  const int64_t ts_base = a.chunk_base[0], seq_base = a.chunk_base[1];
  CMqQuery* qc = (CMqQuery*)a.q;
  const MqCtx<NC> c0{ts_base, seq_base, 0, 0, 0, a.lmap[0], a.lmap[1], a.lmap[2], a.lmap[3], a.in_seq, a.err, a.ablate,
                        lg, bucket, a.key_stride, a.key_offset};
  MQ_STAMP(0);
  for (int q = tid; q < a.nq; q += NT) {
    MqHot& h = L.hot[q];
    CMqQuery& Q = qc[q];
    uint64_t viw = 0;
    for (int x = 0; x < kMqMaxSel; ++x) {
      h.col[x] = x < Q.nsel ? (uint64_t)Q.out_col[x] : 0ull;
      if (x < Q.nsel) viw |= (uint64_t)((uint32_t)Q.sel_vi[x] | ((uint32_t)Q.sel_w[x] << 4)) << (8 * x);
    }
    h.viw = viw;
    h.ts = (uint64_t)Q.out_ts;
    h.seq = (uint64_t)Q.out_seq;
    h.cap = Q.out_cap;
    h.hconst = Q.hav_cconst;
    h.fbit = (uint32_t)Q.filter_bit;
  }
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
    for (int k = tid; k < 257; k += NT) L.lhist[k] = 0;
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
    MQ_STAMP(1);
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
    // counting sort by key into a scratch array (the wave staging rows are
    // free until the items run), then each record's arrival rank inside its
    // key run (rows are unique in a chunk) places it: one short independent
    // loop per record instead of one serial insertion sort per key
    static_assert(W * sizeof(uint16_t) <= sizeof(L.stg), "sort scratch in the staging rows");
    uint16_t* tmp = reinterpret_cast<uint16_t*>(&L.stg[0][0]);
    for (uint32_t p = tid; p < nw; p += NT) {
      const uint32_t slot = atomicAdd(&L.kcur[mq_key(L.w1[p])], 1u);
      tmp[slot] = (uint16_t)p;
    }
    lds_barrier();
    for (uint32_t q = tid; q < nw; q += NT) {
      const uint16_t e = tmp[q];
      const uint32_t k = mq_key(L.w1[e]);
      const uint32_t q0 = L.kstart[k], q1 = L.kstart[k + 1];
      const uint32_t re = mq_row(L.w0[e]);
      uint32_t rank = 0;
      for (uint32_t j = q0; j < q1; ++j) rank += mq_row(L.w0[tmp[j]]) < re ? 1u : 0u;
      L.sorted[q0 + rank] = e;
    }
    // keys by descending run length: a wave's loop runs to the longest run
    // of its 64 keys, so blocks of alike runs keep the lanes busy
    auto bin_of = [&](int k) {
      const uint32_t len = L.kstart[k + 1] - L.kstart[k];
      return 255u - (len < 255u ? len : 255u);
    };
    for (int k = tid; k < kpb; k += NT) atomicAdd(&L.lhist[bin_of(k)], 1u);
    lds_barrier();
    {
      const uint32_t c = tid < 256 ? L.lhist[tid] : 0u;
      uint32_t tot;
      const uint32_t off = bscan<NT>(c, L.scratch, &tot);
      if (tid < 256) L.lhist[tid] = off;
    }
    lds_barrier();
    for (int k = tid; k < kpb; k += NT) L.korder[atomicAdd(&L.lhist[bin_of(k)], 1u)] = (uint16_t)k;
    lds_barrier();
    // longest run per 64-key block (the wave loops' trip count)
    for (int b = wave; b < nblk; b += NWV) {
      const int k = b * 64 + lane < kpb ? L.korder[b * 64 + lane] : kpb;
      uint32_t len = k < kpb ? L.kstart[k + 1] - L.kstart[k] : 0u;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = __shfl_xor(len, o, 64);
        len = y > len ? y : len;
      }
      if (lane == 0) L.bmax[b] = len;
    }
    lds_barrier();
    MQ_STAMP(2);
    const int nitems = a.nunits * nblk;
    CMqUnit* units = (CMqUnit*)a.units;
    // a unit over one 64-key block (lane = key); cur: the wave's per-query
    // row counters (count pass) / output cursors (emit pass)
    auto run_unit = [&](auto emit, int u, int b) {
      constexpr bool kE = decltype(emit)::value;
      CMqUnit& U = units[u];
      const uint32_t maxlen = L.bmax[b];
      unsigned long long* cur = L.wcur[wave];
      if (!maxlen) return;
      const int k = b * 64 + lane < kpb ? L.korder[b * 64 + lane] : kpb;
      MqCtx<NC> c = c0;
      if (k < kpb) {
        c.r0 = L.kstart[k];
        c.len = L.kstart[k + 1] - c.r0;
        c.keyv = ((((int64_t)k << lg) | bucket) * a.key_stride) + a.key_offset;
      }
      const int64_t kidx = k < kpb ? k : 0;
      if (U.kind == MQU_SEQ) {
        CMqQuery& Q = qc[U.q0];
        const unsigned long long rows = mq_seq<kE, NC>(L, c, Q, L.hot[U.q0], state_b + Q.st_off * ks + kidx, ks,
                                                       maxlen, kE ? cur[0] : 0ull);
        if (!kE && lane == 0) cur[0] = rows;
      } else if (U.kind == MQU_SEQ_BP) {
        mq_seq_bp<kE, NC>(L, c, U, qc, state_b + U.st_off * ks + kidx, ks, maxlen, cur);
      } else if (U.fast) {
        // the shapes built in (the rest run mq_agg_unit): compile time and
        // code size grow with every instance
        switch (U.fast) {
          case 1: mq_agg_fast<kE, NC, 4, 0, 0>(L, c, U, qc, state_b, kidx, ks, maxlen, cur); break;
          case 2: mq_agg_fast<kE, NC, 4, 1, 0>(L, c, U, qc, state_b, kidx, ks, maxlen, cur); break;
          default: mq_agg_fast<kE, NC, 4, 4, 0>(L, c, U, qc, state_b, kidx, ks, maxlen, cur); break;
        }
      } else if (U.nu == 8) {
        mq_agg_unit<kE, NC, 8, 1>(L, c, U, qc, state_b, kidx, ks, maxlen, cur);
      } else if (U.nu == 4) {
        mq_agg_unit<kE, NC, 4, 2>(L, c, U, qc, state_b, kidx, ks, maxlen, cur);
      } else {
        mq_agg_unit<kE, NC, 2, 4>(L, c, U, qc, state_b, kidx, ks, maxlen, cur);
      }
    };
    // Each item (unit x 64-key block) is complete inside its wave: a count
    // pass, one output reservation per query of the unit with rows (lane q
    // reserves for query q0 + q), the emit pass with the state commit.  No
    // workgroup barrier between the passes: waves run their items
    // independently, and a key's rows of one query come from one item, so
    // they stay in arrival order.  The emit pass re-reads the state the count
    // pass just read (L1 / L2).
    for (int it = wave; it < nitems; it += NWV) {
      const int u = __builtin_amdgcn_readfirstlane(it / nblk);
      const int b = __builtin_amdgcn_readfirstlane(it - u * nblk);
      const int q0 = units[u].q0, nqu = units[u].nq;
      for (int q = lane; q < nqu; q += 64) L.wcur[wave][q] = 0;
      wave_lds_sync();
      const uint64_t tu = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
      run_unit(std::false_type{}, u, b);
      MQ_UNIT_TICKS(0, u, tu);
      wave_lds_sync();
      for (int q = lane; q < nqu; q += 64) {
        const unsigned long long n = L.wcur[wave][q];
        L.wcur[wave][q] = n ? atomicAdd(qc[q0 + q].out_count, n) : 0ull;
      }
      wave_lds_sync();
      const uint64_t tv = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
      run_unit(std::true_type{}, u, b);
      MQ_UNIT_TICKS(1, u, tv);
    }
    MQ_STAMP(3);
    // the next window re-reads state this one wrote and reuses the LDS arrays
    if (t0 < ntiles) __syncthreads();
    MQ_STAMP(4);
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
