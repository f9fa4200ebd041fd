// gfx950 kernels of the closed-form fast path for the keyed pattern
//   partition with (k of A, k of B) begin
//     from every s1=A[f] -> s2=B[g] within W select ... insert into O;
//   end;
// (the Siddhi work behind AbstractSiddhiOperator.java:130 for BASELINE
// config 3; semantics: SURVEY.md App. A.3 — every A matches the next B of its
// key that passes g, if that B is within W of it; a B consumes every pending
// A it completes; A's older than W are pruned).
//
//   k_cfpart  one 1024-lane workgroup per 8192-row tile: 16-byte column
//             loads of every row a lane owns issued back to back, f / g as
//             term lists, rows no state can use dropped, LDS histogram over
//             the P key buckets, LDS scan, 16-byte records staged in LDS and
//             stored as one contiguous run per tile (coalesced).
//   k_cfwalk  one 1024-lane workgroup per key bucket (<= 512 keys): gathers
//             the bucket's segment of every tile (tile order = arrival
//             order), counting sort by key in LDS + arrival sort per key run,
//             closed-form matching (segmented next-B), one block scan for the
//             output rows, one atomic per window for the output cursor.  A
//             key's pending partials live in per-key SoA state in HBM; the
//             lane that owns the key prefetches its first two slots into
//             registers at kernel start, so the state read is off the
//             critical path.
//
// Versus k_partition / k_walk (kernels.hip) this path trades generality for
// 4x larger tiles and chunks: a bucket's segment per tile holds ~1.3
// records at config 3 (0.33 in the general path) and a walk workgroup
// resolves ~2.7 k records per launch instead of ~0.7 k.
#include <hip/hip_runtime.h>

#include "dev_common.h"
#include "kernels.h"
#include "vm.h"

namespace cep {

namespace {

constexpr uint16_t kNoB = 0xffff;
constexpr int kCfStageBytes = 48 * 1024;    // a tile keeps ~1/3 of its rows at config 3

// Block-wide exclusive scan of one value per thread, NT <= 1024 threads;
// scratch holds NT / 64 + 1 words.
template <int NT>
__device__ __forceinline__ uint32_t bscan(uint32_t v, uint32_t* scratch, uint32_t* total) {
  constexpr int NWV = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) scratch[wave + 1] = x;
  lds_barrier();
  if (wave == 0) {
    uint32_t s = (lane < NWV) ? scratch[lane + 1] : 0u;
#pragma unroll
    for (int o = 1; o < NWV; o <<= 1) {
      const uint32_t y = __shfl_up(s, o, 64);
      if (lane >= o) s += y;
    }
    if (lane < NWV) scratch[lane + 1] = s;   // inclusive prefix of wave totals
    if (lane == 0) scratch[0] = 0;
  }
  lds_barrier();
  const uint32_t r = scratch[wave] + x - v;
  *total = scratch[NWV];
  lds_barrier();
  return r;
}

// Record field accessors (w0).
__device__ __forceinline__ uint32_t rec_row(uint64_t w0) { return (uint32_t)(w0 >> 32) & 0x1fffu; }
__device__ __forceinline__ uint32_t rec_role(uint64_t w0) { return (uint32_t)(w0 >> 45) & 0x7u; }
__device__ __forceinline__ uint32_t rec_key(uint64_t w0) { return (uint32_t)(w0 >> 48); }

}  // namespace

// ============================================================== k_cfpart ==
template <int NW>
__global__ __launch_bounds__(kCfPartThreads) void k_cfpart(CfPartArgs a) {
  constexpr int E = kCfItems, NT = kCfPartThreads, RW = 1 + NW;
  constexpr int kStageRecs = kCfStageBytes / (8 * RW);
  __shared__ uint32_t scratch[NT / 64 + 1];
  __shared__ __attribute__((aligned(16))) uint64_t stage[kStageRecs * RW];
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];   // P + 1 (dynamic)
  const int tid = threadIdx.x;
  const int64_t tile = blockIdx.x;
  const PatternArgs& p = a.pat;
  const int lg = p.buckets_log2;
  const int P = 1 << lg;
  for (int i = tid; i <= P; i += NT) hist[i] = 0;

  const int64_t ts_base = a.rows.ts[a.rows.row0];
  if (tile == 0 && tid == 0) {
    a.chunk_base[0] = ts_base;
    a.chunk_base[1] = a.rows.seq0 + a.rows.row0;
  }
  const int64_t r0 = tile * kCfTile + (int64_t)tid * E;   // chunk-relative first row of this lane
  const int64_t nvalid = a.rows.n - r0;
  const int64_t row0 = a.rows.row0 + r0;                  // batch row
  uint32_t role_a = 0, role_b = 0;
  uint64_t tsv[E];
  uint64_t pv[kPref][E];
#pragma unroll
  for (int e = 0; e < E; ++e) tsv[e] = 0;
  if (nvalid > 0) {
    // issue every load of the lane's rows before any use (no branches between
    // them; unused prefetch slots repeat column col[0], set by the host)
    const bool full = nvalid >= 16;   // 16-byte loads of 1-byte columns stay in bounds
    const int64_t prev_ld = a.rows.ts[row0 > 0 ? row0 - 1 : row0];
    uint64_t sbytes = 0;
    if (full) {
      uint4 rt[E / 2], rc[kPref][E / 2];
      load_raw<E>(a.rows.ts, 8, row0, rt);
#pragma unroll
      for (int q = 0; q < kPref; ++q)
        load_raw<E>(a.rows.cols.p[a.pref.col[q]], type_width(a.rows.cols.t[a.pref.col[q]]), row0, rc[q]);
      if (a.rows.stream) sbytes = *(const __attribute__((address_space(1))) uint64_t*)(a.rows.stream + row0);
      decode<E>(rt, T_LONG, tsv);
#pragma unroll
      for (int q = 0; q < kPref; ++q) decode<E>(rc[q], a.rows.cols.t[a.pref.col[q]], pv[q]);
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        tsv[e] = e < nvalid ? (uint64_t)a.rows.ts[row0 + e] : 0;
        if (a.rows.stream && e < nvalid) sbytes |= (uint64_t)a.rows.stream[row0 + e] << (8 * e);
#pragma unroll
        for (int q = 0; q < kPref; ++q)
          pv[q][e] = (q < a.pref.n && e < nvalid)
                         ? load_col(a.rows.cols.p[a.pref.col[q]], a.rows.cols.t[a.pref.col[q]], row0 + e)
                         : 0;
      }
    }
    int64_t prev = row0 > 0 ? prev_ld : a.rows.prev_ts;
    uint32_t is_a = 0, is_b = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int sid = a.rows.stream ? (int)((sbytes >> (8 * e)) & 0xffu) : a.rows.input;
      if (e < nvalid) {
        is_a |= (sid == p.a_stream ? 1u : 0u) << e;
        is_b |= (sid == p.b_stream ? 1u : 0u) << e;
      }
    }
    if (p.within >= 0) {   // event-time order check (`within` pruning relies on it)
      bool bad = false;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (e < nvalid) {
          bad |= (int64_t)tsv[e] < prev;
          prev = (int64_t)tsv[e];
        }
      }
      if (bad) set_err(a.err, ERR_ORDER);
    }
    const uint32_t all = (1u << E) - 1u;
    if (is_a) role_a = is_a & (p.f_prog < 0 ? all : eval_terms_regs<E>(p.f_terms, a.pref.f_slot, a.rows.cols, pv));
    if (is_b) role_b = is_b & (p.g_raw_prog < 0 ? all : eval_terms_regs<E>(p.g_terms, a.pref.g_slot, a.rows.cols, pv));
  }
  lds_barrier();   // hist zeroed

  // bits 0-12 rank in tile, 13-24 bucket, 25-26 role (never all ones)
  uint32_t packed[E];
  uint32_t lkey[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    packed[e] = 0xffffffffu;
    lkey[e] = 0;
    const uint32_t role = ((role_a >> e) & 1u) * ROLE_A | ((role_b >> e) & 1u) * ROLE_B;
    if (!role) continue;
    const int64_t key = a.pref.key_slot >= 0 ? (int64_t)pick<E>(pv, a.pref.key_slot, e) : 0;
    if (key < 0 || (key % p.key_stride) != p.key_offset) {
      set_err(a.err, ERR_KEY_RANGE);
      continue;
    }
    const int64_t kfield = key / p.key_stride;
    if (kfield >= p.key_capacity) {
      set_err(a.err, ERR_KEY_RANGE);
      continue;
    }
    const uint32_t bucket = (uint32_t)(kfield & (P - 1));
    lkey[e] = (uint32_t)(kfield >> lg);
    const uint32_t rank = atomicAdd(&hist[bucket], 1u);
    packed[e] = (role << 25) | (bucket << 13) | rank;
  }
  lds_barrier();
  {
    // exclusive scan of the P bucket counts (P <= 4096: <= 4 per thread)
    const int per = (P + NT - 1) / NT;
    uint32_t c[4];
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid * per + i;
      c[i] = (i < per && idx < P) ? hist[idx] : 0u;
      sum += c[i];
    }
    uint32_t total;
    uint32_t off = bscan<NT>(sum, scratch, &total);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid * per + i;
      if (i < per && idx < P) {
        hist[idx] = off;
        off += c[i];
      }
    }
    if (tid == 0) hist[P] = total;
  }
  lds_barrier();
  const uint32_t total = hist[P];
  const bool staged = total <= (uint32_t)kStageRecs;   // uniform
  uint64_t* trecs = a.recs + tile * (int64_t)kCfTile * RW;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if (packed[e] == 0xffffffffu) continue;
    const uint32_t b = (packed[e] >> 13) & 0xfffu, rank = packed[e] & 0x1fffu;
    const uint32_t role = packed[e] >> 25;
    const uint32_t slot = hist[b] + rank;
    const int64_t dts = (int64_t)tsv[e] - ts_base;
    if (dts < 0 || dts > 0xffffffffll) set_err(a.err, ERR_ORDER);
    const uint64_t w0 = (uint64_t)(uint32_t)dts | ((uint64_t)(tid * E + e) << 32) |
                        ((uint64_t)role << 45) | ((uint64_t)lkey[e] << 48);
    const bool isa = (role & ROLE_A) != 0;
    uint64_t c0 = 0, c1 = 0;
    if (NW > 0) c0 = pick<E>(pv, isa ? a.cf.a_slot[0] : a.cf.b_slot[0], e);
    if (NW > 1) c1 = pick<E>(pv, isa ? a.cf.a_slot[1] : a.cf.b_slot[1], e);
    // explicit address spaces (a generic pointer would make these flat stores)
    if (staged) {
      stage[slot * RW] = w0;
      if (NW > 0) stage[slot * RW + 1] = c0;
      if (NW > 1) stage[slot * RW + 2] = c1;
    } else {
      uint64_t* g = trecs + (int64_t)slot * RW;
      g[0] = w0;
      if (NW > 0) g[1] = c0;
      if (NW > 1) g[2] = c1;
    }
  }
  uint16_t* toff = a.tile_off + tile * (int64_t)(P + 1);
  for (int i = tid; i <= P; i += NT) toff[i] = (uint16_t)hist[i];
  if (staged) {
    lds_barrier();
    // the tile's records are contiguous in HBM: 16-byte coalesced stores
    const int64_t words = (int64_t)total * RW;
    for (int64_t w = 2 * tid; w < words; w += 2 * NT) {
      if (w + 1 < words) *(uint4*)(trecs + w) = *(const uint4*)(stage + w);
      else trecs[w] = stage[w];
    }
  }
}

// ============================================================== k_cfwalk ==
namespace {

// Records per LDS window: 4096 with <= 1 carried word, 3072 with 2 (LDS).
template <int NW>
constexpr int cf_window() { return NW > 1 ? 3072 : kCfWindow; }

template <int NW, int WIN = cf_window<NW>()>
struct CfWalkLds {
  uint32_t seg[kCfMaxTiles + 1];       // exclusive prefix of the bucket's segment sizes
  uint16_t lo[kCfMaxTiles];            // segment start inside each tile's run
  uint32_t kstart[kCfMaxKeys + 1];     // key runs in `sorted`
  uint32_t kcur[kCfMaxKeys];           // counting-sort cursors
  uint32_t wts[WIN];             // ts - chunk ts base
  uint32_t wseq[WIN];            // chunk-relative row (arrival order)
  uint16_t wkr[WIN];             // key in bucket | role << 12
  uint16_t sorted[WIN];          // window slots grouped by key, arrival order per key
  union {
    struct {
      uint16_t nextb[WIN];       // sorted position of the next B of the key, or kNoB
      uint16_t v[WIN];           // output row offset per sorted position
    };
    uint16_t rowmap[kCfTile];          // oversize tile: segment index per tile row
  };
  uint16_t ord[kCfTile];               // oversize tile: segment indices in arrival order
  uint64_t wcap[NW > 0 ? NW : 1][WIN];   // physical carried words
  uint8_t cm[kCfMaxKeys];              // carried partials completed by the key's first B
  uint32_t scratch[kCfWalkThreads / 64 + 1];
  unsigned long long base;
};

// One output row.  acap = the A's logical captures, b0 / b1 = the completing
// B's physical words, bts / seq = its event ts and arrival number.
__device__ __forceinline__ void cf_emit(const CfWalkArgs& a, unsigned long long pos, int64_t key,
                                        uint64_t acap0, uint64_t acap1, uint64_t b0, uint64_t b1,
                                        int64_t bts, int64_t seq) {
  if ((int64_t)pos >= a.out.cap) {
    set_err(a.err, ERR_OUT_CAP);
    return;
  }
  for (int c = 0; c < a.out.ncols; ++c) {
    const int src = a.out.src[c];
    uint64_t v;
    if (src == SRC_KEY) {
      v = (uint64_t)key;
    } else if (src >= SRC_CAP && src < SRC_REC) {
      v = (src - SRC_CAP) == 0 ? acap0 : acap1;
    } else {
      const int ph = a.cf.bcol_phys[src - SRC_REC];
      v = ph < 0 ? (uint64_t)bts : (ph == 0 ? b0 : b1);
    }
    store_col(a.out.col[c], a.out.type[c], (int64_t)pos, v);
  }
  a.out.ts[pos] = bts;
  a.out.seq[pos] = seq;
}

}  // namespace

template <int NW>
__global__ __launch_bounds__(kCfWalkThreads) void k_cfwalk(CfWalkArgs a) {
  constexpr int NT = kCfWalkThreads, RW = 1 + NW, WIN = cf_window<NW>();
  __shared__ CfWalkLds<NW> L;
  const int tid = threadIdx.x;
  const PatternArgs& p = a.pat;
  const int lg = p.buckets_log2;
  const int P = 1 << lg;
  const int bucket = xcd_bucket(blockIdx.x, P);
  const int kpb = (int)((p.key_capacity + P - 1) >> lg);
  const int ntiles = a.ntiles;
  const int64_t ks = a.kstride;
  const int sw = p.slot_words;   // 2 + ncap
  const int S = p.pending_slots;
  const int64_t W = p.within;

  // ---- key lane (tid < kpb): pending count + slots 0 / 1 in registers,
  // loaded now so the state read overlaps the gather below
  const bool klane = tid < kpb;
  const int64_t kidx = (int64_t)bucket * kpb + tid;
  uint64_t* ksl = a.kslot + kidx;   // slot j word w: ksl[(j * sw + w) * ks]
  uint32_t hdr = klane ? a.khdr[kidx] : 0u;
  int n = (int)(hdr & 0xffu);
  // (named scalars, not an array: a dynamically indexed array lands in scratch)
  uint64_t s00 = 0, s01 = 0, s02 = 0, s03 = 0, s10 = 0, s11 = 0, s12 = 0, s13 = 0;
  auto load_regs = [&]() {
    s00 = n > 0 ? ksl[0] : 0ull;
    s01 = n > 0 ? ksl[ks] : 0ull;
    s02 = n > 0 && sw > 2 ? ksl[2 * ks] : 0ull;
    s03 = n > 0 && sw > 3 ? ksl[3 * ks] : 0ull;
    s10 = n > 1 ? ksl[(int64_t)sw * ks] : 0ull;
    s11 = n > 1 ? ksl[(int64_t)(sw + 1) * ks] : 0ull;
    s12 = n > 1 && sw > 2 ? ksl[(int64_t)(sw + 2) * ks] : 0ull;
    s13 = n > 1 && sw > 3 ? ksl[(int64_t)(sw + 3) * ks] : 0ull;
  };
  load_regs();
  const int64_t ts_base = a.chunk_base[0];
  const int64_t seq_base = a.chunk_base[1];
  for (int k = tid; k <= kpb; k += NT) L.kstart[k] = 0;

  // ---- the bucket's segment in every tile -> exclusive prefix over tiles
  {
    constexpr int TPT = kCfMaxTiles / NT;
    uint32_t cnt[TPT];
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < TPT; ++i) {
      const int t = tid * TPT + i;
      cnt[i] = 0;
      if (t < ntiles) {
        const uint16_t* o = a.tile_off + (int64_t)t * (P + 1) + bucket;
        const uint32_t lo = o[0], hi = o[1];
        L.lo[t] = (uint16_t)lo;
        cnt[i] = hi - lo;
      }
      sum += cnt[i];
    }
    uint32_t total;
    uint32_t off = bscan<NT>(sum, L.scratch, &total);
#pragma unroll
    for (int i = 0; i < TPT; ++i) {
      const int t = tid * TPT + i;
      if (t < ntiles) {
        L.seg[t] = off;
        off += cnt[i];
      }
    }
    if (tid == 0) L.seg[ntiles] = total;
  }
  lds_barrier();
  const uint32_t nall = L.seg[ntiles];

  // the closed form keeps, per key and window, `n` pending partials (slots
  // 0..n-1, ts-ordered) and walks the window's records of the key
  auto slot_word = [&](int j, int w) -> uint64_t {
    if (j >= 2) return ksl[((int64_t)j * sw + w) * ks];
    const uint64_t m0 = 0ull - (uint64_t)(w == 0), m1 = 0ull - (uint64_t)(w == 1);
    const uint64_t m2 = 0ull - (uint64_t)(w == 2), m3 = 0ull - (uint64_t)(w == 3);
    return j == 0 ? ((s00 & m0) | (s01 & m1) | (s02 & m2) | (s03 & m3))
                  : ((s10 & m0) | (s11 & m1) | (s12 & m2) | (s13 & m3));
  };

  // One LDS record per window position.
  auto put = [&](uint32_t pos, uint32_t trow, const uint4 x, uint64_t y) {
    const uint64_t w0 = ((uint64_t)x.y << 32) | x.x;
    const uint32_t k = rec_key(w0);
    L.wts[pos] = x.x;
    L.wseq[pos] = trow + rec_row(w0);
    L.wkr[pos] = (uint16_t)(k | (rec_role(w0) << 12));
    if (NW > 0) L.wcap[0][pos] = ((uint64_t)x.w << 32) | x.z;
    if (NW > 1) L.wcap[NW > 1 ? 1 : 0][pos] = y;
    atomicAdd(&L.kstart[k + 1], 1u);
  };

  // Windows are runs of whole tiles: a tile's segment is in bucket-rank
  // order, not arrival order, so a window never splits one — except a single
  // segment larger than a window (a key holding most of a tile), which is
  // first put in arrival order in LDS (`ord`; rows are unique in a tile) and
  // then walked in pieces.
  int t0 = 0;
  bool over = false;        // tile t0's segment is being walked in pieces
  uint32_t piece = 0;       // next piece start (index into ord)
  while (t0 < ntiles && L.seg[t0] < nall) {
    int t1 = t0;
    uint32_t nw;
    if (!over) {
      const uint32_t lim = L.seg[t0] + (uint32_t)WIN;
      int lo = t0, hi = ntiles;
      while (lo < hi) {   // largest t1 with seg[t1] <= lim (uniform)
        const int mid = (lo + hi + 1) >> 1;
        if (L.seg[mid] <= lim) lo = mid;
        else hi = mid - 1;
      }
      t1 = lo;
      if (t1 == t0) {
        // ---- oversize segment: arrival order by a scatter over tile rows
        over = true;
        piece = 0;
        const uint32_t c = L.seg[t0 + 1] - L.seg[t0];
        const uint64_t* tr = a.recs + ((int64_t)t0 * kCfTile + L.lo[t0]) * RW;
        for (int r = tid; r < kCfTile; r += NT) L.rowmap[r] = kNoB;
        lds_barrier();
        for (uint32_t j = tid; j < c; j += NT) L.rowmap[rec_row(tr[(int64_t)j * RW])] = (uint16_t)j;
        lds_barrier();
        constexpr int RPT = kCfTile / NT;
        uint32_t cnt = 0;
#pragma unroll
        for (int i = 0; i < RPT; ++i) cnt += L.rowmap[tid * RPT + i] != kNoB ? 1u : 0u;
        uint32_t total;
        uint32_t off = bscan<NT>(cnt, L.scratch, &total);
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
          const uint16_t j = L.rowmap[tid * RPT + i];
          if (j != kNoB) L.ord[off++] = j;
        }
        lds_barrier();
      }
    }
    if (over) {
      const uint32_t c = L.seg[t0 + 1] - L.seg[t0];
      nw = min((uint32_t)WIN, c - piece);
      const uint64_t* tr = a.recs + ((int64_t)t0 * kCfTile + L.lo[t0]) * RW;
      const uint32_t trow = (uint32_t)t0 * (uint32_t)kCfTile;
      for (uint32_t q = tid; q < nw; q += NT) {
        const uint64_t* r = tr + (int64_t)L.ord[piece + q] * RW;
        put(q, trow, gload4(r), NW > 1 ? r[2] : 0ull);
      }
    } else {
      nw = L.seg[t1] - L.seg[t0];
      // ---- gather whole tiles (tile order = arrival order)
      const uint32_t wb = L.seg[t0];
      constexpr int TPT = kCfMaxTiles / NT;
#pragma unroll
      for (int i = 0; i < TPT; ++i) {
        const int t = tid * TPT + i;
        if (t < t0 || t >= t1) continue;
        const uint32_t s0 = L.seg[t], s1 = L.seg[t + 1];
        if (s0 >= s1) continue;
        const uint32_t trow = (uint32_t)t * (uint32_t)kCfTile;
        const uint64_t* tr = a.recs + ((int64_t)t * kCfTile + L.lo[t]) * RW;
        for (uint32_t g = s0; g < s1; g += 2) {
          // two independent record loads in flight per step
          const bool two = g + 1 < s1;
          const uint64_t* r = tr + (int64_t)(g - s0) * RW;
          const uint4 x0 = gload4(r);
          const uint4 x1 = two ? gload4(r + RW) : make_uint4(0, 0, 0, 0);
          const uint64_t y0 = NW > 1 ? r[2] : 0ull;
          const uint64_t y1 = (NW > 1 && two) ? r[RW + 2] : 0ull;
          put(g - wb, trow, x0, y0);
          if (two) put(g + 1 - wb, trow, x1, y1);
        }
      }
    }
    lds_barrier();
    // ---- counting sort by key
    {
      const uint32_t c = tid < kpb ? L.kstart[tid + 1] : 0u;
      uint32_t total;
      const uint32_t off = bscan<NT>(c, L.scratch, &total);
      if (tid < kpb) {
        L.kstart[tid] = off;
        L.kcur[tid] = off;
      }
      if (tid == 0) L.kstart[kpb] = total;
    }
    lds_barrier();
    for (uint32_t w = tid; w < nw; w += NT) {
      const uint32_t slot = atomicAdd(&L.kcur[L.wkr[w] & 0xfffu], 1u);
      L.sorted[slot] = (uint16_t)w;
    }
    lds_barrier();

    // ---- key lanes: arrival order per run, next-B links, carried matches
    uint32_t r0 = 0, r1 = 0;
    int fb = -1, lb = -1;            // first / last B (sorted positions)
    int64_t last_a_ts = INT64_MIN;
    int cfirst = 0, cm = 0;
    if (klane) {
      r0 = L.kstart[tid];
      r1 = L.kstart[tid + 1];
      const uint32_t len = r1 - r0;
      if (len > 1) {
        for (uint32_t gap = len > 64 ? len / 3 : 1;; gap = gap / 3 ? gap / 3 : 1) {
          for (uint32_t i = r0 + gap; i < r1; ++i) {
            const uint16_t x = L.sorted[i];
            const uint32_t sx = L.wseq[x];
            uint32_t j = i;
            while (j >= r0 + gap && L.wseq[L.sorted[j - gap]] > sx) {
              L.sorted[j] = L.sorted[j - gap];
              j -= gap;
            }
            L.sorted[j] = x;
          }
          if (gap == 1) break;
        }
      }
      uint16_t nb = kNoB;
      for (uint32_t q = r1; q-- > r0;) {
        const uint16_t x = L.sorted[q];
        const uint32_t role = (uint32_t)L.wkr[x] >> 12;
        L.nextb[q] = nb;
        if (role & ROLE_B) {
          nb = (uint16_t)q;
          if (lb < 0) lb = (int)q;
        }
        if ((role & ROLE_A) && last_a_ts == INT64_MIN) last_a_ts = ts_base + (int64_t)L.wts[x];
      }
      fb = nb == kNoB ? -1 : (int)nb;
      if (r1 > r0 && fb >= 0 && n > 0) {
        const int64_t tb = ts_base + (int64_t)L.wts[L.sorted[fb]];
        cfirst = n;
        for (int j = 0; j < n; ++j) {
          const int64_t d = tb - (int64_t)slot_word(j, 0);
          if (W < 0 || (d < 0 ? -d : d) <= W) {
            cfirst = j;
            break;
          }
        }
        cm = n - cfirst;
      }
      L.cm[tid] = (uint8_t)cm;
    }
    lds_barrier();

    // ---- match flag per sorted position (+ carried matches at run start)
    {
      constexpr int PER = WIN / NT;
      uint32_t vals[PER];
      uint32_t sum = 0;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const uint32_t q = tid * PER + i;
        uint32_t val = 0;
        if (q < nw) {
          const uint16_t x = L.sorted[q];
          const uint32_t kr = L.wkr[x];
          const uint32_t k = kr & 0xfffu;
          if (((kr >> 12) & ROLE_A) && L.nextb[q] != kNoB) {
            const int64_t d = (int64_t)L.wts[L.sorted[L.nextb[q]]] - (int64_t)L.wts[x];
            val = (W < 0 || (d < 0 ? -d : d) <= W) ? 1u : 0u;
          }
          if (q == L.kstart[k]) val += L.cm[k];
        }
        vals[i] = val;
        sum += val;
      }
      uint32_t total;
      uint32_t off = bscan<NT>(sum, L.scratch, &total);
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const uint32_t q = tid * PER + i;
        if (q < (uint32_t)WIN) L.v[q] = (uint16_t)off;
        off += vals[i];
      }
      if (tid == 0) L.base = total ? atomicAdd(a.out.count, (unsigned long long)total) : 0ull;
    }
    lds_barrier();
    const unsigned long long base = L.base;

    // ---- emit record matches (lane per sorted position; LDS reads + stores)
    for (uint32_t q = tid; q < nw; q += NT) {
      const uint16_t x = L.sorted[q];
      const uint32_t kr = L.wkr[x];
      if (!((kr >> 12) & ROLE_A) || L.nextb[q] == kNoB) continue;
      const uint16_t xb = L.sorted[L.nextb[q]];
      const int64_t d = (int64_t)L.wts[xb] - (int64_t)L.wts[x];
      if (W >= 0 && (d < 0 ? -d : d) > W) continue;
      const uint32_t k = kr & 0xfffu;
      const uint32_t extra = q == L.kstart[k] ? L.cm[k] : 0u;
      const int64_t ats = ts_base + (int64_t)L.wts[x];
      const int64_t bts = ts_base + (int64_t)L.wts[xb];
      const uint64_t a0 = NW > 0 ? L.wcap[0][x] : 0ull, a1 = NW > 1 ? L.wcap[NW > 1 ? 1 : 0][x] : 0ull;
      const int cp0 = a.cf.cap_phys[0], cp1 = a.cf.cap_phys[1];
      const uint64_t c0 = cp0 < 0 ? (uint64_t)ats : (cp0 == 0 ? a0 : a1);
      const uint64_t c1 = cp1 < 0 ? (uint64_t)ats : (cp1 == 0 ? a0 : a1);
      const int64_t kl = ((int64_t)k << lg) | bucket;
      cf_emit(a, base + L.v[q] + extra, kl * p.key_stride + p.key_offset, c0, c1,
              NW > 0 ? L.wcap[0][xb] : 0ull, NW > 1 ? L.wcap[NW > 1 ? 1 : 0][xb] : 0ull, bts,
              seq_base + (int64_t)L.wseq[xb]);
    }

    // ---- key lanes: carried matches, survivors, state commit
    if (klane && r1 > r0) {
      const int64_t kl = ((int64_t)tid << lg) | bucket;
      const int64_t kv = kl * p.key_stride + p.key_offset;
      if (cm) {
        const uint16_t xb = L.sorted[fb];
        const int64_t bts = ts_base + (int64_t)L.wts[xb];
        const uint64_t b0 = NW > 0 ? L.wcap[0][xb] : 0ull, b1 = NW > 1 ? L.wcap[NW > 1 ? 1 : 0][xb] : 0ull;
        for (int j = 0; j < cm; ++j) {
          const int js = cfirst + j;
          cf_emit(a, base + L.v[r0] + j, kv, slot_word(js, 2), slot_word(js, 3), b0, b1, bts,
                  seq_base + (int64_t)L.wseq[xb]);
        }
      }
      const bool prune = W >= 0 && last_a_ts != INT64_MIN;
      int nn = 0;
      if (lb < 0) {
        // no B: the carried partials survive, minus those pruned by the
        // run's last start (ts-ordered, so a prefix)
        int drop = 0;
        while (drop < n && prune && last_a_ts - (int64_t)slot_word(drop, 0) > W) ++drop;
        if (drop) {
          for (int j = drop; j < n; ++j)
            for (int w = 0; w < sw; ++w) ksl[((int64_t)(j - drop) * sw + w) * ks] = slot_word(j, w);
        }
        nn = n - drop;
      }
      // partials created after the last B (a record that is both B and A
      // starts a partial after completing others)
      for (uint32_t q = (lb < 0 ? r0 : (uint32_t)lb); q < r1; ++q) {
        const uint16_t x = L.sorted[q];
        if (!((L.wkr[x] >> 12) & ROLE_A)) continue;
        const int64_t ats = ts_base + (int64_t)L.wts[x];
        if (prune && last_a_ts - ats > W) continue;
        if (nn >= S) {
          set_err(a.err, ERR_PENDING);
          break;
        }
        const uint64_t a0 = NW > 0 ? L.wcap[0][x] : 0ull, a1 = NW > 1 ? L.wcap[NW > 1 ? 1 : 0][x] : 0ull;
        uint64_t* dst = ksl + (int64_t)nn * sw * ks;
        dst[0] = (uint64_t)ats;
        dst[ks] = (uint64_t)(seq_base + (int64_t)L.wseq[x]);
        for (int c = 0; c < sw - 2; ++c) {
          const int cp = a.cf.cap_phys[c];
          dst[(2 + c) * ks] = cp < 0 ? (uint64_t)ats : (cp == 0 ? a0 : a1);
        }
        ++nn;
      }
      n = nn;
      hdr = (hdr & ~0xffu) | (uint32_t)nn;
      a.khdr[kidx] = hdr;
    }
    if (over) {
      piece += nw;
      if (piece >= L.seg[t0 + 1] - L.seg[t0]) {
        over = false;
        t0 = t0 + 1;
      }
    } else {
      t0 = t1;
    }
    if (!over && (t0 >= ntiles || L.seg[t0] >= nall)) break;
    // next window: the key lanes re-read the slots they just wrote; the LDS
    // arrays are reused
    __syncthreads();
    if (klane) load_regs();
    for (int k = tid; k <= kpb; k += NT) L.kstart[k] = 0;
    lds_barrier();
  }
}

void launch_cf_partition(const CfPartArgs& a, int64_t ntiles, hipStream_t s) {
  const int P = 1 << a.pat.buckets_log2;
  const size_t dyn = ((size_t)(P + 1) * 4 + 15) & ~(size_t)15;
  switch (a.cf.nw) {
    case 0: hipLaunchKernelGGL(k_cfpart<0>, dim3((unsigned)ntiles), dim3(kCfPartThreads), dyn, s, a); break;
    case 1: hipLaunchKernelGGL(k_cfpart<1>, dim3((unsigned)ntiles), dim3(kCfPartThreads), dyn, s, a); break;
    default: hipLaunchKernelGGL(k_cfpart<2>, dim3((unsigned)ntiles), dim3(kCfPartThreads), dyn, s, a); break;
  }
}

void launch_cf_walk(const CfWalkArgs& a, int nbuckets, hipStream_t s) {
  switch (a.cf.nw) {
    case 0: hipLaunchKernelGGL(k_cfwalk<0>, dim3((unsigned)nbuckets), dim3(kCfWalkThreads), 0, s, a); break;
    case 1: hipLaunchKernelGGL(k_cfwalk<1>, dim3((unsigned)nbuckets), dim3(kCfWalkThreads), 0, s, a); break;
    default: hipLaunchKernelGGL(k_cfwalk<2>, dim3((unsigned)nbuckets), dim3(kCfWalkThreads), 0, s, a); break;
  }
}

}  // namespace cep
