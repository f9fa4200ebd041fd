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
// Order-tolerant records (TOL builds, cep_options.ts_order 0): a B-stream row
// that fails g is kept with this role — it completes nothing but expires the
// partials it is more than W away from (App. A.3, on every event of the
// waiting stream) — and record ts are stored as ts - chunk base + 2^31.
constexpr uint32_t kRolePB = 4;
constexpr int64_t kTolBias = 1ll << 31;
// skr bit 15 (TOL walk): the A at this sorted position survives every B-stream
// row up to its next g-passing B (or to the end of its run)
constexpr uint32_t kSkrAlive = 0x8000u;
constexpr int kCfStageBytes = (kCfTile / 8192 * 20 + 36) * 1024;    // a tile keeps ~1/3 of its rows at config 3

// Diagnostics (CEP_STAMPS=1): s_memtime at phase i of block b.
#ifdef CF_WAVESTAMP
#define CF_STAMP(i) do { } while (0)
#else
#define CF_STAMP(i)                                                                 \
  do {                                                                              \
    if (a.stamps && threadIdx.x == 0 && blockIdx.x < 4096)                          \
      a.stamps[(int64_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memtime();      \
  } while (0)
#endif

// Diagnostics build (-DCF_WAVESTAMP, CEP_STAMPS=1): window 0 of each block,
// slot 0 = wave 0 after the output-scan barrier, slots 1-8 = each wave at the
// end of its key-lane commit, slots 9-15 = waves 0-6 at the end of the
// record emission (which wave holds the window-end barrier, and why).
#ifdef CF_WAVESTAMP
#define CF_WSTAMP(slot)                                                             \
  do {                                                                              \
    if (a.stamps && (threadIdx.x & 63) == 0 && blockIdx.x < 4096 && wi == 0 &&     \
        (slot) < 16)                                                                \
      a.stamps[(int64_t)blockIdx.x * 16 + (slot)] = __builtin_amdgcn_s_memtime();  \
  } while (0)
#else
#define CF_WSTAMP(slot) do { } while (0)
#endif

// Diagnostics (CEP_STAMPS=1 CEP_ABLATE=256): event counters of the walk (last launch).
#define CF_COUNT(i, v)                                                                       \
  do {                                                                                       \
    if (a.stamps && (a.ablate & 256))                                                        \
      atomicAdd((unsigned long long*)&a.stamps[4095 * 16 + (i)], (unsigned long long)(v));   \
  } while (0)

// Carried word of each row: slot sa on A rows (role_a bit set), sb otherwise;
// both slots uniform.
template <int E, int Q = kPref>
__device__ __forceinline__ void pick_carried(const uint64_t (&pv)[Q][E], int sa, int sb,
                                             uint32_t role_a, uint64_t (&out)[E]) {
  take_slot<E, Q>(pv, sa, out);
  if (sb != sa) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      if (sb == q) {
        asm volatile("");
#pragma unroll
        for (int e = 0; e < E; ++e) out[e] = ((role_a >> e) & 1u) ? out[e] : pv[q][e];
      }
    }
  }
}

// Record field accessors (w0).
__device__ __forceinline__ uint32_t rec_row(uint64_t w0) { return (uint32_t)(w0 >> 32) & 0x1fffu; }
__device__ __forceinline__ uint32_t rec_role(uint64_t w0) { return (uint32_t)(w0 >> 45) & 0x7u; }
__device__ __forceinline__ uint32_t rec_key(uint64_t w0) { return (uint32_t)(w0 >> 48); }

}  // namespace

// ============================================================== k_cfpart ==
#ifndef CF_PART_MINW   // waves per SIMD the register budget is set for
#define CF_PART_MINW (kCfPartThreads == 512 ? 4 : 1)
#endif
// FR: rows are received shuffle records; NP prefetched columns; TOL: order-tolerant records
template <int NW, bool FR, int NP = kPref, bool TOL = false>
__global__ __launch_bounds__(kCfPartThreads, CF_PART_MINW) void k_cfpart(CfPartArgs a) {
  constexpr int E = kCfItems, NT = kCfPartThreads, RW = 1 + NW;
  // received records (FR: every row is kept) and order-tolerant tiles (~3/4
  // kept) need a larger stage to store their tile as one coalesced run; the
  // kernel runs one workgroup per CU either way (128 VGPRs x 1024 lanes)
  constexpr int kStageBytesT = (FR || TOL) ? 128 * 1024 : kCfStageBytes;
  constexpr int kStageRecs = kStageBytesT / (8 * RW);
  __shared__ uint32_t scratch[NT / 64 + 1];
  __shared__ __attribute__((aligned(16))) uint64_t stage[kStageRecs * RW];
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];   // NB + 1 (dynamic)
  const int tid = threadIdx.x;
  const int64_t tile = xcd_tile(blockIdx.x, a.ntiles);
  const PatternArgs& p = a.pat;
  const int lg = p.buckets_log2;
  const int P = 1 << lg;
  const int NB = P + a.nhot;   // key buckets, then one bucket per hot key (hot.hip)
  CF_STAMP(0);
  for (int i = tid; i <= NB; i += NT) hist[i] = 0;

  const int64_t ts_base = FR ? (int64_t)a.in_recs[a.rows.row0 * a.in_rec_words + 2] : a.rows.ts[a.rows.row0];
  if (tile == 0 && tid == 0) {
    a.chunk_base[0] = ts_base;
    a.chunk_base[1] = FR ? (int64_t)a.in_recs[a.rows.row0 * a.in_rec_words + 1] : a.rows.seq0 + a.rows.row0;
  }
  // Lane-interleaved rows: lane l of wave w owns rows w*64*E + 64*e + l
  // (e < E), so every load instruction reads one contiguous 64-row segment
  // of a column (fully coalesced).
  const int lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = tile * kCfTile + (int64_t)wave * 64 * E + lane;   // chunk-relative row of e = 0
  const int64_t row0 = a.rows.row0 + r0;                                 // batch row of e = 0
  uint32_t valid = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) valid |= (r0 + 64 * e < a.rows.n ? 1u : 0u) << e;
  uint32_t role_a = 0, role_b = 0, role_pb = 0;
  uint64_t tsv[E];
  uint64_t pv[NP][E];
#pragma unroll
  for (int e = 0; e < E; ++e) tsv[e] = 0;
  uint64_t fkey[E], fc0[E], fc1[E];   // key and carried words per row
#pragma unroll
  for (int e = 0; e < E; ++e) fkey[e] = fc0[e] = fc1[e] = 0;
  if (FR && valid) {
    // received records: roles and keys were computed by the sender (k_route)
    const int rw = a.in_rec_words;
    uint64_t hv[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const bool ok = (valid >> e) & 1u;
      const uint64_t* r = a.in_recs + (row0 + 64 * e) * rw;
      hv[e] = ok ? r[0] : 0ull;
      tsv[e] = ok ? r[2] : 0ull;
      const bool isa = ((hv[e] >> 32) & ROLE_A) != 0;
      fc0[e] = (ok && NW > 0) ? r[3 + (isa ? a.cf.a_log[0] : a.cf.b_log[0])] : 0ull;
      fc1[e] = (ok && NW > 1) ? r[3 + (isa ? a.cf.a_log[1] : a.cf.b_log[1])] : 0ull;
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint32_t role = (uint32_t)(hv[e] >> 32) & 0xffu;
      role_a |= ((role & ROLE_A) ? 1u : 0u) << e;
      role_b |= ((role & ROLE_B) && (role & ROLE_G) ? 1u : 0u) << e;
      fkey[e] = (uint64_t)(uint32_t)hv[e];
    }
    if (p.within >= 0) {
      const int64_t before = row0 > 0 ? (int64_t)a.in_recs[(row0 - 1) * rw + 2] : batch_prev_ts(a.rows);
      bool bad = false;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const uint64_t up = __shfl_up(tsv[e], 1, 64);
        const uint64_t last = e > 0 ? __shfl(tsv[e > 0 ? e - 1 : 0], 63, 64) : 0ull;
        const int64_t prev = lane > 0 ? (int64_t)up : (e > 0 ? (int64_t)last : before);
        if ((valid >> e) & 1u) bad |= (int64_t)tsv[e] < prev;
      }
      if (bad) report_descent(a.rows, a.err);
    }
  }
  if (!FR && valid) {
    uint32_t sb[E];
    cf_load_cols<E, NP>(a.rows, a.pref, a.ts_slot, row0, valid, tsv, sb, pv);
    uint32_t is_a = 0, is_b = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if ((valid >> e) & 1u) {
        is_a |= ((int)sb[e] == p.a_stream ? 1u : 0u) << e;
        is_b |= ((int)sb[e] == p.b_stream ? 1u : 0u) << e;
      }
    }
    if (p.within >= 0 && !TOL) {
      // event-time order check (`within` pruning relies on it): row r - 1 is
      // held by the previous lane (same e), lane 63 (e - 1), or loaded
      const int64_t before = row0 > 0 ? a.rows.ts[row0 - 1] : batch_prev_ts(a.rows);
      bool bad = false;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const uint64_t up = __shfl_up(tsv[e], 1, 64);
        const uint64_t last = e > 0 ? __shfl(tsv[e > 0 ? e - 1 : 0], 63, 64) : 0ull;
        const int64_t prev = lane > 0 ? (int64_t)up : (e > 0 ? (int64_t)last : before);
        if ((valid >> e) & 1u) bad |= (int64_t)tsv[e] < prev;
      }
      if (bad) report_descent(a.rows, a.err);
    }
    const uint32_t all = (1u << E) - 1u;
    if (is_a) role_a = is_a & (p.f_prog < 0 ? all : eval_terms_regs<E, NP>(p.f_terms, a.pref.f_slot, a.rows.cols, pv));
    if (is_b) role_b = is_b & (p.g_raw_prog < 0 ? all : eval_terms_regs<E, NP>(p.g_terms, a.pref.g_slot, a.rows.cols, pv));
    if (TOL) role_pb = is_b & ~role_b;
    // key (the host puts the key column in slot 0) and carried words (A
    // rows: the A's columns, else the B's) picked now, so pv dies here
    if (NW > 0) pick_carried<E, NP>(pv, a.cf.a_slot[0], a.cf.b_slot[0], role_a, fc0);
    if (NW > 1) pick_carried<E, NP>(pv, a.cf.a_slot[1], a.cf.b_slot[1], role_a, fc1);
    if (a.pref.key_slot >= 0) {
#pragma unroll
      for (int e = 0; e < E; ++e) fkey[e] = pv[0][e];
    }
  }
  lds_barrier();   // hist zeroed
  CF_STAMP(1);

  // bits 0-12 rank in tile, 13-24 bucket, 25-27 role (never all ones)
  uint32_t packed[E];
  uint32_t lkey[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    packed[e] = 0xffffffffu;
    lkey[e] = 0;
    const uint32_t role = ((role_a >> e) & 1u) * ROLE_A | ((role_b >> e) & 1u) * ROLE_B |
                          (TOL ? ((role_pb >> e) & 1u) * kRolePB : 0u);
    if (!role) continue;
    int64_t key;
    key = (int64_t)fkey[e];
    const int64_t kfield = shard_key(key, p.key_stride, p.key_offset);
    if (kfield < 0 || kfield >= p.key_capacity) {
      set_err(a.err, ERR_KEY_RANGE);
      continue;
    }
    uint32_t bucket = (uint32_t)(kfield & (P - 1));
    lkey[e] = (uint32_t)(kfield >> lg);
    if (a.nhot) {
      const uint32_t hs = a.hot_id[kfield];
      if (hs != kNotHot) {   // hot key: its own bucket; the key field holds the slot
        bucket = (uint32_t)P + hs;
        lkey[e] = hs;
      }
    }
    const uint32_t rank = atomicAdd(&hist[bucket], 1u);
    packed[e] = (role << 25) | (bucket << 13) | rank;
  }
  lds_barrier();
  CF_STAMP(2);
  {
    // exclusive scan of the NB bucket counts (NB <= 4096: <= 8 per thread)
    constexpr int MAXPER = kCfMaxBuckets / NT;
    const int per = (NB + NT - 1) / NT;
    uint32_t c[MAXPER];
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < MAXPER; ++i) {
      const int idx = tid * per + i;
      c[i] = (i < per && idx < NB) ? hist[idx] : 0u;
      sum += c[i];
    }
    uint32_t total;
    uint32_t off = bscan<NT>(sum, scratch, &total);
#pragma unroll
    for (int i = 0; i < MAXPER; ++i) {
      const int idx = tid * per + i;
      if (i < per && idx < NB) {
        hist[idx] = off;
        off += c[i];
      }
    }
    if (tid == 0) hist[NB] = total;
  }
  lds_barrier();
  CF_STAMP(3);
  const uint32_t total = hist[NB];
  const bool staged = total <= (uint32_t)kStageRecs;   // uniform
  uint64_t* trecs = a.recs + tile * (int64_t)kCfTile * RW;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if (packed[e] == 0xffffffffu) continue;
    const uint32_t b = (packed[e] >> 13) & 0xfffu;
    const uint32_t role = packed[e] >> 25;
    const uint32_t slot = hist[b] + (packed[e] & 0x1fffu);
    const int64_t dts = (int64_t)tsv[e] - ts_base + (TOL ? kTolBias : 0);
    if (dts < 0) {
      if (TOL) set_err(a.err, ERR_TS_SPAN);
      else report_descent(a.rows, a.err);
    } else if (dts > 0xffffffffll) {
      set_err(a.err, ERR_TS_SPAN);
    }
    const uint64_t w0 = (uint64_t)(uint32_t)dts | ((uint64_t)(wave * 64 * E + 64 * e + lane) << 32) |
                        ((uint64_t)role << 45) | ((uint64_t)lkey[e] << 48);
    const uint64_t c0 = fc0[e], c1 = fc1[e];
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
  for (int i = tid; i <= NB; i += NT) a.tile_off[(int64_t)i * a.ntiles + tile] = (uint16_t)hist[i];
  if (staged) {
    lds_barrier();
    CF_STAMP(4);
    // the tile's records are contiguous in HBM: 16-byte coalesced stores
    const int64_t words = (int64_t)total * RW;
    for (int64_t w = 2 * tid; w < words; w += 2 * NT) {
      if (w + 1 < words) *(uint4*)(trecs + w) = *(const uint4*)(stage + w);
      else trecs[w] = stage[w];
    }
  }
  CF_STAMP(5);
}

// ============================================================= k_cfroute ==
// Sender side of the key shuffle: the k_cfpart load path,
// predicate push-down (rows no state can use are not shipped), owner =
// key % world, owner ranks stable in arrival order (wave ballots per owner,
// then a prefix over waves), wide records [key | role << 32 | stream << 40,
// global seq, ts, logical carried words] staged in LDS and stored as one
// contiguous owner-grouped run per tile.  k_route_scan / k_route_gather
// (kernels.hip) then make each owner's records contiguous.
constexpr int kCfRouteStage = 112 * 1024;   // bytes of staged wide records
constexpr int kRouteSmallWorld = 8;          // owners ranked with scalar counters
__global__ __launch_bounds__(kCfPartThreads, 1) void k_cfroute(CfRouteArgs ca) {
  constexpr int E = kCfItems, NT = kCfPartThreads, NWV = NT / 64;
  const RouteArgs& a = ca.r;
  const PatternArgs& p = a.pat;
  __shared__ uint32_t wcnt[NWV][kMaxWorld];   // per wave, per owner: rows so far / then wave base
  __shared__ uint32_t obase[kMaxWorld + 1];   // owner segment starts in the tile
  __shared__ __attribute__((aligned(16))) uint64_t stage[kCfRouteStage / 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int world = a.world, wrw = a.wrw;
  const int64_t tile = blockIdx.x;
  for (int i = tid; i < NWV * kMaxWorld; i += NT) wcnt[i / kMaxWorld][i % kMaxWorld] = 0;

  const int64_t r0 = tile * kCfTile + (int64_t)wave * 64 * E + lane;
  const int64_t row0 = a.rows.row0 + r0;
  uint32_t valid = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) valid |= (r0 + 64 * e < a.rows.n ? 1u : 0u) << e;
  uint64_t tsv[E], pv[kPref][E];
#pragma unroll
  for (int e = 0; e < E; ++e) tsv[e] = 0;
  uint32_t is_a = 0, role_a = 0, role_b = 0, role_g = 0;
  uint64_t fkey[E], fc0[E], fc1[E];
#pragma unroll
  for (int e = 0; e < E; ++e) fkey[e] = fc0[e] = fc1[e] = 0;
  if (valid) {
    uint32_t sb[E];
    cf_load_cols<E>(a.rows, ca.pref, ca.ts_slot, row0, valid, tsv, sb, pv);
    uint32_t is_b = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if ((valid >> e) & 1u) {
        is_a |= ((int)sb[e] == p.a_stream ? 1u : 0u) << e;
        is_b |= ((int)sb[e] == p.b_stream ? 1u : 0u) << e;
      }
    }
    const uint32_t all = (1u << E) - 1u;
    if (is_a) role_a = is_a & (p.f_prog < 0 ? all : eval_terms_regs<E>(p.f_terms, ca.pref.f_slot, a.rows.cols, pv));
    if (is_b) {
      if (p.g_walk_prog >= 0) {   // g reads s1: decided by the owner's walk
        role_b = is_b;
      } else {
        role_b = is_b & (p.g_raw_prog < 0 ? all : eval_terms_regs<E>(p.g_terms, ca.pref.g_slot, a.rows.cols, pv));
        role_g = role_b;
      }
    }
    // logical carried words: the A stream's columns on A rows, else the B's
    if (p.nrec_a > 0 || p.nrec_b > 0)
      pick_carried<E>(pv, p.nrec_a > 0 ? ca.pref.reca_slot[0] : -1, p.nrec_b > 0 ? ca.pref.recb_slot[0] : -1,
                      is_a, fc0);
    if (p.nrec_a > 1 || p.nrec_b > 1)
      pick_carried<E>(pv, p.nrec_a > 1 ? ca.pref.reca_slot[1] : -1, p.nrec_b > 1 ? ca.pref.recb_slot[1] : -1,
                      is_a, fc1);
    if (ca.pref.key_slot >= 0) {
#pragma unroll
      for (int e = 0; e < E; ++e) fkey[e] = pv[0][e];
    }
  }
  __syncthreads();   // wcnt zeroed

  // owner per kept row, stable rank inside (wave, owner): rows of a wave are
  // in arrival order by (e, lane)
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int dest[E];
  uint32_t wr[E];
  uint32_t pre[kRouteSmallWorld];   // world <= 8: rows per owner so far in this wave (uniform)
#pragma unroll
  for (int d = 0; d < kRouteSmallWorld; ++d) pre[d] = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    dest[e] = -1;
    wr[e] = 0;
    if ((((role_a | role_b) >> e) & 1u)) {
      const int64_t key = (int64_t)fkey[e];
      if (key < 0 || key > 0xffffffffll) set_err(a.err, ERR_KEY_RANGE);
      else dest[e] = (int)((uint32_t)key % (uint32_t)world);
    }
    if (world > kRouteSmallWorld) {
      // owners met in this row group, one at a time (counts in LDS)
      uint64_t rem = __ballot(dest[e] >= 0);
      while (rem) {
        const int leader = __ffsll((long long)rem) - 1;
        const int d0 = __shfl(dest[e], leader, 64);
        const uint64_t m = __ballot(dest[e] == d0);
        const uint32_t c0 = wcnt[wave][d0];
        if (dest[e] == d0) wr[e] = c0 + (uint32_t)__popcll(m & lt);
        if (lane == leader) wcnt[wave][d0] = c0 + (uint32_t)__popcll(m);
        rem &= ~m;
      }
    } else {
      // every owner, counts in scalar registers: no LDS round trip per owner
#pragma unroll
      for (int d = 0; d < kRouteSmallWorld; ++d) {
        const uint64_t m = __ballot(dest[e] == d);
        if (dest[e] == d) wr[e] = pre[d] + (uint32_t)__popcll(m & lt);
        pre[d] += (uint32_t)__popcll(m);
      }
    }
  }
  if (world <= kRouteSmallWorld) {
    uint32_t mine = 0;
#pragma unroll
    for (int d = 0; d < kRouteSmallWorld; ++d) mine = lane == d ? pre[d] : mine;
    if (lane < kRouteSmallWorld) wcnt[wave][lane] = mine;
  }
  __syncthreads();
  // tile totals per owner -> owner segment starts; per (wave, owner) bases
  if (tid < 64) {
    uint32_t tot = 0;
    if (tid < world)
      for (int w = 0; w < NWV; ++w) tot += wcnt[w][tid];
    uint32_t x = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (tid < world) {
      obase[tid] = x - tot;
      a.tcount[tile * world + tid] = tot;
    }
    if (tid == 63) obase[world] = x;   // kept rows of the tile
  }
  __syncthreads();
  if (tid < world) {
    uint32_t run = obase[tid];
    for (int w = 0; w < NWV; ++w) {
      const uint32_t c = wcnt[w][tid];
      wcnt[w][tid] = run;
      run += c;
    }
  }
  __syncthreads();
  const uint32_t total = obase[world];
  const bool staged = (int64_t)total * wrw * 8 <= kCfRouteStage;   // uniform
  uint64_t* tout = a.arena + tile * (int64_t)kCfTile * wrw;
  const int nrc = wrw - 3;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if (dest[e] < 0) continue;
    const uint32_t pos = wcnt[wave][dest[e]] + wr[e];
    const uint32_t role = ((role_a >> e) & 1u) * ROLE_A | ((role_b >> e) & 1u) * ROLE_B |
                          ((role_g >> e) & 1u) * ROLE_G;
    const int64_t r = row0 + 64 * e;
    uint64_t w[5];
    const uint32_t sid = ((is_a >> e) & 1u) ? (uint32_t)p.a_stream : (uint32_t)p.b_stream;   // kept rows are A or B
    w[0] = (uint64_t)(uint32_t)fkey[e] | ((uint64_t)role << 32) | ((uint64_t)sid << 40);
    w[1] = (uint64_t)(a.seq0 + (r - a.rows.row0));
    w[2] = tsv[e];
    w[3] = fc0[e];
    w[4] = fc1[e];
    uint64_t* o = staged ? stage + (int64_t)pos * wrw : tout + (int64_t)pos * wrw;
#pragma unroll
    for (int c = 0; c < 5; ++c)
      if (c < 3 + nrc) o[c] = w[c];
  }
  if (staged) {
    __syncthreads();
    const int64_t words = (int64_t)total * wrw;
    for (int64_t w = 2 * tid; w < words; w += 2 * NT) {
      if (w + 1 < words) *(uint4*)(tout + w) = *(const uint4*)(stage + w);
      else tout[w] = stage[w];
    }
  }
}

void launch_cf_route(const CfRouteArgs& a, int64_t ntiles, hipStream_t s) {
  hipLaunchKernelGGL(k_cfroute, dim3((unsigned)ntiles), dim3(kCfPartThreads), 0, s, a);
}

// ============================================================== k_cfwalk ==
namespace {

// Records per LDS window: the LDS budget keeps 2 workgroups per CU.
template <int NW>
constexpr int cf_window() { return NW > 1 ? 1536 : kCfWindow; }

// Window layout.  The gather loads only each record's header; the window is
// sorted by (key, arrival) on compact entries, then the full records are
// re-read (L2) in sorted order, so every later phase reads LDS contiguously.
template <int NW, int WIN = cf_window<NW>()>
struct CfWalkLds {
  uint32_t seg[kCfMaxTiles + 1];       // exclusive prefix of the bucket's segment sizes
  uint32_t kstart[2][kCfMaxKeys + 1];  // key runs (sorted positions); alternating windows
  union {
    uint32_t kcur[kCfMaxKeys];         // counting-sort cursors (p3)
    uint32_t klast[kCfMaxKeys];        // ts of the run's last A (if khasa; p4 - p6)
  };
  union {
    uint32_t wrec[WIN];                // arena record index per window slot (gather, reload)
    uint64_t pcache[WIN / 2];          // from p4: key lanes' pending slots >= 2 (ts, captures);
                                       // its last kCfOmap / 4 words hold omap (record-match positions)
  };
  uint32_t pc_used;                    // pcache words handed out this window
  uint32_t nrec;                       // record matches of the window (omap entries)
  union {
    uint64_t kent[WIN];                // seq << 20 | key << 11 | slot, grouped by key
    uint64_t scap[NW > 0 ? NW : 1][WIN];   // sorted: physical carried words
  };
  union alignas(16) {
    uint16_t sorted[WIN];              // window slot per sorted position
    uint16_t nextb[WIN];               // sorted position of the run's next B, or kNoB
  };
  alignas(16) uint32_t sts[WIN];       // sorted: ts - chunk ts base
  uint32_t sseq[WIN];                  // sorted: chunk-relative row (arrival order)
  alignas(16) uint16_t skr[WIN];       // sorted: key in bucket | role << 12
  alignas(16) uint16_t v[WIN];         // output row offset per sorted position
  uint16_t kfb[kCfMaxKeys];            // first B of the key's run, or kNoB
  uint16_t klb[kCfMaxKeys];            // last B of the key's run, or kNoB
  uint8_t khasa[kCfMaxKeys];
  uint8_t cm[kCfMaxKeys];              // carried partials completed by the key's first B
  uint32_t obits[kCfTile / 32];        // oversize segment: tile-row presence bitmap
  uint16_t opre[kCfTile / 32];         // oversize segment: popcount prefix per bitmap word
  uint32_t scratch[kCfWalkThreads / 64 + 1];
  uint32_t scratch2[kCfWalkThreads / 64 + 1];   // the output scan's (no tail barrier)
  unsigned long long base;
};

// Record matches a window lists for the compacted emission (lane per output
// row): the top of the pcache region, which holds no key's slots then.
constexpr int kCfOmap = 1024;

// One output row.  acap = the A's logical captures, b0 / b1 = the completing
// B's physical words, bts / seq = its event ts and arrival number.
template <bool KR>   // KR: sparse keys (output the partition value, key_rev)
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
      v = KR ? a.key_rev[key] : (uint64_t)key;
    } else if (src >= SRC_CAP && src < SRC_REC) {
      v = (src - SRC_CAP) == 0 ? acap0 : acap1;
    } else {
      const int ph = a.cf.bcol_phys[src - SRC_REC];
      v = ph < 0 ? (uint64_t)bts : (ph == 0 ? b0 : b1);
    }
    store_col(a.out.col[c], a.out.type[c], (int64_t)pos, v);
  }
  a.out.ts[pos] = bts;
  if (a.out.write_seq) a.out.seq[pos] = seq;
}

}  // namespace

// NC: captured words per pending slot (slot_words - 2); TOL: order-tolerant
// records (ts in any order, App. A.3's |ts - ts(s1)| > W on every B-stream row)
template <int NW, bool KR, int NC, bool TOL = false>
__global__ __launch_bounds__(kCfWalkThreads, 4) void k_cfwalk(CfWalkArgs a) {   // 2 workgroups per CU
  constexpr int NT = kCfWalkThreads, RW = 1 + NW, WIN = cf_window<NW>();
  constexpr int TPT = kCfMaxTiles / NT;   // tiles per thread
  constexpr int PER = WIN / NT;           // window slots per thread
  __shared__ CfWalkLds<NW> L;
  const int tid = threadIdx.x;
  const PatternArgs& p = a.pat;
  const int lg = p.buckets_log2;
  const int P = 1 << lg;
  const int bucket = xcd_bucket(blockIdx.x, P);
  const int kpb = (int)((p.key_capacity + P - 1) >> lg);
  const int ntiles = a.ntiles;
  const int64_t ks = a.kstride;
  constexpr int sw = 2 + NC;     // p.slot_words
  const int S = p.pending_slots;
  const int64_t W = p.within;
  CF_STAMP(0);

  // ---- key lane (tid < kpb): pending count + slots 0 / 1 in registers,
  // loaded now so the state read overlaps the gather below.  A hot key's
  // records were diverted to the hot path this launch: its state is not ours.
  const bool klane = tid < kpb && !(a.hot_id && a.hot_id[((int64_t)tid << lg) | bucket] != kNotHot);
  uint32_t kcnt = 0;   // the key's records this launch (hot-key candidates)
  const int64_t kidx = (int64_t)bucket * kpb + tid;
  // slot j word w of this key at byte kb + (j * sw + w) * pb of kslot: 32-bit
  // offsets from the kernel-argument base (the host checks the state fits
  // 4 GiB) keep no 64-bit per-slot addresses live in registers
  const uint32_t kb = (uint32_t)kidx * 8u, pb = (uint32_t)ks * 8u;
  auto sl_ld = [&](int j, int w) -> uint64_t {
    return *(const uint64_t*)((const char*)a.kslot + (kb + (uint32_t)(j * sw + w) * pb));
  };
  auto sl_st = [&](int j, int w, uint64_t v) {
    *(uint64_t*)((char*)a.kslot + (kb + (uint32_t)(j * sw + w) * pb)) = v;
  };
  const uint32_t hdr = klane ? a.khdr[kidx] : 0u;
  // A pending list longer than the S inline slots keeps slots [S, n) in an
  // overflow run of the pending pool: header bit kHdrOvf set, kext = n |
  // run offset << 32 in this launch's read pool.  Runs are rewritten into the
  // write pool whenever the list is rebuilt (and moved there at kernel end
  // otherwise): the host swaps the two pools per launch.  The run lives in
  // one register: ovo = offset | kOvoWr (run in the write pool); the host
  // keeps pool offsets below 2^31.
  const bool ovf0 = klane && (hdr & kHdrOvf);
  const uint64_t ext0 = ovf0 ? a.kext[kidx] : 0ull;
  uint32_t ovo = (uint32_t)(ext0 >> 32);
  constexpr uint32_t kOvoWr = 0x80000000u;
  auto ovp = [&]() -> const uint64_t* {
    return ((ovo & kOvoWr) ? a.pool_wr : a.pool_rd) + (uint64_t)(ovo & ~kOvoWr) * (uint64_t)sw;
  };
  // bucket-major offset table, loaded before the slot loads below (those
  // wait for hdr; these need not)
  const uint16_t* rlo = a.tile_off + (int64_t)bucket * ntiles;
  const uint16_t* rhi = rlo + ntiles;
  const int tb = tid * TPT;
  // packed u16 offsets of tiles tid*TPT + i in one row of the bucket-major
  // table: one 8- or 16-byte load when the row is whole, else per tile
  auto load_tile_off = [&](const uint16_t* row, uint32_t (&o)[TPT / 2]) {
    if ((ntiles & (TPT - 1)) == 0 && tb + TPT <= ntiles) {
      if constexpr (TPT == 8) {
        const uint4 x = *(const uint4*)(row + tb);
        o[0] = x.x; o[1 % (TPT / 2)] = x.y; o[2 % (TPT / 2)] = x.z; o[3 % (TPT / 2)] = x.w;
      } else {
        const uint2 x = *(const uint2*)(row + tb);
        o[0] = x.x; o[1 % (TPT / 2)] = x.y;
      }
    } else {
#pragma unroll
      for (int i = 0; i < TPT / 2; ++i) o[i] = 0;
#pragma unroll
      for (int i = 0; i < TPT; ++i) {
        const int t = tb + i;
        o[i >> 1] |= (t < ntiles ? (uint32_t)row[t] : 0u) << (16 * (i & 1));
      }
    }
  };
  uint32_t lop[TPT / 2];   // packed u16 segment starts (prefix phase only)
  uint32_t ys[TPT / 2];    // packed u16 segment ends
  load_tile_off(rlo, lop);
  load_tile_off(rhi, ys);

  int n = ovf0 ? (int)(uint32_t)ext0 : (int)(hdr & 0xffu);
  // Slots 0 / 1 (ts + captures) live in registers for the whole kernel: read
  // once here, rewritten by the commit of each window (named scalars: a
  // dynamically indexed array lands in scratch).  Word 1 of a slot (the A's
  // arrival number) is not needed by the closed form and is neither read nor
  // written here; slots >= 2 stay in HBM.
  constexpr bool c1 = NC > 0, c2 = NC > 1;
  uint64_t t0r = 0, t1r = 0, a0c0 = 0, a0c1 = 0, a1c0 = 0, a1c1 = 0;
  bool dirty = false;   // header / slots 0-1 changed: stored at kernel end
  if (n > 0) {
    t0r = sl_ld(0, 0);
    if (c1) a0c0 = sl_ld(0, 2);
    if (c2) a0c1 = sl_ld(0, 3);
  }
  if (n > 1) {
    t1r = sl_ld(1, 0);
    if (c1) a1c0 = sl_ld(1, 2);
    if (c2) a1c1 = sl_ld(1, 3);
  }
  // (masked selects: a select chain on j / w is turned into a stack array)
  // Per window, a key lane copies its slots >= 2 (one batch of independent
  // loads, before any of the window's stores) to pcache: words pcb + (j - 2)
  // * cw + {0: ts, 1: capture 0, 2: capture 1} for j - 2 < cn.
  constexpr int cw = 1 + (c1 ? 1 : 0) + (c2 ? 1 : 0);
  int cn = 0;
  uint32_t pcb = 0;
  auto slot_word = [&](int j, int w) -> uint64_t {
    if (j >= 2) {
      if (j >= S) return ovp()[(int64_t)(j - S) * sw + w];
      if (j - 2 < cn) return L.pcache[pcb + (uint32_t)((j - 2) * cw + (w == 0 ? 0 : w - 1))];
      return sl_ld(j, w);
    }
    const uint64_t m0 = 0ull - (uint64_t)(j == 0), m1 = ~m0;
    const uint64_t w0 = 0ull - (uint64_t)(w == 0), w2 = 0ull - (uint64_t)(w == 2);
    const uint64_t w3 = 0ull - (uint64_t)(w == 3);
    return (m0 & ((t0r & w0) | (a0c0 & w2) | (a0c1 & w3))) |
           (m1 & ((t1r & w0) | (a1c0 & w2) | (a1c1 & w3)));
  };
  const int64_t ts_base = a.chunk_base[0] - (TOL ? kTolBias : 0);   // record ts = ts_base + sts
  const int64_t seq_base = a.chunk_base[1];
  int kbuf = 0;   // this window's key-run buffer
  for (int k = tid; k <= kpb; k += NT) L.kstart[0][k] = 0;

  // ---- segment sizes -> exclusive prefix over tiles; this thread's segment
  // starts stay in registers (lop) for the gather
  {
    uint32_t cnt[TPT];
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < TPT; ++i)
      cnt[i] = ((ys[i >> 1] >> (16 * (i & 1))) & 0xffffu) - ((lop[i >> 1] >> (16 * (i & 1))) & 0xffffu);
#pragma unroll
    for (int i = 0; i < TPT; ++i) sum += cnt[i];
    uint32_t total;
    uint32_t off = bscan<NT>(sum, L.scratch, &total);
#pragma unroll
    for (int i = 0; i < TPT; ++i) {
      const int t = tb + i;
      if (t < ntiles) {
        L.seg[t] = off;
        off += cnt[i];
      }
    }
    if (tid == 0) L.seg[ntiles] = total;
  }
  lds_barrier();
  CF_STAMP(1);
  const uint32_t nall = L.seg[ntiles];

  // Windows are runs of whole tiles: a tile's segment is in bucket-rank
  // order, not arrival order, so a window never splits one — except a single
  // segment larger than a window (a key holding most of a tile), which is
  // walked in pieces of consecutive arrival rank (rows are unique in a tile:
  // rank = popcount of the row-presence bitmap below the row).
  int t0 = 0;
  int wi = 0;               // window index (diagnostic stamps: windows 0 and 1)
  bool over = false;        // tile t0's segment is being walked in pieces
  uint32_t piece = 0;       // next piece's first arrival rank
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
        over = true;
        piece = 0;
        const uint32_t c = L.seg[t0 + 1] - L.seg[t0];
        const uint64_t* tr = a.recs + ((int64_t)t0 * kCfTile + a.tile_off[(int64_t)bucket * ntiles + t0]) * RW;
        for (int w = tid; w < kCfTile / 32; w += NT) L.obits[w] = 0;
        lds_barrier();
        for (uint32_t j = tid; j < c; j += NT) {
          const uint32_t row = rec_row(tr[(int64_t)j * RW]);
          atomicOr(&L.obits[row >> 5], 1u << (row & 31));
        }
        lds_barrier();
        const uint32_t pc = tid < kCfTile / 32 ? (uint32_t)__popc(L.obits[tid]) : 0u;
        uint32_t total;
        const uint32_t off = bscan<NT>(pc, L.scratch, &total);
        if (tid < kCfTile / 32) L.opre[tid] = (uint16_t)off;
        lds_barrier();
      }
    }
    // ---- window slot -> arena record index (LDS only)
    if (over) {
      const uint32_t c = L.seg[t0 + 1] - L.seg[t0];
      nw = min((uint32_t)WIN, c - piece);
      const int64_t g0 = (int64_t)t0 * kCfTile + a.tile_off[(int64_t)bucket * ntiles + t0];
      const uint64_t* tr = a.recs + g0 * RW;
      for (uint32_t j = tid; j < c; j += NT) {
        const uint32_t row = rec_row(tr[(int64_t)j * RW]);
        const uint32_t rank = L.opre[row >> 5] + (uint32_t)__popc(L.obits[row >> 5] & ((1u << (row & 31)) - 1u));
        if (rank >= piece && rank < piece + nw) L.wrec[rank - piece] = (uint32_t)(g0 + j);
      }
    } else {
      nw = L.seg[t1] - L.seg[t0];
      const uint32_t wb = L.seg[t0];
      // this thread's segment starts, re-read (L2) per window rather than
      // held in registers across the whole walk
      uint32_t lop[TPT / 2];
      load_tile_off(rlo, lop);
#pragma unroll
      for (int i = 0; i < TPT; ++i) {
        const int t = tid * TPT + i;
        if (t < t0 || t >= t1) continue;
        const uint32_t s0 = L.seg[t], s1 = L.seg[t + 1];
        const uint32_t g0 = (uint32_t)t * (uint32_t)kCfTile + ((lop[i >> 1] >> (16 * (i & 1))) & 0xffffu);
        for (uint32_t g = s0; g < s1; ++g) L.wrec[g - wb] = g0 + (g - s0);
      }
    }
    if (klane) {
      if (tid == 0) L.pc_used = 0;
      L.kfb[tid] = kNoB;
      L.klb[tid] = kNoB;
      L.khasa[tid] = 0;
    }
    lds_barrier();
    if (wi == 1) CF_STAMP(9);   // window 1: the window's record table is built
    // ---- every record of the window in flight at once (one pass over the
    // scattered segments: the records stay in registers through the sort);
    // key counts
    uint32_t hk[PER], hs[PER];
    uint4 x[PER];
    uint64_t y[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const uint32_t q = tid + i * NT;
      x[i] = make_uint4(0, 0, 0, 0);
      y[i] = 0;
      if (q < nw) {
        const uint64_t* r = a.recs + (int64_t)L.wrec[q] * RW;
        x[i] = gload4(r);
        if (NW > 1) y[i] = r[2];
      }
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const uint32_t q = tid + i * NT;
      const uint64_t h = ((uint64_t)x[i].y << 32) | x[i].x;
      hk[i] = rec_key(h);
      hs[i] = (L.wrec[q < nw ? q : 0] & ~(uint32_t)(kCfTile - 1)) + rec_row(h);
      if (q < nw) atomicAdd(&L.kstart[kbuf][hk[i] + 1], 1u);
    }
    lds_barrier();
    CF_STAMP(wi * 8 + 2);
    // ---- counting sort by key of (seq, key, slot) entries, then each entry's
    // arrival rank inside its key run -> sorted position of window slot q
    {
      const uint32_t c = tid < kpb ? L.kstart[kbuf][tid + 1] : 0u;
      uint32_t total;
      const uint32_t off = bscan<NT, false>(c, L.scratch, &total);
      if (tid < kpb) {
        L.kstart[kbuf][tid] = off;
        L.kcur[tid] = off;
      }
      if (tid == 0) L.kstart[kbuf][kpb] = total;
    }
    lds_barrier();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const uint32_t q = tid + i * NT;
      if (q >= nw) continue;
      const uint32_t slot = atomicAdd(&L.kcur[hk[i]], 1u);
      L.kent[slot] = ((uint64_t)hs[i] << 20) | ((uint64_t)hk[i] << 11) | q;
    }
    lds_barrier();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const uint32_t s = tid + i * NT;
      if (s >= nw) continue;
      const uint64_t e = L.kent[s];
      const uint32_t k = (uint32_t)(e >> 11) & 0x1ffu;
      const uint32_t r0 = L.kstart[kbuf][k], r1 = L.kstart[kbuf][k + 1];
      uint32_t rank = 0;
      for (uint32_t j = r0; j < r1; ++j) rank += (L.kent[j] >> 20) < (e >> 20) ? 1u : 0u;
      L.sorted[e & 0x7ffu] = (uint16_t)(r0 + rank);
    }
    lds_barrier();
    // ---- the records (registers) -> contiguous LDS arrays in sorted order
    {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const uint32_t q = tid + i * NT;
        if (q >= nw) continue;
        const uint32_t s = L.sorted[q];
        const uint64_t w0 = ((uint64_t)x[i].y << 32) | x[i].x;
        L.sts[s] = x[i].x;
        L.sseq[s] = hs[i];
        // received records: global arrival number - chunk base (read only
        // when the output stores seq: a scattered load per record)
        if (a.in_seq && a.out.write_seq)
          L.sseq[s] = (uint32_t)((int64_t)a.in_seq[(int64_t)hs[i] * a.in_rec_words] - seq_base);
        L.skr[s] = (uint16_t)(rec_key(w0) | (rec_role(w0) << 12));
        if (NW > 0) L.scap[0][s] = ((uint64_t)x[i].w << 32) | x[i].z;
        if (NW > 1) L.scap[NW > 1 ? 1 : 0][s] = y[i];
      }
    }
    lds_barrier();
    CF_STAMP(wi * 8 + 3);
    // ---- key lanes: slots >= 2 of the pending list -> pcache (wrec is dead
    // from here to the next window).  The first two are loaded now and
    // written after the position scan below, so their latency is hidden; a
    // lane that finds pcache full reads HBM instead.
    cn = 0;
    uint64_t pv0[2], pv1[2], pv2[2];
    uint32_t pco = 0;
    const int ni = min(n, S);   // inline slots in use (overflow slots are read from the pool)
    const bool fill = klane && ni > 2 && L.kstart[kbuf][tid + 1] > L.kstart[kbuf][tid];
    if (fill) {
      const uint32_t need = (uint32_t)((ni - 2) * cw);
      pco = atomicAdd(&L.pc_used, need);
      if (pco + need <= (uint32_t)(WIN / 2 - kCfOmap / 4)) {
        pcb = pco;
        cn = ni - 2;
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = 2 + u;
      const bool ld = cn > 0 && j < ni;
      pv0[u] = ld ? sl_ld(j, 0) : 0ull;
      pv1[u] = (ld && c1) ? sl_ld(j, 2) : 0ull;
      pv2[u] = (ld && c2) ? sl_ld(j, 3) : 0ull;
    }
    // ---- per sorted position: next B and next A of its key run, as two
    // segmented suffix-min scans over the window (O(log) steps, not a walk
    // of the run per position); then first / last B and last A per key.
    // Thread t holds positions 4 (NT - 1 - t) .. + 3, so the suffix scan over
    // positions is a prefix scan over lanes (DPP) and waves (LDS).
    {
      constexpr uint32_t kInf = kNoB, kCut = 0x10000u;
      const uint32_t pb = (uint32_t)(NT - 1 - tid) * PER;
      uint32_t kq[PER + 1], rq[PER], krw[PER + 1];
      if constexpr (PER == 4) {   // one 8-byte read (lane-consecutive) + the next thread's first
        const uint2 k2 = *(const uint2*)&L.skr[pb];
        krw[0] = k2.x & 0xffffu; krw[1] = k2.x >> 16; krw[2] = k2.y & 0xffffu; krw[3] = k2.y >> 16;
        krw[4] = pb + 4 < nw ? (uint32_t)L.skr[pb + 4] : 0xffffu;
      } else {
#pragma unroll
        for (int i = 0; i <= PER; ++i) krw[i] = pb + i < nw ? (uint32_t)L.skr[pb + i] : 0xffffu;
      }
#pragma unroll
      for (int i = 0; i <= PER; ++i) {
        const uint32_t q = pb + i;
        const uint32_t kr = krw[i];
        kq[i] = q < nw ? (kr & 0xfffu) : 0xffffffffu - (uint32_t)i;   // past the window: all distinct
        if (i < PER) rq[i] = q < nw ? kr >> 12 : 0u;
      }
      const uint32_t kprev = (pb > 0 && pb - 1 < nw) ? ((uint32_t)L.skr[pb - 1] & 0xfffu) : 0xfffffff0u;
      uint32_t vb[PER], va[PER];
      bool st[PER + 1];   // run start at position pb + i
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const uint32_t q = pb + i;
        vb[i] = (q < nw && (rq[i] & ROLE_B)) ? q : kInf;
        va[i] = (q < nw && (rq[i] & ROLE_A)) ? q : kInf;
        st[i] = q >= nw || kq[i] != (i == 0 ? kprev : kq[i - 1]);
      }
      st[PER] = pb + PER >= nw || kq[PER] != kq[PER - 1];
      // the thread's element: (cut, min from its first position to the first
      // run start after it)
      uint32_t lb = vb[0], la = va[0];
      bool cut = false;
#pragma unroll
      for (int i = 1; i < PER; ++i) {
        cut = cut || st[i];
        if (!cut) {
          lb = min(lb, vb[i]);
          la = min(la, va[i]);
        }
      }
      cut = cut || st[PER];
      // combine(earlier = positions further right, own)
      auto comb = [](uint32_t e, uint32_t o) -> uint32_t {
        return ((e | o) & kCut) | ((o & kCut) ? (o & 0xffffu) : min(e & 0xffffu, o & 0xffffu));
      };
      auto scan = [&](uint32_t x) -> uint32_t {
        constexpr int ident = (int)kInf;
        x = comb((uint32_t)__builtin_amdgcn_update_dpp(ident, (int)x, 0x111, 0xf, 0xf, false), x);   // row_shr:1
        x = comb((uint32_t)__builtin_amdgcn_update_dpp(ident, (int)x, 0x112, 0xf, 0xf, false), x);   // row_shr:2
        x = comb((uint32_t)__builtin_amdgcn_update_dpp(ident, (int)x, 0x114, 0xf, 0xf, false), x);   // row_shr:4
        x = comb((uint32_t)__builtin_amdgcn_update_dpp(ident, (int)x, 0x118, 0xf, 0xf, false), x);   // row_shr:8
        x = comb((uint32_t)__builtin_amdgcn_update_dpp(ident, (int)x, 0x142, 0xa, 0xf, false), x);   // row_bcast:15
        x = comb((uint32_t)__builtin_amdgcn_update_dpp(ident, (int)x, 0x143, 0xc, 0xf, false), x);   // row_bcast:31
        return x;
      };
      const uint32_t ib = scan((cut ? kCut : 0u) | lb), ia = scan((cut ? kCut : 0u) | la);
      const int lane = tid & 63, wv = tid >> 6;
      if (lane == 63) {
        L.scratch[wv] = ib;
        L.scratch2[wv] = ia;
      }
      lds_barrier();
      uint32_t cb = kInf, ca = kInf;   // the waves to the right
      for (int w = 0; w < wv; ++w) {
        cb = comb(cb, L.scratch[w]);
        ca = comb(ca, L.scratch2[w]);
      }
      const uint32_t pbv = (uint32_t)__shfl_up((int)ib, 1, 64), pav = (uint32_t)__shfl_up((int)ia, 1, 64);
      const uint32_t xb = lane == 0 ? cb : comb(cb, pbv), xa = lane == 0 ? ca : comb(ca, pav);
      // this thread's positions, right to left: next B / A of p_i is the
      // suffix min at p_{i+1} unless p_{i+1} starts a run
      uint32_t nbn = st[PER] ? kInf : (xb & 0xffffu), nan_ = st[PER] ? kInf : (xa & 0xffffu);
      uint32_t nbo[PER];
#pragma unroll
      for (int i = PER - 1; i >= 0; --i) {
        const uint32_t q = pb + i;
        const uint32_t nbi = nbn, nai = nan_;
        const uint32_t sbi = min(vb[i], nbi), sai = min(va[i], nai);
        nbn = st[i] ? kInf : sbi;
        nan_ = st[i] ? kInf : sai;
        nbo[i] = nbi;
        if (q >= nw) continue;
        const uint32_t k = kq[i], role = rq[i];
        if constexpr (PER != 4) L.nextb[q] = (uint16_t)nbi;
        if ((role & ROLE_A) && nai == kInf) {
          L.klast[k] = L.sts[q];
          L.khasa[k] = 1;
        }
        if ((role & ROLE_B) && nbi == kInf) L.klb[k] = (uint16_t)q;
        if (st[i]) L.kfb[k] = (role & ROLE_B) ? (uint16_t)q : (uint16_t)nbi;
      }
      if constexpr (PER == 4)   // positions past the window get kNoB, never read
        *(uint2*)&L.nextb[pb] = make_uint2((nbo[0] & 0xffffu) | (nbo[1] << 16), (nbo[2] & 0xffffu) | (nbo[3] << 16));
    }
    if (cn > 0) {
      auto put_pc = [&](int j, uint64_t t, uint64_t x0, uint64_t x1) {
        const uint32_t o = pcb + (uint32_t)((j - 2) * cw);
        L.pcache[o] = t;
        if (c1) L.pcache[o + 1] = x0;
        if (c2) L.pcache[o + 1 + (c1 ? 1 : 0)] = x1;
      };
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (2 + u < n) put_pc(2 + u, pv0[u], pv1[u], pv2[u]);
      // longer lists (a few per wave): four slots' loads in flight at a time,
      // not one dependent round trip per slot
      for (int j0 = 4; j0 < ni; j0 += 4) {
        uint64_t t[4], x0[4], x1[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool ok = j0 + u < ni;
          t[u] = ok ? sl_ld(j0 + u, 0) : 0ull;
          x0[u] = (ok && c1) ? sl_ld(j0 + u, 2) : 0ull;
          x1[u] = (ok && c2) ? sl_ld(j0 + u, 3) : 0ull;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (j0 + u < ni) put_pc(j0 + u, t[u], x0[u], x1[u]);
      }
    }
    lds_barrier();
    // ---- key lanes: carried partials completed by the run's first B
    uint32_t r0 = 0, r1 = 0;
    int cfirst = 0, cm = 0;
    uint64_t e00 = 0, e01 = 0, e10 = 0, e11 = 0;
    // TOL: ts range [tmn, tmx] (sts units) of the B-stream rows from the run
    // start to its first g-passing B inclusive (the whole run without one)
    uint32_t tmn = 0xffffffffu, tmx = 0u;
    bool thave = false;
    auto tol_alive = [&](int64_t pts) {   // a partial started at pts survives that range
      return !thave || W < 0 ||
             (pts - (ts_base + (int64_t)tmn) <= W && (ts_base + (int64_t)tmx) - pts <= W);
    };
    if (klane) {
      r0 = L.kstart[kbuf][tid];
      r1 = L.kstart[kbuf][tid + 1];
      kcnt += r1 - r0;
      const uint16_t fb = L.kfb[tid];
      if (TOL && r1 > r0) {
        // right to left over the key's run: each A learns whether every
        // B-stream row after it up to its next g-passing B (inclusive) is
        // within W of it (skr bit 15); the range restarts at each such B
        for (uint32_t q = r1; q-- > r0;) {
          const uint32_t kr = L.skr[q];
          const uint32_t role = (kr >> 12) & 7u;
          const uint32_t t = L.sts[q];
          if (role & ROLE_A) {
            const bool ok = !thave || W < 0 ||
                            ((int64_t)t - (int64_t)tmn <= W && (int64_t)tmx - (int64_t)t <= W);
            L.skr[q] = (uint16_t)((kr & 0x7fffu) | (ok ? kSkrAlive : 0u));
          }
          if (role & ROLE_B) {
            tmn = tmx = t;
            thave = true;
          } else if (role & kRolePB) {
            tmn = t < tmn ? t : tmn;
            tmx = t > tmx ? t : tmx;
            thave = true;
          }
        }
        // carried partials completed by the first g-passing B: every one
        // that survives the rows before it (not a prefix when ts go back)
        if (fb != kNoB)
          for (int j = 0; j < n; ++j) cm += tol_alive((int64_t)slot_word(j, 0)) ? 1 : 0;
      } else if (!TOL && r1 > r0 && fb != kNoB && n > 0) {
        const int64_t tb = ts_base + (int64_t)L.sts[fb];
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
      // captures of the first two completed carried partials (registers
      // unless the partial sits in slot >= 2)
      if (!TOL && cm > 0) {
        e00 = c1 ? slot_word(cfirst, 2) : 0ull;
        e01 = c2 ? slot_word(cfirst, 3) : 0ull;
      }
      if (!TOL && cm > 1) {
        e10 = c1 ? slot_word(cfirst + 1, 2) : 0ull;
        e11 = c2 ? slot_word(cfirst + 1, 3) : 0ull;
      }
    }
    lds_barrier();
    CF_STAMP(wi * 8 + 4);

    // ---- match flag per sorted position (+ carried matches at run start);
    // one scan yields both the output offsets (low 20 bits) and each record
    // match's rank among the window's record matches (bits 20-31), which
    // lists it in omap for the compacted emission
    uint16_t* omap = (uint16_t*)&L.pcache[WIN / 2 - kCfOmap / 4];
    {
      uint32_t vals[PER];
      uint32_t sum = 0;
      // a thread's PER contiguous positions: one wide LDS read per array
      // (lane-consecutive, no bank conflicts) where PER is 4
      uint32_t krv[PER], nbv[PER], stv[PER];
      if constexpr (PER == 4) {
        const uint2 k2 = *(const uint2*)&L.skr[tid * 4];
        const uint2 n2 = *(const uint2*)&L.nextb[tid * 4];
        const uint4 t4 = *(const uint4*)&L.sts[tid * 4];
        krv[0] = k2.x & 0xffffu; krv[1 % PER] = k2.x >> 16; krv[2 % PER] = k2.y & 0xffffu; krv[3 % PER] = k2.y >> 16;
        nbv[0] = n2.x & 0xffffu; nbv[1 % PER] = n2.x >> 16; nbv[2 % PER] = n2.y & 0xffffu; nbv[3 % PER] = n2.y >> 16;
        stv[0] = t4.x; stv[1 % PER] = t4.y; stv[2 % PER] = t4.z; stv[3 % PER] = t4.w;
      } else {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
          const uint32_t q = tid * PER + i;
          krv[i] = q < nw ? L.skr[q] : 0u;
          nbv[i] = q < nw ? L.nextb[q] : kNoB;
          stv[i] = q < nw ? L.sts[q] : 0u;
        }
      }
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const uint32_t q = tid * PER + i;
        uint32_t val = 0;
        if (q < nw) {
          const uint32_t kr = krv[i];
          const uint32_t k = kr & 0xfffu;
          const uint32_t nb = nbv[i];
          if (((kr >> 12) & ROLE_A) && nb != kNoB) {
            if (TOL) {
              val = (kr & kSkrAlive) ? (1u << 20) | 1u : 0u;
            } else {
              const int64_t d = (int64_t)L.sts[nb] - (int64_t)stv[i];
              val = (W < 0 || (d < 0 ? -d : d) <= W) ? (1u << 20) | 1u : 0u;
            }
          }
          if (q == L.kstart[kbuf][k]) val += L.cm[k];
        }
        vals[i] = val;
        sum += val;
      }
      uint32_t total;
      uint32_t off = bscan<NT, false>(sum, L.scratch2, &total);
      uint32_t vv[PER];
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const uint32_t q = tid * PER + i;
        vv[i] = off & 0xfffffu;
        if ((vals[i] >> 20) && (off >> 20) < (uint32_t)kCfOmap) omap[off >> 20] = (uint16_t)q;
        off += vals[i];
      }
      if constexpr (PER == 4) {
        *(uint2*)&L.v[tid * 4] = make_uint2((vv[0] & 0xffffu) | (vv[1 % PER] << 16),
                                            (vv[2 % PER] & 0xffffu) | (vv[3 % PER] << 16));
      } else {
#pragma unroll
        for (int i = 0; i < PER; ++i) L.v[tid * PER + i] = (uint16_t)vv[i];
      }
      const uint32_t rows = total & 0xfffffu;
      if (tid == 0) {
        L.base = rows ? atomicAdd(a.out.count, (unsigned long long)rows) : 0ull;
        L.nrec = total >> 20;
      }
      if (tid == 0) { CF_COUNT(1, rows); CF_COUNT(5, 1); }
    }
    lds_barrier();
#ifndef CF_WAVESTAMP
    CF_STAMP(wi * 8 + 5);
#else
    if ((threadIdx.x >> 6) == 0) CF_WSTAMP(0);
#endif
    const unsigned long long base = L.base;
    const int cp0 = a.cf.cap_phys[0], cp1 = a.cf.cap_phys[1];

    // ---- key lanes: carried matches, survivors, state commit.  Runs before
    // the record emission: a slot read (slots >= 2 live in HBM) issued after
    // a wave's output stores waits for all of them (vmcnt counts loads and
    // stores in issue order), so the state work goes first.
    if (klane && r1 > r0) {
      const int64_t kl = ((int64_t)tid << lg) | bucket;
      const int64_t kv = kl * p.key_stride + p.key_offset;
      const uint16_t fb = L.kfb[tid], lb = L.klb[tid];
      CF_COUNT(7, 1);
      if (n > 2) CF_COUNT(2, 1);
      if (cm) {
        CF_COUNT(0, cm);
        const int64_t bts = ts_base + (int64_t)L.sts[fb];
        const uint64_t b0 = NW > 0 ? L.scap[0][fb] : 0ull, b1 = NW > 1 ? L.scap[NW > 1 ? 1 : 0][fb] : 0ull;
        if (TOL) {   // the carried partials that survived to the first B, in slot order
          int o = 0;
          for (int j = 0; j < n && o < cm; ++j) {
            if (!tol_alive((int64_t)slot_word(j, 0))) continue;
            cf_emit<KR>(a, base + L.v[r0] + o, kv, c1 ? slot_word(j, 2) : 0ull, c2 ? slot_word(j, 3) : 0ull,
                        b0, b1, bts, seq_base + (int64_t)L.sseq[fb]);
            ++o;
          }
        } else {
          for (int j = 0; j < cm; ++j) {
            const int js = cfirst + j;
            const uint64_t x0 = j == 0 ? e00 : (j == 1 ? e10 : (c1 ? slot_word(js, 2) : 0ull));
            const uint64_t x1 = j == 0 ? e01 : (j == 1 ? e11 : (c2 ? slot_word(js, 3) : 0ull));
            cf_emit<KR>(a, base + L.v[r0] + j, kv, x0, x1, b0, b1, bts, seq_base + (int64_t)L.sseq[fb]);
          }
        }
      }
      // (TOL: no pruning at A arrivals — a later row may carry an older ts)
      const bool prune = !TOL && W >= 0 && L.khasa[tid];
      const int64_t last_a_ts = ts_base + (int64_t)L.klast[tid];
      // new pending list, built in place: (no B in the run) the carried
      // partials minus the pruned prefix, then the starts after the last B
      // minus pruned ones.  Slot j is written only after every old slot it
      // could overwrite has been read (old slot j' >= j is read at step j').
      int nn = 0;
      // capacity of the new list: the kept old entries + every record from
      // the run's last B on; past S the tail goes to a fresh overflow run in
      // the write pool (rare: a key with more than S live partials)
      const uint32_t from = (lb == kNoB ? r0 : (uint32_t)lb);
      int cap = (lb == kNoB ? n : 0) + (int)(r1 - from);
      // the new overflow run: pool_wr slot noff on (kNoOff: none / pool full)
      constexpr uint32_t kNoOff = 0xffffffffu;
      uint32_t noff = kNoOff;
      if (cap > S) {
        const unsigned long long cnt = (unsigned long long)(cap - S);
        const unsigned long long o = atomicAdd(a.pool_cursor, cnt);
        if (o + cnt > a.pool_cap) {
          set_err(a.err, ERR_POOL);
          cap = S;
        } else {
          noff = (uint32_t)o;
        }
      }
      auto put_slot = [&](uint64_t ts, uint64_t x0, uint64_t x1) {
        const uint64_t m0 = 0ull - (uint64_t)(nn == 0), m1 = 0ull - (uint64_t)(nn == 1);
        t0r = (ts & m0) | (t0r & ~m0);
        a0c0 = (x0 & m0) | (a0c0 & ~m0);
        a0c1 = (x1 & m0) | (a0c1 & ~m0);
        t1r = (ts & m1) | (t1r & ~m1);
        a1c0 = (x0 & m1) | (a1c0 & ~m1);
        a1c1 = (x1 & m1) | (a1c1 & ~m1);
        if (nn >= 2) CF_COUNT(4, 1);
        if (nn >= S) {   // overflow run
          if (noff == kNoOff) {   // the pool ran out (ERR_POOL set): keep the device safe
            ++nn;
            return;
          }
          uint64_t* o = a.pool_wr + ((uint64_t)noff + (uint64_t)(nn - S)) * (uint64_t)sw;
          o[0] = ts;
          if (c1) o[2] = x0;
          if (c2) o[3] = x1;
        } else if (nn >= 2) {   // slots 0 / 1 are stored once, at kernel end
          sl_st(nn, 0, ts);
          if (c1) sl_st(nn, 2, x0);
          if (c2) sl_st(nn, 3, x1);
        }
        ++nn;
        dirty = true;
      };
      if (lb == kNoB && (a.ablate & 1)) {
        nn = 0;
      } else if (TOL && lb == kNoB) {
        // no g-passing B: the carried partials that survive the run's B-stream rows
        bool all = true;
        for (int j = 0; j < n && all; ++j) all = tol_alive((int64_t)slot_word(j, 0));
        if (all && cap <= S) {
          nn = n;   // unchanged, in place
        } else {
          for (int j = 0; j < n; ++j) {
            const uint64_t ts = slot_word(j, 0);
            if (!tol_alive((int64_t)ts)) continue;
            const uint64_t x0 = c1 ? slot_word(j, 2) : 0ull, x1 = c2 ? slot_word(j, 3) : 0ull;
            put_slot(ts, x0, x1);
          }
        }
      } else if (lb == kNoB) {
        int drop = 0;
        while (drop < n && prune && last_a_ts - (int64_t)slot_word(drop, 0) > W) ++drop;
        if (drop == 0 && cap <= S) {
          nn = n;   // unchanged, in place
        } else {
          if (n > 2) CF_COUNT(3, 1);
          for (int j = drop; j < n; ++j) {
            const uint64_t ts = slot_word(j, 0);
            const uint64_t x0 = c1 ? slot_word(j, 2) : 0ull, x1 = c2 ? slot_word(j, 3) : 0ull;
            put_slot(ts, x0, x1);
          }
        }
      }
      // partials created after the last B (a record that is both B and A
      // starts a partial after completing others)
      for (uint32_t q = (lb == kNoB ? r0 : (uint32_t)lb); q < r1 && !(a.ablate & 2); ++q) {
        if (!((L.skr[q] >> 12) & ROLE_A)) continue;
        if (TOL && !(L.skr[q] & kSkrAlive)) continue;   // expired before the run ended
        const int64_t ats = ts_base + (int64_t)L.sts[q];
        if (prune && last_a_ts - ats > W) continue;
        if (nn >= cap) {   // only after the pool ran out (ERR_POOL is set)
          set_err(a.err, ERR_POOL);
          break;
        }
        const uint64_t a0 = NW > 0 ? L.scap[0][q] : 0ull, a1 = NW > 1 ? L.scap[NW > 1 ? 1 : 0][q] : 0ull;
        put_slot((uint64_t)ats, cp0 < 0 ? (uint64_t)ats : (cp0 == 0 ? a0 : a1),
                 cp1 < 0 ? (uint64_t)ats : (cp1 == 0 ? a0 : a1));
      }
      dirty |= nn != n;
      if (nn > S) ovo = noff | kOvoWr;
      n = nn;
    }
#ifndef CF_WAVESTAMP
    CF_STAMP(wi * 8 + 6);
#else
    CF_WSTAMP(1 + (int)(threadIdx.x >> 6));
#endif

    // ---- emit record matches: lane per output row from omap (consecutive
    // lanes write consecutive rows, every lane busy), or lane per sorted
    // position when the window has more record matches than omap lists
    const uint32_t nrec = L.nrec;
    const bool compact = nrec <= (uint32_t)kCfOmap && !(a.ablate & 8);   // ablate 8: per position
    const uint32_t nemit = compact ? nrec : (uint32_t)(PER * NT);
#pragma unroll 1
    for (uint32_t j = tid; j < nemit; j += NT) {
      const uint32_t q = compact ? (uint32_t)omap[j] : j;
      if (q >= nw || (a.ablate & 4)) continue;   // ablate 4 (diagnostics): no record-match stores
      const uint32_t kr = L.skr[q];
      const uint16_t nb = L.nextb[q];
      if (!((kr >> 12) & ROLE_A) || nb == kNoB) continue;
      if (TOL) {
        if (!(kr & kSkrAlive)) continue;
      } else {
        const int64_t d = (int64_t)L.sts[nb] - (int64_t)L.sts[q];
        if (W >= 0 && (d < 0 ? -d : d) > W) continue;
      }
      const uint32_t k = kr & 0xfffu;
      const uint32_t extra = q == L.kstart[kbuf][k] ? L.cm[k] : 0u;
      const int64_t ats = ts_base + (int64_t)L.sts[q];
      const int64_t bts = ts_base + (int64_t)L.sts[nb];
      const uint64_t a0 = NW > 0 ? L.scap[0][q] : 0ull, a1 = NW > 1 ? L.scap[NW > 1 ? 1 : 0][q] : 0ull;
      const uint64_t x0 = cp0 < 0 ? (uint64_t)ats : (cp0 == 0 ? a0 : a1);
      const uint64_t x1 = cp1 < 0 ? (uint64_t)ats : (cp1 == 0 ? a0 : a1);
      const int64_t kl = ((int64_t)k << lg) | bucket;
      cf_emit<KR>(a, base + L.v[q] + extra, kl * p.key_stride + p.key_offset, x0, x1,
              NW > 0 ? L.scap[0][nb] : 0ull, NW > 1 ? L.scap[NW > 1 ? 1 : 0][nb] : 0ull, bts,
              seq_base + (int64_t)L.sseq[nb]);
    }
#ifndef CF_WAVESTAMP
    CF_STAMP(wi * 8 + 7);
#else
    CF_WSTAMP(9 + (int)(threadIdx.x >> 6));
#endif
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
    wi = 1;
    // next window: the LDS arrays are reused (a key's slots >= 2 are read
    // back only by the lane that wrote them).  Its key-run buffer is the one
    // the previous window used, read by nobody since: zeroed without a
    // second barrier (its counts are added after the next window's first)
    lds_barrier();
    CF_STAMP(8);   // window 1 only: after the window-end barrier
    kbuf ^= 1;
    for (int k = tid; k <= kpb; k += NT) L.kstart[kbuf][k] = 0;
  }
  // ---- hot-key candidates: keys that made this bucket long (hot.hip)
  if (klane && a.hot_thresh && kcnt > a.hot_thresh) {
    // two tiers, so the busiest keys are never crowded out by many merely
    // warm ones: [0, kCfHotMax) for keys over 8x the threshold, the rest after
    const uint32_t key = (uint32_t)(((int64_t)tid << lg) | bucket);
    const uint64_t v = ((uint64_t)kcnt << 32) | key;
    bool put = false;
    if (kcnt >= 8u * a.hot_thresh) {
      const uint32_t i = atomicAdd(&a.hot_ncand[0], 1u);
      if (i < (uint32_t)kCfHotMax) {
        a.hot_cand[i] = v;
        put = true;
      }
    }
    if (!put) {
      const uint32_t j = atomicAdd(&a.hot_ncand[1], 1u);
      if (j < 3u * kCfHotMax) a.hot_cand[kCfHotMax + j] = v;
    }
  }
  // ---- an overflow run still in the read pool moves to the write pool
  // (the read pool is the next launch's write pool)
  if (klane && n > S && !(ovo & kOvoWr)) {
    const unsigned long long cnt = (unsigned long long)(n - S);
    const unsigned long long off = atomicAdd(a.pool_cursor, cnt);
    if (off + cnt > a.pool_cap) {
      set_err(a.err, ERR_POOL);
    } else {
      uint64_t* o = a.pool_wr + off * (uint64_t)sw;
      const uint64_t* src = ovp();
      for (int64_t i = 0; i < (int64_t)cnt * sw; ++i) o[i] = src[i];
      ovo = (uint32_t)off | kOvoWr;
      dirty = true;
    }
  }
  // ---- the key's header and register-resident slots 0 / 1, once
  if (klane && dirty) {
    const uint32_t h1 = (a.khdr[kidx] & ~(0xffu | kHdrOvf)) | (n > S ? ((uint32_t)S | kHdrOvf) : (uint32_t)n);
    if (n > S) a.kext[kidx] = (uint64_t)(uint32_t)n | ((uint64_t)(ovo & ~kOvoWr) << 32);
    if (n > 0) {
      sl_st(0, 0, t0r);
      if (c1) sl_st(0, 2, a0c0);
      if (c2) sl_st(0, 3, a0c1);
    }
    if (n > 1) {
      sl_st(1, 0, t1r);
      if (c1) sl_st(1, 2, a1c0);
      if (c2) sl_st(1, 3, a1c1);
    }
    a.khdr[kidx] = h1;
  }
}

void launch_cf_partition(const CfPartArgs& a, int64_t ntiles, hipStream_t s) {
  const int P = 1 << a.pat.buckets_log2;
  const size_t dyn = ((size_t)(P + a.nhot + 1) * 4 + 15) & ~(size_t)15;
  const dim3 g((unsigned)ntiles), b(kCfPartThreads);
  if (a.in_recs) {
    switch (a.cf.nw) {
      case 0: hipLaunchKernelGGL((k_cfpart<0, true>), g, b, dyn, s, a); break;
      case 1: hipLaunchKernelGGL((k_cfpart<1, true>), g, b, dyn, s, a); break;
      default: hipLaunchKernelGGL((k_cfpart<2, true>), g, b, dyn, s, a); break;
    }
    return;
  }
  // the local-rows build holds only the prefetched columns the plan reads
  const int np = a.pref.n <= 2 ? 2 : a.pref.n;
  if (a.pat.tolerant) {   // order-tolerant records (cep_options.ts_order 0)
    switch (a.cf.nw * 8 + np) {
      case 0 * 8 + 2: hipLaunchKernelGGL((k_cfpart<0, false, 2, true>), g, b, dyn, s, a); break;
      case 0 * 8 + 3: hipLaunchKernelGGL((k_cfpart<0, false, 3, true>), g, b, dyn, s, a); break;
      case 0 * 8 + 4: hipLaunchKernelGGL((k_cfpart<0, false, 4, true>), g, b, dyn, s, a); break;
      case 1 * 8 + 2: hipLaunchKernelGGL((k_cfpart<1, false, 2, true>), g, b, dyn, s, a); break;
      case 1 * 8 + 3: hipLaunchKernelGGL((k_cfpart<1, false, 3, true>), g, b, dyn, s, a); break;
      case 1 * 8 + 4: hipLaunchKernelGGL((k_cfpart<1, false, 4, true>), g, b, dyn, s, a); break;
      case 2 * 8 + 2: hipLaunchKernelGGL((k_cfpart<2, false, 2, true>), g, b, dyn, s, a); break;
      case 2 * 8 + 3: hipLaunchKernelGGL((k_cfpart<2, false, 3, true>), g, b, dyn, s, a); break;
      default: hipLaunchKernelGGL((k_cfpart<2, false, 4, true>), g, b, dyn, s, a); break;
    }
    return;
  }
  switch (a.cf.nw * 8 + np) {
    case 0 * 8 + 2: hipLaunchKernelGGL((k_cfpart<0, false, 2>), g, b, dyn, s, a); break;
    case 0 * 8 + 3: hipLaunchKernelGGL((k_cfpart<0, false, 3>), g, b, dyn, s, a); break;
    case 0 * 8 + 4: hipLaunchKernelGGL((k_cfpart<0, false, 4>), g, b, dyn, s, a); break;
    case 1 * 8 + 2: hipLaunchKernelGGL((k_cfpart<1, false, 2>), g, b, dyn, s, a); break;
    case 1 * 8 + 3: hipLaunchKernelGGL((k_cfpart<1, false, 3>), g, b, dyn, s, a); break;
    case 1 * 8 + 4: hipLaunchKernelGGL((k_cfpart<1, false, 4>), g, b, dyn, s, a); break;
    case 2 * 8 + 2: hipLaunchKernelGGL((k_cfpart<2, false, 2>), g, b, dyn, s, a); break;
    case 2 * 8 + 3: hipLaunchKernelGGL((k_cfpart<2, false, 3>), g, b, dyn, s, a); break;
    default: hipLaunchKernelGGL((k_cfpart<2, false, 4>), g, b, dyn, s, a); break;
  }
}

template <int NW, bool KR, bool TOL = false>
static void launch_cf_walk_nc(const CfWalkArgs& a, int nbuckets, hipStream_t s) {
  const dim3 g((unsigned)nbuckets), b(kCfWalkThreads);
  switch (a.pat.slot_words - 2) {
    case 0: hipLaunchKernelGGL((k_cfwalk<NW, KR, 0, TOL>), g, b, 0, s, a); break;
    case 1: hipLaunchKernelGGL((k_cfwalk<NW, KR, 1, TOL>), g, b, 0, s, a); break;
    default: hipLaunchKernelGGL((k_cfwalk<NW, KR, 2, TOL>), g, b, 0, s, a); break;
  }
}

void launch_cf_walk(const CfWalkArgs& a, int nbuckets, hipStream_t s) {
  const bool kr = a.key_rev != nullptr;
  if (a.pat.tolerant) {   // order-tolerant records (dense keys only: the engine refuses sparse + tolerant)
    switch (a.cf.nw) {
      case 0: launch_cf_walk_nc<0, false, true>(a, nbuckets, s); break;
      case 1: launch_cf_walk_nc<1, false, true>(a, nbuckets, s); break;
      default: launch_cf_walk_nc<2, false, true>(a, nbuckets, s); break;
    }
    return;
  }
  switch (a.cf.nw) {
    case 0: kr ? launch_cf_walk_nc<0, true>(a, nbuckets, s) : launch_cf_walk_nc<0, false>(a, nbuckets, s); break;
    case 1: kr ? launch_cf_walk_nc<1, true>(a, nbuckets, s) : launch_cf_walk_nc<1, false>(a, nbuckets, s); break;
    default: kr ? launch_cf_walk_nc<2, true>(a, nbuckets, s) : launch_cf_walk_nc<2, false>(a, nbuckets, s); break;
  }
}

}  // namespace cep
