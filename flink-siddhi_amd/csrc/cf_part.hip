// gfx950 partition pass of the closed-form keyed pattern, persistent build
// (the Siddhi work behind AbstractSiddhiOperator.java:130 for BASELINE
// config 3; same records and bucket-major tile offsets as k_cfpart,
// cf_kernels.hip, byte for byte).
//
// k_cfpart runs one 1024-lane workgroup per 8192-row tile: its loads, then
// its LDS histogram / scan / staging phases, during which the CU's memory
// pipe idles (one workgroup fills the register file).  k_cfpart2 keeps one
// such workgroup per CU for the whole chunk and software-pipelines it: the
// next tile's column loads are issued as soon as the current tile's rows are
// decoded, so they are in flight through the current tile's LDS phases and
// record stores.  Tiles go to workgroups XCD-contiguously (xcd_tile's
// layout), so the 64 tiles sharing a line of the bucket-major offset table
// are written from one XCD's L2.
#include <hip/hip_runtime.h>

#include "dev_common.h"
#include "kernels.h"
#include "vm.h"

namespace cep {

namespace {

constexpr int kP2StageBytes = 56 * 1024;   // staged records (a tile keeps ~1/3 of its rows at config 3)

template <int E, int Q>
__device__ __forceinline__ void p2_pick_carried(const uint64_t (&pv)[Q][E], int sa, int sb, uint32_t role_a,
                                                uint64_t (&out)[E]) {
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

// Raw column words of a lane's E rows (row0 + 64 e), as loaded: 64-bit
// columns whole, narrower ones in the low word (decoded after the wait).
template <int E, int Q>
struct P2Raw {
  uint64_t ts[E];
  uint32_t sb[E];
  uint64_t v[Q][E];
};

template <int E, int Q>
__device__ __forceinline__ void p2_issue(const RowsArgs& rows, const PrefPlan& pref, int ts_slot, int64_t row0,
                                         uint32_t valid, P2Raw<E, Q>& r) {
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const bool ok = (valid >> e) & 1u;
    r.ts[e] = ok ? (uint64_t)rows.ts[row0 + 64 * e] : 0ull;
    r.sb[e] = (ok && rows.stream) ? (uint32_t)rows.stream[row0 + 64 * e] : (uint32_t)rows.input;
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = pref.col[q];
    const int ty = rows.cols.t[c];
    if (q < pref.n && q != ts_slot) {
      const void* base = rows.cols.p[c];
      if (ty == T_LONG || ty == T_DOUBLE) {
#pragma unroll
        for (int e = 0; e < E; ++e) r.v[q][e] = ((valid >> e) & 1u) ? ((const uint64_t*)base)[row0 + 64 * e] : 0ull;
      } else if (ty == T_BOOL) {
#pragma unroll
        for (int e = 0; e < E; ++e) r.v[q][e] = ((valid >> e) & 1u) ? ((const uint8_t*)base)[row0 + 64 * e] : 0u;
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) r.v[q][e] = ((valid >> e) & 1u) ? ((const uint32_t*)base)[row0 + 64 * e] : 0u;
      }
    }
  }
}

// load_col semantics of the raw words (cf_load_cols' decode)
template <int E, int Q>
__device__ __forceinline__ void p2_decode(const RowsArgs& rows, const PrefPlan& pref, int ts_slot,
                                          const P2Raw<E, Q>& r, uint64_t (&pv)[Q][E]) {
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int ty = rows.cols.t[pref.col[q]];
    if (q == ts_slot) {
#pragma unroll
      for (int e = 0; e < E; ++e) pv[q][e] = r.ts[e];
    } else if (q >= pref.n) {
#pragma unroll
      for (int e = 0; e < E; ++e) pv[q][e] = 0;
    } else if (ty == T_LONG || ty == T_DOUBLE) {
#pragma unroll
      for (int e = 0; e < E; ++e) pv[q][e] = r.v[q][e];
    } else if (ty == T_BOOL) {
#pragma unroll
      for (int e = 0; e < E; ++e) pv[q][e] = (r.v[q][e] & 0xffu) ? 1ull : 0ull;
    } else if (ty == T_FLOAT) {
#pragma unroll
      for (int e = 0; e < E; ++e) pv[q][e] = (uint32_t)r.v[q][e];
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) pv[q][e] = from_i32((int32_t)(uint32_t)r.v[q][e]);
    }
  }
}

}  // namespace

template <int NW, int NP>
__global__ __launch_bounds__(kCfPartThreads, 1) void k_cfpart2(CfPartArgs a) {
  constexpr int E = kCfItems, NT = kCfPartThreads, RW = 1 + NW;
  constexpr int kStageRecs = kP2StageBytes / (8 * RW);
  __shared__ uint32_t scratch[NT / 64 + 1];
  __shared__ __attribute__((aligned(16))) uint64_t stage[kStageRecs * RW];
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];   // NB + 1 (dynamic)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const PatternArgs& p = a.pat;
  const int lg = p.buckets_log2;
  const int P = 1 << lg;
  const int NB = P + a.nhot;
  const int ntiles = a.ntiles;
  const int G = (int)gridDim.x;
  // XCD-contiguous tile order: workgroup w (XCD w % 8) walks the XCD's tile
  // range [x n/8, (x+1) n/8) with stride G/8 (speed only, never correctness)
  const bool xcd = (G & 7) == 0 && (ntiles & 7) == 0 && ntiles >= 8;
  const int per_x = ntiles >> 3, wx = G >> 3;
  auto tile_of = [&](int it) -> int {
    if (!xcd) return (int)blockIdx.x + it * G;
    const int j = ((int)blockIdx.x >> 3) + it * wx;
    return j < per_x ? ((int)blockIdx.x & 7) * per_x + j : ntiles;
  };
  const int64_t ts_base = a.rows.ts[a.rows.row0];
  const uint32_t all = (1u << E) - 1u;

  int it = 0;
  int tile = tile_of(0);
  P2Raw<E, NP> raw;
  auto valid_of = [&](int t) -> uint32_t {
    const int64_t r0 = (int64_t)t * kCfTile + (int64_t)wave * 64 * E + lane;
    uint32_t v = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) v |= (r0 + 64 * e < a.rows.n ? 1u : 0u) << e;
    return v;
  };
  auto row_of = [&](int t) -> int64_t { return a.rows.row0 + (int64_t)t * kCfTile + (int64_t)wave * 64 * E + lane; };
  if (tile < ntiles) {
    const uint32_t v = valid_of(tile);
    if (v) p2_issue<E, NP>(a.rows, a.pref, a.ts_slot, row_of(tile), v, raw);
  }
  for (int i = tid; i <= NB; i += NT) hist[i] = 0;
  while (tile < ntiles) {
    const int next = tile_of(it + 1);
    if (tile == 0 && tid == 0) {
      a.chunk_base[0] = ts_base;
      a.chunk_base[1] = a.rows.seq0 + a.rows.row0;
    }
    const int64_t row0 = row_of(tile);
    const uint32_t valid = valid_of(tile);
    // ---- decode this tile's rows: roles, key, carried words, ts
    uint32_t role_a = 0, role_b = 0;
    uint64_t tsv[E], fkey[E], fc0[E], fc1[E];
#pragma unroll
    for (int e = 0; e < E; ++e) tsv[e] = fkey[e] = fc0[e] = fc1[e] = 0;
    if (valid) {
      uint64_t pv[NP][E];
      p2_decode<E, NP>(a.rows, a.pref, a.ts_slot, raw, pv);
#pragma unroll
      for (int e = 0; e < E; ++e) tsv[e] = raw.ts[e];
      uint32_t is_a = 0, is_b = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if ((valid >> e) & 1u) {
          is_a |= ((int)raw.sb[e] == p.a_stream ? 1u : 0u) << e;
          is_b |= ((int)raw.sb[e] == p.b_stream ? 1u : 0u) << e;
        }
      }
      if (p.within >= 0) {
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
      if (is_a) role_a = is_a & (p.f_prog < 0 ? all : eval_terms_regs<E, NP>(p.f_terms, a.pref.f_slot, a.rows.cols, pv));
      if (is_b) role_b = is_b & (p.g_raw_prog < 0 ? all : eval_terms_regs<E, NP>(p.g_terms, a.pref.g_slot, a.rows.cols, pv));
      if (NW > 0) p2_pick_carried<E, NP>(pv, a.cf.a_slot[0], a.cf.b_slot[0], role_a, fc0);
      if (NW > 1) p2_pick_carried<E, NP>(pv, a.cf.a_slot[1], a.cf.b_slot[1], role_a, fc1);
      if (a.pref.key_slot >= 0) {
#pragma unroll
        for (int e = 0; e < E; ++e) fkey[e] = pv[0][e];
      }
    }
    // ---- the next tile's loads go out now, in flight through this tile's
    // LDS phases and stores
    if (next < ntiles) {
      const uint32_t v = valid_of(next);
      if (v) p2_issue<E, NP>(a.rows, a.pref, a.ts_slot, row_of(next), v, raw);
    }
    lds_barrier();   // hist zeroed (and the previous tile's stage drained)
    // bits 0-12 rank in tile, 13-24 bucket, 25-26 role
    uint32_t packed[E];
    uint64_t w0v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      packed[e] = 0xffffffffu;
      w0v[e] = 0;
      const uint32_t role = ((role_a >> e) & 1u) * ROLE_A | ((role_b >> e) & 1u) * ROLE_B;
      if (!role) continue;
      const int64_t kfield = shard_key((int64_t)fkey[e], p.key_stride, p.key_offset);
      if (kfield < 0 || kfield >= p.key_capacity) {
        set_err(a.err, ERR_KEY_RANGE);
        continue;
      }
      uint32_t bucket = (uint32_t)(kfield & (P - 1));
      uint32_t lkey = (uint32_t)(kfield >> lg);
      if (a.nhot) {
        const uint32_t hs = a.hot_id[kfield];
        if (hs != kNotHot) {
          bucket = (uint32_t)P + hs;
          lkey = hs;
        }
      }
      const uint32_t rank = atomicAdd(&hist[bucket], 1u);
      packed[e] = (role << 25) | (bucket << 13) | rank;
      const int64_t dts = (int64_t)tsv[e] - ts_base;
      if (dts < 0 || dts > 0xffffffffll) set_err(a.err, ERR_ORDER);
      w0v[e] = (uint64_t)(uint32_t)dts | ((uint64_t)(wave * 64 * E + 64 * e + lane) << 32) | ((uint64_t)role << 45) |
               ((uint64_t)lkey << 48);
    }
    lds_barrier();
    {
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
    const uint32_t total = hist[NB];
    const bool staged = total <= (uint32_t)kStageRecs;   // uniform
    uint64_t* trecs = a.recs + (int64_t)tile * (int64_t)kCfTile * RW;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (packed[e] == 0xffffffffu) continue;
      const uint32_t b = (packed[e] >> 13) & 0xfffu;
      const uint32_t slot = hist[b] + (packed[e] & 0x1fffu);
      const uint64_t c0 = fc0[e], c1 = fc1[e];
      if (staged) {
        stage[slot * RW] = w0v[e];
        if (NW > 0) stage[slot * RW + 1] = c0;
        if (NW > 1) stage[slot * RW + 2] = c1;
      } else {
        uint64_t* g = trecs + (int64_t)slot * RW;
        g[0] = w0v[e];
        if (NW > 0) g[1] = c0;
        if (NW > 1) g[2] = c1;
      }
    }
    for (int i = tid; i <= NB; i += NT) a.tile_off[(int64_t)i * ntiles + tile] = (uint16_t)hist[i];
    lds_barrier();   // stage complete; hist read
    if (staged) {
      const int64_t words = (int64_t)total * RW;
      for (int64_t w = 2 * tid; w < words; w += 2 * NT) {
        if (w + 1 < words) *(uint4*)(trecs + w) = *(const uint4*)(stage + w);
        else trecs[w] = stage[w];
      }
    }
    for (int i = tid; i <= NB; i += NT) hist[i] = 0;   // the next tile's histogram (ordered by its first barrier)
    ++it;
    tile = next;
  }
}

int cf_partition2_ok(const CfPartArgs& a) { return a.in_recs == nullptr; }

void launch_cf_partition2(const CfPartArgs& a, int64_t ntiles, int nblocks, hipStream_t s) {
  const int P = 1 << a.pat.buckets_log2;
  const size_t dyn = ((size_t)(P + a.nhot + 1) * 4 + 15) & ~(size_t)15;
  const dim3 g((unsigned)std::min<int64_t>(ntiles, nblocks)), b(kCfPartThreads);
  const int np = a.pref.n <= 2 ? 2 : a.pref.n;
  switch (a.cf.nw * 8 + np) {
    case 0 * 8 + 2: hipLaunchKernelGGL((k_cfpart2<0, 2>), g, b, dyn, s, a); break;
    case 0 * 8 + 3: hipLaunchKernelGGL((k_cfpart2<0, 3>), g, b, dyn, s, a); break;
    case 0 * 8 + 4: hipLaunchKernelGGL((k_cfpart2<0, 4>), g, b, dyn, s, a); break;
    case 1 * 8 + 2: hipLaunchKernelGGL((k_cfpart2<1, 2>), g, b, dyn, s, a); break;
    case 1 * 8 + 3: hipLaunchKernelGGL((k_cfpart2<1, 3>), g, b, dyn, s, a); break;
    case 1 * 8 + 4: hipLaunchKernelGGL((k_cfpart2<1, 4>), g, b, dyn, s, a); break;
    case 2 * 8 + 2: hipLaunchKernelGGL((k_cfpart2<2, 2>), g, b, dyn, s, a); break;
    case 2 * 8 + 3: hipLaunchKernelGGL((k_cfpart2<2, 3>), g, b, dyn, s, a); break;
    default: hipLaunchKernelGGL((k_cfpart2<2, 4>), g, b, dyn, s, a); break;
  }
}

}  // namespace cep
