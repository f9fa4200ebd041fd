// Device helpers shared by the pattern kernels (kernels.hip, cf_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "vm.h"

namespace cep {
namespace {

__device__ __forceinline__ void set_err(unsigned int* err, unsigned int bit) {
  if (err) atomicOr(err, bit);
}

// ts of the row before a batch's first row (host-known, or the device word
// the previous batch left: RowsArgs::prev_ts_dev).
__device__ __forceinline__ int64_t batch_prev_ts(const RowsArgs& r) {
  int64_t p = r.prev_ts;
  if (r.prev_ts_dev) {
    const int64_t d = *r.prev_ts_dev;
    p = d > p ? d : p;
  }
  return p;
}

// A ts descent in a slice that promised event-time order (ts_order = 1).
__device__ __forceinline__ void report_descent(const RowsArgs&, unsigned int* err) {
  set_err(err, ERR_ORDER);
}

// Workgroup barrier that orders LDS only.  __syncthreads() also releases
// global memory, which makes every wave drain its outstanding global loads
// and stores (s_waitcnt vmcnt(0)) before the barrier; phases that only hand
// LDS data to each other keep their global traffic in flight with this one.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Block-wide exclusive scan of one value per thread (blockDim <= 512).
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* scratch /*>=9*/,
                                                    uint32_t* total) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwaves = (int)(blockDim.x >> 6);
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) scratch[wave] = x;
  lds_barrier();
  if (tid == 0) {
    uint32_t s = 0;
    for (int w = 0; w < nwaves; ++w) {
      uint32_t t = scratch[w];
      scratch[w] = s;
      s += t;
    }
    scratch[8] = s;
  }
  lds_barrier();
  uint32_t r = scratch[wave] + x - v;
  *total = scratch[8];
  lds_barrier();
  return r;
}

// Block-wide exclusive scan of one value per thread, NT <= 1024 threads;
// scratch holds NT / 64 + 1 words.
// kTail = false: no trailing barrier; the caller must not write `scratch`
// again before another barrier (the walk alternates two scratch buffers).
template <int NT, bool kTail = true>
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
  if (kTail) lds_barrier();
  return r;
}

// Shard-local dense key of partition key `key` (cep_options key_stride /
// key_offset: this shard owns key % stride == offset), or -1 when the key is
// negative or not owned.  stride == 1 (one shard) skips the division; else a
// 32-bit division (keys are int attributes).
__device__ __forceinline__ int64_t shard_key(int64_t key, int32_t stride, int32_t offset) {
  if (stride == 1) return (key < 0 || offset != 0) ? -1 : key;
  if (key < 0 || key > 0xffffffffll) return -1;
  const uint32_t k = (uint32_t)key, q = k / (uint32_t)stride;
  return (k - q * (uint32_t)stride) == (uint32_t)offset ? (int64_t)q : -1;
}

// ---- fast partition path helpers (PrefPlan) --------------------------------
// Raw 16-byte loads of E consecutive rows of a column of width w; branch
// free (surplus loads repeat the last address), all issued before any use.
template <int E>
__device__ __forceinline__ void load_raw(const void* p, int w, int64_t row, uint4 (&r)[E / 2]) {
  const char* b = (const char*)p + row * w;
  const int nl = w == 8 ? E / 2 : (w == 4 ? (E / 4 > 0 ? E / 4 : 1) : 1);
#pragma unroll
  for (int i = 0; i < E / 2; ++i) r[i] = gload4(b + 16 * (i < nl ? i : nl - 1));
}

// Decode E rows of raw column data into VM words (load_col semantics).
template <int E>
__device__ __forceinline__ void decode(const uint4 (&r)[E / 2], int type, uint64_t (&v)[E]) {
  uint32_t x[2 * E];
#pragma unroll
  for (int i = 0; i < E / 2; ++i) {
    x[4 * i] = r[i].x;
    x[4 * i + 1] = r[i].y;
    x[4 * i + 2] = r[i].z;
    x[4 * i + 3] = r[i].w;
  }
  if (type == T_LONG || type == T_DOUBLE) {
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = ((uint64_t)x[2 * e + 1] << 32) | x[2 * e];
  } else if (type == T_BOOL) {
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = ((x[e >> 2] >> (8 * (e & 3))) & 0xffu) ? 1u : 0u;
  } else if (type == T_FLOAT) {
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = (uint64_t)x[e];
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = from_i32((int32_t)x[e]);
  }
}

// Value of prefetched slot `slot` (uniform) for row e.
template <int N, int Q = kPref>
__device__ __forceinline__ uint64_t pick(const uint64_t (&v)[Q][N], int slot, int e) {
  // masked OR rather than selects: a select chain on slot == q gets rewritten
  // into a dynamically indexed (scratch) array access
  uint64_t x = 0;
#pragma unroll
  for (int q = 0; q < Q; ++q) x |= v[q][e] & (0ull - (uint64_t)(slot == q));
  return x;
}

// Rows of prefetched slot `slot` (uniform): one uniform branch per slot value,
// so only the taken slot's copies execute.  A select chain or masked OR over
// every slot costs kPref times the VALU per row; the empty asm keeps each
// branch a branch (it is not if-converted into selects).
template <int N, int Q = kPref>
__device__ __forceinline__ void take_slot(const uint64_t (&v)[Q][N], int slot, uint64_t (&out)[N]) {
#pragma unroll
  for (int e = 0; e < N; ++e) out[e] = 0;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    if (slot == q) {
      asm volatile("");
#pragma unroll
      for (int e = 0; e < N; ++e) out[e] = v[q][e];
    }
  }
}

// Term-list predicate over prefetched rows (eval_terms_run without loads).
template <int N, int Q = kPref>
__device__ __forceinline__ uint32_t eval_terms_regs(const TermList& tl, const int32_t* slot,
                                                    const ColSet& cols,
                                                    const uint64_t (&vals)[Q][N]) {
  uint32_t acc = tl.any ? 0u : ((N >= 32) ? 0xffffffffu : ((1u << N) - 1u));
#pragma unroll
  for (int i = 0; i < kMaxTerms; ++i) {   // fixed indices: term descriptors load once (SGPRs)
    if (i >= tl.n) break;
    const Term& t = tl.t[i];
    uint64_t v[N];
    take_slot<N, Q>(vals, slot[i], v);   // one uniform branch, not a masked OR over every slot
    int ty = (t.coltype == T_BOOL || t.coltype == T_STRING) ? T_INT : t.coltype;
    uint32_t nullm = 0;
    if (t.aop) {
      convert_run<N>(v, ty, t.atype);
      arith_run<N>(v, t.aop, t.atype, t.aconst, &nullm);
      ty = t.atype;
    }
    convert_run<N>(v, ty, t.ctype);
    const uint32_t bits = compare_run<N>(v, t.cop, t.ctype, t.cconst) & ~nullm;
    acc = tl.any ? (acc | bits) : (acc & bits);
  }
  return acc;
}

// Columns of a lane's E rows (row0 + 64 e) for the fast paths: event ts,
// stream handle and every prefetched slot, all loads issued before any use;
// unused slots and the ts alias issue none (uniform branches).
template <int E, int Q = kPref>
__device__ __forceinline__ void cf_load_cols(const RowsArgs& rows, const PrefPlan& pref, int ts_slot,
                                             int64_t row0, uint32_t valid, uint64_t (&tsv)[E],
                                             uint32_t (&sb)[E], uint64_t (&pv)[Q][E]) {
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const bool ok = (valid >> e) & 1u;
    tsv[e] = ok ? (uint64_t)rows.ts[row0 + 64 * e] : 0ull;
    sb[e] = (ok && rows.stream) ? (uint32_t)rows.stream[row0 + 64 * e] : (uint32_t)rows.input;
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = pref.col[q];
    const int ty = rows.cols.t[c];
    if (q < pref.n && q != ts_slot) {
      const void* base = rows.cols.p[c];
      if (ty == T_LONG || ty == T_DOUBLE) {
#pragma unroll
        for (int e = 0; e < E; ++e)
          pv[q][e] = ((valid >> e) & 1u) ? ((const uint64_t*)base)[row0 + 64 * e] : 0ull;
      } else if (ty == T_BOOL) {
#pragma unroll
        for (int e = 0; e < E; ++e)
          pv[q][e] = ((valid >> e) & 1u) ? (((const uint8_t*)base)[row0 + 64 * e] ? 1ull : 0ull) : 0ull;
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const uint32_t v = ((valid >> e) & 1u) ? ((const uint32_t*)base)[row0 + 64 * e] : 0u;
          pv[q][e] = ty == T_FLOAT ? (uint64_t)v : from_i32((int32_t)v);
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) pv[q][e] = 0;
    }
  }
#pragma unroll
  for (int q = 0; q < Q; ++q)
    if (q == ts_slot) {
#pragma unroll
      for (int e = 0; e < E; ++e) pv[q][e] = tsv[e];
    }
}

// Inclusive scan over the 64 lanes with DPP row shifts and row broadcasts
// (VALU-only: no LDS round trip per step, unlike __shfl_up).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  // within each row of 16 lanes: shifts 1, 2, 4, 8 (lanes without a source add 0)
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);   // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);   // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);   // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);   // row_shr:8
  // across rows: lane 15 into rows 1 and 3, then lane 31 into rows 2 and 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);   // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);   // row_bcast:31
  return x;
}

// XCD-aware bucket order: blocks b and b+8 share an XCD (MI355X_MICROARCH.md
// §Workgroup dispatch), so consecutive buckets — which share tile-offset
// cache lines — are given to blocks of one XCD.  Speed only, never correctness.
// Tile order for streaming passes: XCD x (blocks b with b % 8 == x) takes
// the contiguous tile range [x * n/8, (x+1) * n/8), so the lines of a
// bucket-major per-tile table that 64 consecutive tiles write stay in one
// XCD's L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_tile(int bid, int n) {
  if (n < 8 || (n & 7)) return bid;
  return (bid & 7) * (n >> 3) + (bid >> 3);
}

__device__ __forceinline__ int xcd_bucket(int bid, int nb) {
  if (nb < 8 || (nb & 7)) return bid;
  return (bid & 7) * (nb >> 3) + (bid >> 3);
}

}  // namespace
}  // namespace cep
