// k_filterc — `from S[expr] select attrs insert into O` as one
// coalesced stream-compaction pass (the per-event filter branch of
// operator/AbstractSiddhiOperator.java:130 -> Siddhi's FilterProcessor, for
// term-list predicates and plain attribute projections; k_filter keeps the
// rest).
//
// Layout of a tile: 1024 lanes, wave w owns rows [2 P 64 w, 2 P 64 (w + 1));
// lane l holds row pairs 128 i + 2 l + {0, 1}, i < P (P = 4: 8192-row
// tiles), so every load instruction of a column reads one contiguous 512 B
// (4-byte column) or 1 KiB (8-byte column) span: a wave's loads are fully
// coalesced, and all of a lane's loads are issued before the first is used.
// Selected rows are ranked per wave (DPP scans of per-pair counts, four pairs
// packed per word); the global output position comes from a decoupled
// look-back over tile tickets.
//
// Selected rows are compacted
// per wave in LDS, then the projection runs lane per selected row, so each
// output column is written as consecutive rows by consecutive lanes; the
// projection's loads for the first 64 selected rows of every wave are in
// flight while the look-back runs.
#include <hip/hip_runtime.h>

#include "dev_common.h"
#include "kernels.h"
#include "vm.h"

namespace cep {

namespace {

#ifndef FC_THREADS
#define FC_THREADS 1024
#endif
constexpr int kFcThreads = FC_THREADS;
constexpr int kFcWaves = kFcThreads / 64;
#ifndef FC_PAIRS
#define FC_PAIRS 4
#endif
#ifndef FC_REGCOLS
#define FC_REGCOLS 4
#endif
#ifndef FC_MINW
#define FC_MINW 4
#endif
constexpr int kFcPairs = FC_PAIRS;               // row pairs per lane
constexpr int kFcWaveRows = 64 * 2 * kFcPairs;   // 512 rows per wave
constexpr int kFcTile = kFcWaves * kFcWaveRows;  // 8192
constexpr int kFcRegCols = FC_REGCOLS;                    // projected columns loaded ahead of the look-back
constexpr uint64_t kFcStatusShift = 62;
constexpr uint64_t kFcValueMask = (1ull << 62) - 1;

// Rows r, r + 1 of a typed column as VM words (r even; `two`: both in range).
__device__ __forceinline__ void fc_load_pair(const void* p, int type, int64_t r, bool two, uint64_t& v0,
                                             uint64_t& v1) {
  const int w = type_width(type);
  if (!two) {
    v0 = load_col(p, type, r);
    v1 = 0;
    return;
  }
  if (w == 8) {
    const uint4 x = gload4((const uint64_t*)p + r);
    v0 = ((uint64_t)x.y << 32) | x.x;
    v1 = ((uint64_t)x.w << 32) | x.z;
  } else if (w == 4) {
    const uint2 x = *(const uint2*)((const uint32_t*)p + r);
    v0 = type == T_FLOAT ? (uint64_t)x.x : from_i32((int32_t)x.x);
    v1 = type == T_FLOAT ? (uint64_t)x.y : from_i32((int32_t)x.y);
  } else {
    const uint32_t x = *(const uint16_t*)((const uint8_t*)p + r);
    v0 = (x & 0xffu) ? 1u : 0u;
    v1 = (x >> 8) ? 1u : 0u;
  }
}

// Decoupled look-back (one wave): lane l reads the flag of tile base - l;
// publishes this tile's aggregate, then its inclusive prefix; *s_prefix gets
// the rows of every earlier tile.
__device__ __forceinline__ void fc_lookback(const FilterArgs& a, int64_t tile, uint32_t total, int lane,
                                            unsigned long long* s_prefix) {
  unsigned long long* flags = a.tile_state;
  unsigned long long prefix = 0;
  if (tile == 0) {
    prefix = __hip_atomic_load(a.out.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    if (lane == 0)
      __hip_atomic_store(&flags[tile], (1ull << kFcStatusShift) | total, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    int64_t b = tile - 1;
    unsigned spins = 0;
    while (true) {
      const int64_t j = b - lane;
      const unsigned long long v =
          j >= 0 ? __hip_atomic_load(&flags[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
      const uint32_t st = (uint32_t)(v >> kFcStatusShift);
      const uint64_t ready = __ballot(st != 0);
      const uint64_t incl = __ballot(st == 2);
      const int f = incl ? __ffsll((long long)incl) - 1 : 63;
      const uint64_t need = f == 63 ? ~0ull : ((2ull << f) - 1ull);   // lanes 0..f
      if ((ready & need) != need) {
        if (++spins > (1u << 22)) {   // a predecessor never published: fail loudly
          if (lane == 0) set_err(a.err, ERR_WINDOW);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      unsigned long long x = ((need >> lane) & 1ull) ? (v & kFcValueMask) : 0ull;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
      prefix += x;
      if (incl) break;
      b -= 64;
    }
  }
  if (lane == 0) {
    __hip_atomic_store(&flags[tile], (2ull << kFcStatusShift) | (prefix + total), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    *s_prefix = prefix;
    if (tile == (int64_t)gridDim.x - 1)
      __hip_atomic_store(a.out.count, prefix + total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

template <int Q>   // distinct predicate columns (1..3)
__global__ __launch_bounds__(kFcThreads, FC_MINW) void k_filterc(FilterArgs a) {
  __shared__ uint16_t rows_sel[kFcWaves][kFcWaveRows];   // wave-relative row of each selected row
  __shared__ uint32_t wtot[kFcWaves];
  __shared__ uint32_t s_tile;
  __shared__ unsigned long long s_prefix;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s_tile = atomicAdd(a.ticket, 1u);
  __syncthreads();
  const int64_t tile = s_tile;
  const int64_t n = a.rows.n;
  const int64_t wrow0 = tile * kFcTile + (int64_t)wave * kFcWaveRows;   // slice-relative
  const int64_t brow0 = a.rows.row0 + wrow0;                            // batch row

  // ---- predicate columns and stream handles, every load issued up front
  uint64_t pv[Q][2 * kFcPairs];
  uint32_t okp = 0;   // bit 2i + j: row in range
#pragma unroll
  for (int i = 0; i < kFcPairs; ++i) {
    const int64_t r = wrow0 + 128 * i + 2 * lane;
    okp |= (r < n ? 1u : 0u) << (2 * i);
    okp |= (r + 1 < n ? 1u : 0u) << (2 * i + 1);
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = a.pcol[q];
    const void* p = a.rows.cols.p[c];
    const int ty = a.rows.cols.t[c];
#pragma unroll
    for (int i = 0; i < kFcPairs; ++i) {
      const int64_t r = brow0 + 128 * i + 2 * lane;
      pv[q][2 * i] = pv[q][2 * i + 1] = 0;
      if ((okp >> (2 * i)) & 1u) fc_load_pair(p, ty, r, (okp >> (2 * i + 1)) & 1u, pv[q][2 * i], pv[q][2 * i + 1]);
    }
  }
  uint32_t sel = okp;
  if (a.rows.stream) {
#pragma unroll
    for (int i = 0; i < kFcPairs; ++i) {
      const int64_t r = brow0 + 128 * i + 2 * lane;
      if ((okp >> (2 * i)) & 1u) {
        uint32_t s0, s1;
        if ((okp >> (2 * i + 1)) & 1u) {
          const uint32_t x = *(const uint16_t*)(a.rows.stream + r);
          s0 = x & 0xffu;
          s1 = x >> 8;
        } else {
          s0 = a.rows.stream[r];
          s1 = 0xffu;
        }
        if ((int)s0 != a.in_stream) sel &= ~(1u << (2 * i));
        if ((int)s1 != a.in_stream) sel &= ~(1u << (2 * i + 1));
      }
    }
  } else if (a.rows.input != a.in_stream) {
    sel = 0;
  }
  if (sel && a.filter_prog >= 0) sel &= eval_terms_regs<2 * kFcPairs, Q>(a.filter_terms, a.fslot, a.rows.cols, pv);

  // ---- per-wave compaction in row order (pair i major, lane, row of the pair)
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < kFcPairs; ++i) {
    const uint32_t c = (uint32_t)__popc((sel >> (2 * i)) & 3u);
    if (i < 4) lo |= c << (8 * i);
    else hi |= c << (8 * (i - 4));
  }
  const uint32_t ilo = wave_incl_scan(lo), ihi = wave_incl_scan(hi);
  const uint32_t tlo = (uint32_t)__builtin_amdgcn_readlane((int)ilo, 63);
  const uint32_t thi = (uint32_t)__builtin_amdgcn_readlane((int)ihi, 63);
  const uint32_t elo = ilo - lo, ehi = ihi - hi;
  uint32_t base = 0;
#pragma unroll
  for (int i = 0; i < kFcPairs; ++i) {
    const uint32_t ex = i < 4 ? (elo >> (8 * i)) & 0xffu : (ehi >> (8 * (i - 4))) & 0xffu;
    const uint32_t t = i < 4 ? (tlo >> (8 * i)) & 0xffu : (thi >> (8 * (i - 4))) & 0xffu;
    uint32_t k = base + ex;
    if ((sel >> (2 * i)) & 1u) rows_sel[wave][k++] = (uint16_t)(128 * i + 2 * lane);
    if ((sel >> (2 * i + 1)) & 1u) rows_sel[wave][k] = (uint16_t)(128 * i + 2 * lane + 1);
    base += t;
  }
  const uint32_t wt = base;   // this wave's selected rows (uniform)
  if (lane == 0) wtot[wave] = wt;
  __syncthreads();
  uint32_t woff = 0, total = 0;
#pragma unroll
  for (int w = 0; w < kFcWaves; ++w) {
    const uint32_t c = wtot[w];
    woff += w < wave ? c : 0u;
    total += c;
  }

  // ---- projection loads of the first 64 selected rows (lane per row): in
  // flight while wave 0 looks back
  const int nc = a.out.ncols;
  uint64_t val[kFcRegCols];
  int64_t vts = 0, vseq = 0;
  auto load_row = [&](uint32_t k) {
    const int64_t row = brow0 + rows_sel[wave][k];
#pragma unroll
    for (int c = 0; c < kFcRegCols; ++c) {
      if (c < nc) {
        const int col = a.out.src[c] - SRC_REC;
        val[c] = load_col(a.rows.cols.p[col], a.rows.cols.t[col], row);
      }
    }
    vts = a.rows.ts[row];
    vseq = row_seq(a.rows, row);
  };
  if ((uint32_t)lane < wt) load_row((uint32_t)lane);

  // ---- decoupled look-back (wave 0)
  if (wave == 0) fc_lookback(a, tile, total, lane, &s_prefix);
  __syncthreads();
  const int64_t obase = (int64_t)s_prefix + woff;
  // ---- stores: consecutive lanes -> consecutive output rows
  for (uint32_t k0 = 0; k0 < wt; k0 += 64) {
    const uint32_t k = k0 + (uint32_t)lane;
    if (k0 > 0 && k < wt) load_row(k);
    if (k < wt) {
      const int64_t pos = obase + k;
      if (pos < a.out.cap) {
#pragma unroll
        for (int c = 0; c < kFcRegCols; ++c)
          if (c < nc) store_col(a.out.col[c], a.out.type[c], pos, val[c]);
        const int64_t row = brow0 + rows_sel[wave][k];
        for (int c = kFcRegCols; c < nc; ++c) {   // wide projections: the rest directly
          const int col = a.out.src[c] - SRC_REC;
          store_col(a.out.col[c], a.out.type[c], pos, load_col(a.rows.cols.p[col], a.rows.cols.t[col], row));
        }
        a.out.ts[pos] = vts;
        if (a.out.write_seq) a.out.seq[pos] = vseq;
      }
    }
  }
}

int filterc_rows_per_tile() { return kFcTile; }



void launch_filterc(const FilterArgs& a, int64_t ntiles, hipStream_t s) {
  switch (a.npref) {
    case 1: hipLaunchKernelGGL(k_filterc<1>, dim3((unsigned)ntiles), dim3(kFcThreads), 0, s, a); break;
    case 2: hipLaunchKernelGGL(k_filterc<2>, dim3((unsigned)ntiles), dim3(kFcThreads), 0, s, a); break;
    default: hipLaunchKernelGGL(k_filterc<3>, dim3((unsigned)ntiles), dim3(kFcThreads), 0, s, a); break;
  }
}

}  // namespace cep
