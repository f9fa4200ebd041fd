// gfx950 walk of the closed-form keyed pattern, owner-wave build
//   partition with (k of A, k of B) begin
//     from every s1=A[f] -> s2=B[g] within W select ... insert into O;
//   end;
// (the Siddhi work behind AbstractSiddhiOperator.java:130 for BASELINE
// config 3; semantics: SURVEY.md App. A.3 as in k_cfwalk, cf_kernels.hip,
// whose results this kernel reproduces row for row).
//
// One 512-lane workgroup per key bucket (<= 512 keys), the bucket's records
// walked in windows of WIN records made of whole tile segments.  Wave w owns
// the bucket's keys [64 w, 64 w + 64): lane l is the key lane of key 64 w + l
// and keeps its pending partials in registers for the whole launch.  A window
// costs three workgroup barriers:
//   A  the window's records (prefetched into registers during the previous
//      window) go to LDS by window slot; wave ballots count them per owner
//      wave; the next window's extent is proposed (LDS atomicMax);
//   B  one 64-entry scan per wave gives every record its place in its owner
//      wave's range; the next window's record table is built;
//   C  (no barrier) the next window's records are loaded, then each wave
//      alone sorts its range by (key, arrival), finds every A's next B, counts
//      its output rows (one atomic per wave), emits them and commits its keys'
//      pending lists — waves never wait for each other inside a window.
// k_cfwalk (cf_kernels.hip) does the same work with ~11 workgroup barriers
// per window and no prefetch; it stays the default until this build beats
// it (CEP_CF_WALK=2 selects this one).
#include <hip/hip_runtime.h>

#include "dev_common.h"
#include "kernels.h"
#include "vm.h"

namespace cep {

namespace {

constexpr uint16_t kNoSlot = 0xffff;
constexpr uint32_t kNoPos = 0xffffffffu;
constexpr int kOwners = kCfWalkThreads / 64;   // owner waves per workgroup
static_assert(kOwners * 64 == kCfMaxKeys, "one owner wave per 64 keys of a bucket");

// Records per window, and the waves per SIMD the register budget is set for
// (4: two workgroups per CU, 128 VGPRs).
#ifndef W2_WIN
#define W2_WIN 1024
#endif
#ifndef W2_MINW
#define W2_MINW 4
#endif
template <int NW>
constexpr int w2_window() { return NW > 1 ? (W2_WIN > 1024 ? 1024 : W2_WIN) : W2_WIN; }

// Diagnostics (CEP_STAMPS=1): s_memtime at point i of block b (wave 0), per
// block 16 slots: 0 start, 1 setup done, window 0: 2 phase A, 3 barrier 1,
// 4 phase B, 5 barrier 2 + prefetch issue, 6 C1 sort, 7 C2 / C3, 8 C4
// reservation, 9 C5 key lanes, 10 C6 emission, 11 barrier 3; window 1: 12
// barrier 1, 13 barrier 2, 14 phase C; 15 kernel end.
#define W2_STAMP(i)                                                                 \
  do {                                                                              \
    if (a.stamps && threadIdx.x == 0 && blockIdx.x < 4096)                          \
      a.stamps[(int64_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memtime();      \
  } while (0)
#define W2_STAMPW(w, i0, i1)                                                        \
  do {                                                                              \
    if ((w) == 0) W2_STAMP(i0);                                                     \
    else if ((w) == 1 && (i1) >= 0) W2_STAMP(i1);                                   \
  } while (0)

__device__ __forceinline__ uint32_t w2_row(uint64_t w0) { return (uint32_t)(w0 >> 32) & 0x1fffu; }
__device__ __forceinline__ uint32_t w2_role(uint64_t w0) { return (uint32_t)(w0 >> 45) & 0x7u; }
__device__ __forceinline__ uint32_t w2_key(uint64_t w0) { return (uint32_t)(w0 >> 48); }

// LDS written by some lanes of a wave, then read by others: one wave's LDS
// operations are performed in issue order, so only the compiler must not
// reorder them (mq_kernels.hip wave_lds_sync).
__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// Entry of one record in its owner wave's range: window slot (11) | key in
// the owner's 64 (6) << 11 | role (3) << 17 | counting-sort rank (11) << 20.
__device__ __forceinline__ uint32_t e_slot(uint32_t e) { return e & 0x7ffu; }
__device__ __forceinline__ uint32_t e_key(uint32_t e) { return (e >> 11) & 63u; }
__device__ __forceinline__ uint32_t e_role(uint32_t e) { return (e >> 17) & 7u; }

// Per owner wave: a window's copy of its keys' pending slots 2 .. S-1 (ts,
// captures), loaded with independent loads at the window's start, so the key
// lanes never wait on a dependent global load in phase C (at config 3 a
// quarter of the active keys hold more than two partials).
constexpr int kW2Scr = 64;   // slots per wave

template <int NW, int WIN, int NC>
struct W2Lds {
  uint32_t wrec[2][WIN];                   // arena record index per window slot (this window / the next)
  uint32_t rts[WIN];                       // by slot: ts - chunk ts base
  uint32_t rseq[WIN];                      // by slot: chunk-relative arrival number
  uint64_t rcap[NW > 0 ? NW : 1][WIN];     // by slot: physical carried words
  uint32_t ent[WIN];                       // owner ranges: entries, then sorted by (key, arrival)
  uint32_t ent2[WIN];                      // owner ranges grouped by key (counting sort)
  uint16_t nextb[WIN];                     // by sorted position: slot of the run's next B (kNoSlot)
  uint32_t vout[WIN];                      // by sorted position: output rows before it in the owner range
  uint32_t ocnt[kOwners][kOwners];         // per producer wave, per owner wave: records
  uint32_t wk[kOwners][64];                // per owner wave: key counters, then key run starts
  unsigned long long bound[2];             // next window extent proposals: end tile << 32 | its record index
  uint32_t tseg[kCfMaxTiles / kCfWalkThreads + 1][kCfWalkThreads];   // [i][thread]: seg of the thread's tile i (+ end)
  uint32_t tlop[kCfMaxTiles / kCfWalkThreads / 2][kCfWalkThreads];   // [i][thread]: packed u16 segment starts
  uint32_t obits[kCfTile / 32];            // oversize segment: tile-row presence bitmap
  uint16_t opre[kCfTile / 32];             // oversize segment: popcount prefix per bitmap word
  uint32_t scratch[kCfWalkThreads / 64 + 1];
  uint64_t scr[kOwners][kW2Scr * (1 + NC)];   // [wave][slot * (1 + NC) + word]
  uint32_t wrows[kOwners];                 // output rows of each owner wave (this window)
  unsigned long long wbase[kOwners];       // their first output row
};

// One output row (as k_cfwalk's cf_emit).
template <bool KR>
__device__ __forceinline__ void w2_emit(const CfWalkArgs& a, unsigned long long pos, int64_t key, uint64_t acap0,
                                        uint64_t acap1, uint64_t b0, uint64_t b1, int64_t bts, int64_t seq) {
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
  a.out.seq[pos] = seq;
}

}  // namespace

template <int NW, bool KR, int NC, int WIN>
__global__ __launch_bounds__(kCfWalkThreads, W2_MINW) void k_cfwalk2(CfWalkArgs a) {
  constexpr int NT = kCfWalkThreads, RW = 1 + NW;
  constexpr int TPT = kCfMaxTiles / NT;   // tiles per thread
  constexpr int PER = (WIN + NT - 1) / NT;   // window slots per thread
  static_assert(WIN <= 2048, "entry slot field is 11 bits");
  __shared__ W2Lds<NW, WIN, NC> L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
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
  const int64_t ts_base = a.chunk_base[0];
  const int64_t seq_base = a.chunk_base[1];
  const int cp0 = a.cf.cap_phys[0], cp1 = a.cf.cap_phys[1];
  W2_STAMP(0);
  int wi = 0;   // window index (diagnostic stamps)

  // ---- key lane (tid < kpb; key = tid = 64 * wave + lane): pending count +
  // slots 0 / 1 in registers for the whole launch (as k_cfwalk).  A hot key's
  // records were diverted to the hot path this launch: its state is not ours.
  const bool klane = tid < kpb && !(a.hot_id && a.hot_id[((int64_t)tid << lg) | bucket] != kNotHot);
  uint32_t kcnt = 0;
  const int64_t kidx = (int64_t)bucket * kpb + tid;
  const uint32_t kb = (uint32_t)kidx * 8u, pb = (uint32_t)ks * 8u;
  auto sl_ld = [&](int j, int w) -> uint64_t {
    return *(const uint64_t*)((const char*)a.kslot + (kb + (uint32_t)(j * sw + w) * pb));
  };
  auto sl_st = [&](int j, int w, uint64_t v) {
    *(uint64_t*)((char*)a.kslot + (kb + (uint32_t)(j * sw + w) * pb)) = v;
  };
  const uint32_t hdr = klane ? a.khdr[kidx] : 0u;
  const bool ovf0 = klane && (hdr & kHdrOvf);
  const uint64_t ext0 = ovf0 ? a.kext[kidx] : 0ull;
  uint32_t ovo = (uint32_t)(ext0 >> 32);
  constexpr uint32_t kOvoWr = 0x80000000u;
  auto ovp = [&]() -> const uint64_t* {
    return ((ovo & kOvoWr) ? a.pool_wr : a.pool_rd) + (uint64_t)(ovo & ~kOvoWr) * (uint64_t)sw;
  };
  // bucket-major tile offsets: this thread's TPT tiles
  const uint16_t* rlo = a.tile_off + (int64_t)bucket * ntiles;
  const uint16_t* rhi = rlo + ntiles;
  const int tb = tid * TPT;
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
  uint32_t lop[TPT / 2];   // packed u16 segment starts inside each tile (setup only)
  uint32_t ys[TPT / 2];
  load_tile_off(rlo, lop);
  load_tile_off(rhi, ys);

  int n = ovf0 ? (int)(uint32_t)ext0 : (int)(hdr & 0xffu);
  constexpr bool c1 = NC > 0, c2 = NC > 1;
  uint64_t t0r = 0, t1r = 0, a0c0 = 0, a0c1 = 0, a1c0 = 0, a1c1 = 0;
  bool dirty = false;
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
  int scb = -1;   // this window's scratch copy of slots 2 .. min(n, S) - 1 (slot index base), or -1
  auto slot_word = [&](int j, int w) -> uint64_t {
    if (j >= 2) {
      if (j >= S) return ovp()[(int64_t)(j - S) * sw + w];
      if (scb >= 0) return L.scr[wave][(scb + j - 2) * (1 + NC) + (w == 0 ? 0 : w - 1)];
      return sl_ld(j, w);
    }
    const uint64_t m0 = 0ull - (uint64_t)(j == 0), m1 = ~m0;
    const uint64_t w0 = 0ull - (uint64_t)(w == 0), w2 = 0ull - (uint64_t)(w == 2);
    const uint64_t w3 = 0ull - (uint64_t)(w == 3);
    return (m0 & ((t0r & w0) | (a0c0 & w2) | (a0c1 & w3))) | (m1 & ((t1r & w0) | (a1c0 & w2) | (a1c1 & w3)));
  };

  // ---- segment sizes -> this thread's exclusive prefix over its tiles, kept
  // in LDS (thread-major columns: conflict-free) with the segment starts
  uint32_t nall;
  {
    uint32_t cnt[TPT];
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < TPT; ++i) {
      cnt[i] = ((ys[i >> 1] >> (16 * (i & 1))) & 0xffffu) - ((lop[i >> 1] >> (16 * (i & 1))) & 0xffffu);
      sum += cnt[i];
    }
    uint32_t off = bscan<NT>(sum, L.scratch, &nall);
#pragma unroll
    for (int i = 0; i < TPT; ++i) {
      L.tseg[i][tid] = off;
      off += cnt[i];
    }
    L.tseg[TPT][tid] = off;
#pragma unroll
    for (int i = 0; i < TPT / 2; ++i) L.tlop[i][tid] = lop[i];
  }
  if (tid < 2) L.bound[tid] = 0ull;
  // window extent: the largest tile t > ts with seg[t] <= lim (whole tiles);
  // every thread proposes from its own tiles
  auto propose = [&](int ts, uint32_t lim, int par) {
#ifdef W2_NO_PROP
    return;
#endif
    unsigned long long best = 0;
    int tbv = tb;
    asm volatile("" : "+v"(tbv));   // per-tile constants are recomputed, not hoisted and held
    if (tbv + TPT <= ts) return;   // all of this thread's tiles lie before the window
#pragma unroll
    for (int i = 0; i < TPT; ++i) {
      const int t = tbv + i + 1;
      const uint32_t sg = L.tseg[i + 1][tid];
      if (t > ts && t <= ntiles && sg <= lim) best = ((unsigned long long)t << 32) | sg;
    }
    if (best) atomicMax(&L.bound[par], best);
  };
  // wrec for whole tiles [t0, t1) of a window starting at record wb
  auto build_wrec = [&](int t0, int t1, uint32_t wb, int bufi) {
#ifdef W2_NO_BW
    return;
#endif
    int tbv = tb;
    asm volatile("" : "+v"(tbv));
    if (tbv + TPT <= t0 || tbv >= t1) return;
#pragma unroll 1
    for (int i = 0; i < TPT; ++i) {
      const int t = tbv + i;
      if (t < t0 || t >= t1) continue;
      const uint32_t s0 = L.tseg[i][tid], s1 = L.tseg[i + 1][tid];
      const uint32_t g0 = (uint32_t)t * (uint32_t)kCfTile + ((L.tlop[i >> 1][tid] >> (16 * (i & 1))) & 0xffffu) - s0;
      for (uint32_t g = s0; g < s1; ++g) L.wrec[bufi][g - wb] = g0 + g;
    }
  };
  lds_barrier();   // bound[] zeroed (bscan's barriers ordered the rest)
  W2_STAMP(1);

  // ---- window state (uniform)
  int t0 = 0, t1 = 0;          // whole-tile window [t0, t1), or the oversize tile t0
  uint32_t wb = 0, nw = 0;     // first record (bucket order) and records of the window
  bool over = false;           // window is a piece of tile t0's oversize segment
  uint32_t piece = 0, osz = 0; // piece's first arrival rank in the segment; segment size
  int buf = 0;
  bool pref = false;           // this window's records are already in x[] / wq[]
  int wpar = 0;                // window index parity (bound[] slot of the next window)
  uint4 x[PER];
  uint64_t y[PER];
  uint32_t wq[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    x[i] = make_uint4(0, 0, 0, 0);
    y[i] = 0;
    wq[i] = 0;
  }
  if (nall > 0) {
    propose(0, (uint32_t)WIN, 0);
    lds_barrier();
    const unsigned long long bd = L.bound[0];
    const int tn = (int)(bd >> 32);
    if (bd == 0ull || tn <= 0) {
      over = true;
      t0 = 0;
    } else {
      t1 = tn;
      nw = (uint32_t)bd;
    }
    lds_barrier();
    if (tid == 0) L.bound[0] = 0ull;   // read by everyone before the barrier above
  }
  // (an oversize window at tile 0 only starts once empty leading tiles are
  // skipped: seg[0] = 0 <= WIN always proposes t >= 1 unless tile 0 alone
  // exceeds WIN)
  while (nall > 0 && wb < nall) {
    // ---- oversize piece: its record table needs the tile's row bitmap
    // (rows are unique in a tile: rank = popcount below the row)
#ifndef W2_NO_OVER
    if (over) {
      const int64_t g0 = (int64_t)t0 * kCfTile + a.tile_off[(int64_t)bucket * ntiles + t0];
      const uint64_t* tr = a.recs + g0 * RW;
      if (piece == 0) {
        osz = (uint32_t)a.tile_off[(int64_t)(bucket + 1) * ntiles + t0] - (uint32_t)a.tile_off[(int64_t)bucket * ntiles + t0];
        for (int w = tid; w < kCfTile / 32; w += NT) L.obits[w] = 0;
        lds_barrier();
        for (uint32_t j = tid; j < osz; j += NT) {
          const uint32_t row = w2_row(tr[(int64_t)j * RW]);
          atomicOr(&L.obits[row >> 5], 1u << (row & 31));
        }
        lds_barrier();
        const uint32_t pc = tid < kCfTile / 32 ? (uint32_t)__popc(L.obits[tid]) : 0u;
        uint32_t tot;
        const uint32_t off = bscan<NT>(pc, L.scratch, &tot);
        if (tid < kCfTile / 32) L.opre[tid] = (uint16_t)off;
        lds_barrier();
      }
      nw = min((uint32_t)WIN, osz - piece);
      for (uint32_t j = tid; j < osz; j += NT) {
        const uint32_t row = w2_row(tr[(int64_t)j * RW]);
        const uint32_t rank = L.opre[row >> 5] + (uint32_t)__popc(L.obits[row >> 5] & ((1u << (row & 31)) - 1u));
        if (rank >= piece && rank < piece + nw) L.wrec[buf][rank - piece] = (uint32_t)(g0 + j);
      }
      lds_barrier();
      pref = false;
    } else
#endif
    if (!pref) {
      build_wrec(t0, t1, wb, buf);
      lds_barrier();
    }
    if (!pref) {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const uint32_t q = tid + i * NT;
        if (q < nw) {
          wq[i] = L.wrec[buf][q];
          const uint64_t* r = a.recs + (int64_t)wq[i] * RW;
          x[i] = gload4(r);
          if (NW > 1) y[i] = r[2];
        }
      }
    }

    // ================= scratch: key lanes' slots 2 .. min(n, S) - 1, loads
    // issued before this window's records are waited for (they overlap)
    {
      const int need = (klane && n > 2) ? min(n, S) - 2 : 0;
      const uint32_t incl = wave_incl_scan((uint32_t)need);
      const int off = (int)(incl - (uint32_t)need);
      scb = (need > 0 && off + need <= kW2Scr) ? off : -1;
      if (scb >= 0) {
        for (int j0 = 0; j0 < need; j0 += 4) {
          uint64_t v[4][1 + NC];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const bool ok = j0 + u < need;
            v[u][0] = ok ? sl_ld(2 + j0 + u, 0) : 0ull;
#pragma unroll
            for (int c = 0; c < NC; ++c) v[u][1 + c] = ok ? sl_ld(2 + j0 + u, 2 + c) : 0ull;
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (j0 + u < need) {
#pragma unroll
              for (int c = 0; c <= NC; ++c) L.scr[wave][(scb + j0 + u) * (1 + NC) + c] = v[u][c];
            }
        }
      }
    }
    // ================= phase A: records -> LDS by slot, owner counts, next extent
    uint32_t own[PER], rk[PER], entv[PER];
    {
      uint32_t cnt[kOwners];
#pragma unroll
      for (int o = 0; o < kOwners; ++o) cnt[o] = 0;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const uint32_t q = tid + i * NT;
        const bool v = q < nw;
        const uint64_t w0 = ((uint64_t)x[i].y << 32) | x[i].x;
        const uint32_t k = w2_key(w0);
        own[i] = v ? (k >> 6) : (uint32_t)kOwners;
        entv[i] = q | ((k & 63u) << 11) | (w2_role(w0) << 17);
        if (v) {
          const uint32_t hs = (wq[i] & ~(uint32_t)(kCfTile - 1)) + w2_row(w0);
          L.rts[q] = (uint32_t)w0;
          L.rseq[q] = a.in_seq ? (uint32_t)((int64_t)a.in_seq[(int64_t)hs * a.in_rec_words] - seq_base) : hs;
          if (NW > 0) L.rcap[0][q] = ((uint64_t)x[i].w << 32) | x[i].z;
          if (NW > 1) L.rcap[NW > 1 ? 1 : 0][q] = y[i];
        }
#pragma unroll
        for (int o = 0; o < kOwners; ++o) {
          const uint64_t m = __ballot(own[i] == (uint32_t)o);
          if (own[i] == (uint32_t)o) rk[i] = cnt[o] + (uint32_t)__popcll(m & lt);
          cnt[o] += (uint32_t)__popcll(m);
        }
      }
      uint32_t mine = 0;
#pragma unroll
      for (int o = 0; o < kOwners; ++o) mine = lane == o ? cnt[o] : mine;
      if (lane < kOwners) L.ocnt[wave][lane] = mine;
    }
    // the next window: pieces of this oversize segment, or whole tiles from
    // the tile after this window
    const bool more_pieces = over && piece + nw < osz;
    const int nts = over ? t0 + 1 : t1;
    const uint32_t nwb = wb + nw;
    if (!more_pieces && nwb < nall) propose(nts, nwb + (uint32_t)WIN, wpar ^ 1);
    W2_STAMPW(wi, 2, -1);
    lds_barrier();   // #1
    W2_STAMPW(wi, 3, 12);

    // ================= phase B: owner ranges, next window's record table
    uint32_t os, oe;
    {
      const uint32_t c = L.ocnt[lane & (kOwners - 1)][lane >> 3];   // lane = owner * 8 + producer
      const uint32_t incl = wave_incl_scan(kOwners == 8 ? c : 0u);
      const uint32_t ex = incl - c;
      const uint32_t total = __shfl(incl, 63, 64);
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int src = (int)(own[i] < (uint32_t)kOwners ? own[i] : 0u) * kOwners + wave;
        const uint32_t base = __shfl(ex, src, 64);
        if (own[i] < (uint32_t)kOwners) L.ent[base + rk[i]] = entv[i];
      }
      os = __shfl(ex, wave * kOwners, 64);
      oe = wave + 1 < kOwners ? __shfl(ex, (wave + 1) * kOwners, 64) : total;
    }
    bool next_over = false, next_none = false;
    int nt1 = 0;
    uint32_t nnw = 0;
    if (more_pieces) {
      next_over = true;
    } else if (nwb >= nall) {
      next_none = true;
    } else {
      const unsigned long long bd = L.bound[wpar ^ 1];
      const int tn = (int)(bd >> 32);
      if (bd == 0ull || tn <= nts) {
        next_over = true;
      } else {
        nt1 = tn;
        nnw = (uint32_t)bd - nwb;
        build_wrec(nts, nt1, nwb, buf ^ 1);
      }
    }
    W2_STAMPW(wi, 4, -1);
    lds_barrier();   // #2

#ifdef W2_NOPREF   // experiment: no prefetch (the next window loads at its start)
    const bool next_pref = false;
#else
    const bool next_pref = !next_over && !next_none;
#endif

    // ================= phase C: this wave's keys, no workgroup barrier
    const uint32_t nl = oe - os;   // records of this wave's keys (uniform)
    W2_STAMPW(wi, 5, 13);
#ifndef W2_NO_C
    // C1: counting sort by key, then arrival order inside each key run
    L.wk[wave][lane] = 0;
    wsync();
    for (uint32_t e = lane; e < nl; e += 64) {
      const uint32_t en = L.ent[os + e];
      const uint32_t r = atomicAdd(&L.wk[wave][e_key(en)], 1u);
      L.ent[os + e] = en | (r << 20);
    }
    wsync();
    const uint32_t kc = L.wk[wave][lane];        // records of this lane's key
    const uint32_t kst = wave_incl_scan(kc) - kc;   // its run start in the owner range
    L.wk[wave][lane] = kst;
    wsync();
    for (uint32_t e = lane; e < nl; e += 64) {
      const uint32_t en = L.ent[os + e];
      L.ent2[os + L.wk[wave][e_key(en)] + (en >> 20)] = en & 0xfffffu;
    }
    wsync();
    for (uint32_t e = lane; e < nl; e += 64) {
      const uint32_t en = L.ent2[os + e];
      const uint32_t k6 = e_key(en);
      const uint32_t r0 = L.wk[wave][k6];
      const uint32_t r1 = k6 < 63 ? L.wk[wave][k6 + 1] : nl;
      const uint32_t mys = L.rseq[e_slot(en)];
      uint32_t ar = 0;
      for (uint32_t j = r0; j < r1; ++j) ar += L.rseq[e_slot(L.ent2[os + j])] < mys ? 1u : 0u;
      L.ent[os + r0 + ar] = en;
    }
    wsync();
    W2_STAMPW(wi, 6, -1);
    // C2: key lane: next B of every record (backward over the run), first /
    // last B, last A
    const uint32_t r0 = os + kst, r1 = r0 + kc;
    kcnt += kc;
    uint16_t fbs = kNoSlot;        // first B of the run (slot)
    uint32_t lbp = kNoPos;         // last B of the run (position)
    bool hasa = false;
    uint32_t last_a = 0;           // ts - base of the run's last A
    for (uint32_t s = r1; s-- > r0;) {
      const uint32_t en = L.ent[s];
      const uint32_t role = e_role(en);
      L.nextb[s] = fbs;
      if ((role & ROLE_A) && !hasa) {
        hasa = true;
        last_a = L.rts[e_slot(en)];
      }
      if (role & ROLE_B) {
        if (lbp == kNoPos) lbp = s;
        fbs = (uint16_t)e_slot(en);
      }
    }
    if (a.stamps && (a.ablate & 256) && klane && kc > 0) {   // diagnostics: list lengths of active keys
      unsigned long long* c = (unsigned long long*)&a.stamps[4095 * 16];
      atomicAdd(&c[0], 1ull);
      if (n > 2) atomicAdd(&c[1], 1ull);
      if (n > 4) atomicAdd(&c[2], 1ull);
      if (n > 6) atomicAdd(&c[3], 1ull);
      if (n > 8) atomicAdd(&c[4], 1ull);
      if (__ballot(n > 2) && lane == __ffsll((long long)__ballot(klane && kc > 0)) - 1) atomicAdd(&c[5], 1ull);
      if (__ballot(n > 4) && lane == __ffsll((long long)__ballot(klane && kc > 0)) - 1) atomicAdd(&c[6], 1ull);
      if (lane == __ffsll((long long)__ballot(klane && kc > 0)) - 1) atomicAdd(&c[7], 1ull);
    }
    // C3: key lane: carried partials completed by the run's first B.  Lists of
    // at most two partials (the common case) are decided from registers: no
    // global load in this phase may wait for the next window's loads.
    int cfirst = 0, cm = 0;
    uint64_t e00 = 0, e01 = 0, e10 = 0, e11 = 0;
    auto within_of = [&](int64_t d) { return W < 0 || (d < 0 ? -d : d) <= W; };
    if (klane && kc > 0 && fbs != kNoSlot && n > 0) {
      const int64_t tbs = ts_base + (int64_t)L.rts[fbs];
      if (n <= 2 && !(a.ablate & 16)) {
        const bool w0 = within_of(tbs - (int64_t)t0r);
        const bool w1 = n > 1 && within_of(tbs - (int64_t)t1r);
        cfirst = w0 ? 0 : (w1 ? 1 : n);
        cm = n - cfirst;
        e00 = cfirst == 0 ? a0c0 : a1c0;
        e01 = cfirst == 0 ? a0c1 : a1c1;
        e10 = a1c0;
        e11 = a1c1;
      } else {
        cfirst = n;
        for (int j = 0; j < n; ++j) {
          if (within_of(tbs - (int64_t)slot_word(j, 0))) {
            cfirst = j;
            break;
          }
        }
        cm = n - cfirst;
        if (cm > 0) {
          e00 = c1 ? slot_word(cfirst, 2) : 0ull;
          e01 = c2 ? slot_word(cfirst, 3) : 0ull;
        }
        if (cm > 1) {
          e10 = c1 ? slot_word(cfirst + 1, 2) : 0ull;
          e11 = c2 ? slot_word(cfirst + 1, 3) : 0ull;
        }
      }
    }
    W2_STAMPW(wi, 7, -1);
    wsync();   // nextb written by key lanes, read by position lanes below
    // C4: output rows per sorted position (record matches + carried matches
    // at the run start), one reservation per wave
    uint32_t rows = 0;
    for (uint32_t e0 = 0; e0 < nl; e0 += 64) {
      const uint32_t e = e0 + lane;
      const uint32_t en = e < nl ? L.ent[os + e] : 0u;
      const uint32_t k6 = e_key(en);
      const int cmk = __shfl(cm, (int)k6, 64);
      const uint32_t kstk = __shfl(kst, (int)k6, 64);
      uint32_t val = 0;
      if (e < nl) {
        const uint16_t nb = L.nextb[os + e];
        if ((e_role(en) & ROLE_A) && nb != kNoSlot)
          val = within_of((int64_t)L.rts[nb] - (int64_t)L.rts[e_slot(en)]) ? 1u : 0u;
        if (e == kstk) val += (uint32_t)cmk;
      }
      const uint32_t incl = wave_incl_scan(val);
      if (e < nl) L.vout[os + e] = rows + incl - val;
      rows += __shfl(incl, 63, 64);
    }
    if (lane == 0) L.wrows[wave] = rows;
#endif
    // ================= the window's output reservation: one atomic per
    // workgroup (one per wave on the single output cursor serialises every
    // wave of the chip); the key lanes' commit runs while it is in flight
    lds_barrier();   // #C: every wave's row count
    if (tid == 0) {
      unsigned long long tot = 0;
#pragma unroll
      for (int w = 0; w < kOwners; ++w) tot += L.wrows[w];
      unsigned long long b = tot ? atomicAdd(a.out.count, tot) : 0ull;
#pragma unroll
      for (int w = 0; w < kOwners; ++w) {
        L.wbase[w] = b;
        b += L.wrows[w];
      }
    }
#ifndef W2_NO_C
    W2_STAMPW(wi, 8, -1);
    // C5: key lane: survivors and state commit (no output yet: the carried
    // rows are emitted after the reservation, from values read before it)
    int nn_new = n;
    uint32_t ovo_new = ovo;
    // a lane whose carried rows read slots >= 2 from HBM (no scratch copy)
    // commits only after emitting them: the commit rewrites those slots
    const bool late = klane && kc > 0 && cm > 2 && scb < 0;
    auto commit = [&]() {
      const bool prune = W >= 0 && hasa;
      const int64_t last_a_ts = ts_base + (int64_t)last_a;
      int nn = 0;
      const uint32_t from = (lbp == kNoPos ? r0 : lbp);
      int cap = (lbp == kNoPos ? n : 0) + (int)(r1 - from);
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
      if (lbp == kNoPos) {
        if (n <= 2 && !(a.ablate & 32)) {   // registers only
          const bool d0 = n > 0 && prune && last_a_ts - (int64_t)t0r > W;
          const bool d1 = d0 && n > 1 && prune && last_a_ts - (int64_t)t1r > W;
          const int drop = d0 ? (d1 ? 2 : 1) : 0;
          if (drop == 0 && cap <= S) {
            nn = n;
          } else {
            const uint64_t s1t = t1r, s1a = a1c0, s1b = a1c1;
            if (drop == 0 && n > 0) put_slot(t0r, a0c0, a0c1);
            if (drop <= 1 && n > 1) put_slot(s1t, s1a, s1b);
          }
        } else {
          int drop = 0;
          while (drop < n && prune && last_a_ts - (int64_t)slot_word(drop, 0) > W) ++drop;
          if (drop == 0 && cap <= S) {
            nn = n;   // unchanged, in place
          } else {
            for (int j = drop; j < n; ++j) {
              const uint64_t ts = slot_word(j, 0);
              const uint64_t x0 = c1 ? slot_word(j, 2) : 0ull, x1 = c2 ? slot_word(j, 3) : 0ull;
              put_slot(ts, x0, x1);
            }
          }
        }
      }
      // partials created after the last B (a record that is both B and A
      // starts a partial after completing others)
      for (uint32_t q = from; q < r1; ++q) {
        const uint32_t en = L.ent[q];
        if (!(e_role(en) & ROLE_A)) continue;
        const uint32_t sl = e_slot(en);
        const int64_t ats = ts_base + (int64_t)L.rts[sl];
        if (prune && last_a_ts - ats > W) continue;
        if (nn >= cap) {   // only after the pool ran out (ERR_POOL is set)
          set_err(a.err, ERR_POOL);
          break;
        }
        const uint64_t a0 = NW > 0 ? L.rcap[0][sl] : 0ull, a1 = NW > 1 ? L.rcap[NW > 1 ? 1 : 0][sl] : 0ull;
        put_slot((uint64_t)ats, cp0 < 0 ? (uint64_t)ats : (cp0 == 0 ? a0 : a1),
                 cp1 < 0 ? (uint64_t)ats : (cp1 == 0 ? a0 : a1));
      }
      dirty |= nn != n;
      nn_new = nn;
      if (nn > S) ovo_new = noff | kOvoWr;
    };
    if (klane && kc > 0 && !late) commit();
#endif
    lds_barrier();   // #D: the output bases
    const unsigned long long obase = L.wbase[wave];
    W2_STAMPW(wi, 9, -1);
    // ================= C0: the next window's records go out only now: from
    // here on this wave issues stores only, so nothing waits for these loads
    // until the next window's phase A (vmcnt counts loads and stores in issue
    // order: the reservation atomic and the key lanes' slot loads above would
    // wait for them)
    if (next_pref) {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const uint32_t q = tid + i * NT;
        if (q < nnw) {
          wq[i] = L.wrec[buf ^ 1][q];
          const uint64_t* r = a.recs + (int64_t)wq[i] * RW;
          x[i] = gload4(r);
          if (NW > 1) y[i] = r[2];
        }
      }
    }
#ifndef W2_NO_C
    // C5b: key lane: carried rows completed by the run's first B (captures
    // read before the commit; slots >= 2 from this window's scratch copy)
    if (klane && kc > 0 && cm) {
      const int64_t kv = (((int64_t)tid << lg) | bucket) * p.key_stride + p.key_offset;
      const int64_t bts = ts_base + (int64_t)L.rts[fbs];
      const uint64_t b0 = NW > 0 ? L.rcap[0][fbs] : 0ull, b1 = NW > 1 ? L.rcap[NW > 1 ? 1 : 0][fbs] : 0ull;
      const unsigned long long rb = obase + L.vout[r0];
      const int64_t bseq = seq_base + (int64_t)L.rseq[fbs];
#ifndef W2_NO_EMIT
      w2_emit<KR>(a, rb, kv, e00, e01, b0, b1, bts, bseq);
      if (cm > 1) w2_emit<KR>(a, rb + 1, kv, e10, e11, b0, b1, bts, bseq);
      for (int j = 2; j < cm; ++j)   // long lists (rare)
        w2_emit<KR>(a, rb + j, kv, c1 ? slot_word(cfirst + j, 2) : 0ull, c2 ? slot_word(cfirst + j, 3) : 0ull, b0, b1,
                    bts, bseq);
#endif
    }
    if (late) commit();
    n = nn_new;
    ovo = ovo_new;
    // C6: record matches, lane per sorted position (stores only)
    for (uint32_t e0 = 0; e0 < nl; e0 += 64) {
      const uint32_t e = e0 + lane;
      const uint32_t en = e < nl ? L.ent[os + e] : 0u;
      const uint32_t k6 = e_key(en);
      const int cmk = __shfl(cm, (int)k6, 64);
      const uint32_t kstk = __shfl(kst, (int)k6, 64);
      if (e >= nl || !(e_role(en) & ROLE_A)) continue;
      const uint16_t nb = L.nextb[os + e];
      if (nb == kNoSlot) continue;
      const uint32_t sl = e_slot(en);
      if (!within_of((int64_t)L.rts[nb] - (int64_t)L.rts[sl])) continue;
      const int64_t ats = ts_base + (int64_t)L.rts[sl];
      const int64_t bts = ts_base + (int64_t)L.rts[nb];
      const uint64_t a0 = NW > 0 ? L.rcap[0][sl] : 0ull, a1 = NW > 1 ? L.rcap[NW > 1 ? 1 : 0][sl] : 0ull;
      const uint64_t x0 = cp0 < 0 ? (uint64_t)ats : (cp0 == 0 ? a0 : a1);
      const uint64_t x1 = cp1 < 0 ? (uint64_t)ats : (cp1 == 0 ? a0 : a1);
      const int64_t kl = ((int64_t)(wave * 64 + (int)k6) << lg) | bucket;
      const unsigned extra = e == kstk ? (unsigned)cmk : 0u;
#ifndef W2_NO_EMIT
      w2_emit<KR>(a, obase + L.vout[os + e] + extra, kl * p.key_stride + p.key_offset, x0, x1,
                  NW > 0 ? L.rcap[0][nb] : 0ull, NW > 1 ? L.rcap[NW > 1 ? 1 : 0][nb] : 0ull, bts,
                  seq_base + (int64_t)L.rseq[nb]);
#endif
    }
#endif
    W2_STAMPW(wi, 10, 14);
    // ================= window end: the next window
    if (tid == 0) L.bound[wpar] = 0ull;   // read in the previous window's phase B
    lds_barrier();   // #3: LDS arrays are reused
    W2_STAMPW(wi, 11, -1);
    ++wi;
    if (next_none) break;
    if (over && more_pieces) {
      piece += nw;
    } else if (over) {
      over = false;
    }
    wb = nwb;
    if (next_over) {
      if (!more_pieces) {   // a new oversize tile
        over = true;
        piece = 0;
        t0 = nts;
      }
      pref = false;
    } else {
      t0 = nts;
      t1 = nt1;
      nw = nnw;
      pref = next_pref;
      buf ^= 1;
    }
    wpar ^= 1;
  }

  W2_STAMP(15);
  // ---- hot-key candidates: keys that made this bucket long (hot.hip)
  if (klane && a.hot_thresh && kcnt > a.hot_thresh) {
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

template <int NW, bool KR>
static void launch_cf_walk2_nc(const CfWalkArgs& a, int nbuckets, hipStream_t s) {
  const dim3 g((unsigned)nbuckets), b(kCfWalkThreads);
  constexpr int WIN = w2_window<NW>();
#ifdef W2_ONE   // resource-usage experiments: one instantiation
  if constexpr (NW == 1 && !KR) hipLaunchKernelGGL((k_cfwalk2<NW, KR, 1, WIN>), g, b, 0, s, a);
#else
  switch (a.pat.slot_words - 2) {
    case 0: hipLaunchKernelGGL((k_cfwalk2<NW, KR, 0, WIN>), g, b, 0, s, a); break;
    case 1: hipLaunchKernelGGL((k_cfwalk2<NW, KR, 1, WIN>), g, b, 0, s, a); break;
    default: hipLaunchKernelGGL((k_cfwalk2<NW, KR, 2, WIN>), g, b, 0, s, a); break;
  }
#endif
}

void launch_cf_walk2(const CfWalkArgs& a, int nbuckets, hipStream_t s) {
  const bool kr = a.key_rev != nullptr;
  switch (a.cf.nw) {
    case 0: kr ? launch_cf_walk2_nc<0, true>(a, nbuckets, s) : launch_cf_walk2_nc<0, false>(a, nbuckets, s); break;
    case 1: kr ? launch_cf_walk2_nc<1, true>(a, nbuckets, s) : launch_cf_walk2_nc<1, false>(a, nbuckets, s); break;
    default: kr ? launch_cf_walk2_nc<2, true>(a, nbuckets, s) : launch_cf_walk2_nc<2, false>(a, nbuckets, s); break;
  }
}

}  // namespace cep
