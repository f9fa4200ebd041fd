// gfx950 kernels for the flink-siddhi hot path (the Siddhi work behind
// AbstractSiddhiOperator.java:130 `InputHandler.send(ts, row)`):
//
//   k_filter     `from S[expr] select ... insert into O`: columnar predicate
//                evaluation + order-preserving compaction (64-bit wave ballot,
//                mbcnt ranks, single-pass decoupled look-back across tiles) +
//                projection.  HBM-bound: reads the predicate columns once,
//                writes the selected rows once.
//   k_partition  keyed pattern, pass 1: evaluates the state filters f / g on
//                the event columns, drops events no state can use (exact for
//                `->` patterns) and scatters the rest as
//                fixed-size records into per-tile key-bucket segments
//                (LDS histogram + LDS scan; no global atomics).
//   k_walk       keyed pattern, pass 2: one workgroup per key bucket gathers
//                its segments (tile order = arrival order), groups them by
//                key in LDS, and runs one NFA lane per key: `within` pruning,
//                completion of pending partials in creation order, `every`
//                re-arming.  Matches are reserved with one atomic per window
//                and projected in place.
//   k_generate   counter-based synthetic workload.
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "vm.h"

namespace cep {

namespace {

constexpr uint64_t kStatusShift = 62;
constexpr uint64_t kValueMask = (1ull << 62) - 1;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ void set_err(unsigned int* err, unsigned int bit) {
  if (err) atomicOr(err, bit);
}

// Block-wide exclusive scan of one value per thread (256 threads).
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* scratch /*>=5*/,
                                                    uint32_t* total) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) scratch[wave] = x;
  __syncthreads();
  if (tid == 0) {
    uint32_t s = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
      uint32_t t = scratch[w];
      scratch[w] = s;
      s += t;
    }
    scratch[4] = s;
  }
  __syncthreads();
  uint32_t r = scratch[wave] + x - v;
  *total = scratch[4];
  __syncthreads();
  return r;
}

struct RowEnv {
  const RowsArgs* r;
  int64_t row;
  __device__ uint64_t col(int c, int type) const { return load_col(r->cols.p[c], type, row); }
  __device__ uint64_t cap(int) const { return 0; }
  __device__ uint64_t outv(int, bool* n) const { *n = true; return 0; }
  __device__ uint64_t agg(int, bool* n) const { *n = true; return 0; }
  __device__ int64_t ts() const { return r->ts[row]; }
};

__device__ __forceinline__ bool eval_pred(const VmArgs& vm, int prog, uint64_t* R,
                                          const RowEnv& env) {
  if (prog < 0) return true;
  bool isnull = false;
  uint64_t v = vm_eval(vm.code, vm.konst, prog, R, threadIdx.x, blockDim.x, env, &isnull);
  return !isnull && (v & 1u);
}

}  // namespace

// ============================================================== k_filter ==
__global__ __launch_bounds__(kFilterThreads) void k_filter(FilterArgs a) {
  __shared__ uint64_t R[kMaxRegs * kFilterThreads];
  __shared__ uint32_t cnt[kFilterItems * 4];
  __shared__ uint32_t s_tile;
  __shared__ unsigned long long s_prefix;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int kTile = kFilterThreads * kFilterItems;

  if (tid == 0) s_tile = atomicAdd(a.ticket, 1u);
  __syncthreads();
  const int64_t tile = s_tile;
  const int64_t base = tile * kTile;

  uint32_t selmask = 0;
#pragma unroll 1
  for (int e = 0; e < kFilterItems; ++e) {
    const int64_t r = base + (int64_t)e * kFilterThreads + tid;
    bool sel = false;
    if (r < a.rows.n) {
      const int64_t row = a.rows.row0 + r;
      const int s = a.rows.stream ? (int)a.rows.stream[row] : a.rows.input;
      if (s == a.in_stream) sel = eval_pred(a.vm, a.filter_prog, R, RowEnv{&a.rows, row});
    }
    const uint64_t bal = __ballot(sel);
    if (lane == 0) cnt[e * 4 + wave] = (uint32_t)__popcll(bal);
    selmask |= (sel ? 1u : 0u) << e;
  }
  __syncthreads();
  // exclusive scan over (item, wave) in row order
  if (tid == 0) {
    uint32_t s = 0;
    for (int i = 0; i < kFilterItems * 4; ++i) {
      uint32_t t = cnt[i];
      cnt[i] = s;
      s += t;
    }
    const unsigned long long total = s;
    unsigned long long* flags = a.tile_state;
    // publish the aggregate, then look back for the exclusive prefix
    unsigned long long prefix = 0;
    if (tile == 0) {
      prefix = __hip_atomic_load(a.out.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_store(&flags[tile], (1ull << kStatusShift) | total, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      int64_t j = tile - 1;
      while (j >= 0) {
        unsigned long long v;
        unsigned spins = 0;
        do {
          v = __hip_atomic_load(&flags[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((v >> kStatusShift) == 0) {
            __builtin_amdgcn_s_sleep(1);
            ++spins;
          }
        } while ((v >> kStatusShift) == 0 && spins < (1u << 22));
        if ((v >> kStatusShift) == 0) {   // predecessor never published: give up loudly
          set_err(a.err, ERR_WINDOW);
          break;
        }
        prefix += v & kValueMask;
        if ((v >> kStatusShift) == 2) break;
        --j;
      }
    }
    __hip_atomic_store(&flags[tile], (2ull << kStatusShift) | (prefix + total),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_prefix = prefix;
    if (tile == (int64_t)gridDim.x - 1)
      __hip_atomic_store(a.out.count, prefix + total, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const unsigned long long prefix = s_prefix;
#pragma unroll 1
  for (int e = 0; e < kFilterItems; ++e) {
    const bool sel = (selmask >> e) & 1u;
    const uint64_t bal = __ballot(sel);
    if (!sel) continue;
    const int64_t r = base + (int64_t)e * kFilterThreads + tid;
    const int64_t row = a.rows.row0 + r;
    const int64_t pos = (int64_t)prefix + cnt[e * 4 + wave] + mbcnt(bal);
    if (pos >= a.out.cap) continue;
    RowEnv env{&a.rows, row};
    for (int c = 0; c < a.out.ncols; ++c) {
      bool isnull = false;
      uint64_t v = vm_eval(a.vm.code, a.vm.konst, a.out.prog[c], R, tid, kFilterThreads, env,
                           &isnull);
      store_col(a.out.col[c], a.out.type[c], pos, isnull ? 0 : v);
    }
    a.out.ts[pos] = a.rows.ts[row];
    a.out.seq[pos] = a.rows.seq0 + row;
  }
}

void launch_filter(const FilterArgs& a, int64_t ntiles, hipStream_t s) {
  hipLaunchKernelGGL(k_filter, dim3((unsigned)ntiles), dim3(kFilterThreads), 0, s, a);
}

// =========================================================== k_partition ==
// Record layout (8-byte words):
//   w0 = dense key (low 32) | role << 32 | input handle << 40
//   w1 = arrival sequence number,  w2 = event timestamp,
//   w3.. = carried columns (rec_a for A-stream rows, rec_b for B-stream rows)
__global__ __launch_bounds__(kPartThreads) void k_partition(PartArgs a) {
  __shared__ uint64_t R[kMaxRegs * kPartThreads];
  __shared__ uint32_t hist[4096 + 1];
  __shared__ uint32_t scratch[8];
  const int tid = threadIdx.x;
  const int64_t tile = blockIdx.x;
  const PatternArgs& p = a.pat;
  const int P = a.route_world > 0 ? a.route_world : (1 << p.buckets_log2);
  for (int i = tid; i <= P; i += kPartThreads) hist[i] = 0;
  __syncthreads();

  uint32_t packed[kPartItems];
  const int64_t tbase = tile * (int64_t)a.tile_rows;
#pragma unroll
  for (int e = 0; e < kPartItems; ++e) {
    packed[e] = 0xffffffffu;
    const int64_t r = tbase + (int64_t)e * kPartThreads + tid;
    if (r >= a.rows.n) continue;
    uint32_t role = 0;
    int s;
    int64_t key = 0;
    if (a.from_records) {
      const uint64_t* rec = a.in_recs + r * p.rec_words;
      const uint64_t h = rec[0];
      role = (uint32_t)(h >> 32) & 0xffu;
      s = (int)(h >> 40) & 0xff;
      key = (int64_t)(uint32_t)h;
    } else {
      const int64_t row = a.rows.row0 + r;
      s = a.rows.stream ? (int)a.rows.stream[row] : a.rows.input;
      if (p.within >= 0) {
        const int64_t prev = row > 0 ? a.rows.ts[row - 1] : a.rows.prev_ts;
        if (a.rows.ts[row] < prev) set_err(a.err, ERR_ORDER);
      }
      RowEnv env{&a.rows, row};
      if (s == p.a_stream && eval_pred(a.vm, p.f_prog, R, env)) role |= ROLE_A;
      if (s == p.b_stream) {
        if (p.g_walk_prog >= 0) role |= ROLE_B;
        else if (eval_pred(a.vm, p.g_raw_prog, R, env)) role |= ROLE_B | ROLE_G;
      }
      if (role) {
        const int kc = s == p.a_stream ? p.key_col_a : p.key_col_b;
        if (kc >= 0) key = (int64_t)load_col(a.rows.cols.p[kc], a.rows.cols.t[kc], row);
      }
    }
    if (!role) continue;
    int bucket;
    if (a.route_world > 0) {
      if (key < 0) { set_err(a.err, ERR_KEY_RANGE); continue; }
      bucket = (int)(key % a.route_world);
    } else {
      if (key < 0 || (key % p.key_stride) != p.key_offset) {
        set_err(a.err, ERR_KEY_RANGE);
        continue;
      }
      const int64_t kl = key / p.key_stride;
      if (kl >= p.key_capacity) { set_err(a.err, ERR_KEY_RANGE); continue; }
      bucket = (int)(kl & (P - 1));
    }
    const uint32_t rank = atomicAdd(&hist[bucket], 1u);
    // bits 0-10 rank in tile, 11-13 role, 14-25 bucket
    packed[e] = ((uint32_t)bucket << 14) | (role << 11) | rank;
  }
  __syncthreads();
  // exclusive scan of the P bucket counts (P <= 4096: 16 per thread)
  {
    const int per = (P + kPartThreads - 1) / kPartThreads;
    uint32_t local[16];
    uint32_t sum = 0;
    for (int i = 0; i < per; ++i) {
      const int idx = tid * per + i;
      local[i] = idx < P ? hist[idx] : 0u;
      sum += local[i];
    }
    uint32_t total;
    uint32_t off = block_excl_scan(sum, scratch, &total);
    for (int i = 0; i < per; ++i) {
      const int idx = tid * per + i;
      if (idx < P) hist[idx] = off;
      off += local[i];
    }
    if (tid == 0) hist[P] = total;
  }
  __syncthreads();
  uint16_t* toff = a.tile_off + tile * (int64_t)(P + 1);
  for (int i = tid; i <= P; i += kPartThreads) toff[i] = (uint16_t)hist[i];

#pragma unroll
  for (int e = 0; e < kPartItems; ++e) {
    if (packed[e] == 0xffffffffu) continue;
    const int64_t r = tbase + (int64_t)e * kPartThreads + tid;
    const uint32_t b = packed[e] >> 14, rank = packed[e] & 0x7ffu;
    const uint32_t role = (packed[e] >> 11) & 7u;
    const int64_t pos = tbase + hist[b] + rank;
    uint64_t* out = a.recs + pos * p.rec_words;
    if (a.from_records) {
      const uint64_t* in = a.in_recs + r * p.rec_words;
      for (int w = 0; w < p.rec_words; ++w) out[w] = in[w];
      if (a.route_world <= 0) {
        const int64_t kl = (int64_t)(uint32_t)in[0] / p.key_stride;
        out[0] = (in[0] & ~0xffffffffull) | (uint64_t)(uint32_t)kl;
      }
      continue;
    }
    const int64_t row = a.rows.row0 + r;
    const int s = a.rows.stream ? (int)a.rows.stream[row] : a.rows.input;
    const int kc = s == p.a_stream ? p.key_col_a : p.key_col_b;
    const int64_t key = kc >= 0 ? (int64_t)load_col(a.rows.cols.p[kc], a.rows.cols.t[kc], row) : 0;
    const uint64_t kfield = a.route_world > 0 ? (uint64_t)(uint32_t)key
                                              : (uint64_t)(uint32_t)(key / p.key_stride);
    out[0] = kfield | ((uint64_t)role << 32) | ((uint64_t)(uint32_t)s << 40);
    out[1] = (uint64_t)(a.rows.seq0 + row);
    out[2] = (uint64_t)a.rows.ts[row];
    const int nrc = s == p.a_stream ? p.nrec_a : p.nrec_b;
    for (int c = 0; c < nrc; ++c) {
      const int col = s == p.a_stream ? p.rec_a[c] : p.rec_b[c];
      out[3 + c] = load_col(a.rows.cols.p[col], a.rows.cols.t[col], row);
    }
  }
}

void launch_partition(const PartArgs& a, int64_t ntiles, hipStream_t s) {
  hipLaunchKernelGGL(k_partition, dim3((unsigned)ntiles), dim3(kPartThreads), 0, s, a);
}

// ================================================================ k_walk ==
namespace {

constexpr int kEntryRec = 64;   // working-list ids >= 64 name window records

struct WalkLds {
  uint32_t seg[kWalkMaxTiles + 1];   // exclusive prefix of segment sizes
  uint32_t wrec[kWalkWindow];        // global record index per window slot
  uint32_t wseq[kWalkWindow];        // chunk-relative sequence number
  uint16_t wkey[kWalkWindow];        // key within the bucket
  uint16_t sorted[kWalkWindow];      // window slots grouped by key, arrival order
  uint32_t kstart[kWalkMaxKeys + 1];
  uint32_t kcur[kWalkMaxKeys];
  uint16_t plist[kMaxPending * kWalkThreads]; // per-thread working list [i][tid]
  uint64_t R[kMaxRegs * kWalkThreads];
  uint32_t scratch[8];
  unsigned long long base;
  uint32_t t1;
};

struct MatchEnv {
  const uint64_t* slot;    // pending entry captured words (slot+2) or nullptr
  const uint64_t* arec;    // pending entry as an A record (rec+3) or nullptr
  const int32_t* cap_from_rec;
  const uint64_t* brec;    // completing B record
  __device__ uint64_t col(int c, int) const { return brec[3 + c]; }
  __device__ uint64_t cap(int i) const { return slot ? slot[2 + i] : arec[3 + cap_from_rec[i]]; }
  __device__ uint64_t outv(int, bool* n) const { *n = true; return 0; }
  __device__ uint64_t agg(int, bool* n) const { *n = true; return 0; }
  __device__ int64_t ts() const { return (int64_t)brec[2]; }
};

template <bool kEmit>
__device__ uint32_t walk_key(const WalkArgs& a, WalkLds& L, int key_in_bucket, int bucket,
                             unsigned long long out_pos) {
  const PatternArgs& p = a.pat;
  const int tid = threadIdx.x;
  const int S = p.pending_slots;
  const int sw = p.slot_words;
  const int rw = p.rec_words;
  const int64_t kl = ((int64_t)key_in_bucket << p.buckets_log2) | bucket;
  uint64_t* sl = a.slots + kl * (int64_t)S * sw;
  int n = a.pcnt[kl];
  bool started = p.every ? false : (a.started[kl] != 0);
#define PL(i) L.plist[(i) * kWalkThreads + tid]
  for (int i = 0; i < n; ++i) PL(i) = (uint16_t)i;
  auto entry_ts = [&](int e) -> int64_t {
    return e < kEntryRec ? (int64_t)sl[e * sw] : (int64_t)a.recs[(int64_t)L.wrec[e - kEntryRec] * rw + 2];
  };
  uint32_t matches = 0;
  const uint32_t r0 = L.kstart[key_in_bucket], r1 = L.kstart[key_in_bucket + 1];
  for (uint32_t q = r0; q < r1; ++q) {
    const int w = L.sorted[q];
    const uint64_t* rec = a.recs + (int64_t)L.wrec[w] * rw;
    const uint64_t h = rec[0];
    const uint32_t role = (uint32_t)(h >> 32) & 0xffu;
    const int64_t ts = (int64_t)rec[2];
    if (role & ROLE_B) {
      int m = 0;
      for (int i = 0; i < n; ++i) {
        const int e = PL(i);
        const int64_t ets = entry_ts(e);
        if (p.within >= 0) {
          const int64_t d = ts - ets;
          if ((d < 0 ? -d : d) > p.within) continue;   // expired: dropped
        }
        bool g = (role & ROLE_G) != 0;
        MatchEnv env{e < kEntryRec ? sl + (int64_t)e * sw : nullptr,
                     e < kEntryRec ? nullptr : a.recs + (int64_t)L.wrec[e - kEntryRec] * rw,
                     p.cap_from_rec, rec};
        if (!g && p.g_walk_prog >= 0) {
          bool isnull = false;
          uint64_t v = vm_eval(a.vm.code, a.vm.konst, p.g_walk_prog, L.R, tid, kWalkThreads, env,
                               &isnull);
          g = !isnull && (v & 1u);
        }
        if (g) {
          if (kEmit) {
            const unsigned long long pos = out_pos + matches;
            if ((int64_t)pos < a.out.cap) {
              for (int c = 0; c < a.out.ncols; ++c) {
                bool isnull = false;
                uint64_t v = vm_eval(a.vm.code, a.vm.konst, a.out.prog[c], L.R, tid,
                                     kWalkThreads, env, &isnull);
                store_col(a.out.col[c], a.out.type[c], (int64_t)pos, isnull ? 0 : v);
              }
              a.out.ts[pos] = ts;
              a.out.seq[pos] = (int64_t)rec[1];
            } else {
              set_err(a.err, ERR_OUT_CAP);
            }
          }
          ++matches;
          continue;   // completed partial is consumed (s2 is not `every`)
        }
        PL(m) = (uint16_t)e;
        ++m;
      }
      n = m;
    }
    if ((role & ROLE_A) && (p.every || !started)) {
      started = true;
      if (p.within >= 0) {
        // event-time order: partials older than W can never complete again
        int drop = 0;
        while (drop < n && ts - entry_ts(PL(drop)) > p.within) ++drop;
        if (drop) {
          for (int i = drop; i < n; ++i) PL(i - drop) = PL(i);
          n -= drop;
        }
      }
      if (n >= S) {
        set_err(a.err, ERR_PENDING);
      } else {
        PL(n) = (uint16_t)(kEntryRec + w);
        ++n;
      }
    }
  }
  if (kEmit) {
    for (int j = 0; j < n; ++j) {
      const int e = PL(j);
      uint64_t* dst = sl + (int64_t)j * sw;
      if (e < kEntryRec) {
        if (e != j)
          for (int x = 0; x < sw; ++x) dst[x] = sl[(int64_t)e * sw + x];
      } else {
        const uint64_t* rec = a.recs + (int64_t)L.wrec[e - kEntryRec] * rw;
        dst[0] = rec[2];
        dst[1] = rec[1];
        for (int c = 0; c < p.ncap; ++c) dst[2 + c] = rec[3 + p.cap_from_rec[c]];
      }
    }
    a.pcnt[kl] = (uint8_t)n;
    if (!p.every) a.started[kl] = started ? 1 : 0;
  }
#undef PL
  return matches;
}

}  // namespace

__global__ __launch_bounds__(kWalkThreads) void k_walk(WalkArgs a) {
  __shared__ WalkLds L;
  const int tid = threadIdx.x;
  const int bucket = blockIdx.x;
  const PatternArgs& p = a.pat;
  const int P = 1 << p.buckets_log2;
  const int kpb = (int)((p.key_capacity + P - 1) >> p.buckets_log2);
  const int ntiles = a.ntiles;

  // segment sizes -> exclusive prefix over tiles
  {
    const int per = (ntiles + kWalkThreads - 1) / kWalkThreads;   // <= 8
    uint32_t local[8];
    uint32_t sum = 0;
    for (int i = 0; i < per; ++i) {
      const int t = tid * per + i;
      uint32_t c = 0;
      if (t < ntiles) {
        const uint16_t* o = a.tile_off + (int64_t)t * (P + 1) + bucket;
        c = (uint32_t)o[1] - (uint32_t)o[0];
      }
      local[i] = c;
      sum += c;
    }
    uint32_t total;
    uint32_t off = block_excl_scan(sum, L.scratch, &total);
    for (int i = 0; i < per; ++i) {
      const int t = tid * per + i;
      if (t < ntiles) L.seg[t] = off;
      off += local[i];
    }
    if (tid == 0) L.seg[ntiles] = total;
  }
  __syncthreads();

  int t0 = 0;
  while (t0 < ntiles) {
    if (tid == 0) {
      // largest t1 with seg[t1] - seg[t0] <= window (a single tile always fits)
      int lo = t0 + 1, hi = ntiles;
      const uint32_t lim = L.seg[t0] + kWalkWindow;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (L.seg[mid] <= lim) lo = mid;
        else hi = mid - 1;
      }
      L.t1 = (uint32_t)lo;
    }
    for (int k = tid; k <= kpb; k += kWalkThreads) L.kstart[k] = 0;
    __syncthreads();
    const int t1 = (int)L.t1;
    const uint32_t wbase = L.seg[t0];
    const uint32_t nrec = L.seg[t1] - wbase;
    if (nrec > kWalkWindow) set_err(a.err, ERR_WINDOW);
    // gather the window: one thread per tile segment
    for (int t = t0 + tid; t < t1; t += kWalkThreads) {
      const uint16_t* o = a.tile_off + (int64_t)t * (P + 1) + bucket;
      const uint32_t lo = o[0], hi = o[1];
      const uint32_t pos = L.seg[t] - wbase;
      for (uint32_t j = lo; j < hi; ++j) {
        const uint32_t w = pos + (j - lo);
        if (w >= kWalkWindow) break;
        const uint32_t gi = (uint32_t)t * (uint32_t)a.tile_rows + j;
        const uint64_t* rec = a.recs + (int64_t)gi * p.rec_words;
        L.wrec[w] = gi;
        L.wkey[w] = (uint16_t)((uint32_t)rec[0] >> p.buckets_log2);
        L.wseq[w] = (uint32_t)((int64_t)rec[1] - a.seq_chunk0);
      }
    }
    __syncthreads();
    const uint32_t nw = nrec < (uint32_t)kWalkWindow ? nrec : (uint32_t)kWalkWindow;
    for (uint32_t w = tid; w < nw; w += kWalkThreads) atomicAdd(&L.kstart[L.wkey[w] + 1], 1u);
    __syncthreads();
    // exclusive scan of key counts (kstart[1..kpb] -> kstart[0..kpb])
    {
      const int per = (kpb + kWalkThreads - 1) / kWalkThreads;   // <= 8
      uint32_t local[8];
      uint32_t sum = 0;
      for (int i = 0; i < per; ++i) {
        const int k = tid * per + i;
        local[i] = k < kpb ? L.kstart[k + 1] : 0u;
        sum += local[i];
      }
      uint32_t total;
      uint32_t off = block_excl_scan(sum, L.scratch, &total);
      for (int i = 0; i < per; ++i) {
        const int k = tid * per + i;
        if (k < kpb) {
          L.kstart[k] = off;
          L.kcur[k] = off;
        }
        off += local[i];
      }
      if (tid == 0) L.kstart[kpb] = total;
    }
    __syncthreads();
    for (uint32_t w = tid; w < nw; w += kWalkThreads) {
      const uint32_t slot = atomicAdd(&L.kcur[L.wkey[w]], 1u);
      L.sorted[slot] = (uint16_t)w;
    }
    __syncthreads();
    // restore arrival order inside each key run (insertion / shell sort on seq)
    for (int k = tid; k < kpb; k += kWalkThreads) {
      const uint32_t r0 = L.kstart[k], r1 = L.kstart[k + 1];
      const uint32_t len = r1 - r0;
      if (len < 2) continue;
      for (uint32_t gap = len > 64 ? len / 3 : 1;; gap = gap / 3 ? gap / 3 : 1) {
        for (uint32_t i = r0 + gap; i < r1; ++i) {
          const uint16_t v = L.sorted[i];
          const uint32_t sv = L.wseq[v];
          uint32_t j = i;
          while (j >= r0 + gap && L.wseq[L.sorted[j - gap]] > sv) {
            L.sorted[j] = L.sorted[j - gap];
            j -= gap;
          }
          L.sorted[j] = v;
        }
        if (gap == 1) break;
      }
    }
    __syncthreads();
    // pass 1: count matches per thread
    uint32_t mine = 0;
    for (int k = tid; k < kpb; k += kWalkThreads)
      if (L.kstart[k + 1] > L.kstart[k]) mine += walk_key<false>(a, L, k, bucket, 0);
    uint32_t total;
    const uint32_t off = block_excl_scan(mine, L.scratch, &total);
    if (tid == 0) L.base = total ? atomicAdd(a.out.count, (unsigned long long)total) : 0ull;
    __syncthreads();
    // pass 2: emit + commit state
    unsigned long long pos = L.base + off;
    for (int k = tid; k < kpb; k += kWalkThreads)
      if (L.kstart[k + 1] > L.kstart[k]) pos += walk_key<true>(a, L, k, bucket, pos);
    __syncthreads();
    t0 = t1;
  }
}

void launch_walk(const WalkArgs& a, int nbuckets, hipStream_t s) {
  hipLaunchKernelGGL(k_walk, dim3((unsigned)nbuckets), dim3(kWalkThreads), 0, s, a);
}

// ============================================================ k_generate ==
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_generate(int64_t first, int64_t n, uint64_t seed, int64_t keys, int64_t rate,
                           int64_t t0, int single, int32_t* key, int64_t* ts, uint8_t* stream,
                           int32_t* id, double* price) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t g = (uint64_t)(first + i);
    const uint64_t b = seed ^ (g * 0x9E3779B97F4A7C15ull);
    if (key) key[i] = (int32_t)(splitmix64(b ^ 0) % (uint64_t)keys);
    if (stream) stream[i] = single ? 0 : (uint8_t)(splitmix64(b ^ 1) >> 63);
    if (id) id[i] = (int32_t)(splitmix64(b ^ 2) % 50u);
    if (price) price[i] = (double)(splitmix64(b ^ 3) >> 11) * 0x1.0p-53;
    if (ts) ts[i] = t0 + (int64_t)(g / (uint64_t)rate);
  }
}

void launch_generate(int64_t first, int64_t n, uint64_t seed, int64_t keys, int64_t rate,
                     int64_t t0, int single_stream, int32_t* key, int64_t* ts, uint8_t* stream,
                     int32_t* id, double* price, hipStream_t s) {
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 256 * 64);
  hipLaunchKernelGGL(k_generate, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, s,
                     first, n, seed, keys, rate, t0, single_stream, key, ts, stream, id, price);
}

}  // namespace cep
