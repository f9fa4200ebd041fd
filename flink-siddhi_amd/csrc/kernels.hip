// gfx950 kernels for the flink-siddhi hot path (the Siddhi work behind
// AbstractSiddhiOperator.java:130 `InputHandler.send(ts, row)`):
//
//   k_filter     `from S[expr] select ... insert into O`: columnar predicate
//                evaluation (16 consecutive rows per lane, 16-byte loads) +
//                order-preserving compaction (block scan + single-pass
//                decoupled look-back across tiles) + projection.
//   k_partition  keyed pattern, pass 1: evaluates the state filters f / g on
//                the event columns, drops events no state can use (exact for
//                `->` patterns) and scatters the rest as
//                fixed-size records into per-tile key-bucket segments
//                (LDS histogram + LDS scan; no global atomics).
//   k_walk       keyed pattern, pass 2: one workgroup per key bucket gathers
//                its segments (tile order = arrival order), groups them by
//                key in LDS and resolves the pattern:
//                  closed form (`every`, g independent of s1, SURVEY.md
//                  App. A.3): every A matches the next B of its key within W
//                  -> segmented next-B scan, per-record match flags, one block
//                  scan for output positions; fully data-parallel;
//                  general form: one NFA lane per key walking its records
//                  (count pass + emit pass), pending partials in LDS lists.
//   k_generate   counter-based synthetic workload.
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "vm.h"
#include "dev_common.h"

namespace cep {

namespace {

constexpr uint64_t kStatusShift = 62;
constexpr uint64_t kValueMask = (1ull << 62) - 1;
constexpr uint16_t kNone16 = 0xffff;



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

__device__ __forceinline__ uint64_t eval_word(const VmArgs& vm, int prog, uint64_t* R,
                                                        const RowEnv& env) {
  bool isnull = false;
  uint64_t v = vm_eval(vm.code, vm.konst, prog, R, threadIdx.x, blockDim.x, env, &isnull);
  return isnull ? 0 : v;
}

// Load N consecutive elements [row, row + N) of a typed column as VM words,
// with 16-byte vector loads when the run is full and aligned.
template <int N>
__device__ __forceinline__ void load_run(const void* p, int type, int64_t row, int64_t nvalid,
                                         uint64_t (&v)[N]) {
  const int w = type_width(type);
  const uintptr_t addr = (uintptr_t)p + (uintptr_t)(row * w);
  if (nvalid >= N && (addr & 15u) == 0 && (w * N) % 16 == 0) {
    if (w == 8) {
#pragma unroll
      for (int i = 0; i < N / 2; ++i) {
        const uint4 x = gload4((const void*)(addr + 16 * i));
        v[2 * i] = ((uint64_t)x.y << 32) | x.x;
        v[2 * i + 1] = ((uint64_t)x.w << 32) | x.z;
      }
    } else if (w == 4) {
#pragma unroll
      for (int i = 0; i < N / 4; ++i) {
        const uint4 x = gload4((const void*)(addr + 16 * i));
        const uint32_t e[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v[4 * i + j] = type == T_FLOAT ? (uint64_t)e[j] : from_i32((int32_t)e[j]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < N / 16; ++i) {
        const uint4 x = gload4((const void*)(addr + 16 * i));
        const uint32_t e[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int j = 0; j < 16; ++j)
          v[16 * i + j] = ((e[j >> 2] >> (8 * (j & 3))) & 0xffu) ? 1u : 0u;
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = i < nvalid ? load_col(p, type, row + i) : 0;
}

// Interpreter-free predicate over N consecutive rows -> bit i set when row i
// passes.  Stage-wise: one switch per stage, straight loops over the N values.
template <int N>
__device__ __forceinline__ uint32_t eval_terms_run(const TermList& tl, const RowsArgs& rows,
                                                   int64_t row, int64_t nvalid) {
  uint32_t acc = tl.any ? 0u : ((N >= 32) ? 0xffffffffu : ((1u << N) - 1u));
  for (int i = 0; i < tl.n; ++i) {
    const Term& t = tl.t[i];
    uint64_t v[N];
    load_run<N>(rows.cols.p[t.col], t.coltype, row, nvalid, v);
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

// Predicate over N consecutive rows: term list when available, else the VM.
template <int N, bool kVm>
__device__ __forceinline__ uint32_t eval_run(const TermList& tl, const VmArgs& vm, int prog,
                                             uint64_t* R, const RowsArgs& rows, int64_t row,
                                             int64_t nvalid) {
  const uint32_t full = (N >= 32) ? 0xffffffffu : ((1u << N) - 1u);
  if (prog < 0) return full;
  if (!kVm || tl.n >= 0) return eval_terms_run<N>(tl, rows, row, nvalid);
  uint32_t bits = 0;
  for (int e = 0; e < N; ++e)
    if (e < nvalid && eval_pred(vm, prog, R, RowEnv{&rows, row + e})) bits |= 1u << e;
  return bits;
}

}  // namespace

// ============================================================== k_filter ==
// kVm = false: filter and projection are TermList / direct copies (no interpreter).
template <bool kVm>
__global__ __launch_bounds__(kFilterThreads) void k_filter(FilterArgs a) {
  constexpr int kStageWords = 16 * kFilterThreads;   // plain-copy output stage (16 words per lane)
  __shared__ uint64_t R[kVm ? kMaxRegs * kFilterThreads : kStageWords];
  __shared__ uint32_t scratch[16];
  __shared__ uint32_t s_tile;
  __shared__ unsigned long long s_prefix;
  const int tid = threadIdx.x;
  constexpr int kTile = kFilterThreads * kFilterItems;

  if (tid == 0) s_tile = atomicAdd(a.ticket, 1u);
  __syncthreads();
  const int64_t tile = s_tile;
  const int64_t r0 = tile * kTile + (int64_t)tid * kFilterItems;   // first row of this lane
  const int64_t nvalid = a.rows.n - r0;
  const int64_t row0 = a.rows.row0 + r0;

  uint32_t sel = 0;
  if (nvalid > 0) {
    uint32_t in_stream = (1u << kFilterItems) - 1u;
    if (a.rows.stream) {
      in_stream = 0;
#pragma unroll
      for (int e = 0; e < kFilterItems; ++e)
        if (e < nvalid && (int)a.rows.stream[row0 + e] == a.in_stream) in_stream |= 1u << e;
    } else if (a.rows.input != a.in_stream) {
      in_stream = 0;
    }
    if (in_stream)
      sel = in_stream & eval_run<kFilterItems, kVm>(a.filter_terms, a.vm, a.filter_prog, R, a.rows,
                                               row0, nvalid);
    if (nvalid < kFilterItems) sel &= (1u << nvalid) - 1u;
  }
  uint32_t total;
  const uint32_t mine = (uint32_t)__popc(sel);
  uint32_t off;
  {   // block exclusive scan (up to 16 waves)
    const int lane = tid & 63, wave = tid >> 6;
    constexpr int NWV = kFilterThreads / 64;
    uint32_t x = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) scratch[wave] = x;
    __syncthreads();
    uint32_t wb = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
      const uint32_t c = scratch[w];
      wb += w < wave ? c : 0u;
      tot += c;
    }
    off = wb + x - mine;
    total = tot;
  }

  // Plain-copy projection (kVm = false): the tile's selected rows are staged
  // in LDS column by column, then each column's run [prefix, prefix + total)
  // is written with consecutive lanes on consecutive rows.  The in-tile
  // offsets are known before the tile's prefix, so the staging loads are
  // issued before the look-back (wave 0 looks back first, the other waves
  // stage meanwhile).  A tile selecting more rows than the stage holds, or
  // one that would pass the output capacity, stores directly.
  const int nc = a.out.ncols;
  const uint32_t cap = (uint32_t)(kStageWords / (nc + 2));
  const bool stage = !kVm && total <= cap;   // uniform
  auto stage_rows = [&]() {
    uint32_t slot = off;
    for (uint32_t m = sel; m; m &= m - 1) {
      const int64_t row = row0 + (__ffs(m) - 1);
      for (int c = 0; c < nc; ++c) {
        const int col = a.out.src[c] - SRC_REC;
        R[c * cap + slot] = load_col(a.rows.cols.p[col], a.rows.cols.t[col], row);
      }
      R[nc * cap + slot] = (uint64_t)a.rows.ts[row];
      R[(nc + 1) * cap + slot] = (uint64_t)row_seq(a.rows, row);
      ++slot;
    }
  };
  if (stage && tid >= 64) stage_rows();

  // Decoupled look-back, one wave wide: lane l reads the flag of tile
  // (base - l); the nearest inclusive prefix among the 64 ends the walk once
  // every nearer predecessor has published its aggregate, otherwise all 64
  // aggregates are added and the window moves 64 tiles back.
  if (tid < 64) {
    const int lane = tid;
    unsigned long long* flags = a.tile_state;
    unsigned long long prefix = 0;
    if (tile == 0) {
      prefix = __hip_atomic_load(a.out.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0)
        __hip_atomic_store(&flags[tile], (1ull << kStatusShift) | total, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      int64_t base = tile - 1;
      unsigned spins = 0;
      while (true) {
        const int64_t j = base - lane;
        const unsigned long long v =
            j >= 0 ? __hip_atomic_load(&flags[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        const uint32_t st = (uint32_t)(v >> kStatusShift);
        const uint64_t ready = __ballot(st != 0);
        const uint64_t incl = __ballot(st == 2);
        const int f = incl ? __ffsll((long long)incl) - 1 : 63;
        const uint64_t need = f == 63 ? ~0ull : ((2ull << f) - 1ull);   // lanes 0..f
        if ((ready & need) != need) {   // a nearer predecessor has not published yet
          if (++spins > (1u << 22)) {   // never published: give up loudly
            if (lane == 0) set_err(a.err, ERR_WINDOW);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        unsigned long long x = ((need >> lane) & 1ull) ? (v & kValueMask) : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        prefix += x;
        if (incl) break;
        base -= 64;
      }
    }
    if (lane == 0) {
      __hip_atomic_store(&flags[tile], (2ull << kStatusShift) | (prefix + total), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      s_prefix = prefix;
      if (tile == (int64_t)gridDim.x - 1)
        __hip_atomic_store(a.out.count, prefix + total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (stage && tid < 64) stage_rows();
  __syncthreads();
  int64_t pos = (int64_t)s_prefix + off;
  if (stage && (int64_t)s_prefix + (int64_t)total <= a.out.cap) {   // uniform
    const int64_t prefix = (int64_t)s_prefix;
    for (int c = 0; c < nc; ++c)
      for (uint32_t j = tid; j < total; j += kFilterThreads)
        store_col(a.out.col[c], a.out.type[c], prefix + j, R[c * cap + j]);
    for (uint32_t j = tid; j < total; j += kFilterThreads) {
      a.out.ts[prefix + j] = (int64_t)R[nc * cap + j];
      a.out.seq[prefix + j] = (int64_t)R[(nc + 1) * cap + j];
    }
    return;
  }
  while (sel) {
    const int e = __ffs(sel) - 1;
    sel &= sel - 1;
    const int64_t row = row0 + e;
    if (pos < a.out.cap) {
      RowEnv env{&a.rows, row};
      for (int c = 0; c < a.out.ncols; ++c) {
        const int src = a.out.src[c];
        uint64_t v;
        if (!kVm || (src >= SRC_REC && src < SRC_TS)) {
          v = load_col(a.rows.cols.p[src - SRC_REC], a.rows.cols.t[src - SRC_REC], row);
        } else {
          v = eval_word(a.vm, a.out.prog[c], R, env);
        }
        store_col(a.out.col[c], a.out.type[c], pos, v);
      }
      a.out.ts[pos] = a.rows.ts[row];
      if (a.out.write_seq) a.out.seq[pos] = row_seq(a.rows, row);
    }
    ++pos;
  }
}

void launch_filter(const FilterArgs& a, int64_t ntiles, bool vm, hipStream_t s) {
  if (vm) hipLaunchKernelGGL(k_filter<true>, dim3((unsigned)ntiles), dim3(kFilterThreads), 0, s, a);
  else hipLaunchKernelGGL(k_filter<false>, dim3((unsigned)ntiles), dim3(kFilterThreads), 0, s, a);
}



// =========================================================== k_partition ==
// Record layout (8-byte words, chunk-relative):
//   w0 = dense key (low 32) | role << 32 | input handle << 40
//   w1 = seq - chunk seq base (low 32) | ts - chunk ts base (high 32, signed)
//   w2.. = carried columns (rec_a for A-stream rows, rec_b for B-stream rows)
// Records of a tile are staged in LDS in bucket order and written out with
// coalesced 16-byte stores (the tile's region is contiguous).
constexpr int kStageBytes = 32 * 1024;   // a tile keeps ~1/3 of its rows at config 3 (24 B each)

#define PART_STAMP(i)                                                              \
  do {                                                                              \
    if (a.stamps && threadIdx.x == 0 && blockIdx.x < 4096)                          \
      a.stamps[(int64_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memtime();      \
  } while (0)   // typical tiles keep ~10% of rows

// kPf: PrefPlan fast path (term-list predicates, <= kPref columns, aligned).
template <bool kVm, bool kPf>
__global__ __launch_bounds__(kPartThreads) void k_partition(PartArgs a) {
  __shared__ uint64_t R[kVm ? kMaxRegs * kPartThreads : 1];
  __shared__ uint32_t scratch[16];
  __shared__ __attribute__((aligned(16))) uint64_t stage[kStageBytes / 8];
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];   // P + 1 (dynamic)
  const int tid = threadIdx.x;
  const int64_t tile = blockIdx.x;
  const PatternArgs& p = a.pat;
  const int P = 1 << p.buckets_log2;
  const int rw = p.rec_words;
  PART_STAMP(0);
  for (int i = tid; i <= P; i += kPartThreads) hist[i] = 0;

  // chunk bases: relative seq / ts in records
  int64_t ts_base, seq_base;
  if (a.from_records) {
    ts_base = (int64_t)a.in_recs[a.rows.row0 * a.in_rec_words + 2];
    seq_base = (int64_t)a.in_recs[a.rows.row0 * a.in_rec_words + 1];
  } else {
    ts_base = a.rows.ts[a.rows.row0];
    seq_base = row_seq(a.rows, a.rows.row0);
  }
  if (tile == 0 && tid == 0 && a.chunk_base) {
    a.chunk_base[0] = ts_base;
    a.chunk_base[1] = seq_base;
  }
  lds_barrier();
  PART_STAMP(1);

  constexpr int E = kPartItems;
  const int64_t r0 = tile * (int64_t)a.tile_rows + (int64_t)tid * E;   // first row of this lane
  const int64_t nvalid = a.rows.n - r0;
  uint32_t packed[E];
#pragma unroll
  for (int e = 0; e < E; ++e) packed[e] = 0xffffffffu;

  int64_t key[E];
#pragma unroll
  for (int e = 0; e < E; ++e) key[e] = 0;
  uint32_t nrole[kVm ? E : 1];   // N-state pattern / sequence roles (VM path)
  // fast path: the lane's rows stay in registers for the record build
  uint64_t tsv[kPf ? E : 1];
  uint64_t pv[kPf ? kPref : 1][kPf ? E : 1];
  int sid[kPf ? E : 1];
  if (nvalid > 0) {
    uint32_t role_a = 0, role_b = 0, role_g = 0;
    if (a.from_records) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (e < nvalid) {
          const uint64_t h = a.in_recs[(a.rows.row0 + r0 + e) * a.in_rec_words];
          const uint32_t role = (uint32_t)(h >> 32) & 0xffu;
          role_a |= ((role & ROLE_A) ? 1u : 0u) << e;
          role_b |= ((role & ROLE_B) ? 1u : 0u) << e;
          role_g |= ((role & ROLE_G) ? 1u : 0u) << e;
          key[e] = (int64_t)(uint32_t)h;
        }
      }
    } else if constexpr (kPf) {
      const int64_t row0 = a.rows.row0 + r0;
      const bool full = nvalid >= 16;   // 16-byte loads of 1-byte columns stay in bounds
      // issue every load of the lane's rows before any use
      // (no branches between the loads: a branch join makes the compiler
      // drain them; unused slots repeat column col[0], set by the host)
      const int64_t prev_ld = a.rows.ts[row0 > 0 ? row0 - 1 : row0];
      uint64_t sbytes = 0;
      if (full) {
        uint4 rt[E / 2], rc[kPref][E / 2];
        load_raw<E>(a.rows.ts, 8, row0, rt);
#pragma unroll
        for (int q = 0; q < kPref; ++q)
          load_raw<E>(a.rows.cols.p[a.pref.col[q]], type_width(a.rows.cols.t[a.pref.col[q]]), row0,
                      rc[q]);
        const uint8_t* sp = a.rows.stream ? a.rows.stream + row0 : (const uint8_t*)a.rows.ts + row0 * 8;
        if constexpr (E == 8) sbytes = *(const __attribute__((address_space(1))) uint64_t*)sp;
        else sbytes = *(const __attribute__((address_space(1))) uint32_t*)sp;
        decode<E>(rt, T_LONG, tsv);
#pragma unroll
        for (int q = 0; q < kPref; ++q)
          if (q < a.pref.n) decode<E>(rc[q], a.rows.cols.t[a.pref.col[q]], pv[q]);
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
      int64_t prev = row0 > 0 ? prev_ld : batch_prev_ts(a.rows);
      uint32_t is_a = 0, is_b = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        sid[e] = a.rows.stream ? (int)((sbytes >> (8 * e)) & 0xffu) : a.rows.input;
        if (e < nvalid) {
          is_a |= (sid[e] == p.a_stream ? 1u : 0u) << e;
          is_b |= (sid[e] == p.b_stream ? 1u : 0u) << e;
        }
      }
      if (p.within >= 0 && !p.tolerant) {   // event-time order check (`within` pruning relies on it)
        bool bad = false;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          if (e < nvalid) {
            bad |= (int64_t)tsv[e] < prev;
            prev = (int64_t)tsv[e];
          }
        }
        if (bad) report_descent(a.rows, a.err);
      }
      const uint32_t all = (1u << E) - 1u;
      if (is_a) role_a = is_a & (p.f_prog < 0 ? all : eval_terms_regs<E>(p.f_terms, a.pref.f_slot, a.rows.cols, pv));
      if (is_b) {
        if (p.g_walk_prog >= 0) {
          role_b = is_b;
        } else {
          role_g = is_b & (p.g_raw_prog < 0 ? all : eval_terms_regs<E>(p.g_terms, a.pref.g_slot, a.rows.cols, pv));
          // tolerant: a g-failing B still prunes (|ts(B) - ts(s1)| > W)
          role_b = p.tolerant ? is_b : role_g;
        }
      }
#pragma unroll
      for (int e = 0; e < E; ++e) key[e] = a.pref.key_slot >= 0 ? (int64_t)pick<E>(pv, a.pref.key_slot, e) : 0;
    } else {
      const int64_t row0 = a.rows.row0 + r0;
      uint32_t is_a = 0, is_b = 0;
      int sid[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        sid[e] = a.rows.stream ? (e < nvalid ? (int)a.rows.stream[row0 + e] : -1) : a.rows.input;
        if (e < nvalid) {
          is_a |= (sid[e] == p.a_stream ? 1u : 0u) << e;
          is_b |= (sid[e] == p.b_stream ? 1u : 0u) << e;
        }
      }
      if (p.within >= 0 && !p.tolerant) {   // event-time order check (`within` pruning relies on it)
        uint64_t t[E];
        load_run<E>(a.rows.ts, T_LONG, row0, nvalid, t);
        int64_t prev = row0 > 0 ? a.rows.ts[row0 - 1] : batch_prev_ts(a.rows);
        bool bad = false;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          if (e < nvalid) {
            bad |= (int64_t)t[e] < prev;
            prev = (int64_t)t[e];
          }
        }
        if (bad) report_descent(a.rows, a.err);
      }
      bool nfa = false;
      if constexpr (kVm) nfa = p.nfa_mode != 0 && !p.nfa_pair;
      if (nfa) {
        // N-state pattern / sequence: role bit j = state j's own condition
        // accepts the row (or it is checked in the walk); bit 7 = row kept.
        // Sequences keep every row of their streams (strict contiguity).
#pragma unroll
        for (int e = 0; e < E; ++e) {
          key[e] = 0;
          if constexpr (kVm) {
            nrole[e] = 0;
            if (e >= nvalid || sid[e] < 0 || !((p.stream_mask >> sid[e]) & 1)) continue;
            uint32_t r = 0x80u;
            for (int j = 0; j < p.nstates; ++j) {
              if (p.st_stream[j] != sid[e]) continue;
              if (p.st_raw[j] < 0 || eval_pred(a.vm, p.st_raw[j], R, RowEnv{&a.rows, row0 + e}))
                r |= 1u << j;
            }
            // patterns: no state can use it (tolerant: it may still expire partials)
            if (!p.nfa_seq && r == 0x80u && !p.tolerant) continue;
            nrole[e] = r;
            const int kc = p.key_col_s[sid[e]];
            if (kc >= 0) key[e] = (int64_t)load_col(a.rows.cols.p[kc], a.rows.cols.t[kc], row0 + e);
          }
        }
      } else {
        if (is_a) role_a = is_a & eval_run<E, kVm>(p.f_terms, a.vm, p.f_prog, R, a.rows, row0, nvalid);
        if (is_b) {
          if (p.g_walk_prog >= 0) {
            role_b = is_b;
          } else {
            role_g = is_b & eval_run<E, kVm>(p.g_terms, a.vm, p.g_raw_prog, R, a.rows, row0, nvalid);
            role_b = p.tolerant ? is_b : role_g;
          }
        }
#pragma unroll
        for (int e = 0; e < E; ++e) key[e] = 0;
        if (role_a | role_b) {
          if (p.key_col_a >= 0 && p.key_col_a == p.key_col_b) {
            uint64_t k[E];
            load_run<E>(a.rows.cols.p[p.key_col_a], a.rows.cols.t[p.key_col_a], row0, nvalid, k);
#pragma unroll
            for (int e = 0; e < E; ++e) key[e] = (int64_t)k[e];
          } else {
#pragma unroll
            for (int e = 0; e < E; ++e) {
              if (((role_a | role_b) >> e) & 1u) {
                const int kc = sid[e] == p.a_stream ? p.key_col_a : p.key_col_b;
                if (kc >= 0) key[e] = (int64_t)load_col(a.rows.cols.p[kc], a.rows.cols.t[kc], row0 + e);
              }
            }
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      uint32_t role = ((role_a >> e) & 1u) * ROLE_A | ((role_b >> e) & 1u) * ROLE_B |
                      ((role_g >> e) & 1u) * ROLE_G;
      if constexpr (kVm) {
        if (p.nfa_mode && !p.nfa_pair) role = nrole[e];
      }
      if (!role) continue;
      const int64_t kfield = shard_key(key[e], p.key_stride, p.key_offset);
      if (kfield < 0 || kfield >= p.key_capacity) { set_err(a.err, ERR_KEY_RANGE); continue; }
      const int bucket = (int)(kfield & (P - 1));
      key[e] = kfield;
      const uint32_t rank = atomicAdd(&hist[bucket], 1u);
      // bits 0-10 rank in tile, 11-22 bucket, 23-30 role (never all ones)
      packed[e] = (role << 23) | ((uint32_t)bucket << 11) | rank;
    }
  }
  lds_barrier();
  PART_STAMP(2);
  // exclusive scan of the P bucket counts (P <= 4096: 16 per thread); every
  // thread of the block takes part (barriers inside)
  {
      const int per = (P + kPartThreads - 1) / kPartThreads;
      uint32_t sum = 0;
      for (int i = 0; i < per; ++i) {
        const int idx = tid * per + i;
        sum += idx < P ? hist[idx] : 0u;
      }
      uint32_t total;
      uint32_t off = block_excl_scan(sum, scratch, &total);
      for (int i = 0; i < per; ++i) {
        const int idx = tid * per + i;
        if (idx < P) {
          const uint32_t c = hist[idx];
          hist[idx] = off;
          off += c;
        }
      }
      if (tid == 0) hist[P] = total;
  }
  lds_barrier();
  PART_STAMP(3);
  const bool staged = (int64_t)hist[P] * rw * 8 <= kStageBytes;   // uniform
  {
    // build the records (LDS stage when they fit, else straight to HBM)
    const int64_t tbase = tile * (int64_t)a.tile_rows;
    const int sa0 = a.pref.reca_slot[0], sa1 = a.pref.reca_slot[1];
    const int sb0 = a.pref.recb_slot[0], sb1 = a.pref.recb_slot[1];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (packed[e] == 0xffffffffu) continue;
      const uint32_t b = (packed[e] >> 11) & 0xfffu, rank = packed[e] & 0x7ffu;
      const uint32_t role = (packed[e] >> 23) & 0xffu;
      const uint32_t slot = hist[b] + rank;
      // explicit address spaces (a generic pointer would make these flat stores)
      const int64_t so = (int64_t)slot * rw;
      uint64_t* gout = a.recs + (tbase + slot) * rw;
      auto put = [&](int w, uint64_t v) {
        if (staged) stage[so + w] = v;
        else gout[w] = v;
      };
      const int64_t r = a.rows.row0 + r0 + e;
      if constexpr (!kPf) {
        if (a.from_records) {
          const uint64_t* in = a.in_recs + r * a.in_rec_words;
          const int64_t dseq = (int64_t)in[1] - seq_base, dts = (int64_t)in[2] - ts_base;
          if (dseq < 0 || dseq > 0xffffffffll || dts > 0x7fffffffll || dts < -0x7fffffffll)
            set_err(a.err, ERR_ORDER);
          put(0, (in[0] & ~0xffffffffull) | (uint64_t)(uint32_t)key[e]);
          put(1, (uint64_t)(uint32_t)((int64_t)in[1] - seq_base) |
                   ((uint64_t)(uint32_t)(int32_t)((int64_t)in[2] - ts_base) << 32));
          for (int w = 2; w < rw; ++w) put(w, in[w + 1]);
          continue;
        }
      }
      int s;
      int64_t dts;
      if constexpr (kPf) {
        s = sid[e];
        dts = (int64_t)tsv[e] - ts_base;
      } else {
        s = a.rows.stream ? (int)a.rows.stream[r] : a.rows.input;
        dts = a.rows.ts[r] - ts_base;
      }
      if (dts > 0x7fffffffll || dts < -0x7fffffffll) set_err(a.err, ERR_ORDER);
      put(0, (uint64_t)(uint32_t)key[e] | ((uint64_t)role << 32) | ((uint64_t)(uint32_t)s << 40));
      int64_t dseq = r - a.rows.row0;
      if (a.rows.seq) {   // shuffled rows: global arrival numbers, increasing
        dseq = a.rows.seq[r] - seq_base;
        if (dseq < 0 || dseq > 0xffffffffll) set_err(a.err, ERR_ORDER);
      }
      put(1, (uint64_t)(uint32_t)dseq | ((uint64_t)(uint32_t)(int32_t)dts << 32));
      const bool isa = s == p.a_stream;
      if constexpr (kPf) {
        // at most kPfRec carried words (host-checked); slots are uniform
        const int nrc = isa ? p.nrec_a : p.nrec_b;
        if (nrc > 0) put(2, pick<E>(pv, isa ? sa0 : sb0, e));
        if (nrc > 1) put(3, pick<E>(pv, isa ? sa1 : sb1, e));
      } else {
        const int nrc = isa ? p.nrec_a : p.nrec_b;
        for (int c = 0; c < nrc; ++c) {
          const int col = isa ? p.rec_a[c] : p.rec_b[c];
          put(2 + c, load_col(a.rows.cols.p[col], a.rows.cols.t[col], r));
        }
      }
    }
  }
  lds_barrier();
  PART_STAMP(4);
  uint16_t* toff = a.tile_off + tile * (int64_t)(P + 1);
  for (int i = tid; i <= P; i += kPartThreads) toff[i] = (uint16_t)hist[i];
  if (staged) {
    // the tile's records are contiguous in HBM: 16-byte coalesced stores
    const int64_t words = (int64_t)hist[P] * rw;
    uint64_t* dst = a.recs + tile * (int64_t)a.tile_rows * rw;
    for (int64_t w = 2 * tid; w < words; w += 2 * kPartThreads) {
      if (w + 1 < words) {
        *(uint4*)(dst + w) = *(const uint4*)(stage + w);
      } else {
        dst[w] = stage[w];
      }
    }
  }
  lds_barrier();
  PART_STAMP(5);
}

void launch_partition(const PartArgs& a, int64_t ntiles, bool vm, hipStream_t s) {
  const int P = 1 << a.pat.buckets_log2;
  const size_t dyn = ((size_t)(P + 1) * 4 + 15) & ~(size_t)15;
  if (vm) hipLaunchKernelGGL((k_partition<true, false>), dim3((unsigned)ntiles), dim3(kPartThreads), dyn, s, a);
  else if (a.pref.n >= 0 && !a.from_records)
    hipLaunchKernelGGL((k_partition<false, true>), dim3((unsigned)ntiles), dim3(kPartThreads), dyn, s, a);
  else hipLaunchKernelGGL((k_partition<false, false>), dim3((unsigned)ntiles), dim3(kPartThreads), dyn, s, a);
}


// ============================================================== k_route ==
// Multi-GPU key shuffle, sender side (router/HashPartitioner.java:24-26:
// owner = abs(hashCode(key)) % n; for the engine's non-negative int keys that
// is key % world).  Predicates are pushed down (rows no state
// can use never leave the GPU).  Each tile writes its kept rows as wide
// records [hdr, seq, ts, carried...] grouped by owner, in arrival order (one
// block scan per owner gives stable ranks); k_route_scan / k_route_gather
// then concatenate every owner's segments over tiles into one contiguous run.
template <bool kVm>
__global__ __launch_bounds__(kPartThreads) void k_route(RouteArgs a) {
  __shared__ uint64_t R[kVm ? kMaxRegs * kPartThreads : 1];
  __shared__ uint32_t scratch[16];
  __shared__ uint32_t dbase[kMaxWorld + 1];
  const int tid = threadIdx.x;
  const int64_t tile = blockIdx.x;
  const PatternArgs& p = a.pat;
  constexpr int E = kPartItems;
  const int64_t r0 = tile * (int64_t)a.tile_rows + (int64_t)tid * E;
  const int64_t nvalid = a.rows.n - r0;
  const int64_t row0 = a.rows.row0 + r0;
  uint32_t role_a = 0, role_b = 0, role_g = 0;
  int sid[E];
  int64_t key[E];
  int dest[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    key[e] = 0;
    dest[e] = -1;
    sid[e] = -1;
  }
  if (nvalid > 0) {
    uint32_t is_a = 0, is_b = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      sid[e] = a.rows.stream ? (e < nvalid ? (int)a.rows.stream[row0 + e] : -1) : a.rows.input;
      if (e < nvalid) {
        is_a |= (sid[e] == p.a_stream ? 1u : 0u) << e;
        is_b |= (sid[e] == p.b_stream ? 1u : 0u) << e;
      }
    }
    if (is_a) role_a = is_a & eval_run<E, kVm>(p.f_terms, a.vm, p.f_prog, R, a.rows, row0, nvalid);
    if (is_b) {
      if (p.g_walk_prog >= 0) {
        role_b = is_b;
      } else {
        role_b = is_b & eval_run<E, kVm>(p.g_terms, a.vm, p.g_raw_prog, R, a.rows, row0, nvalid);
        role_g = role_b;
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (!(((role_a | role_b) >> e) & 1u)) continue;
      const int kc = sid[e] == p.a_stream ? p.key_col_a : p.key_col_b;
      key[e] = kc >= 0 ? (int64_t)load_col(a.rows.cols.p[kc], a.rows.cols.t[kc], row0 + e) : 0;
      if (key[e] < 0 || key[e] > 0xffffffffll) {
        set_err(a.err, ERR_KEY_RANGE);
        continue;
      }
      dest[e] = (int)(key[e] % a.world);
    }
  }
  // stable per-owner ranks: one block scan per owner
  uint32_t rank[E];
  for (int d = 0; d < a.world; ++d) {
    uint32_t c = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) c += dest[e] == d ? 1u : 0u;
    uint32_t total;
    uint32_t off = block_excl_scan(c, scratch, &total);
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (dest[e] == d) rank[e] = off++;
    if (tid == 0) {
      dbase[d] = d == 0 ? 0u : dbase[d - 1] + a.tcount[tile * a.world + d - 1];
      a.tcount[tile * a.world + d] = total;
    }
    lds_barrier();
  }
  if (tid == 0) dbase[a.world] = 0;
  lds_barrier();
  const int wrw = a.wrw;
  uint64_t* base = a.arena + tile * (int64_t)a.tile_rows * wrw;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if (dest[e] < 0) continue;
    const int64_t r = row0 + e;
    const uint32_t role = ((role_a >> e) & 1u) * ROLE_A | ((role_b >> e) & 1u) * ROLE_B |
                          ((role_g >> e) & 1u) * ROLE_G;
    uint64_t* o = base + (int64_t)(dbase[dest[e]] + rank[e]) * wrw;
    o[0] = (uint64_t)(uint32_t)key[e] | ((uint64_t)role << 32) | ((uint64_t)(uint32_t)sid[e] << 40);
    o[1] = (uint64_t)(a.seq0 + (r - a.rows.row0));
    o[2] = (uint64_t)a.rows.ts[r];
    const bool isa = sid[e] == p.a_stream;
    const int nrc = isa ? p.nrec_a : p.nrec_b;
    for (int c = 0; c < nrc; ++c) {
      const int col = isa ? p.rec_a[c] : p.rec_b[c];
      o[3 + c] = load_col(a.rows.cols.p[col], a.rows.cols.t[col], r);
    }
  }
}

// Row shuffle for multi-query apps (sequences, aggregations, several
// patterns): no predicate push-down (a sequence needs every row of its
// streams for strict contiguity), whole rows shipped as
// [stream, seq, ts, column words] grouped by owner in arrival order.
__global__ __launch_bounds__(kPartThreads) void k_route_rows(RowRouteArgs a) {
  __shared__ uint32_t scratch[16];
  __shared__ uint32_t dbase[kMaxWorld + 1];
  const int tid = threadIdx.x;
  const int64_t tile = blockIdx.x;
  constexpr int E = kPartItems;
  const int64_t r0 = tile * (int64_t)a.tile_rows + (int64_t)tid * E;
  const int64_t nvalid = a.rows.n - r0;
  const int64_t row0 = a.rows.row0 + r0;
  int dest[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    dest[e] = -1;
    if (e >= nvalid) continue;
    const int sid = a.rows.stream ? (int)a.rows.stream[row0 + e] : a.rows.input;
    const int kc = sid < 8 ? a.key_col_s[sid] : -2;
    if (kc == -2) continue;   // no query reads the stream
    if (kc == -1) {           // read by stateless filters only: round-robin
      dest[e] = (int)((uint64_t)(a.seq0 + (row0 + e - a.rows.row0)) % (uint64_t)a.world);
      continue;
    }
    const int64_t key = (int64_t)load_col(a.rows.cols.p[kc], a.rows.cols.t[kc], row0 + e);
    if (key < 0 || key > 0xffffffffll) {
      set_err(a.err, ERR_KEY_RANGE);
      continue;
    }
    dest[e] = (int)(key % a.world);
  }
  uint32_t rank[E];
  for (int d = 0; d < a.world; ++d) {
    uint32_t c = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) c += dest[e] == d ? 1u : 0u;
    uint32_t total;
    uint32_t off = block_excl_scan(c, scratch, &total);
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (dest[e] == d) rank[e] = off++;
    if (tid == 0) {
      dbase[d] = d == 0 ? 0u : dbase[d - 1] + a.tcount[tile * a.world + d - 1];
      a.tcount[tile * a.world + d] = total;
    }
    lds_barrier();
  }
  const int wrw = a.wrw;
  uint64_t* base = a.arena + tile * (int64_t)a.tile_rows * wrw;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if (dest[e] < 0) continue;
    const int64_t r = row0 + e;
    uint64_t* o = base + (int64_t)(dbase[dest[e]] + rank[e]) * wrw;
    o[0] = a.rows.stream ? (uint64_t)a.rows.stream[r] : (uint64_t)a.rows.input;
    o[1] = (uint64_t)(a.seq0 + (r - a.rows.row0));
    o[2] = (uint64_t)a.rows.ts[r];
    for (int c = 0; c < a.rows.cols.n; ++c) o[3 + c] = load_col(a.rows.cols.p[c], a.rows.cols.t[c], r);
  }
}

// Owner side of the row shuffle: received rows -> SoA columns + per-row
// stream handle and global arrival number.
__global__ __launch_bounds__(256) void k_unpack_rows(RowUnpackArgs a) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t* r = a.recs + i * a.wrw;
    a.stream[i] = (uint8_t)r[0];
    a.seq[i] = (int64_t)r[1];
    a.ts[i] = (int64_t)r[2];
    for (int c = 0; c < a.ncols; ++c) store_col(a.col[c], a.type[c], i, r[3 + c]);
  }
}

void launch_route_rows(const RowRouteArgs& a, int64_t ntiles, uint32_t* toffs,
                       unsigned long long* dcount, uint64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_route_rows, dim3((unsigned)ntiles), dim3(kPartThreads), 0, s, a);
  RouteArgs ra{};
  ra.rows = a.rows;
  ra.world = a.world;
  ra.wrw = a.wrw;
  ra.tile_rows = a.tile_rows;
  ra.seq0 = a.seq0;
  ra.arena = a.arena;
  ra.tcount = a.tcount;
  ra.err = a.err;
  ra.seg_cap = a.seg_cap;
  ra.row_mode = 1;
  ra.spill = a.spill;
  ra.spill_cap = a.spill_cap;
  ra.spill_counts = a.spill_counts;
  launch_route_collect(ra, ntiles, toffs, dcount, out, s);
  if (a.seg_cap > 0) launch_route_pad(ra, dcount, out, s);
}

void launch_unpack_rows(const RowUnpackArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  const int64_t blocks = (a.n + 255) / 256 < 8192 ? (a.n + 255) / 256 : 8192;
  hipLaunchKernelGGL(k_unpack_rows, dim3((unsigned)blocks), dim3(256), 0, s, a);
}

// Per owner: exclusive prefix of its segment sizes over tiles.
__global__ __launch_bounds__(512) void k_route_scan(const uint32_t* tcount, int64_t ntiles, int world,
                                                    uint32_t* toffs, unsigned long long* dcount) {
  __shared__ uint32_t scratch[16];
  __shared__ uint32_t carry;
  const int d = blockIdx.x;
  if (threadIdx.x == 0) carry = 0;
  lds_barrier();
  for (int64_t t0 = 0; t0 < ntiles; t0 += 512) {
    const int64_t t = t0 + threadIdx.x;
    const uint32_t c = t < ntiles ? tcount[t * world + d] : 0u;
    uint32_t total;
    const uint32_t off = block_excl_scan(c, scratch, &total);
    if (t < ntiles) toffs[(int64_t)d * ntiles + t] = carry + off;
    lds_barrier();
    if (threadIdx.x == 0) carry += total;
    lds_barrier();
  }
  if (threadIdx.x == 0) dcount[d] = carry;
}

// Copy every tile's owner segments to the owner-contiguous output.
__global__ __launch_bounds__(256) void k_route_gather(RouteArgs a, int64_t ntiles, const uint32_t* toffs,
                                                      const unsigned long long* dcount, uint64_t* out) {
  const int64_t t = blockIdx.x;
  const int wrw = a.wrw;
  unsigned long long obase = 0;
  int64_t sbase = 0;   // spill: records past seg_cap of the owners before d
  uint32_t src = 0;
  for (int d = 0; d < a.world; ++d) {
    const uint32_t c = a.tcount[t * a.world + d];
    const uint64_t* s = a.arena + (t * (int64_t)a.tile_rows + src) * wrw;
    const uint32_t to = toffs[(int64_t)d * ntiles + t];
    int64_t n = c;
    uint64_t* o;
    if (a.seg_cap > 0) {   // padded: owner d's segment, records past seg_cap spilled or dropped (k_route_pad flags them)
      n = (int64_t)to >= a.seg_cap ? 0 : (c < a.seg_cap - (int64_t)to ? (int64_t)c : a.seg_cap - (int64_t)to);
      o = out + ((int64_t)d * (1 + a.seg_cap) + 1 + to) * wrw;
      if (a.spill && n < (int64_t)c) {
        // the rest of this tile's run: spill slots (to + n - seg_cap) on
        const int64_t k0 = sbase + (int64_t)to + n - a.seg_cap;
        const int64_t m = (int64_t)c - n;
        const int64_t fit = k0 >= a.spill_cap ? 0 : (m < a.spill_cap - k0 ? m : a.spill_cap - k0);
        uint64_t* so = a.spill + k0 * wrw;
        const uint64_t* ss = s + n * wrw;
        for (int64_t w = threadIdx.x; w < fit * wrw; w += blockDim.x) so[w] = ss[w];
      }
      const int64_t tot = (int64_t)dcount[d];
      sbase += tot > a.seg_cap ? tot - a.seg_cap : 0;
    } else {
      o = out + (int64_t)(obase + to) * wrw;
    }
    for (int64_t w = threadIdx.x; w < n * wrw; w += blockDim.x) o[w] = s[w];
    src += c;
    obase += dcount[d];
  }
}

// Padded key shuffle, sender side: owner d's segment is one header record
// then seg_cap record slots.  The header and the unused slots are null
// records (role 0: every partition skips them) whose ts / seq keep the
// receiver's concatenation in event-time order: the header carries the
// batch's first row, the tail its last (rank r's batch precedes rank r + 1's).
// Header word 0 = the owner's true record count (low 32 bits) | route error
// bits << 40 | 1 << 63 when the count exceeds seg_cap; owners check it
// (k_route_check) without a host round trip.
__global__ __launch_bounds__(256) void k_route_pad(RouteArgs a, const unsigned long long* dcount, uint64_t* out) {
  const int d = blockIdx.y;
  const int wrw = a.wrw;
  const unsigned long long cnt = dcount[d];
  const int64_t used = (int64_t)cnt < a.seg_cap ? (int64_t)cnt : a.seg_cap;
  const int64_t r0 = a.rows.row0, r1 = a.rows.row0 + a.rows.n - 1;
  uint64_t* seg = out + (int64_t)d * (1 + a.seg_cap) * wrw;
  const uint64_t ovf = (int64_t)cnt > a.seg_cap ? 1ull << 63 : 0ull;
  if (a.spill_counts && blockIdx.x == 0 && threadIdx.x == 0) {
    // records past seg_cap, all of them in the spill unless it ran out
    int64_t before = 0;
    for (int e = 0; e < d; ++e) {
      const int64_t c = (int64_t)dcount[e];
      before += c > a.seg_cap ? c - a.seg_cap : 0;
    }
    const int64_t over = (int64_t)cnt > a.seg_cap ? (int64_t)cnt - a.seg_cap : 0;
    a.spill_counts[d] = over;
    if (before + over > a.spill_cap) set_err(a.err, ERR_SHUFFLE_CAP);
  }
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)wrw) {
    const unsigned int e = *(volatile unsigned int*)a.err;
    uint64_t h = 0;
    if (threadIdx.x == 0)   // records: count | errors << 40 (role 0); rows: null stream | errors << 8 | count << 32
      h = a.row_mode ? (uint64_t)kRowNullStream | ((uint64_t)(e & 0xffffffu) << 8) | ((cnt & 0x7fffffffull) << 32) | ovf
                     : (cnt & 0xffffffffull) | ((uint64_t)(e & 0xffffu) << 40) | ovf;
    else if (threadIdx.x == 1)
      h = (uint64_t)a.seq0;
    else if (threadIdx.x == 2)
      h = (uint64_t)a.rows.ts[r0];
    seg[threadIdx.x] = h;
  }
  const uint64_t tseq = (uint64_t)(a.seq0 + a.rows.n - 1), tts = (uint64_t)a.rows.ts[r1];
  const int64_t nul = (a.seg_cap - used) * wrw;
  uint64_t* tail = seg + (1 + used) * wrw;
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nul; w += (int64_t)gridDim.x * blockDim.x) {
    const int f = (int)(w % wrw);
    tail[w] = f == 1 ? tseq : (f == 2 ? tts : (f == 0 && a.row_mode ? (uint64_t)kRowNullStream : 0ull));
  }
}

// Owner side: a flagged header (overflowed segment or a sender-side route
// error) becomes the owner's error word, reported by its next flush.
__global__ void k_route_check(const uint64_t* segs, int world, int64_t seg_cap, int wrw, int row_mode,
                              unsigned int* err) {
  const int d = threadIdx.x;
  if (d >= world) return;
  const uint64_t h = segs[(int64_t)d * (1 + seg_cap) * wrw];
  unsigned int e = row_mode ? (unsigned int)((h >> 8) & 0xffffffu) : (unsigned int)((h >> 40) & 0xffffu);
  if (h >> 63) e |= ERR_SHUFFLE_CAP;
  if (e) atomicOr(err, e);
}

void launch_route_pad(const RouteArgs& a, const unsigned long long* dcount, uint64_t* out, hipStream_t s) {
  const int64_t per = (a.seg_cap * a.wrw + 255) / 256;
  const unsigned bx = (unsigned)(per < 1 ? 1 : (per > 1024 ? 1024 : per));
  hipLaunchKernelGGL(k_route_pad, dim3(bx, (unsigned)a.world), dim3(256), 0, s, a, dcount, out);
}

void launch_route_check(const uint64_t* segs, int world, int64_t seg_cap, int wrw, int row_mode, unsigned int* err,
                        hipStream_t s) {
  hipLaunchKernelGGL(k_route_check, dim3(1), dim3(64), 0, s, segs, world, seg_cap, wrw, row_mode, err);
}

void launch_route(const RouteArgs& a, int64_t ntiles, bool vm, uint32_t* toffs,
                  unsigned long long* dcount, uint64_t* out, hipStream_t s) {
  if (vm) hipLaunchKernelGGL(k_route<true>, dim3((unsigned)ntiles), dim3(kPartThreads), 0, s, a);
  else hipLaunchKernelGGL(k_route<false>, dim3((unsigned)ntiles), dim3(kPartThreads), 0, s, a);
  launch_route_collect(a, ntiles, toffs, dcount, out, s);
}

// Owner-contiguous output from per-tile owner segments (k_route / k_cfroute).
void launch_route_collect(const RouteArgs& a, int64_t ntiles, uint32_t* toffs,
                          unsigned long long* dcount, uint64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_route_scan, dim3((unsigned)a.world), dim3(512), 0, s, a.tcount, ntiles, a.world,
                     toffs, dcount);
  hipLaunchKernelGGL(k_route_gather, dim3((unsigned)ntiles), dim3(256), 0, s, a, ntiles, toffs, dcount, out);
}

// ================================================================ k_walk ==
namespace {

constexpr int kEntryRec = 64;   // working-list ids >= 64 name window records
constexpr int kWalkSlotStage = 2048;   // u64 words of staged per-key state (closed form)

// Tiles per chunk the walk's segment tables hold: the VM build (sequences,
// aggregates: one LDS-heavy workgroup per CU either way) takes 16 Mi-row
// chunks so per-key state is loaded and committed once per 16 Mi events;
// the 2-state build keeps 4 Mi-row chunks and two workgroups per CU.
template <bool kVm>
constexpr int walk_max_tiles() { return kVm ? kWalkMaxTiles : kWalkMaxTiles / 4; }

struct WalkLds {
  uint32_t wrec[kWalkWindow];        // global record index per window slot
  uint16_t wkey[kWalkWindow];        // key within the bucket
  uint16_t sorted[kWalkWindow];      // window slots grouped by key, arrival order
  uint32_t wseq[kWalkWindow];        // chunk-relative sequence number
  uint32_t kstart[kWalkMaxKeys + 1];
  uint32_t khdr[kWalkMaxKeys];       // per-key state headers of this bucket (prefetched)
  uint32_t kcur[kWalkMaxKeys];       // counting-sort cursors, then closed-form first B
  union {
    struct {
      int32_t wts[kWalkWindow];      // chunk-relative event ts per window slot
      uint32_t v[kWalkWindow];       // output position scan
      uint16_t nextb[kWalkWindow];   // next B in the key run (sorted pos), or kNone16
      uint8_t wrole[kWalkWindow];
      uint8_t cm[kWalkMaxKeys];      // carried partials completed by the first B
      uint8_t cfirst[kWalkMaxKeys];  // first completed carried slot
      uint64_t wcap[kWalkWindow][kWalkCapLds];   // carried record words
      uint64_t sstage[kWalkSlotStage];           // carried state slots of touched keys
      uint16_t soff[kWalkMaxKeys];               // key's offset in sstage, or kNone16
    } cf;
    uint16_t plist[kMaxPending * kWalkThreads];   // general form: working lists [i][tid]
  };
  uint32_t scratch[16];
  unsigned long long base;
  uint32_t t1;
};

// Chunk-relative record fields.
__device__ __forceinline__ int64_t rec_ts(const uint64_t* rec, int64_t ts_base) {
  return ts_base + (int64_t)(int32_t)(rec[1] >> 32);
}
__device__ __forceinline__ int64_t rec_seq(const uint64_t* rec, int64_t seq_base) {
  return seq_base + (int64_t)(uint32_t)rec[1];
}

// Match environment of the general walk (records read from HBM).
struct MatchEnv {
  const uint64_t* slot;    // pending entry as state slot word 0 (stride `sstride`) or nullptr
  const uint64_t* arec;    // pending entry as an A record, or nullptr
  const int32_t* cap_from_rec;
  const uint64_t* brec;    // completing B record
  int64_t ts_base;
  int64_t sstride;         // words between consecutive words of one slot
  __device__ uint64_t col(int c, int) const { return brec[2 + c]; }
  __device__ uint64_t cap(int i) const {
    return slot ? slot[(2 + i) * sstride] : arec[2 + cap_from_rec[i]];
  }
  __device__ uint64_t outv(int, bool* n) const { *n = true; return 0; }
  __device__ uint64_t agg(int, bool* n) const { *n = true; return 0; }
  __device__ int64_t ts() const { return rec_ts(brec, ts_base); }
};

// Match environment of the closed form (record words already in LDS).
struct CfEnv {
  const uint64_t* acap;    // A words: LDS record words, or state slot word 0 (stride astride)
  int64_t astride;         // 0: LDS record; else slot stride
  const int32_t* cap_from_rec;
  const uint64_t* bcap;    // completing B record words (LDS)
  int64_t bts;
  __device__ uint64_t col(int c, int) const { return bcap[c]; }
  __device__ uint64_t cap(int i) const {
    return astride ? acap[(2 + i) * astride] : acap[cap_from_rec[i]];
  }
  __device__ uint64_t outv(int, bool* n) const { *n = true; return 0; }
  __device__ uint64_t agg(int, bool* n) const { *n = true; return 0; }
  __device__ int64_t ts() const { return bts; }
};

template <class Env>
__device__ __forceinline__ uint64_t eval_env(const VmArgs& vm, int prog, uint64_t* R,
                                             const Env& env, bool* isnull) {
  return vm_eval(vm.code, vm.konst, prog, R, threadIdx.x, kWalkThreads, env, isnull);
}

// One output row.  `bword(c)` = completing event word c (src SRC_REC + c).
template <bool kVm, class Env>
__device__ __forceinline__ void emit_row(const WalkArgs& a, uint64_t* R, const Env& env,
                                         int64_t key, int64_t seq, unsigned long long pos) {
  if ((int64_t)pos >= a.out.cap) {
    set_err(a.err, ERR_OUT_CAP);
    return;
  }
  for (int c = 0; c < a.out.ncols; ++c) {
    const int src = a.out.src[c];
    uint64_t v;
    if (src >= SRC_CAP && src < SRC_REC) {
      v = env.cap(src - SRC_CAP);
    } else if (src == SRC_KEY) {
      v = (uint64_t)key;
    } else if (src >= SRC_AGG && src < SRC_AGG + kMaxAggs) {
      bool isnull = false;
      v = env.agg(src - SRC_AGG, &isnull);
      if (isnull) v = 0;
    } else if (!kVm || (src >= SRC_REC && src < SRC_TS)) {
      v = env.col(src - SRC_REC, 0);
    } else {
      bool isnull = false;
      v = eval_env(a.vm, a.out.prog[c], R, env, &isnull);
      if (isnull) v = 0;
    }
    store_col(a.out.col[c], a.out.type[c], (int64_t)pos, v);
  }
  a.out.ts[pos] = env.ts();
  if (a.out.write_seq) a.out.seq[pos] = seq;
}

// Original key value of dense key kl (shard ownership: key = kl*stride + offset).
__device__ __forceinline__ int64_t key_value(const PatternArgs& p, int64_t kl) {
  return kl * p.key_stride + p.key_offset;
}

// Diagnostic phase stamps (null pointer = off).
#define WALK_STAMP(i)                                                              \
  do {                                                                              \
    if (a.stamps && threadIdx.x == 0 && (i) < 16)                                   \
      a.stamps[(int64_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memtime();      \
  } while (0)

// General form: one lane walks one key's records in arrival order.
template <bool kEmit, bool kVm>
__device__ uint32_t walk_key(const WalkArgs& a, WalkLds& L, uint64_t* R, int key_in_bucket,
                             int bucket, int kpb, int64_t ts_base, int64_t seq_base,
                             unsigned long long out_pos) {
  const PatternArgs& p = a.pat;
  const int tid = threadIdx.x;
  const int S = p.pending_slots;
  const int sw = p.slot_words;
  const int rw = p.rec_words;
  const int64_t kl = ((int64_t)key_in_bucket << p.buckets_log2) | bucket;
  const int64_t idx = (int64_t)bucket * kpb + key_in_bucket;
  const int64_t ks = a.kstride;
  uint64_t* sl = a.kslot + idx;                       // slot j word w: sl[(j * sw + w) * ks]
  const uint32_t hdr = L.khdr[key_in_bucket];
  int n = (int)(hdr & 0xffu);
  bool started = p.every ? false : ((hdr >> 8) & 1u) != 0;
#define PL(i) L.plist[(i) * kWalkThreads + tid]
#define SW(j, w) sl[((int64_t)(j) * sw + (w)) * ks]
  for (int i = 0; i < n; ++i) PL(i) = (uint16_t)i;
  auto entry_ts = [&](int e) -> int64_t {
    return e < kEntryRec ? (int64_t)SW(e, 0)
                         : rec_ts(a.recs + (int64_t)L.wrec[e - kEntryRec] * rw, ts_base);
  };
  uint32_t matches = 0;
  const uint32_t r0 = L.kstart[key_in_bucket], r1 = L.kstart[key_in_bucket + 1];
  for (uint32_t q = r0; q < r1; ++q) {
    const int w = L.sorted[q];
    const uint64_t* rec = a.recs + (int64_t)L.wrec[w] * rw;
    const uint64_t h = rec[0];
    const uint32_t role = (uint32_t)(h >> 32) & 0xffu;
    const int64_t ts = rec_ts(rec, ts_base);
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
        const MatchEnv env{e < kEntryRec ? &SW(e, 0) : nullptr,
                           e < kEntryRec ? nullptr : a.recs + (int64_t)L.wrec[e - kEntryRec] * rw,
                           p.cap_from_rec, rec, ts_base, ks};
        if (kVm && !g && p.g_walk_prog >= 0) {
          bool isnull = false;
          uint64_t v = eval_env(a.vm, p.g_walk_prog, R, env, &isnull);
          g = !isnull && (v & 1u);
        }
        if (g) {
          if (kEmit)
            emit_row<kVm>(a, R, env, key_value(p, kl), rec_seq(rec, seq_base), out_pos + matches);
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
      if (p.within >= 0 && !p.tolerant) {
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
      if (e < kEntryRec) {
        if (e != j)
          for (int x = 0; x < sw; ++x) SW(j, x) = SW(e, x);
      } else {
        const uint64_t* rec = a.recs + (int64_t)L.wrec[e - kEntryRec] * rw;
        SW(j, 0) = (uint64_t)rec_ts(rec, ts_base);
        SW(j, 1) = (uint64_t)rec_seq(rec, seq_base);
        for (int c = 0; c < p.ncap; ++c) SW(j, 2 + c) = rec[2 + p.cap_from_rec[c]];
      }
    }
    const uint32_t nh = (uint32_t)n | ((started ? 1u : 0u) << 8);
    L.khdr[key_in_bucket] = nh;   // next window of this bucket reads the LDS copy
    a.khdr[idx] = nh;
  }
#undef SW
#undef PL
  return matches;
}

// ---- group-by / having (agg_mode) -----------------------------------------
// Running aggregates per group in arrival order, following the restatement in
// oracle/siddhi_oracle.py (_Agg): sum over int/long wraps in 64 bits, sum /
// avg over float/double accumulate in double, min/max compare in the argument
// type, count counts; every aggregate of a group sees every kept row.
struct AggState {
  uint64_t acc[kMaxAggs];
  uint64_t cnt[kMaxAggs];
};

__device__ __forceinline__ double agg_as_double(uint64_t v, int t) {
  switch (t) {
    case T_INT: return (double)(int32_t)v;
    case T_LONG: return (double)(int64_t)v;
    case T_FLOAT: return (double)as_f32(v);
    default: return as_f64(v);
  }
}

__device__ __forceinline__ bool agg_less(uint64_t a, uint64_t b, int t) {
  switch (t) {
    case T_LONG: return (int64_t)a < (int64_t)b;
    case T_FLOAT: return as_f32(a) < as_f32(b);
    case T_DOUBLE: return as_f64(a) < as_f64(b);
    default: return (int32_t)a < (int32_t)b;
  }
}

__device__ __forceinline__ void agg_update(const PatternArgs& p, AggState& s, const uint64_t* rec) {
#pragma unroll
  for (int j = 0; j < kMaxAggs; ++j) {
    if (j >= p.nagg) break;
    const int fn = p.agg_fn[j], at = p.agg_arg_type[j];
    const uint64_t v = p.agg_word[j] >= 0 ? rec[2 + p.agg_word[j]] : 0;
    const bool first = s.cnt[j] == 0;
    s.cnt[j] += 1;
    if (fn == AGG_SUM) {
      s.acc[j] = p.agg_out_type[j] == T_LONG ? s.acc[j] + v
                                             : from_f64(as_f64(s.acc[j]) + agg_as_double(v, at));
    } else if (fn == AGG_AVG) {
      s.acc[j] = from_f64(as_f64(s.acc[j]) + agg_as_double(v, at));
    } else if (fn == AGG_MIN) {
      if (first || agg_less(v, s.acc[j], at)) s.acc[j] = v;
    } else if (fn == AGG_MAX) {
      if (first || agg_less(s.acc[j], v, at)) s.acc[j] = v;
    }
  }
}

struct AggEnv {
  const PatternArgs* p;
  const uint64_t* rec;     // current record (carried words at rec[2..])
  int64_t ev_ts;
  AggState s;
  __device__ uint64_t col(int c, int) const { return rec[2 + c]; }
  __device__ uint64_t cap(int) const { return 0; }
  __device__ uint64_t outv(int, bool* n) const { *n = true; return 0; }
  __device__ uint64_t agg(int i, bool* isnull) const {
    // masked pick (a select chain on i would become a scratch array access)
    uint64_t acc = 0, cnt = 0;
#pragma unroll
    for (int j = 0; j < kMaxAggs; ++j) {
      const uint64_t m = 0ull - (uint64_t)(i == j);
      acc |= s.acc[j] & m;
      cnt |= s.cnt[j] & m;
    }
    const int fn = p->agg_fn[i];
    if (fn == AGG_COUNT) {
      *isnull = false;
      return cnt;
    }
    *isnull = cnt == 0;
    if (fn == AGG_AVG) return from_f64(as_f64(acc) / (double)(int64_t)cnt);
    return acc;
  }
  __device__ int64_t ts() const { return ev_ts; }
};

// One group's records of the window, sequentially (count pass / emit pass).
template <bool kEmit, bool kVm>
__device__ uint32_t agg_key(const WalkArgs& a, WalkLds& L, uint64_t* R, int k, int bucket, int kpb,
                            int64_t ts_base, int64_t seq_base, unsigned long long out_pos) {
  const PatternArgs& p = a.pat;
  const int64_t idx = (int64_t)bucket * kpb + k;
  const int64_t kl = ((int64_t)k << p.buckets_log2) | bucket;
  const int64_t ks = a.kstride;
  const int rw = p.rec_words;
  AggEnv env{&p, nullptr, 0, {}};
  const bool live = (L.khdr[k] & 0xffu) != 0;
#pragma unroll
  for (int j = 0; j < kMaxAggs; ++j) {
    env.s.acc[j] = (live && j < p.nagg) ? a.kslot[(int64_t)(2 * j) * ks + idx] : 0;
    env.s.cnt[j] = (live && j < p.nagg) ? a.kslot[(int64_t)(2 * j + 1) * ks + idx] : 0;
  }
  uint32_t emitted = 0;
  for (uint32_t q = L.kstart[k]; q < L.kstart[k + 1]; ++q) {
    const uint64_t* rec = a.recs + (int64_t)L.wrec[L.sorted[q]] * rw;
    agg_update(p, env.s, rec);
    env.rec = rec;
    env.ev_ts = rec_ts(rec, ts_base);
    bool pass = true;
    if (kVm && p.having_prog >= 0) {
      bool isnull = false;
      const uint64_t v = eval_env(a.vm, p.having_prog, R, env, &isnull);
      pass = !isnull && (v & 1u);
    }
    if (!pass) continue;
    if (kEmit) emit_row<kVm>(a, R, env, key_value(p, kl), rec_seq(rec, seq_base), out_pos + emitted);
    ++emitted;
  }
  if (kEmit) {
#pragma unroll
    for (int j = 0; j < kMaxAggs; ++j) {
      if (j >= p.nagg) break;
      a.kslot[(int64_t)(2 * j) * ks + idx] = env.s.acc[j];
      a.kslot[(int64_t)(2 * j + 1) * ks + idx] = env.s.cnt[j];
    }
    L.khdr[k] = 1u;
    a.khdr[idx] = 1u;
  }
  return emitted;
}

// ---- N-state patterns / sequences (nfa_mode) --------------------------------
// One lane walks one key's records in arrival order over the key's partial
// matches, kept in its state slots {start ts, state | count << 8, captures}.
// Restates oracle/siddhi_oracle.py _pattern_event / _sequence_event (SURVEY
// App. A.3-A.5).  Patterns: a partial advances when the event is on its next
// state's stream and the condition holds (else it stays), expired partials
// are dropped, advanced partials move behind the ones that stayed, a start
// event appends a new partial.  Sequences: every event of the query's streams
// either advances a partial (staying in a count state, or moving to a later
// state skipping optional ones) or discards it.  Matches reserve output rows
// one by one (a lane's rows of one event stay in creation order).
// Reserve `need` slots of a pool without pushing its cursor past `cap`:
// ~0 when they do not fit (a failed booking leaves the cursor as it was, so
// smaller bookings later in the launch can still succeed).
__device__ __forceinline__ unsigned long long pool_reserve(unsigned long long* cursor, unsigned long long need,
                                                           unsigned long long cap) {
  unsigned long long o = *(volatile unsigned long long*)cursor;
  while (true) {
    if (o + need > cap) return ~0ull;
    const unsigned long long prev = atomicCAS(cursor, o, o + need);
    if (prev == o) return o;
    o = prev;
  }
}

template <bool kVm>
__device__ __forceinline__ bool nfa_cond(const WalkArgs& a, uint64_t* R, int j, uint32_t role,
                                         const uint64_t* slot, int64_t st, const uint64_t* rec, int64_t ts_base) {
  const PatternArgs& p = a.pat;
  if (p.nfa_pair) {   // 2-state record roles: A = s1's condition, G = g passed in the partition
    if (j == 0) return (role & ROLE_A) != 0;
    if (role & ROLE_G) return true;
    if (!(role & ROLE_B) || !kVm || p.g_walk_prog < 0) return false;
    const MatchEnv env{slot, nullptr, p.cap_from_rec, rec, ts_base, st};
    bool isnull = false;
    const uint64_t v = eval_env(a.vm, p.g_walk_prog, R, env, &isnull);
    return !isnull && (v & 1u);
  }
  if (!((role >> j) & 1u)) return false;
  if (!kVm || p.st_walk[j] < 0) return true;
  const MatchEnv env{slot, nullptr, p.cap_from_rec, rec, ts_base, st};
  bool isnull = false;
  const uint64_t v = eval_env(a.vm, p.st_walk[j], R, env, &isnull);
  return !isnull && (v & 1u);
}

// Collect the event into state j of the partial at `slot` (count c after it).
__device__ __forceinline__ void nfa_collect(const PatternArgs& p, uint64_t* slot, int64_t ks, int j,
                                            int c, const uint64_t* rec) {
  slot[ks] = (uint64_t)(uint32_t)j | ((uint64_t)(uint32_t)c << 8);
  for (int i = 0; i < p.ncap; ++i) {
    if (p.cap_state[i] != j) continue;
    if (p.cap_index[i] < 0 || p.cap_index[i] + 1 == c) slot[(2 + i) * ks] = rec[2 + p.cap_word[i]];
  }
}

template <bool kVm>
__device__ __forceinline__ void nfa_emit(const WalkArgs& a, uint64_t* R, const uint64_t* slot, int64_t st,
                                         const uint64_t* rec, int64_t ts_base, int64_t seq_base,
                                         int64_t kl) {
  const PatternArgs& p = a.pat;
  const MatchEnv env{slot, nullptr, p.cap_from_rec, rec, ts_base, st};
  const unsigned long long pos = atomicAdd(a.out.count, 1ull);
  emit_row<kVm>(a, R, env, key_value(p, kl), rec_seq(rec, seq_base), pos);
}

template <bool kVm>
__device__ __noinline__ void nfa_key(const WalkArgs& a, WalkLds& L, uint64_t* R, int k, int bucket, int kpb,
                        int64_t ts_base, int64_t seq_base) {
  const PatternArgs& p = a.pat;
  const int S = p.pending_slots, sw = p.slot_words, rw = p.rec_words, N = p.nstates;
  const int64_t ks = a.kstride;
  const int64_t idx = (int64_t)bucket * kpb + k;
  const int64_t kl = ((int64_t)k << p.buckets_log2) | bucket;
  uint64_t* sl = a.kslot + idx;
  uint32_t hdr = L.khdr[k];
  const bool ovf0 = (hdr & kHdrOvf) != 0;
  const uint64_t ext0 = ovf0 ? a.kext[idx] : 0ull;
  int n = ovf0 ? (int)(ext0 & 0x7fffffffull) : (int)(hdr & 0xffu);
  bool started = ((hdr >> 8) & 1u) != 0;
  // Working storage.  Inline: list [0, S), staging [S, 2S), word stride ks.
  // Each record adds at most one partial, so a list can outgrow S only once
  // it holds S partials.  Then (lazily, before that record) the key moves to
  // one pool run sized for the rest of the window: list [0, M), staging
  // [M, 2M), word stride 1, M = n + records left; it is written back in the
  // at-rest layout (inline [0, S) + tail run) when the key is done.  A key
  // whose list stays within S books no pool slots at all.
  uint64_t* run = nullptr;
  unsigned long long roff = 0;
  int64_t st = ks;
  int CAP = S;
  bool pool_failed = false;
  auto grow = [&](uint32_t q_next) -> bool {
    // false only when an overflowed key cannot get its run: it keeps its state
    if (run || pool_failed || !a.pool_wr) return true;
    const int64_t M = (int64_t)n + (int64_t)(L.kstart[k + 1] - q_next);
    const unsigned long long need = 2ull * (unsigned long long)M;
    // reserve without pushing the cursor past pool_cap (a failed booking
    // must not make every later booking of the launch fail too)
    const unsigned long long o = pool_reserve(a.pool_cursor, need, a.pool_cap);
    if (o == ~0ull) {
      pool_failed = true;
      if (ovf0) {          // the tail cannot be moved: the key keeps its state, the error is real
        set_err(a.err, ERR_POOL);
        return false;
      }
      return true;         // inline; ERR_POOL only if the list really outgrows S
    }
    roff = o;
    run = a.pool_wr + o * (uint64_t)sw;
    const uint64_t* tail =
        ovf0 ? (((ext0 >> 31) & 1ull) ? (const uint64_t*)a.pool_wr : a.pool_rd) + (ext0 >> 32) * (uint64_t)sw
             : nullptr;
    for (int j = 0; j < n; ++j)
      for (int x = 0; x < sw; ++x)
        run[(int64_t)j * sw + x] = j < S ? sl[((int64_t)j * sw + x) * st] : tail[(int64_t)(j - S) * sw + x];
    st = 1;
    CAP = (int)M;
    return true;
  };
  auto list_full = [&]() { set_err(a.err, pool_failed ? ERR_POOL : ERR_PENDING); };
#define NSLOT(j) (run ? run + (int64_t)(j) * sw : sl + (int64_t)(j) * sw * ks)
  auto copy_slot = [&](int dst, int src) {
    if (dst == src) return;
    for (int x = 0; x < sw; ++x) NSLOT(dst)[x * st] = NSLOT(src)[x * st];
  };
  auto settle = [&](uint64_t* slot, int j, int c, const uint64_t* rec) -> bool {
    // returns whether the partial survives; emits when complete
    const bool done = c >= p.st_min[j] && p.st_tail_opt[j];
    if (!done) return true;
    nfa_emit<kVm>(a, R, slot, st, rec, ts_base, seq_base, kl);
    return j == N - 1 && (p.st_max[j] < 0 || c < p.st_max[j]);
  };
  for (uint32_t q = L.kstart[k]; q < L.kstart[k + 1]; ++q) {
    const uint64_t* rec = a.recs + (int64_t)L.wrec[L.sorted[q]] * rw;
    const uint64_t h = rec[0];
    const uint32_t role = (uint32_t)(h >> 32) & 0xffu;
    const int stream = (int)((h >> 40) & 0xffu);
    const int64_t ts = rec_ts(rec, ts_base);
    if (n >= CAP && !run && !grow(q)) return;
    int m = 0;
    if (!p.nfa_seq) {
      int nf = 0;   // advanced partials, staged in slots [CAP, 2 CAP)
      for (int i = 0; i < n; ++i) {
        uint64_t* si = NSLOT(i);
        // a 2-state pattern's partials all wait on state 1 (its at-rest slots
        // do not hold the state word)
        const int j = p.nfa_pair ? 1 : (int)(si[st] & 0xffu);
        if (p.st_stream[j] != stream) { copy_slot(m++, i); continue; }
        if (p.within >= 0) {
          const int64_t d = ts - (int64_t)si[0];
          if ((d < 0 ? -d : d) > p.within) continue;   // expired: dropped
        }
        if (!nfa_cond<kVm>(a, R, j, role, si, st, rec, ts_base)) { copy_slot(m++, i); continue; }
        if (j + 1 == N) {
          nfa_collect(p, si, st, j, 1, rec);
          nfa_emit<kVm>(a, R, si, st, rec, ts_base, seq_base, kl);   // consumed
          continue;
        }
        copy_slot(CAP + nf, i);
        nfa_collect(p, NSLOT(CAP + nf), st, j + 1 - 1, 1, rec);
        NSLOT(CAP + nf)[st] = (uint64_t)(j + 1);
        ++nf;
      }
      if (p.st_stream[0] == stream && (p.every || !started) &&
          nfa_cond<kVm>(a, R, 0, role, nullptr, st, rec, ts_base)) {
        started = true;
        uint64_t* ns = NSLOT(CAP + nf);
        ns[0] = (uint64_t)ts;
        for (int x = 2; x < sw; ++x) ns[x * st] = p.cap_null[x - 2];
        nfa_collect(p, ns, st, 0, 1, rec);
        if (N == 1) {
          nfa_emit<kVm>(a, R, ns, st, rec, ts_base, seq_base, kl);
        } else {
          ns[st] = 1;
          ++nf;
        }
      }
      if (m + nf > CAP) {
        list_full();
        nf = CAP - m;
      }
      for (int f = 0; f < nf; ++f) copy_slot(m + f, CAP + f);
      n = m + nf;
    } else {
      for (int i = 0; i < n; ++i) {
        uint64_t* si = NSLOT(i);
        if (p.within >= 0) {
          const int64_t d = ts - (int64_t)si[0];
          if ((d < 0 ? -d : d) > p.within) continue;
        }
        const uint64_t jc = si[st];
        const int j = (int)(jc & 0xffu), c = (int)(jc >> 8);
        bool keep = false;
        if (p.st_stream[j] == stream && (p.st_max[j] < 0 || c < p.st_max[j]) &&
            nfa_cond<kVm>(a, R, j, role, si, st, rec, ts_base)) {
          nfa_collect(p, si, st, j, c + 1, rec);              // stay in the count state
          keep = settle(si, j, c + 1, rec);
        } else if (c >= p.st_min[j]) {
          for (int j2 = j + 1; j2 < N; ++j2) {                // move on, skipping optional states
            if (p.st_stream[j2] == stream && nfa_cond<kVm>(a, R, j2, role, si, st, rec, ts_base)) {
              nfa_collect(p, si, st, j2, 1, rec);
              keep = settle(si, j2, 1, rec);
              break;
            }
            if (p.st_min[j2] > 0) break;
          }
        }
        if (keep) copy_slot(m++, i);                          // else discarded (contiguity)
      }
      if (p.st_stream[0] == stream && (p.every || !started) &&
          nfa_cond<kVm>(a, R, 0, role, nullptr, st, rec, ts_base)) {
        started = true;
        if (m >= CAP) {
          list_full();
        } else {
          uint64_t* ns = NSLOT(m);
          ns[0] = (uint64_t)ts;
          for (int x = 2; x < sw; ++x) ns[x * st] = p.cap_null[x - 2];
          nfa_collect(p, ns, st, 0, 1, rec);
          if (settle(ns, 0, 1, rec)) ++m;
        }
      }
      n = m;
    }
  }
#undef NSLOT
  bool ovf = false;
  if (run) {   // back to the at-rest layout: inline [0, S), tail [S, n) in place in the run
    for (int j = 0; j < n && j < S; ++j)
      for (int x = 0; x < sw; ++x) sl[((int64_t)j * sw + x) * ks] = run[(int64_t)j * sw + x];
    if (n > S) {
      ovf = true;
      a.kext[idx] = (uint64_t)(uint32_t)n | (1ull << 31) | ((uint64_t)(roff + (unsigned long long)S) << 32);
    }
  } else if (ovf0) {   // no record this window: the at-rest list (inline + tail run) stays as it is
    ovf = true;
  }
  const uint32_t nh = (uint32_t)(ovf ? S : n) | ((started ? 1u : 0u) << 8) | (ovf ? kHdrOvf : 0u);
  L.khdr[k] = nh;
  a.khdr[idx] = nh;
}

// Kernel end (N-state walk): a key's overflow tail still in the read pool
// moves to the write pool (the host swaps the pools per launch); kext then
// names the run in what the next launch reads.
__device__ void nfa_settle_runs(const WalkArgs& a, WalkLds& L, int bucket, int kpb) {
  const int S = a.pat.pending_slots, sw = a.pat.slot_words;
  for (int k = threadIdx.x; k < kpb; k += kWalkThreads) {
    if (!(L.khdr[k] & kHdrOvf)) continue;
    const int64_t idx = (int64_t)bucket * kpb + k;
    uint64_t e = a.kext[idx];
    const uint64_t n = e & 0x7fffffffull;
    uint64_t off = e >> 32;
    if (!((e >> 31) & 1ull)) {
      const unsigned long long cnt = n - (uint64_t)S;
      const unsigned long long o = pool_reserve(a.pool_cursor, cnt, a.pool_cap);
      if (o == ~0ull) {
        set_err(a.err, ERR_POOL);
        continue;
      }
      const uint64_t* src = a.pool_rd + off * (uint64_t)sw;
      uint64_t* dst = a.pool_wr + o * (uint64_t)sw;
      for (uint64_t i = 0; i < cnt * (uint64_t)sw; ++i) dst[i] = src[i];
      off = o;
    }
    a.kext[idx] = n | (off << 32);
  }
}

}  // namespace

// kVm = false: g is evaluated in the partition pass and every output attribute
// is a direct copy (no interpreter in the walk).
template <bool kVm>
__global__ __launch_bounds__(kWalkThreads) void k_walk(WalkArgs a) {
  __shared__ WalkLds L;
  __shared__ uint64_t R[kVm ? kMaxRegs * kWalkThreads : 1];   // VM registers, [reg][lane]
  __shared__ uint32_t Lseg[walk_max_tiles<kVm>() + 1];        // exclusive prefix of segment sizes
  __shared__ uint16_t Llo[walk_max_tiles<kVm>()];             // segment start inside each tile
  const int tid = threadIdx.x;
  const PatternArgs& p = a.pat;
  const int P = 1 << p.buckets_log2;
  const int bucket = xcd_bucket(blockIdx.x, P);
  const int kpb = (int)((p.key_capacity + P - 1) >> p.buckets_log2);
  const int ntiles = a.ntiles;
  const int rw = p.rec_words;
  const int ncw = rw - 2;   // carried words per record
  WALK_STAMP(0);
  const int64_t ts_base = a.chunk_base[0];
  const int64_t seq_base = a.chunk_base[1];
  const int64_t ks = a.kstride;
  // this bucket's per-key headers: kpb consecutive words (bucket-major index)
  for (int k = tid; k < kpb; k += kWalkThreads) {
    const uint32_t h = a.khdr[(int64_t)bucket * kpb + k];
    // a list that overflowed into the pending pool: the N-state walk works on
    // it (nfa_key); the other walks keep per-key lists of pending_slots
    if ((h & kHdrOvf) && !(kVm && p.nfa_mode && a.kext)) {
      set_err(a.err, ERR_PENDING);
      L.khdr[k] = h & ~kHdrOvf;
    } else {
      L.khdr[k] = h;
    }
  }

  // segment starts and sizes -> exclusive prefix over tiles
  {
    constexpr int MAXPER = walk_max_tiles<kVm>() / kWalkThreads;   // 4 or 16
    const int per = (ntiles + kWalkThreads - 1) / kWalkThreads;   // <= MAXPER
    uint32_t cnt[MAXPER];
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < MAXPER; ++i) {
      const int t = tid * per + i;
      cnt[i] = 0;
      if (i < per && t < ntiles) {
        const uint16_t* o = a.tile_off + (int64_t)t * (P + 1) + bucket;
        const uint32_t lo = o[0], hi = o[1];
        Llo[t] = (uint16_t)lo;
        cnt[i] = hi - lo;
      }
      sum += cnt[i];
    }
    uint32_t total;
    uint32_t off = block_excl_scan(sum, L.scratch, &total);
#pragma unroll
    for (int i = 0; i < MAXPER; ++i) {
      const int t = tid * per + i;
      if (i < per && t < ntiles) {
        Lseg[t] = off;
        off += cnt[i];
      }
    }
    if (tid == 0) Lseg[ntiles] = total;
  }
  lds_barrier();
  WALK_STAMP(1);

  int t0 = 0;
  while (t0 < ntiles) {
    if (tid == 0) {
      // largest t1 with seg[t1] - seg[t0] <= window (a single tile's segment is
      // at most tile_rows = 2048 > window: such a tile is split below)
      int lo = t0 + 1, hi = ntiles;
      const uint32_t lim = Lseg[t0] + kWalkWindow;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (Lseg[mid] <= lim) lo = mid;
        else hi = mid - 1;
      }
      L.t1 = (uint32_t)lo;
    }
    for (int k = tid; k <= kpb; k += kWalkThreads) L.kstart[k] = 0;
    lds_barrier();
    const int t1 = (int)L.t1;
    const uint32_t wbase = Lseg[t0];
    const uint32_t nrec = Lseg[t1] - wbase;
    if (nrec > kWalkWindow) {   // one tile holds more than a window of this bucket
      set_err(a.err, ERR_WINDOW);
    }
    const uint32_t nw = nrec < (uint32_t)kWalkWindow ? nrec : (uint32_t)kWalkWindow;
    // gather the window: record indices per tile segment (LDS only), then one
    // independent 16-byte header load (+ carried words) per record
    for (int t = t0 + tid; t < t1; t += kWalkThreads) {
      const uint32_t pos = Lseg[t] - wbase, cnt = Lseg[t + 1] - Lseg[t];
      const uint32_t g0 = (uint32_t)t * (uint32_t)a.tile_rows + Llo[t];
      for (uint32_t j = 0; j < cnt && pos + j < (uint32_t)kWalkWindow; ++j) L.wrec[pos + j] = g0 + j;
    }
    lds_barrier();
    for (uint32_t w = tid; w < nw; w += kWalkThreads) {
      const uint64_t* rec = a.recs + (int64_t)L.wrec[w] * rw;
      const uint4 hv = gload4(rec);   // w0, w1 in one 16-byte load
      uint4 cv = make_uint4(0, 0, 0, 0);
      if (p.closed_form && ncw > 0) cv = gload4(rec + 2);
      const uint64_t h = ((uint64_t)hv.y << 32) | hv.x;
      L.wkey[w] = (uint16_t)((uint32_t)h >> p.buckets_log2);
      L.wseq[w] = hv.z;
      if (p.closed_form) {
        L.cf.wts[w] = (int32_t)hv.w;
        L.cf.wrole[w] = (uint8_t)(h >> 32);
        L.cf.wcap[w][0] = ((uint64_t)cv.y << 32) | cv.x;
        L.cf.wcap[w][1] = ((uint64_t)cv.w << 32) | cv.z;
      }
      atomicAdd(&L.kstart[((uint32_t)h >> p.buckets_log2) + 1], 1u);
    }
    lds_barrier();
    WALK_STAMP(2);
    // exclusive scan of key counts (kstart[1..kpb] -> kstart[0..kpb])
    {
      const int per = (kpb + kWalkThreads - 1) / kWalkThreads;   // <= 1
      const uint32_t c = (tid < kpb) ? L.kstart[tid + 1] : 0u;
      uint32_t total;
      const uint32_t off = block_excl_scan(per ? c : 0u, L.scratch, &total);
      if (tid < kpb) {
        L.kstart[tid] = off;
        L.kcur[tid] = off;
      }
      if (tid == 0) L.kstart[kpb] = total;
    }
    lds_barrier();
    for (uint32_t w = tid; w < nw; w += kWalkThreads) {
      const uint32_t slot = atomicAdd(&L.kcur[L.wkey[w]], 1u);
      L.sorted[slot] = (uint16_t)w;
    }
    lds_barrier();
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
    lds_barrier();
    WALK_STAMP(3);

    bool nfa = false;
    if constexpr (kVm) nfa = p.nfa_mode != 0;   // (the NFA walk needs the VM build)
    if (nfa) {
      // ---- N-state pattern / sequence: one NFA lane per key -----------------
      if constexpr (kVm) {
        for (int k = tid; k < kpb; k += kWalkThreads)
          if (L.kstart[k + 1] > L.kstart[k]) nfa_key<kVm>(a, L, R, k, bucket, kpb, ts_base, seq_base);
      }
    } else if (kVm && p.agg_mode) {
      // ---- group-by / having: one lane per group, count pass + emit pass ----
      // (VM build only: keeps the pattern fast path lean)
      uint32_t mine = 0;
      if constexpr (kVm)
        for (int k = tid; k < kpb; k += kWalkThreads)
          if (L.kstart[k + 1] > L.kstart[k])
            mine += agg_key<false, kVm>(a, L, R, k, bucket, kpb, ts_base, seq_base, 0);
      uint32_t total;
      const uint32_t off = block_excl_scan(mine, L.scratch, &total);
      if (tid == 0) L.base = total ? atomicAdd(a.out.count, (unsigned long long)total) : 0ull;
      lds_barrier();
      unsigned long long pos = L.base + off;
      if constexpr (kVm)
        for (int k = tid; k < kpb; k += kWalkThreads)
          if (L.kstart[k + 1] > L.kstart[k])
            pos += agg_key<true, kVm>(a, L, R, k, bucket, kpb, ts_base, seq_base, pos);
    } else if (p.closed_form) {
      // ---- closed form: A matches the next B of its key within W -----------
      const int S = p.pending_slots, sw = p.slot_words;
      // stage the carried state slots of every touched key in LDS: all global
      // loads of the window are issued here, back to back, so the emission and
      // commit below are LDS reads + HBM stores only
      {
        uint32_t need = 0;
        if (tid < kpb && L.kstart[tid + 1] > L.kstart[tid]) need = (L.khdr[tid] & 0xffu) * (uint32_t)sw;
        uint32_t total;
        const uint32_t off = block_excl_scan(need, L.scratch, &total);
        if (tid < kpb) {
          const bool fits = off + need <= (uint32_t)kWalkSlotStage;
          L.cf.soff[tid] = fits ? (uint16_t)off : kNone16;
          if (fits && need) {
            const uint64_t* sl = a.kslot + (int64_t)bucket * kpb + tid;
            uint64_t* st = L.cf.sstage + off;
            uint32_t i = 0;
            for (; i + 4 <= need; i += 4) {
              const uint64_t x0 = sl[(int64_t)i * ks], x1 = sl[(int64_t)(i + 1) * ks];
              const uint64_t x2 = sl[(int64_t)(i + 2) * ks], x3 = sl[(int64_t)(i + 3) * ks];
              st[i] = x0; st[i + 1] = x1; st[i + 2] = x2; st[i + 3] = x3;
            }
            for (; i < need; ++i) st[i] = sl[(int64_t)i * ks];
          }
        }
      }
      lds_barrier();
      for (int k = tid; k < kpb; k += kWalkThreads) {
        const uint32_t r0 = L.kstart[k], r1 = L.kstart[k + 1];
        uint32_t nb = 0xffffffffu;
        for (uint32_t q = r1; q-- > r0;) {
          L.cf.nextb[q] = nb == 0xffffffffu ? kNone16 : (uint16_t)nb;
          if (L.cf.wrole[L.sorted[q]] & ROLE_B) nb = q;
        }
        L.kcur[k] = nb;   // first B of the run
        uint8_t cm = 0, cf = 0;
        const int n0 = (int)(L.khdr[k] & 0xffu);
        if (r1 > r0 && nb != 0xffffffffu && n0) {
          const uint16_t so = L.cf.soff[k];
          const uint64_t* sl = a.kslot + (int64_t)bucket * kpb + k;
          const int64_t tb = (int64_t)L.cf.wts[L.sorted[nb]] + ts_base;
          int first = n0;
          for (int j = 0; j < n0; ++j) {
            const int64_t ets = so != kNone16 ? (int64_t)L.cf.sstage[so + j * sw]
                                              : (int64_t)sl[(int64_t)j * sw * ks];
            const int64_t d = tb - ets;
            if (p.within < 0 || (d < 0 ? -d : d) <= p.within) {
              first = j;
              break;
            }
          }
          cm = (uint8_t)(n0 - first);
          cf = (uint8_t)first;
        }
        L.cf.cm[k] = cm;
        L.cf.cfirst[k] = cf;
      }
      lds_barrier();
      WALK_STAMP(4);
      // per-position match flag + carried count at run start -> scan input
      constexpr int per = kWalkWindow / kWalkThreads;   // 2 contiguous positions per lane
      uint32_t vals[per];
      uint32_t sum = 0;
#pragma unroll
      for (int i = 0; i < per; ++i) {
        const uint32_t q = tid * per + i;
        uint32_t v = 0;
        if (q < nw) {
          const int w = L.sorted[q];
          const int k = L.wkey[w];
          if ((L.cf.wrole[w] & ROLE_A) && L.cf.nextb[q] != kNone16) {
            const int64_t d = (int64_t)L.cf.wts[L.sorted[L.cf.nextb[q]]] - (int64_t)L.cf.wts[w];
            v = (p.within < 0 || (d < 0 ? -d : d) <= p.within) ? 1u : 0u;
          }
          if (q == L.kstart[k]) v += L.cf.cm[k];
        }
        vals[i] = v;
        sum += v;
      }
      uint32_t total;
      uint32_t off = block_excl_scan(sum, L.scratch, &total);
#pragma unroll
      for (int i = 0; i < per; ++i) {
        L.cf.v[tid * per + i] = off;
        off += vals[i];
      }
      if (tid == 0) L.base = total ? atomicAdd(a.out.count, (unsigned long long)total) : 0ull;
      lds_barrier();
      WALK_STAMP(5);
      const unsigned long long base = L.base;
      // emit record matches (lane per position; record words in LDS: stores only)
      for (uint32_t q = tid; q < nw; q += kWalkThreads) {
        const int w = L.sorted[q];
        if (!(L.cf.wrole[w] & ROLE_A) || L.cf.nextb[q] == kNone16) continue;
        const int wb = L.sorted[L.cf.nextb[q]];
        const int64_t d = (int64_t)L.cf.wts[wb] - (int64_t)L.cf.wts[w];
        if (p.within >= 0 && (d < 0 ? -d : d) > p.within) continue;
        const int k = L.wkey[w];
        const uint32_t extra = q == L.kstart[k] ? L.cf.cm[k] : 0u;
        const int64_t kl = ((int64_t)k << p.buckets_log2) | bucket;
        const CfEnv env{L.cf.wcap[w], 0, p.cap_from_rec, L.cf.wcap[wb],
                        (int64_t)L.cf.wts[wb] + ts_base};
        emit_row<kVm>(a, R, env, key_value(p, kl), seq_base + L.wseq[wb], base + L.cf.v[q] + extra);
      }
      // (no barrier: the commit below reads nothing the emission writes)
      WALK_STAMP(6);
      // emit carried matches and commit per-key state (lane per key)
      for (int k = tid; k < kpb; k += kWalkThreads) {
        const uint32_t r0 = L.kstart[k], r1 = L.kstart[k + 1];
        if (r1 == r0) continue;
        const int64_t kl = ((int64_t)k << p.buckets_log2) | bucket;
        uint64_t* sl = a.kslot + (int64_t)bucket * kpb + k;   // slot j word w: sl[(j*sw+w)*ks]
        const int n0 = (int)(L.khdr[k] & 0xffu);
        const uint16_t so = L.cf.soff[k];
        const uint64_t* st = L.cf.sstage + (so != kNone16 ? so : 0);
        if (L.cf.cm[k]) {
          const int wb = L.sorted[L.kcur[k]];
          for (int j = 0; j < L.cf.cm[k]; ++j) {
            const int js = L.cf.cfirst[k] + j;
            const CfEnv env{so != kNone16 ? st + js * sw : sl + (int64_t)js * sw * ks,
                            so != kNone16 ? 1 : ks, p.cap_from_rec,
                            L.cf.wcap[wb], (int64_t)L.cf.wts[wb] + ts_base};
            emit_row<kVm>(a, R, env, key_value(p, kl), seq_base + L.wseq[wb],
                          base + L.cf.v[r0] + j);
          }
        }
        // survivors: partials created after the last B (all of them if no B),
        // pruned to those within W of the last start (event-time order).
        uint32_t lastb = 0xffffffffu;
        int64_t last_a_ts = INT64_MIN;
        for (uint32_t q = r0; q < r1; ++q) {
          const int w = L.sorted[q];
          if (L.cf.wrole[w] & ROLE_B) lastb = q;
          if (L.cf.wrole[w] & ROLE_A) last_a_ts = (int64_t)L.cf.wts[w] + ts_base;
        }
        const bool prune = p.within >= 0 && last_a_ts != INT64_MIN;
        int n = 0;
        if (lastb == 0xffffffffu) {   // carried partials survive, minus pruned ones
          for (int j = 0; j < n0; ++j) {
            const int64_t ets = so != kNone16 ? (int64_t)st[j * sw] : (int64_t)sl[(int64_t)j * sw * ks];
            if (prune && last_a_ts - ets > p.within) continue;
            if (n != j) {
              if (so != kNone16) {
                for (int x = 0; x < sw; ++x) sl[((int64_t)n * sw + x) * ks] = st[j * sw + x];
              } else {
                for (int x = 0; x < sw; ++x)
                  sl[((int64_t)n * sw + x) * ks] = sl[((int64_t)j * sw + x) * ks];
              }
            }
            ++n;
          }
        }
        // (a record that is both B and A starts a partial after completing others)
        for (uint32_t q = (lastb == 0xffffffffu ? r0 : lastb); q < r1; ++q) {
          const int w = L.sorted[q];
          if (!(L.cf.wrole[w] & ROLE_A)) continue;
          const int64_t ats = (int64_t)L.cf.wts[w] + ts_base;
          if (prune && last_a_ts - ats > p.within) continue;
          if (n >= S) {
            set_err(a.err, ERR_PENDING);
            break;
          }
          uint64_t* dst = sl + (int64_t)n * sw * ks;
          dst[0] = (uint64_t)ats;
          dst[ks] = (uint64_t)(seq_base + L.wseq[w]);
          for (int c = 0; c < p.ncap; ++c) dst[(2 + c) * ks] = L.cf.wcap[w][p.cap_from_rec[c]];
          ++n;
        }
        const uint32_t nh = (L.khdr[k] & ~0xffu) | (uint32_t)n;
        L.khdr[k] = nh;
        a.khdr[(int64_t)bucket * kpb + k] = nh;
      }
      WALK_STAMP(7);
    } else {
      // ---- general form: one NFA lane per key (count pass, emit pass) -------
      uint32_t mine = 0;
      for (int k = tid; k < kpb; k += kWalkThreads)
        if (L.kstart[k + 1] > L.kstart[k])
          mine += walk_key<false, kVm>(a, L, R, k, bucket, kpb, ts_base, seq_base, 0);
      uint32_t total;
      const uint32_t off = block_excl_scan(mine, L.scratch, &total);
      if (tid == 0) L.base = total ? atomicAdd(a.out.count, (unsigned long long)total) : 0ull;
      lds_barrier();
      unsigned long long pos = L.base + off;
      for (int k = tid; k < kpb; k += kWalkThreads)
        if (L.kstart[k + 1] > L.kstart[k])
          pos += walk_key<true, kVm>(a, L, R, k, bucket, kpb, ts_base, seq_base, pos);
    }
    // the next window re-reads state slots this one wrote (HBM) and reuses
    // the LDS arrays: full barrier; none after the last window
    if (t1 < ntiles) __syncthreads();
    t0 = t1;
  }
  if constexpr (kVm)
    if (p.nfa_mode && a.kext) nfa_settle_runs(a, L, bucket, kpb);
}

void launch_walk(const WalkArgs& a, int nbuckets, bool vm, hipStream_t s) {
  if (vm) hipLaunchKernelGGL(k_walk<true>, dim3((unsigned)nbuckets), dim3(kWalkThreads), 0, s, a);
  else hipLaunchKernelGGL(k_walk<false>, dim3((unsigned)nbuckets), dim3(kWalkThreads), 0, s, a);
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
