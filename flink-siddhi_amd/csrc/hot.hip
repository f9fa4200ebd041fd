// Hot keys of the closed-form pattern path (`every s1=A[f] -> s2=B[g]
// within W` under `partition with`) on skewed streams.
//
// k_cfwalk resolves one key bucket per workgroup.  Under a Zipf-distributed
// key (s = 1.1 over 2^20 keys) the hottest key alone carries
// ~12 % of the records, so its bucket's workgroup walks ~250x the average
// bucket and the launch waits for it.  The closed form has no per-key
// sequential dependency: an A matches the next B of its key if that B is
// within W; the key's carried partials complete at its first B; the A's after
// its last B (minus pruned ones) are the new pending list.  So hot keys are
// taken out of the buckets and matched with grid-wide scans:
//
//   k_cfpart   diverts the records of up to kCfHotMax hot keys into buckets
//              P + h (one per hot slot h) of each tile;
//   k_hot_count / k_hot_base     slot sizes and per-tile offsets;
//   k_hot_gather   per tile: the hot segments sorted by (slot, row) in LDS,
//              stored into one array grouped by slot in arrival order;
//   k_hot_local / k_hot_carry / k_hot_flags   next B of each record inside
//              its slot: LDS segmented suffix scan per 2048-record block, one
//              workgroup resolving the carries between blocks, match flags;
//   k_hot_offsets   block offsets, carried completions per slot, one output
//              atomic for the whole hot set;
//   k_hot_emit / k_hot_commit   output rows; per slot the carried rows and the
//              new pending list (inline slots + overflow run, as k_cfwalk).
//   k_hot_update   after the chunk: slots whose key went cold are freed; keys
//              the walk found with more than `thresh` records take free slots
//              (they are diverted from the next chunk on).
//
// Output rows of a hot key are contiguous per chunk: its carried rows (in the
// carried block of the hot set), then its record matches in arrival order —
// the per-key order the walk produces; Siddhi's global order is restored by
// the flush's stable sort on seq as for every other row.
#include <hip/hip_runtime.h>

#include "dev_common.h"
#include "kernels.h"
#include "vm.h"

namespace cep {

namespace {

constexpr uint32_t kNoPos = 0xffffffffu;
constexpr int kHT = 512;   // threads per workgroup

__device__ __forceinline__ uint32_t h_slot(uint64_t w0) { return (uint32_t)(w0 >> 48); }
__device__ __forceinline__ uint32_t h_role(uint64_t w0) { return (uint32_t)(w0 >> 45) & 0x7u; }
__device__ __forceinline__ uint32_t h_row(uint64_t w0) { return (uint32_t)(w0 >> 32) & 0x1fffu; }

__device__ __forceinline__ int rec_words(const HotArgs& a) { return 1 + a.cf.nw; }

// Per-key state index of a dense key (bucket-major, as k_cfwalk).
__device__ __forceinline__ int64_t key_index(const HotArgs& a, int64_t kf) {
  const int lg = a.pat.buckets_log2;
  const int64_t P = 1ll << lg;
  const int64_t kpb = (a.pat.key_capacity + P - 1) >> lg;
  return (kf & (P - 1)) * kpb + (kf >> lg);
}

// Pending slot j word w of key kidx (inline slots, else the read pool's run).
__device__ __forceinline__ uint64_t slot_word(const HotArgs& a, int64_t kidx, int j, int w, uint64_t ovoff) {
  const int S = a.pat.pending_slots, sw = a.pat.slot_words;
  if (j < S) return a.kslot[(int64_t)(j * sw + w) * a.kstride + kidx];
  return a.pool_rd[(ovoff + (uint64_t)(j - S)) * (uint64_t)sw + (uint64_t)w];
}

__device__ __forceinline__ uint32_t hot_total(const HotArgs& a) { return a.hot_gbase[kCfHotMax]; }

__device__ __forceinline__ bool within_w(int64_t W, int64_t d) { return W < 0 || (d < 0 ? -d : d) <= W; }

// Order-tolerant records (pat.tolerant, as cf_kernels.hip): role 4 = a
// B-stream row failing g (expires partials, completes none); record ts are
// stored as ts - chunk base + 2^31.
constexpr uint32_t kRolePB = 4;
constexpr int64_t kTolBias = 1ll << 31;
constexpr uint32_t kTolEmptyMn = 0xffffffffu, kTolEmptyMx = 0u;   // empty range: mn > mx

__device__ __forceinline__ int64_t hot_ts_base(const HotArgs& a) {
  return a.chunk_base[0] - (a.pat.tolerant ? kTolBias : 0);
}

// a partial started at record ts t (record units) survives every B-stream row
// of the range [mn, mx] (empty: mn > mx)
__device__ __forceinline__ bool tol_ok(int64_t W, int64_t t, uint32_t mn, uint32_t mx) {
  return mn > mx || W < 0 || (t - (int64_t)mn <= W && (int64_t)mx - t <= W);
}

// Arrival number of the record at chunk row r (received shuffle records carry
// their global number; local rows are numbered from the chunk base).
__device__ __forceinline__ int64_t row_seq_of(const HotArgs& a, int64_t seq_base, uint32_t r) {
  // (output seq not stored: not read)
  return (a.in_seq && a.out.write_seq) ? (int64_t)a.in_seq[(int64_t)r * a.in_rec_words] : seq_base + (int64_t)r;
}

// One output row (as k_cfwalk's cf_emit).
__device__ __forceinline__ void hot_emit_row(const HotArgs& a, unsigned long long pos, int64_t kf,
                                             uint64_t acap0, uint64_t acap1, uint64_t b0, uint64_t b1,
                                             int64_t bts, int64_t seq) {
  if ((int64_t)pos >= a.out.cap) {
    set_err(a.err, ERR_OUT_CAP);
    return;
  }
  const int64_t kv = a.key_rev ? (int64_t)a.key_rev[kf] : kf * a.pat.key_stride + a.pat.key_offset;
  for (int c = 0; c < a.out.ncols; ++c) {
    const int src = a.out.src[c];
    uint64_t v;
    if (src == SRC_KEY) {
      v = (uint64_t)kv;
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

// A record's logical captures (cap_phys: -1 = its event ts).
__device__ __forceinline__ void a_caps(const HotArgs& a, const uint64_t* r, int64_t ats, uint64_t* x0,
                                       uint64_t* x1) {
  const int cp0 = a.cf.cap_phys[0], cp1 = a.cf.cap_phys[1];
  const int nw = a.cf.nw;
  const uint64_t a0 = nw > 0 ? r[1] : 0ull, a1 = nw > 1 ? r[2] : 0ull;
  *x0 = cp0 < 0 ? (uint64_t)ats : (cp0 == 0 ? a0 : a1);
  *x1 = cp1 < 0 ? (uint64_t)ats : (cp1 == 0 ? a0 : a1);
}

// ---- per slot: records this chunk and their offsets per tile ---------------
__global__ __launch_bounds__(kHT) void k_hot_count(HotArgs a) {
  __shared__ uint32_t scratch[16];
  __shared__ uint32_t carry;
  const int h = blockIdx.x;
  const int64_t nt = a.ntiles;
  const int P = 1 << a.pat.buckets_log2;
  const uint16_t* lo = a.tile_off + (int64_t)(P + h) * nt;
  const uint16_t* hi = lo + nt;
  if (threadIdx.x == 0) carry = 0;
  lds_barrier();
  for (int64_t t0 = 0; t0 < nt; t0 += kHT) {
    const int64_t t = t0 + threadIdx.x;
    const uint32_t c = t < nt ? (uint32_t)hi[t] - (uint32_t)lo[t] : 0u;
    uint32_t total;
    const uint32_t off = block_excl_scan(c, scratch, &total);
    if (t < nt) a.hoff[(int64_t)h * nt + t] = carry + off;
    lds_barrier();
    if (threadIdx.x == 0) carry += total;
    lds_barrier();
  }
  if (threadIdx.x == 0) a.hot_m[h] = carry;
}

__global__ __launch_bounds__(kHT) void k_hot_base(HotArgs a) {
  constexpr int PT = kCfHotMax / kHT;   // consecutive slots per thread
  __shared__ uint32_t scratch[16];
  uint32_t m[PT], sum = 0;
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    m[i] = a.hot_m[threadIdx.x * PT + i];
    sum += m[i];
  }
  uint32_t total;
  uint32_t off = block_excl_scan(sum, scratch, &total);
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    a.hot_gbase[threadIdx.x * PT + i] = off;
    off += m[i];
  }
  if (threadIdx.x == 0) {
    a.hot_gbase[kCfHotMax] = total;
    a.obase[0] = 0;
    a.obase[1] = 0;
  }
}

// ---- per tile: hot segments in row order -> the slot-grouped array.  The
// tile's hot region is already grouped by slot (k_cfpart's bucket order);
// inside a slot's segment a record's rank is the number of the segment's
// records with a smaller row (rows are unique in a tile).  Segments are
// short except for the very hottest keys, so this costs far less than
// sorting the region.
__global__ __launch_bounds__(kHT) void k_hot_gather(HotArgs a) {
  __shared__ uint16_t sslot[kCfTile], srow[kCfTile];
  __shared__ uint32_t sbase[kCfHotMax];
  __shared__ uint16_t sstart[kCfHotMax], send[kCfHotMax];
  const int64_t t = blockIdx.x;
  const int64_t nt = a.ntiles;
  const int P = 1 << a.pat.buckets_log2;
  const int RW = rec_words(a);
  const uint32_t r0 = a.tile_off[(int64_t)P * nt + t];
  const uint32_t r1 = a.tile_off[(int64_t)(P + kCfHotMax) * nt + t];
  const uint32_t cnt = r1 - r0;
  if (cnt == 0) return;
  const uint64_t* tr = a.recs + (t * kCfTile + r0) * RW;
  for (uint32_t i = threadIdx.x; i < cnt; i += kHT) {
    const uint64_t w0 = tr[(int64_t)i * RW];
    sslot[i] = (uint16_t)h_slot(w0);
    srow[i] = (uint16_t)h_row(w0);
  }
  lds_barrier();
  for (uint32_t p = threadIdx.x; p < cnt; p += kHT) {
    const uint32_t h = sslot[p];
    if (p == 0 || sslot[p - 1] != h) {
      sstart[h] = (uint16_t)p;
      sbase[h] = a.hot_gbase[h] + a.hoff[(int64_t)h * nt + t];
    }
    if (p + 1 == cnt || sslot[p + 1] != h) send[h] = (uint16_t)(p + 1 - 1);   // last position
  }
  lds_barrier();
  for (uint32_t p = threadIdx.x; p < cnt; p += kHT) {
    const uint32_t h = sslot[p];
    const uint32_t row = srow[p];
    const uint32_t s0 = sstart[h], s1 = (uint32_t)send[h] + 1;
    uint32_t rank = 0;
    if (!(a.ablate & 1))
      for (uint32_t q = s0; q < s1; ++q) rank += srow[q] < row ? 1u : 0u;
    const uint32_t dest = sbase[h] + rank;
    if (a.ablate & 2) continue;
    const uint64_t* src = tr + (int64_t)p * RW;
    uint64_t* dst = a.harr + (int64_t)dest * RW;
    for (int w = 0; w < RW; ++w) dst[w] = src[w];
    a.hrow[dest] = (uint32_t)t * (uint32_t)kCfTile + row;
  }
}

// ---- per block: next B inside the block (segmented suffix scan) -----------
template <bool TOL>   // TOL: also the order-tolerant ranges (their LDS only in that build)
__global__ __launch_bounds__(kHT) void k_hot_local(HotArgs a) {
  __shared__ uint16_t sl[kHotBlock];
  __shared__ uint32_t v0[kHotBlock], v1[kHotBlock];
  const uint32_t M = hot_total(a);
  const uint32_t p0 = blockIdx.x * (uint32_t)kHotBlock;
  if (p0 >= M) return;
  const uint32_t n = min((uint32_t)kHotBlock, M - p0);
  const int RW = rec_words(a);
  for (uint32_t i = threadIdx.x; i < n; i += kHT) {
    const uint64_t w0 = a.harr[(int64_t)(p0 + i) * RW];
    sl[i] = (uint16_t)h_slot(w0);
    v0[i] = (h_role(w0) & ROLE_B) ? i : kNoPos;
  }
  lds_barrier();
  uint32_t* cur = v0;
  uint32_t* nxt = v1;
  for (uint32_t d = 1; d < n; d <<= 1) {
    for (uint32_t i = threadIdx.x; i < n; i += kHT) {
      uint32_t x = cur[i];
      if (i + d < n && sl[i + d] == sl[i]) x = min(x, cur[i + d]);
      nxt[i] = x;
    }
    lds_barrier();
    uint32_t* tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
  // cur[i]: first B at or after i in i's slot run inside the block
  for (uint32_t i = threadIdx.x; i < n; i += kHT) {
    const uint32_t nb = (i + 1 < n && sl[i + 1] == sl[i]) ? cur[i + 1] : kNoPos;
    a.hnb[p0 + i] = nb == kNoPos ? kNoPos : p0 + nb;
  }
  if (threadIdx.x == 0) {
    uint32_t* s = a.bsum + (int64_t)blockIdx.x * 4;
    s[0] = sl[0];
    s[1] = cur[0] == kNoPos ? kNoPos : p0 + cur[0];
    s[2] = sl[n - 1];
  }
  if constexpr (TOL) {
    // per record: min / max ts of the B-stream rows from it to the next
    // g-passing B of its slot inclusive, inside the block (segmented suffix
    // scan by doubling; open: the range runs into the next block)
    __shared__ uint32_t tmn[2][kHotBlock], tmx[2][kHotBlock];
    __shared__ uint8_t top[2][kHotBlock];
    lds_barrier();
    for (uint32_t i = threadIdx.x; i < n; i += kHT) {
      const uint64_t w0 = a.harr[(int64_t)(p0 + i) * RW];
      const uint32_t role = h_role(w0), t = (uint32_t)w0;
      const bool bs = (role & (ROLE_B | kRolePB)) != 0;
      tmn[0][i] = bs ? t : kTolEmptyMn;
      tmx[0][i] = bs ? t : kTolEmptyMx;
      top[0][i] = (role & ROLE_B) ? 0 : 1;   // a g-passing B ends the range of the records before it
    }
    lds_barrier();
    int c = 0;
    for (uint32_t d = 1; d < n; d <<= 1) {
      for (uint32_t i = threadIdx.x; i < n; i += kHT) {
        uint32_t mn = tmn[c][i], mx = tmx[c][i];
        uint8_t o = top[c][i];
        if (o && i + d < n) {
          if (sl[i + d] == sl[i]) {
            const uint32_t m2 = tmn[c][i + d], x2 = tmx[c][i + d];
            mn = m2 < mn ? m2 : mn;
            mx = x2 > mx ? x2 : mx;
            o = top[c][i + d];
          } else {
            o = 0;   // the slot ends inside the block
          }
        }
        tmn[c ^ 1][i] = mn;
        tmx[c ^ 1][i] = mx;
        top[c ^ 1][i] = o;
      }
      lds_barrier();
      c ^= 1;
    }
    for (uint32_t i = threadIdx.x; i < n; i += kHT) {
      a.htmn[p0 + i] = tmn[c][i];
      a.htmx[p0 + i] = tmx[c][i];
      a.hflag[p0 + i] = top[c][i];
    }
    if (threadIdx.x == 0) {
      uint32_t* b = a.btol + (int64_t)blockIdx.x * 3;
      b[0] = tmn[c][0];
      b[1] = tmx[c][0];
      b[2] = top[c][0];
    }
  }
}

// ---- order-tolerant builds, one workgroup: the resolved range of every
// block's first record (btol[3b], btol[3b + 1]): its own range, continued
// into the next block's first record's resolved range while open and linked
// (the next block starts with the same slot).  Chunks of blocks per thread,
// chunk heads resolved by doubling, then each chunk re-walked.
__global__ __launch_bounds__(kHT) void k_hot_carry_tol(HotArgs a) {
  __shared__ uint32_t hm[2][kHT], hx[2][kHT];
  __shared__ uint8_t ho[2][kHT];
  const uint32_t M = hot_total(a);
  const int nb = (int)((M + kHotBlock - 1) / kHotBlock);
  if (nb == 0) return;
  const int tid = threadIdx.x;
  const int cpt = (nb + kHT - 1) / kHT;
  const int b0 = tid * cpt, b1 = min(nb, b0 + cpt);
  auto linked = [&](int b) -> bool {
    return b + 1 < nb && a.bsum[(int64_t)b * 4 + 2] == a.bsum[(int64_t)(b + 1) * 4];
  };
  uint32_t mn = kTolEmptyMn, mx = kTolEmptyMx;
  bool open = b0 < b1;
  for (int b = b1 - 1; b >= b0; --b) {
    const uint32_t* t = a.btol + (int64_t)b * 3;
    if (t[2] && linked(b)) {
      mn = t[0] < mn ? t[0] : mn;
      mx = t[1] > mx ? t[1] : mx;
    } else {
      mn = t[0];
      mx = t[1];
      open = false;
    }
  }
  int c = 0;
  hm[0][tid] = mn;
  hx[0][tid] = mx;
  ho[0][tid] = open ? 1 : 0;
  lds_barrier();
  for (int d = 1; d < kHT; d <<= 1) {
    uint32_t m = hm[c][tid], x = hx[c][tid];
    uint8_t o = ho[c][tid];
    if (o) {
      if (tid + d < kHT) {
        const uint32_t m2 = hm[c][tid + d], x2 = hx[c][tid + d];
        m = m2 < m ? m2 : m;
        x = x2 > x ? x2 : x;
        o = ho[c][tid + d];
      } else {
        o = 0;
      }
    }
    hm[c ^ 1][tid] = m;
    hx[c ^ 1][tid] = x;
    ho[c ^ 1][tid] = o;
    lds_barrier();
    c ^= 1;
  }
  // the resolved range at the next chunk's first block, then this chunk right to left
  uint32_t rm = tid + 1 < kHT ? hm[c][tid + 1] : kTolEmptyMn;
  uint32_t rx = tid + 1 < kHT ? hx[c][tid + 1] : kTolEmptyMx;
  for (int b = b1 - 1; b >= b0; --b) {
    uint32_t* t = a.btol + (int64_t)b * 3;
    uint32_t fm = t[0], fx = t[1];
    if (t[2] && linked(b)) {
      fm = rm < fm ? rm : fm;
      fx = rx > fx ? rx : fx;
    }
    t[0] = fm;
    t[1] = fx;
    rm = fm;
    rx = fx;
  }
}

// ---- one workgroup: for each block, the first B at or after its first record
// in that record's slot (R, bsum word 3): R[b] = linked(b) ? R[b + 1] : own
__global__ __launch_bounds__(kHT) void k_hot_carry(HotArgs a) {
  __shared__ uint32_t hv[kHT];
  __shared__ uint8_t hopen[kHT];
  __shared__ uint32_t tv[kHT];
  __shared__ uint8_t topen[kHT];
  const uint32_t M = hot_total(a);
  const int nb = (int)((M + kHotBlock - 1) / kHotBlock);
  if (nb == 0) return;
  const int tid = threadIdx.x;
  const int c = (nb + kHT - 1) / kHT;
  const int b0 = tid * c, b1 = min(nb, b0 + c);
  auto linked = [&](int b) -> bool {
    const uint32_t* s = a.bsum + (int64_t)b * 4;
    return s[1] == kNoPos && s[0] == s[2] && b + 1 < nb && a.bsum[(int64_t)(b + 1) * 4] == s[0];
  };
  // chunk head: open (every block of the chunk links to the right) or a value
  bool open = true;
  uint32_t val = kNoPos;
  for (int b = b1 - 1; b >= b0; --b) {
    if (!linked(b)) {
      open = false;
      val = a.bsum[(int64_t)b * 4 + 1];
    }
  }
  if (b0 >= b1) {
    open = false;
    val = kNoPos;
  }
  // the last chunk's final block links nowhere (linked() checks b + 1 < nb)
  hv[tid] = val;
  hopen[tid] = open ? 1 : 0;
  lds_barrier();
  // suffix "first closed head to the right" by pointer doubling
  for (int d = 1; d < kHT; d <<= 1) {
    uint32_t v = hv[tid];
    uint8_t o = hopen[tid];
    if (o) {
      if (tid + d < kHT) {
        v = hv[tid + d];
        o = hopen[tid + d];
      } else {
        v = kNoPos;
        o = 0;
      }
    }
    lds_barrier();
    tv[tid] = v;
    topen[tid] = o;
    lds_barrier();
    hv[tid] = tv[tid];
    hopen[tid] = topen[tid];
    lds_barrier();
  }
  // resolved head of the chunk to the right
  uint32_t right = tid + 1 < kHT ? hv[tid + 1] : kNoPos;
  if (tid + 1 < kHT && hopen[tid + 1]) right = kNoPos;
  for (int b = b1 - 1; b >= b0; --b) {
    const uint32_t r = linked(b) ? right : a.bsum[(int64_t)b * 4 + 1];
    a.bsum[(int64_t)b * 4 + 3] = r;
    right = r;
  }
}

// ---- per block: final next B of every record, match flags, block count ----
__device__ __forceinline__ uint32_t block_carry(const HotArgs& a, int b, int nb) {
  if (b + 1 >= nb) return kNoPos;
  const uint32_t* s = a.bsum + (int64_t)b * 4;
  const uint32_t* t = s + 4;
  return t[0] == s[2] ? t[3] : kNoPos;
}

__device__ __forceinline__ bool hot_matched(const HotArgs& a, uint32_t p, uint32_t nbv, int RW) {
  if (nbv == kNoPos) return false;
  if (a.pat.tolerant) return (a.hflag[p] & 2u) != 0;   // an A alive at its next B (k_hot_flags)
  const uint64_t w0 = a.harr[(int64_t)p * RW];
  if (!(h_role(w0) & ROLE_A)) return false;
  const uint64_t wb = a.harr[(int64_t)nbv * RW];
  return within_w(a.pat.within, (int64_t)(uint32_t)wb - (int64_t)(uint32_t)w0);
}

template <bool TOL>
__global__ __launch_bounds__(kHT) void k_hot_flags(HotArgs a) {
  __shared__ uint32_t scratch[16];
  const uint32_t M = hot_total(a);
  const uint32_t p0 = blockIdx.x * (uint32_t)kHotBlock;
  if (p0 >= M) return;
  const int nb = (int)((M + kHotBlock - 1) / kHotBlock);
  const uint32_t n = min((uint32_t)kHotBlock, M - p0);
  const int RW = rec_words(a);
  const uint32_t carry = block_carry(a, blockIdx.x, nb);
  const uint32_t last = a.bsum[(int64_t)blockIdx.x * 4 + 2];
  if constexpr (TOL) {
    // resolved ranges (open ones continue into the next block's first
    // record), then each A's flag: alive iff every B-stream row after it up
    // to its next g-passing B (or the slot end) is within W of it
    __shared__ uint32_t fm[kHotBlock], fx[kHotBlock];
    __shared__ uint16_t fs[kHotBlock];
    const bool lk = blockIdx.x + 1 < nb && a.bsum[(int64_t)(blockIdx.x + 1) * 4] == last;
    const uint32_t cm = lk ? a.btol[(int64_t)(blockIdx.x + 1) * 3] : kTolEmptyMn;
    const uint32_t cx = lk ? a.btol[(int64_t)(blockIdx.x + 1) * 3 + 1] : kTolEmptyMx;
    for (uint32_t i = threadIdx.x; i < n; i += kHT) {
      const uint32_t p = p0 + i;
      uint32_t mn = a.htmn[p], mx = a.htmx[p];
      if ((a.hflag[p] & 1u) && lk) {
        mn = cm < mn ? cm : mn;
        mx = cx > mx ? cx : mx;
      }
      fm[i] = mn;
      fx[i] = mx;
      fs[i] = (uint16_t)h_slot(a.harr[(int64_t)p * RW]);
      a.htmn[p] = mn;
      a.htmx[p] = mx;
    }
    lds_barrier();
    for (uint32_t i = threadIdx.x; i < n; i += kHT) {
      const uint32_t p = p0 + i;
      const uint64_t w0 = a.harr[(int64_t)p * RW];
      uint32_t mn = kTolEmptyMn, mx = kTolEmptyMx;   // the range after this record
      if (i + 1 < n) {
        if (fs[i + 1] == fs[i]) {
          mn = fm[i + 1];
          mx = fx[i + 1];
        }
      } else if (lk) {
        mn = cm;
        mx = cx;
      }
      const bool alive = (h_role(w0) & ROLE_A) && tol_ok(a.pat.within, (int64_t)(uint32_t)w0, mn, mx);
      a.hflag[p] = (uint8_t)((a.hflag[p] & 1u) | (alive ? 2u : 0u));
    }
    __threadfence_block();
  }
  uint32_t c = 0;
  for (uint32_t i = threadIdx.x; i < n; i += kHT) {
    const uint32_t p = p0 + i;
    uint32_t nbv = a.hnb[p];
    if (nbv == kNoPos && h_slot(a.harr[(int64_t)p * RW]) == last) {
      nbv = carry;
      a.hnb[p] = nbv;
    }
    c += hot_matched(a, p, nbv, RW) ? 1u : 0u;
  }
  uint32_t total;
  block_excl_scan(c, scratch, &total);
  if (threadIdx.x == 0) a.bcnt[blockIdx.x] = total;
}

// ---- one workgroup: block offsets, carried completions per slot, output base
__global__ __launch_bounds__(kHT) void k_hot_offsets(HotArgs a) {
  __shared__ uint32_t scratch[16];
  __shared__ uint32_t carry;
  const uint32_t M = hot_total(a);
  const int nb = (int)((M + kHotBlock - 1) / kHotBlock);
  const int tid = threadIdx.x;
  if (tid == 0) carry = 0;
  lds_barrier();
  for (int b0 = 0; b0 < nb; b0 += kHT) {
    const int b = b0 + tid;
    const uint32_t c = b < nb ? a.bcnt[b] : 0u;
    uint32_t total;
    const uint32_t off = block_excl_scan(c, scratch, &total);
    if (b < nb) a.boff[b] = carry + off;
    lds_barrier();
    if (tid == 0) carry += total;
    lds_barrier();
  }
  const uint32_t rec_total = carry;
  // carried partials of slot h completed by its first B this chunk (each
  // thread: PT consecutive slots)
  constexpr int PT = kCfHotMax / kHT;
  uint32_t cmv[PT], cfv[PT], cmsum = 0;
  const int RW = rec_words(a);
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int h = tid * PT + i;
    uint32_t cm = 0, cfirst = 0;
    if (a.hot_key[h] >= 0 && a.hot_m[h] > 0) {
      const int64_t kf = a.hot_key[h];
      const int64_t kidx = key_index(a, kf);
      const uint32_t hdr = a.khdr[kidx];
      const bool ovf = (hdr & kHdrOvf) != 0;
      const uint64_t ext = ovf ? a.kext[kidx] : 0ull;
      const int n = ovf ? (int)(uint32_t)ext : (int)(hdr & 0xffu);
      const uint32_t g = a.hot_gbase[h];
      const uint32_t fb = (h_role(a.harr[(int64_t)g * RW]) & ROLE_B) ? g : a.hnb[g];
      if (a.pat.tolerant) {
        // carried partials alive at the first g-passing B: the B-stream rows
        // from the slot start to it inclusive (the resolved range of record g)
        if (n > 0 && fb != kNoPos) {
          const int64_t tb = hot_ts_base(a);
          const uint32_t mn = a.htmn[g], mx = a.htmx[g];
          for (int j = 0; j < n; ++j)
            cm += tol_ok(a.pat.within, (int64_t)slot_word(a, kidx, j, 0, ext >> 32) - tb, mn, mx) ? 1u : 0u;
        }
      } else if (n > 0 && fb != kNoPos) {
        const int64_t tb = a.chunk_base[0] + (int64_t)(uint32_t)a.harr[(int64_t)fb * RW];
        int j = 0;
        while (j < n && !within_w(a.pat.within, tb - (int64_t)slot_word(a, kidx, j, 0, ext >> 32))) ++j;
        cfirst = (uint32_t)j;
        cm = (uint32_t)(n - j);
      }
    }
    cmv[i] = cm;
    cfv[i] = cfirst;
    cmsum += cm;
  }
  uint32_t cm_total;
  uint32_t cm_off = block_excl_scan(cmsum, scratch, &cm_total);
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int h = tid * PT + i;
    a.hcm[h * 3 + 0] = cmv[i];
    a.hcm[h * 3 + 1] = cfv[i];
    a.hcm[h * 3 + 2] = cm_off;
    cm_off += cmv[i];
  }
  if (tid == 0) {
    const unsigned long long tot = (unsigned long long)cm_total + rec_total;
    a.obase[0] = tot ? atomicAdd(a.out.count, tot) : 0ull;
    a.obase[1] = cm_total;
  }
}

// ---- per block: record matches -> output rows ------------------------------
__global__ __launch_bounds__(kHT) void k_hot_emit(HotArgs a) {
  __shared__ uint32_t scratch[16];
  const uint32_t M = hot_total(a);
  const uint32_t p0 = blockIdx.x * (uint32_t)kHotBlock;
  if (p0 >= M) return;
  const uint32_t n = min((uint32_t)kHotBlock, M - p0);
  const int RW = rec_words(a);
  // rounds of kHT consecutive records (lane-interleaved): each round's rows
  // are consecutive positions, so the column stores coalesce
  unsigned long long base = a.obase[0] + a.obase[1] + a.boff[blockIdx.x];
  const int64_t ts_base = hot_ts_base(a), seq_base = a.chunk_base[1];
  for (uint32_t r0 = 0; r0 < n; r0 += kHT) {
    const uint32_t i = r0 + threadIdx.x;
    const uint32_t p = p0 + i;
    const uint32_t nbv = i < n ? a.hnb[p] : kNoPos;
    const bool m = i < n && hot_matched(a, p, nbv, RW);
    uint32_t total;
    const uint32_t off = block_excl_scan(m ? 1u : 0u, scratch, &total);
    if (m) {
      const uint64_t* r = a.harr + (int64_t)p * RW;
      const uint64_t* rb = a.harr + (int64_t)nbv * RW;
      const int64_t ats = ts_base + (int64_t)(uint32_t)r[0];
      const int64_t bts = ts_base + (int64_t)(uint32_t)rb[0];
      uint64_t x0, x1;
      a_caps(a, r, ats, &x0, &x1);
      const int64_t kf = a.hot_key[h_slot(r[0])];
      hot_emit_row(a, base + off, kf, x0, x1, a.cf.nw > 0 ? rb[1] : 0ull, a.cf.nw > 1 ? rb[2] : 0ull, bts,
                   row_seq_of(a, seq_base, a.hrow[nbv]));
    }
    base += total;
  }
}

// ---- per slot (one wave): carried rows, new pending list, state commit ----
__global__ __launch_bounds__(64) void k_hot_commit(HotArgs a) {
  const int h = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t kf = a.hot_key[h];
  if (kf < 0) return;
  const int RW = rec_words(a);
  const int S = a.pat.pending_slots, sw = a.pat.slot_words;
  const bool c1 = sw > 2, c2 = sw > 3;
  const int64_t W = a.pat.within;
  const int64_t kidx = key_index(a, kf);
  const uint32_t hdr = a.khdr[kidx];
  const bool ovf = (hdr & kHdrOvf) != 0;
  const uint64_t ext = ovf ? a.kext[kidx] : 0ull;
  const uint64_t ovoff = ext >> 32;
  const int n = ovf ? (int)(uint32_t)ext : (int)(hdr & 0xffu);
  const uint32_t m = a.hot_m[h];
  const bool tol = a.pat.tolerant != 0;
  const int64_t ts_base = hot_ts_base(a), seq_base = a.chunk_base[1];
  const int cp0 = a.cf.cap_phys[0], cp1 = a.cf.cap_phys[1];
  (void)cp0;
  (void)cp1;
  auto put = [&](int j, uint64_t ts, uint64_t x0, uint64_t x1, uint64_t nov) {
    if (j < S) {
      a.kslot[(int64_t)(j * sw) * a.kstride + kidx] = ts;
      if (c1) a.kslot[(int64_t)(j * sw + 2) * a.kstride + kidx] = x0;
      if (c2) a.kslot[(int64_t)(j * sw + 3) * a.kstride + kidx] = x1;
    } else {
      uint64_t* o = a.pool_wr + (nov + (uint64_t)(j - S)) * (uint64_t)sw;
      o[0] = ts;
      if (c1) o[2] = x0;
      if (c2) o[3] = x1;
    }
  };
  auto finish = [&](int nn, uint64_t nov) {
    if (lane != 0) return;
    const uint32_t h1 = (hdr & ~(0xffu | kHdrOvf)) | (nn > S ? ((uint32_t)S | kHdrOvf) : (uint32_t)nn);
    if (nn > S) a.kext[kidx] = (uint64_t)(uint32_t)nn | (nov << 32);
    a.khdr[kidx] = h1;
  };
  if (m == 0) {
    // no records: the list is unchanged; an overflow run moves to the write pool
    if (n > S) {
      unsigned long long off = 0;
      if (lane == 0) off = atomicAdd(a.pool_cursor, (unsigned long long)(n - S));
      off = __shfl(off, 0, 64);
      if (off + (unsigned long long)(n - S) > a.pool_cap) {
        if (lane == 0) set_err(a.err, ERR_POOL);
        return;
      }
      for (int64_t i = lane; i < (int64_t)(n - S) * sw; i += 64)
        a.pool_wr[off * (uint64_t)sw + (uint64_t)i] = a.pool_rd[ovoff * (uint64_t)sw + (uint64_t)i];
      finish(n, off);
    }
    return;
  }
  const uint32_t g = a.hot_gbase[h], e = g + m;
  // first / last B and last A of the slot (backward wave scans)
  const uint32_t fb = (h_role(a.harr[(int64_t)g * RW]) & ROLE_B) ? g : a.hnb[g];
  uint32_t lb = kNoPos, la = kNoPos;
  for (int64_t base = (int64_t)e - 1; base >= (int64_t)g && (lb == kNoPos || la == kNoPos); base -= 64) {
    const int64_t p = base - lane;
    const uint32_t role = p >= (int64_t)g ? h_role(a.harr[p * RW]) : 0u;
    const unsigned long long bb = __ballot((role & ROLE_B) != 0);
    const unsigned long long ba = __ballot((role & ROLE_A) != 0);
    if (lb == kNoPos && bb) lb = (uint32_t)(base - (__ffsll((long long)bb) - 1));
    if (la == kNoPos && ba) la = (uint32_t)(base - (__ffsll((long long)ba) - 1));
  }
  const bool prune = !tol && W >= 0 && la != kNoPos;   // (tol: no pruning at A arrivals)
  // tol: the slot's first range (B-stream rows up to its first g-passing B)
  const uint32_t tmn0 = tol ? a.htmn[g] : 0u, tmx0 = tol ? a.htmx[g] : 0u;
  auto carried_alive = [&](int j) {
    return tol_ok(W, (int64_t)slot_word(a, kidx, j, 0, ovoff) - ts_base, tmn0, tmx0);
  };
  const int64_t last_a_ts = la != kNoPos ? ts_base + (int64_t)(uint32_t)a.harr[(int64_t)la * RW] : 0;
  // carried rows completed by the first B
  const uint32_t cm = a.hcm[h * 3 + 0], cfirst = a.hcm[h * 3 + 1], cm_off = a.hcm[h * 3 + 2];
  if (cm && tol) {
    // the carried partials alive at the first B, in slot order
    const uint64_t* rb = a.harr + (int64_t)fb * RW;
    const int64_t bts = ts_base + (int64_t)(uint32_t)rb[0];
    const uint64_t b0 = a.cf.nw > 0 ? rb[1] : 0ull, b1 = a.cf.nw > 1 ? rb[2] : 0ull;
    uint32_t o = 0;
    for (int j0 = 0; j0 < n; j0 += 64) {
      const int j = j0 + lane;
      const bool al = j < n && carried_alive(j);
      const unsigned long long bal = __ballot(al);
      if (al)
        hot_emit_row(a, a.obase[0] + cm_off + o + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull)), kf,
                     c1 ? slot_word(a, kidx, j, 2, ovoff) : 0ull, c2 ? slot_word(a, kidx, j, 3, ovoff) : 0ull,
                     b0, b1, bts, row_seq_of(a, seq_base, a.hrow[fb]));
      o += (uint32_t)__popcll(bal);
    }
  } else if (cm) {
    const uint64_t* rb = a.harr + (int64_t)fb * RW;
    const int64_t bts = ts_base + (int64_t)(uint32_t)rb[0];
    const uint64_t b0 = a.cf.nw > 0 ? rb[1] : 0ull, b1 = a.cf.nw > 1 ? rb[2] : 0ull;
    for (uint32_t j = lane; j < cm; j += 64) {
      const int js = (int)(cfirst + j);
      hot_emit_row(a, a.obase[0] + cm_off + j, kf, c1 ? slot_word(a, kidx, js, 2, ovoff) : 0ull,
                   c2 ? slot_word(a, kidx, js, 3, ovoff) : 0ull, b0, b1, bts, row_seq_of(a, seq_base, a.hrow[fb]));
    }
  }
  // the new list: (no B) the carried partials minus the pruned prefix, then
  // every A from the last B on (a record that is both B and A starts a new
  // partial after completing the others) minus pruned ones
  int drop = 0;
  int keep = 0;
  if (tol) {
    // (no B) the carried partials that survive the slot's B-stream rows
    if (lb == kNoPos)
      for (int j0 = 0; j0 < n; j0 += 64) {
        const int j = j0 + lane;
        keep += __popcll(__ballot(j < n && carried_alive(j)));
      }
  } else {
    if (lb == kNoPos) {
      while (drop < n && prune && last_a_ts - (int64_t)slot_word(a, kidx, drop, 0, ovoff) > W) ++drop;
    }
    keep = lb == kNoPos ? n - drop : 0;
  }
  const uint32_t from = lb == kNoPos ? g : lb;
  // count the new partials (wave ballots), then allocate the overflow run
  int nnew = 0;
  for (uint32_t base = from; base < e; base += 64) {
    const uint32_t p = base + lane;
    bool take = false;
    if (p < e) {
      const uint64_t w0 = a.harr[(int64_t)p * RW];
      take = (h_role(w0) & ROLE_A) && !(prune && last_a_ts - (ts_base + (int64_t)(uint32_t)w0) > W) &&
             (!tol || (a.hflag[p] & 2u));
    }
    nnew += __popcll(__ballot(take));
  }
  const int nn = keep + nnew;
  uint64_t nov = 0;
  if (nn > S) {
    unsigned long long off = 0;
    if (lane == 0) off = atomicAdd(a.pool_cursor, (unsigned long long)(nn - S));
    off = __shfl(off, 0, 64);
    if (off + (unsigned long long)(nn - S) > a.pool_cap) {
      if (lane == 0) set_err(a.err, ERR_POOL);
      return;
    }
    nov = off;
  }
  // kept carried partials: slot j <- old slot j + drop (all lanes read a
  // round's old slots before any lane writes: one wave, loads before stores);
  // tol: the alive ones compacted (a write never passes the slot it read)
  if (tol && keep > 0) {
    int w = 0;
    for (int j0 = 0; j0 < n; j0 += 64) {
      const int j = j0 + lane;
      uint64_t ts = 0, x0 = 0, x1 = 0;
      bool al = false;
      if (j < n) {
        ts = slot_word(a, kidx, j, 0, ovoff);
        x0 = c1 ? slot_word(a, kidx, j, 2, ovoff) : 0ull;
        x1 = c2 ? slot_word(a, kidx, j, 3, ovoff) : 0ull;
        al = tol_ok(W, (int64_t)ts - ts_base, tmn0, tmx0);
      }
      const unsigned long long bal = __ballot(al);
      __builtin_amdgcn_wave_barrier();
      if (al) put(w + __popcll(bal & ((1ull << lane) - 1ull)), ts, x0, x1, nov);
      w += __popcll(bal);
    }
  }
  for (int j0 = 0; j0 < (tol ? 0 : keep); j0 += 64) {
    const int j = j0 + lane;
    uint64_t ts = 0, x0 = 0, x1 = 0;
    if (j < keep) {
      ts = slot_word(a, kidx, j + drop, 0, ovoff);
      x0 = c1 ? slot_word(a, kidx, j + drop, 2, ovoff) : 0ull;
      x1 = c2 ? slot_word(a, kidx, j + drop, 3, ovoff) : 0ull;
    }
    __builtin_amdgcn_wave_barrier();
    if (j < keep) put(j, ts, x0, x1, nov);
  }
  int j = keep;
  for (uint32_t base = from; base < e; base += 64) {
    const uint32_t p = base + lane;
    bool take = false;
    uint64_t w0 = 0;
    if (p < e) {
      w0 = a.harr[(int64_t)p * RW];
      take = (h_role(w0) & ROLE_A) && !(prune && last_a_ts - (ts_base + (int64_t)(uint32_t)w0) > W) &&
             (!tol || (a.hflag[p] & 2u));
    }
    const unsigned long long bal = __ballot(take);
    if (take) {
      const int rank = __popcll(bal & ((1ull << lane) - 1ull));
      const int64_t ats = ts_base + (int64_t)(uint32_t)w0;
      uint64_t x0, x1;
      a_caps(a, a.harr + (int64_t)p * RW, ats, &x0, &x1);
      put(j + rank, (uint64_t)ats, x0, x1, nov);
    }
    j += __popcll(bal);
  }
  finish(nn, nov);
}

// ---- after the chunk: free cold slots, admit the walk's candidates, the
// busiest first (they are what makes a bucket a straggler) ------------------
__global__ __launch_bounds__(kCfHotMax) void k_hot_update(HotArgs a, int diverted) {
  constexpr int NC = kCfHotMax * 4;
  __shared__ uint64_t c[NC];
  __shared__ uint64_t sm[kCfHotMax];     // slots by records (ascending): m << 32 | slot
  __shared__ uint32_t freel[kCfHotMax];
  __shared__ uint32_t scan[kCfHotMax];
  __shared__ uint32_t nfree, nrest;
  const int h = threadIdx.x;
  auto block_incl_scan = [&](uint32_t v) -> uint32_t {   // inclusive scan over the block
    scan[h] = v;
    __syncthreads();
    for (int d = 1; d < kCfHotMax; d <<= 1) {
      const uint32_t x = h >= d ? scan[h - d] : 0u;
      __syncthreads();
      scan[h] += x;
      __syncthreads();
    }
    const uint32_t r = scan[h];
    __syncthreads();
    return r;
  };
  if (diverted && a.hot_key[h] >= 0 && a.hot_m[h] < a.thresh / 4) {
    a.hot_id[a.hot_key[h]] = kNotHot;
    a.hot_key[h] = -1;
  }
  const uint32_t n0 = min(a.ncand[0], (uint32_t)kCfHotMax);
  const uint32_t n1 = min(a.ncand[1], 3u * kCfHotMax);
  const uint32_t nc = n0 + n1;
  __syncthreads();
  if (nc > 0) {
    uint32_t N = 2;
    while (N < nc) N <<= 1;
    for (uint32_t i = h; i < N; i += kCfHotMax)
      c[i] = i < n0 ? a.cand[i] : (i < nc ? a.cand[kCfHotMax + (i - n0)] : 0ull);
    // free slots, in slot order
    const uint32_t f = a.hot_key[h] < 0 ? 1u : 0u;
    const uint32_t fs = block_incl_scan(f);
    if (f) freel[fs - 1] = (uint32_t)h;
    if (h == kCfHotMax - 1) nfree = fs;
    __syncthreads();
    // candidates, busiest first (bitonic sort, descending)
    for (uint32_t k = 2; k <= N; k <<= 1) {
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t i = h; i < N; i += kCfHotMax) {
          const uint32_t ixj = i ^ j;
          if (ixj > i) {
            const uint64_t x = c[i], y = c[ixj];
            const bool desc = (i & k) == 0;
            if ((x < y) == desc) {
              c[i] = y;
              c[ixj] = x;
            }
          }
        }
        __syncthreads();
      }
    }
    // the busiest candidates not hot yet take the free slots (one walk lane
    // per key: no key appears twice)
    for (uint32_t i0 = 0; i0 < nc; i0 += kCfHotMax) {
      const uint32_t i = i0 + h;
      const uint32_t k = i < nc ? (uint32_t)c[i] : 0u;
      const uint32_t adm = (i < nc && a.hot_id[k] == kNotHot) ? 1u : 0u;
      const uint32_t rank = block_incl_scan(adm) - adm;
      const uint32_t nf = nfree;
      if (adm && rank < nf) {
        const uint32_t slot = freel[rank];
        a.hot_key[slot] = (int32_t)k;
        a.hot_id[k] = (uint16_t)slot;
        a.hot_m[slot] = a.thresh;   // not evicted before it has been measured
        c[i] = 0;                   // taken
      }
      __syncthreads();
      if (h == kCfHotMax - 1) {
        const uint32_t used = min(scan[h] + 0u, nf);   // scan[] holds the round's inclusive total
        nfree = nf - used;
        for (uint32_t x = 0; x < nf - used; ++x) freel[x] = freel[x + used];
      }
      __syncthreads();
      if (nfree == 0) break;
    }
    // all slots taken: a candidate far busier than a slot's key this chunk
    // replaces it (pairs the i-th busiest waiting candidate with the i-th
    // idlest slot), so the hot set converges on the busiest keys
    if (diverted) {
      // waiting candidates, compacted in order
      uint32_t w = 0;
      for (uint32_t i0 = 0; i0 < nc; i0 += kCfHotMax) {
        const uint32_t i = i0 + h;
        const uint32_t k = i < nc ? (uint32_t)c[i] : 0u;
        const uint32_t wt = (i < nc && c[i] != 0 && a.hot_id[k] == kNotHot) ? 1u : 0u;
        const uint32_t r = block_incl_scan(wt) - wt;
        const uint64_t v = i < nc ? c[i] : 0ull;
        __syncthreads();
        if (wt && w + r < (uint32_t)kCfHotMax) c[w + r] = v;   // (in place: w + r <= i)
        w += scan[kCfHotMax - 1];
        __syncthreads();
      }
      if (h == 0) nrest = min(w, (uint32_t)kCfHotMax);
      const int32_t hk = a.hot_key[h];
      sm[h] = hk >= 0 ? (((uint64_t)a.hot_m[h] << 32) | (uint32_t)h) : ~0ull;
      __syncthreads();
      for (int k = 2; k <= kCfHotMax; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
          const int ixj = h ^ j;
          if (ixj > h) {
            const uint64_t x = sm[h], y = sm[ixj];
            const bool asc = (h & k) == 0;
            if ((x > y) == asc) {
              sm[h] = y;
              sm[ixj] = x;
            }
          }
          __syncthreads();
        }
      }
      if ((uint32_t)h < nrest && sm[h] != ~0ull) {
        const uint64_t cand = c[h];
        const uint32_t cm = (uint32_t)(cand >> 32), k = (uint32_t)cand;
        const uint32_t sm_m = (uint32_t)(sm[h] >> 32), slot = (uint32_t)sm[h];
        if ((uint64_t)cm > 4ull * sm_m) {
          a.hot_id[a.hot_key[slot]] = kNotHot;
          a.hot_key[slot] = (int32_t)k;
          a.hot_id[k] = (uint16_t)slot;
          a.hot_m[slot] = a.thresh;
        }
      }
    }
  }
  __syncthreads();
  if (h == 0) {
    a.ncand[0] = 0;
    a.ncand[1] = 0;
  }
  // slots in use
  scan[h] = a.hot_key[h] >= 0 ? 1u : 0u;
  __syncthreads();
  for (int d = kCfHotMax / 2; d > 0; d >>= 1) {
    if (h < d) scan[h] += scan[h + d];
    __syncthreads();
  }
  if (h == 0) *a.active = scan[0];
}

}  // namespace

void launch_hot_match(const HotArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_hot_count, dim3(kCfHotMax), dim3(kHT), 0, s, a);
  hipLaunchKernelGGL(k_hot_base, dim3(1), dim3(kHT), 0, s, a);
  hipLaunchKernelGGL(k_hot_gather, dim3((unsigned)a.ntiles), dim3(kHT), 0, s, a);
  const bool tol = a.pat.tolerant != 0;
  if (tol) hipLaunchKernelGGL(k_hot_local<true>, dim3((unsigned)a.max_blocks), dim3(kHT), 0, s, a);
  else hipLaunchKernelGGL(k_hot_local<false>, dim3((unsigned)a.max_blocks), dim3(kHT), 0, s, a);
  hipLaunchKernelGGL(k_hot_carry, dim3(1), dim3(kHT), 0, s, a);
  if (tol) {
    hipLaunchKernelGGL(k_hot_carry_tol, dim3(1), dim3(kHT), 0, s, a);
    hipLaunchKernelGGL(k_hot_flags<true>, dim3((unsigned)a.max_blocks), dim3(kHT), 0, s, a);
  } else {
    hipLaunchKernelGGL(k_hot_flags<false>, dim3((unsigned)a.max_blocks), dim3(kHT), 0, s, a);
  }
  hipLaunchKernelGGL(k_hot_offsets, dim3(1), dim3(kHT), 0, s, a);
  hipLaunchKernelGGL(k_hot_emit, dim3((unsigned)a.max_blocks), dim3(kHT), 0, s, a);
  hipLaunchKernelGGL(k_hot_commit, dim3(kCfHotMax), dim3(64), 0, s, a);
}

void launch_hot_update(const HotArgs& a, int diverted, hipStream_t s) {
  hipLaunchKernelGGL(k_hot_update, dim3(1), dim3(kCfHotMax), 0, s, a, diverted);
}

}  // namespace cep
