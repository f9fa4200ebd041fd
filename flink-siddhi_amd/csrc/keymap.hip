// Device partition-key map: arbitrary int / long partition values -> dense
// key slots [0, key_capacity) (cep_options.sparse_keys).
//
// Siddhi's `partition with (k of A, k of B)` accepts any attribute value, and
// flink-siddhi's router hashes whatever the group-by value is
// (router/AddRouteOperator.java:83-92).  The per-key state of the pattern
// kernels is a dense array, so a batch's key column is first mapped through
// an open-addressing hash table in HBM (linear probing, capacity >= 2 x
// key_capacity, load <= 0.5): the first occurrence of a value claims a table
// slot with a 64-bit CAS and a dense id from a counter, later occurrences
// read it back.  rev[id] keeps the value for output rows (`select s1.k`).
//
// Table word encoding: stored = value + 1 (0 = empty); the value -1 (all
// ones) would encode as 0 and owns a dedicated id word instead.
#include <hip/hip_runtime.h>

#include "dev_common.h"
#include "kernels.h"

namespace cep {

namespace {

constexpr uint32_t kNoId = 0xffffffffu;
constexpr uint32_t kClaim = 0xfffffffeu;   // minus_one: being assigned

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t ld_id(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t ld_key(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_keymap(KeyMapArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool row = i < a.n;
  int64_t v = 0;
  bool use = false;
  if (row) {
    const int64_t r = a.row0 + i;
    const int s = a.stream ? (int)a.stream[r] : a.input;
    use = s == a.a_stream || s == a.b_stream;
    if (use) v = a.key_is_long ? ((const int64_t*)a.key)[r] : (int64_t)((const int32_t*)a.key)[r];
  }
  uint32_t id = 0;
  if (use && v == -1) {
    // the value whose table encoding would be "empty": its own id word
    // (kNoId -> kClaim by one lane, which then publishes the id)
    unsigned int cur = ld_id(a.minus_one);
    if (cur == kNoId && atomicCAS(a.minus_one, kNoId, kClaim) == kNoId) {
      const unsigned int mine = atomicAdd(a.count, 1u);
      if (mine >= a.cap) set_err(a.err, ERR_KEYMAP);
      else a.rev[mine] = (uint64_t)v;
      __hip_atomic_store(a.minus_one, mine < a.cap ? mine : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    cur = ld_id(a.minus_one);
    for (int t = 0; t < (1 << 22) && cur >= kClaim; ++t) cur = ld_id(a.minus_one);
    if (cur >= kClaim) set_err(a.err, ERR_KEYMAP);
    id = cur >= kClaim ? 0u : cur;
    use = false;
  }
  // linear probing; every lane of the wave runs each step so a lane waiting
  // for an id runs after the lane of the same wave that claimed the slot
  const uint64_t stored = (uint64_t)v + 1ull;
  const uint64_t mask = a.table_cap - 1;
  uint64_t h = mix64((uint64_t)v) & mask;
  bool done = !use;
  bool wait = false;
  for (uint64_t step = 0; step <= mask && __ballot(!done) != 0; ++step) {
    bool won = false;
    if (!done && !wait) {
      const uint64_t cur = ld_key(&a.tkey[h]);
      if (cur == stored) {
        wait = true;
      } else if (cur == 0ull) {
        const unsigned long long prev = atomicCAS(&a.tkey[h], 0ull, (unsigned long long)stored);
        if (prev == 0ull) won = true;
        else if (prev == stored) wait = true;
        else h = (h + 1) & mask;
      } else {
        h = (h + 1) & mask;
      }
    }
    if (won) {
      const unsigned int mine = atomicAdd(a.count, 1u);
      if (mine >= a.cap) set_err(a.err, ERR_KEYMAP);
      id = mine < a.cap ? mine : 0u;
      if (mine < a.cap) a.rev[id] = (uint64_t)v;
      __hip_atomic_store(&a.tval[h], id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      done = true;
    }
    if (wait) {
      // the claiming lane publishes the id right after its CAS; bounded spin
      uint32_t x = kNoId;
      for (int t = 0; t < (1 << 22) && x == kNoId; ++t) x = ld_id(&a.tval[h]);
      if (x == kNoId) set_err(a.err, ERR_KEYMAP);
      id = x == kNoId ? 0u : x;
      wait = false;
      done = true;
    }
  }
  if (!done) set_err(a.err, ERR_KEYMAP);   // table full (cannot happen at load <= 0.5)
  if (row) a.out[i] = (int32_t)id;
}

// AddRouteOperator's partition key of each row (router/AddRouteOperator.java:
// 83-92): |hashCode(field)| with Java's hashCode per attribute type, then
// HashPartitioner's channel key % n (router/HashPartitioner.java:24-26); no
// key field (-1) goes to a pseudo-random channel (DynamicPartitioner.java:
// 53-55 draws java.util.Random; here a hash of the row's arrival number).
__global__ void k_route_keys(RouteKeyArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  int64_t key = -1;
  if (a.col) {
    int32_t h = 0;
    switch (a.type) {
      case T_INT: h = ((const int32_t*)a.col)[i]; break;
      case T_LONG: {
        const uint64_t v = (uint64_t)((const int64_t*)a.col)[i];
        h = (int32_t)(uint32_t)(v ^ (v >> 32));
        break;
      }
      case T_FLOAT: {
        const float f = ((const float*)a.col)[i];
        h = f != f ? 0x7fc00000 : (int32_t)__float_as_uint(f);
        break;
      }
      case T_DOUBLE: {
        const double d = ((const double*)a.col)[i];
        const uint64_t v = d != d ? 0x7ff8000000000000ull : (uint64_t)__double_as_longlong(d);
        h = (int32_t)(uint32_t)(v ^ (v >> 32));
        break;
      }
      case T_BOOL: h = ((const uint8_t*)a.col)[i] ? 1231 : 1237; break;
      default: {   // STRING: dictionary id -> String.hashCode() of the entry
        const int32_t id = ((const int32_t*)a.col)[i];
        h = (id >= 0 && id < a.nstr) ? a.str_hash[id] : 0;
      }
    }
    key = h < 0 ? -(int64_t)h : (int64_t)h;
  }
  if (a.keys) a.keys[i] = key;
  int32_t ch;
  if (key >= 0) {
    ch = (int32_t)(key % a.nchan);
  } else {
    const uint64_t r = mix64((uint64_t)(a.seq0 + i));
    ch = (int32_t)(r % (uint64_t)a.nchan);
  }
  a.chan[i] = ch;
}

}  // namespace

void launch_route_keys(const RouteKeyArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(k_route_keys, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, s, a);
}

void launch_keymap(const KeyMapArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  const int64_t blocks = (a.n + 255) / 256;
  hipLaunchKernelGGL(k_keymap, dim3((unsigned)blocks), dim3(256), 0, s, a);
}

}  // namespace cep
