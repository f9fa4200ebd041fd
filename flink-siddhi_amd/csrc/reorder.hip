// Event-time reorder on the device: the buffer that
// replaces AbstractSiddhiOperator's PriorityQueue<StreamRecord>
// (core/.../operator/AbstractSiddhiOperator.java:222-231 offer,
// :238-247 processWatermark drain; StreamRecordComparator.java:32-40 orders by
// timestamp only).  Rows buffered since the last watermark are sorted by
// (ts, arrival) with one stable LSD radix sort of the 64-bit timestamps
// carrying a row permutation (rocPRIM onesweep), the prefix with
// ts <= watermark is gathered column by column into a sorted batch, and the
// rest is compacted back into the buffer in the same order.  Ties keep
// arrival order (the reference PQ is not stable: SURVEY App. B a5).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include "kernels.h"

namespace cep {

namespace {

__global__ void k_iota(int32_t* p, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (int32_t)i;
}

// dst[i] = src[perm[first + i]] for i < n, rows of `width` bytes (1, 4, 8)
template <typename T>
__global__ void k_gather(const T* __restrict__ src, T* __restrict__ dst, const int32_t* __restrict__ perm,
                         int64_t first, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[perm[first + i]];
}

// number of sorted keys <= wm (one thread: log2(n) dependent loads)
__global__ void k_upper_bound(const int64_t* __restrict__ sorted, int64_t n, int64_t wm, int64_t* out) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    if (sorted[mid] <= wm) lo = mid + 1;
    else hi = mid;
  }
  out[0] = lo;
  out[1] = n > 0 ? sorted[0] : 0;                 // earliest buffered ts
  out[2] = lo > 0 ? sorted[lo - 1] : 0;           // latest released ts
}

constexpr int kT = 256;
inline unsigned nblk(int64_t n) { return (unsigned)((n + kT - 1) / kT); }
constexpr int kStatsT = 1024;   // k_seq_stats: 1024-lane blocks, one per CU

// Emission order of one output stream (cep_flush, ordered_output = 1).
// out[0] = ~min seq, out[1] = max seq (both biased by the sign bit so unsigned
// atomics order them; the complement lets one zero fill initialise both),
// out[2] = rows whose seq is below their predecessor's.
// The row count is read on the device (the output cursor), so this runs before
// the flush's one readback; the grid strides over min(count, cap) rows.
__global__ void k_seq_stats(const int64_t* __restrict__ seq, const unsigned long long* __restrict__ count,
                            int64_t cap, unsigned long long* __restrict__ out) {
  const int64_t n = (int64_t)min((unsigned long long)cap, *count);
  unsigned long long lo = ~0ull, hi = 0, desc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = seq[i];
    const unsigned long long b = (unsigned long long)v ^ 0x8000000000000000ull;
    lo = min(lo, b);
    hi = max(hi, b);
    desc += (i > 0 && seq[i - 1] > v) ? 1 : 0;
  }
  // wave reduction (64 lanes), block reduction in LDS, one atomic per block
  // and word (per-wave atomics on three words serialise: 312 us at 17.5 M rows)
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, (unsigned long long)__shfl_xor((long long)lo, o));
    hi = max(hi, (unsigned long long)__shfl_xor((long long)hi, o));
    desc += (unsigned long long)__shfl_xor((long long)desc, o);
  }
  __shared__ unsigned long long red[3][kStatsT / 64];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = lo;
    red[1][w] = hi;
    red[2][w] = desc;
  }
  __syncthreads();
  if (threadIdx.x == 0 && n > 0) {
    for (int i = 1; i < kStatsT / 64; ++i) {
      lo = min(lo, red[0][i]);
      hi = max(hi, red[1][i]);
      desc += red[2][i];
    }
    atomicMax(&out[0], ~lo);
    atomicMax(&out[1], hi);
    if (desc) atomicAdd(&out[2], desc);
  }
}

// key[i] = seq[i] - lo (fits `K`), idx[i] = i
template <typename K>
__global__ void k_seq_keys(const int64_t* __restrict__ seq, int64_t lo, int64_t n, K* __restrict__ key,
                           int32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    key[i] = (K)(seq[i] - lo);
    idx[i] = (int32_t)i;
  }
}

}  // namespace

void launch_seq_stats(const int64_t* seq, const unsigned long long* count, int64_t cap, unsigned long long* out3,
                      hipStream_t s) {
  if (cap <= 0) return;
  const unsigned blocks = (unsigned)std::min<int64_t>(256, (cap + kStatsT - 1) / kStatsT);
  hipLaunchKernelGGL(k_seq_stats, dim3(blocks), dim3(kStatsT), 0, s, seq, count, cap, out3);
}

size_t order_temp_bytes(int64_t n) {
  size_t b32 = 0, b64 = 0;
  rocprim::radix_sort_pairs(nullptr, b32, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const int32_t*)nullptr,
                            (int32_t*)nullptr, (size_t)n, 0, 32);
  rocprim::radix_sort_pairs(nullptr, b64, (const uint64_t*)nullptr, (uint64_t*)nullptr, (const int32_t*)nullptr,
                            (int32_t*)nullptr, (size_t)n, 0, 64);
  return std::max(b32, b64);
}

// Stable sort of rows [0, n) by seq: the permutation lands in idx_b.  Only the
// `bits` low bits of seq - lo are sorted (the flush window's seq range), so a
// window of 2^28 arrival numbers costs 4 onesweep passes, not 8.  keys_a /
// keys_b hold n 8-byte keys each.
int order_sort(void* temp, size_t temp_bytes, const int64_t* seq, int64_t n, int64_t lo, int bits, void* keys_a,
               void* keys_b, int32_t* idx_a, int32_t* idx_b, hipStream_t s) {
  if (n <= 0) return 0;
  size_t tb = temp_bytes;
  if (bits <= 32) {
    hipLaunchKernelGGL(k_seq_keys<uint32_t>, dim3(nblk(n)), dim3(kT), 0, s, seq, lo, n, (uint32_t*)keys_a, idx_a);
    return rocprim::radix_sort_pairs(temp, tb, (const uint32_t*)keys_a, (uint32_t*)keys_b, (const int32_t*)idx_a,
                                     idx_b, (size_t)n, 0, std::max(bits, 1), s) == hipSuccess ? 0 : -1;
  }
  hipLaunchKernelGGL(k_seq_keys<uint64_t>, dim3(nblk(n)), dim3(kT), 0, s, seq, lo, n, (uint64_t*)keys_a, idx_a);
  return rocprim::radix_sort_pairs(temp, tb, (const uint64_t*)keys_a, (uint64_t*)keys_b, (const int32_t*)idx_a,
                                   idx_b, (size_t)n, 0, bits, s) == hipSuccess ? 0 : -1;
}

size_t reorder_temp_bytes(int64_t n) {
  size_t bytes = 0;
  rocprim::radix_sort_pairs(nullptr, bytes, (const int64_t*)nullptr, (int64_t*)nullptr,
                                              (const int32_t*)nullptr, (int32_t*)nullptr, (size_t)n, 0, 64);
  return bytes;
}

int reorder_sort(void* temp, size_t temp_bytes, const int64_t* keys_in, int64_t* keys_out, int32_t* idx_in,
                 int32_t* idx_out, int64_t n, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_iota, dim3(nblk(n)), dim3(kT), 0, s, idx_in, n);
  size_t tb = temp_bytes;
  return rocprim::radix_sort_pairs(temp, tb, keys_in, keys_out, (const int32_t*)idx_in, idx_out, (size_t)n, 0,
                                   64, s) == hipSuccess ? 0 : -1;
}

void launch_upper_bound(const int64_t* sorted, int64_t n, int64_t wm, int64_t* out3, hipStream_t s) {
  hipLaunchKernelGGL(k_upper_bound, dim3(1), dim3(1), 0, s, sorted, n, wm, out3);
}

void launch_gather(const void* src, void* dst, const int32_t* perm, int64_t first, int64_t n, int width,
                   hipStream_t s) {
  if (n <= 0) return;
  switch (width) {
    case 1: hipLaunchKernelGGL(k_gather<uint8_t>, dim3(nblk(n)), dim3(kT), 0, s, (const uint8_t*)src, (uint8_t*)dst, perm, first, n); break;
    case 4: hipLaunchKernelGGL(k_gather<uint32_t>, dim3(nblk(n)), dim3(kT), 0, s, (const uint32_t*)src, (uint32_t*)dst, perm, first, n); break;
    default: hipLaunchKernelGGL(k_gather<uint64_t>, dim3(nblk(n)), dim3(kT), 0, s, (const uint64_t*)src, (uint64_t*)dst, perm, first, n); break;
  }
}

}  // namespace cep
