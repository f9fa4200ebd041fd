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

}  // namespace

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
