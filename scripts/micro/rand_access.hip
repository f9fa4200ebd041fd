// Microbenchmark: random 4/8-byte loads, random 8-byte stores and random
// returning u32 atomics into tables of 4-128 MiB (decides whether a per-key
// hash-table design beats the bucket partition + LDS walk).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

template <int MODE>
__global__ void k_rand(uint32_t* tab, uint64_t mask, int64_t n, int per, uint32_t* sink) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (int i = 0; i < per; ++i) {
    const int64_t g = t * per + i;
    if (g >= n) break;
    const uint64_t idx = mix((uint64_t)g) & mask;
    if (MODE == 0) acc += tab[idx];
    else if (MODE == 1) acc += (uint32_t)((const uint64_t*)tab)[idx >> 1];
    else if (MODE == 2) ((uint64_t*)tab)[idx >> 1] = (uint64_t)g;
    else if (MODE == 3) acc += atomicAdd(&tab[idx], 1u);
    else if (MODE == 4) atomicAdd(&tab[idx], 1u);
    else if (MODE == 5) { const uint4 v = ((const uint4*)tab)[idx >> 2]; acc += v.x ^ v.w; }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const int64_t n = 1 << 24;  // ops per launch
  uint32_t* tab; uint32_t* sink;
  hipMalloc(&tab, (size_t)512 << 20);
  hipMalloc(&sink, 64);
  hipMemset(tab, 0, (size_t)512 << 20);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[] = {"load4", "load8", "store8", "atomic_ret", "atomic_noret", "load16"};
  for (int mb : {4, 16, 64, 128, 512}) {
    const uint64_t mask = ((uint64_t)mb << 20) / 4 - 1;
    for (int mode = 0; mode < 6; ++mode) {
      for (int per : {1, 4}) {
        const int threads = 256;
        const int64_t blocks = (n / per + threads - 1) / threads;
        float best = 1e9;
        for (int rep = 0; rep < 4; ++rep) {
          hipEventRecord(e0);
          switch (mode) {
            case 0: k_rand<0><<<blocks, threads>>>(tab, mask, n, per, sink); break;
            case 1: k_rand<1><<<blocks, threads>>>(tab, mask, n, per, sink); break;
            case 2: k_rand<2><<<blocks, threads>>>(tab, mask, n, per, sink); break;
            case 3: k_rand<3><<<blocks, threads>>>(tab, mask, n, per, sink); break;
            case 4: k_rand<4><<<blocks, threads>>>(tab, mask, n, per, sink); break;
            case 5: k_rand<5><<<blocks, threads>>>(tab, mask, n, per, sink); break;
          }
          hipEventRecord(e1); hipEventSynchronize(e1);
          float ms; hipEventElapsedTime(&ms, e0, e1);
          if (rep && ms < best) best = ms;
        }
        printf("table %4d MiB %-13s per=%d  %8.1f us  %7.1f G ops/s\n", mb, names[mode], per,
               best * 1e3, n / (best * 1e-3) / 1e9);
      }
    }
  }
  return 0;
}
