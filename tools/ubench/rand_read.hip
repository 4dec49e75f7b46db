// tools/ubench/rand_read.hip -- random single-byte reads per second over a
// working set of W bytes (L2 / Infinity Cache / HBM resident), the access
// pattern of a bloom probe.  Each lane does R independent reads per round
// (R in flight), persistent grid of 8 x 256-thread workgroups per CU.
// Optionally the reads of a wave are confined to a window of the buffer that
// slides with the wave's progress (the filter-sorted probe order).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16; return x;
}

template <int R>
__global__ __launch_bounds__(256) void rr(const uint8_t *__restrict__ p, uint64_t W, uint32_t iters,
                                          uint32_t *__restrict__ sink) {
  uint32_t x = mix(blockIdx.x * 256 + threadIdx.x + 1), acc = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      x = x * 1664525u + 1013904223u;
      const uint64_t a = ((uint64_t)mix(x) * W) >> 32;
      v[r] = p[a];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) acc += v[r];
  }
  if (acc == 0x12345u) sink[blockIdx.x] = acc;
}

int main() {
  const uint64_t MB = 1ull << 20;
  const uint64_t maxW = 2600 * MB;
  uint8_t *p;
  uint32_t *sink;
  CK(hipMalloc(&p, maxW));
  CK(hipMemset(p, 1, maxW));
  CK(hipMalloc(&sink, 1 << 20));
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const uint64_t sizes[] = {2 * MB, 8 * MB, 16 * MB, 32 * MB, 64 * MB, 128 * MB, 256 * MB, 512 * MB, 2560 * MB};
  const uint32_t grid = cus * 8, iters = 64;
  printf("%10s %14s %14s  (G random byte reads / s)\n", "W MiB", "R=2", "R=4");
  for (uint64_t W : sizes) {
    float g[2];
    for (int v = 0; v < 2; ++v) {
      float best = 0;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0, 0);
        if (v == 0) hipLaunchKernelGGL(rr<2>, dim3(grid), dim3(256), 0, 0, p, W, iters * 2, sink);
        else hipLaunchKernelGGL(rr<4>, dim3(grid), dim3(256), 0, 0, p, W, iters, sink);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double reads = (double)grid * 256 * iters * 4;
        best = fmaxf(best, (float)(reads / (ms * 1e-3) / 1e9));
      }
      g[v] = best;
    }
    printf("%10llu %14.1f %14.1f\n", (unsigned long long)(W / MB), g[0], g[1]);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
