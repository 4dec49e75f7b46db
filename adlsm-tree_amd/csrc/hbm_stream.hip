// adlsm-tree_amd/csrc/hbm_stream.hip -- measurement helper for bench.py (not
// part of the filter path): a streaming HBM read kernel, so each bench line
// can report the read bandwidth this box actually reaches next to the
// vendor peak (SURVEY.md §8d "also report a measured stream-read GB/s").
//
// Persistent grid (8 workgroups of 256 threads per CU), 16 B per lane,
// 4 independent nontemporal loads in flight per lane per iteration.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void hbm_read_kernel(const v4u *__restrict__ p, uint64_t n16,
                                                       uint32_t *__restrict__ sink) {
  v4u acc = {0, 0, 0, 0};
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const v4u a = __builtin_nontemporal_load(p + i), b = __builtin_nontemporal_load(p + i + stride);
    const v4u c = __builtin_nontemporal_load(p + i + 2 * stride), d = __builtin_nontemporal_load(p + i + 3 * stride);
    acc ^= a ^ b ^ c ^ d;
  }
  for (; i < n16; i += stride) acc ^= __builtin_nontemporal_load(p + i);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[blockIdx.x] = acc.x;  // keeps the loads
}

extern "C" int adl_hbm_stream_read(const void *d_buf, uint64_t bytes, uint32_t *d_sink, uint32_t sink_words,
                                   void *stream) {
  if (!d_buf || !d_sink || bytes % 16 || reinterpret_cast<uintptr_t>(d_buf) % 16) return -1;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -3;
  uint32_t grid = (uint32_t)cus * 8u;
  if (grid > sink_words) grid = sink_words;
  if (grid == 0) return -1;
  hipLaunchKernelGGL(hbm_read_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     static_cast<const v4u *>(d_buf), bytes / 16, d_sink);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Random single-byte reads over a working set of W bytes: the access pattern
// of the bloom probe (k dependent-free byte loads per query into filters far
// larger than the Infinity Cache).  Gives bench.py the random-read rate this
// box reaches, the real ceiling of the probe (its 21 B/query are not what
// bounds it).  R = 4 independent loads in flight per lane per iteration.
__device__ __forceinline__ uint32_t rr_mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

__global__ __launch_bounds__(256) void hbm_random_read_kernel(const uint8_t *__restrict__ p, uint64_t W,
                                                              uint32_t iters, uint32_t *__restrict__ sink) {
  uint32_t x = rr_mix(blockIdx.x * 256 + threadIdx.x + 1), acc = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    uint32_t v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      x = x * 1664525u + 1013904223u;
      v[r] = p[((uint64_t)rr_mix(x) * W) >> 32];
    }
    acc += v[0] + v[1] + v[2] + v[3];
  }
  if (acc == 0x12345u) sink[blockIdx.x] = acc;  // keeps the loads
}

// Returns the number of byte reads the launch performs (0 on error).
extern "C" uint64_t adl_hbm_random_read(const void *d_buf, uint64_t bytes, uint32_t iters, uint32_t *d_sink,
                                        uint32_t sink_words, void *stream) {
  if (!d_buf || !d_sink || bytes == 0 || bytes > (1ull << 32) || iters == 0) return 0;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  uint32_t grid = (uint32_t)cus * 8u;
  if (grid > sink_words) grid = sink_words;
  if (grid == 0) return 0;
  hipLaunchKernelGGL(hbm_random_read_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     static_cast<const uint8_t *>(d_buf), bytes, iters, d_sink);
  if (hipGetLastError() != hipSuccess) return 0;
  return (uint64_t)grid * 256u * iters * 4u;
}
