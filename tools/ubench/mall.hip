// tools/ubench/mall.hip -- does a buffer written by one kernel stay in the
// 256 MiB Infinity Cache (MALL) for the next kernel that reads it?  The
// two-pass bloom build writes k*n u32 positions in pass A and reads them back
// in pass B; this measures the read-back rate against a cold read, with and
// without a 160 MB key stream (plain or nontemporal loads) in between.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void wr(v4u *p, uint64_t n16, uint32_t salt) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
    p[i] = v4u{(uint32_t)i, salt, (uint32_t)(i >> 32), salt ^ (uint32_t)i};
}

template <bool NT>
__global__ __launch_bounds__(256) void rd(const v4u *p, uint64_t n16, uint32_t *sink) {
  v4u acc = {0, 0, 0, 0};
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
    v4u v = NT ? __builtin_nontemporal_load(p + i) : p[i];
    acc ^= v;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[blockIdx.x] = acc.x;
}

static const int G = 256 * 16;

int main() {
  const uint64_t MB = 1000000ull;
  const uint64_t maxS = 400 * MB, kS = 160 * MB, fS = 1024 * MB;
  v4u *P, *K, *F;
  uint32_t *sink;
  CK(hipMalloc(&P, maxS)); CK(hipMalloc(&K, kS)); CK(hipMalloc(&F, fS)); CK(hipMalloc(&sink, G * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto flush = [&]() { hipLaunchKernelGGL(wr, dim3(G), dim3(256), 0, 0, F, fS / 16, 7u); };
  auto timed_read = [&](const v4u *b, uint64_t bytes) -> float {
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(rd<false>, dim3(G), dim3(256), 0, 0, b, bytes / 16, sink);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return bytes / (ms * 1e-3) / 1e9;
  };
  const uint64_t sizes[] = {32 * MB, 64 * MB, 128 * MB, 192 * MB, 240 * MB, 320 * MB, 400 * MB};
  printf("%8s %10s %10s %12s %12s %10s  (read GB/s)\n", "MB", "cold", "afterwr", "wr+ntK160", "wr+K160", "reread");
  for (uint64_t S : sizes) {
    float r[5] = {0, 0, 0, 0, 0};
    for (int rep = 0; rep < 3; ++rep) {
      flush(); r[0] += timed_read(P, S);
      flush(); hipLaunchKernelGGL(wr, dim3(G), dim3(256), 0, 0, P, S / 16, rep); r[1] += timed_read(P, S);
      flush(); hipLaunchKernelGGL(wr, dim3(G), dim3(256), 0, 0, P, S / 16, rep);
      hipLaunchKernelGGL(rd<true>, dim3(G), dim3(256), 0, 0, K, kS / 16, sink); r[2] += timed_read(P, S);
      flush(); hipLaunchKernelGGL(wr, dim3(G), dim3(256), 0, 0, P, S / 16, rep);
      hipLaunchKernelGGL(rd<false>, dim3(G), dim3(256), 0, 0, K, kS / 16, sink); r[3] += timed_read(P, S);
      r[4] += timed_read(P, S);
    }
    printf("%8llu %10.0f %10.0f %12.0f %12.0f %10.0f\n", (unsigned long long)(S / MB), r[0] / 3, r[1] / 3, r[2] / 3,
           r[3] / 3, r[4] / 3);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
