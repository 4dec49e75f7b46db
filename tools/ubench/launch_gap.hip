// tools/ubench/launch_gap.hip -- what the launch boundary between the build's
// two persistent passes costs, and what a grid barrier inside one cooperative
// launch costs instead.  Both variants run the same two phases: 1 workgroup of
// 1024 threads per CU with 150 KiB of LDS; phase 1 streams `bytes` of stores
// (like pass A's positions), phase 2 reads them back from a different
// workgroup's region (like pass B).  Prints microseconds per two-phase
// iteration for:
//   two     two plain launches per iteration
//   fused   one hipLaunchCooperativeKernel per iteration, flag barrier between
//           the phases (per-workgroup arrival flags tagged with a launch epoch;
//           workgroup 0 collects them and publishes the release; spins are
//           bounded and report an error instead of hanging)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int kBlock = 1024;
constexpr uint32_t kSpinLimit = 1u << 22;

__device__ __forceinline__ void phase1(uint4 *buf, uint64_t per_wg16, uint32_t wg, uint32_t *lds, uint32_t tag) {
  lds[threadIdx.x] = threadIdx.x;
  uint4 *p = buf + (uint64_t)wg * per_wg16;
  for (uint64_t i = threadIdx.x; i < per_wg16; i += kBlock) p[i] = make_uint4((uint32_t)i, wg, tag, 2);
}

// Reads another workgroup's region (on another XCD) and checks it: the
// returned count of stale words must be 0.
__device__ __forceinline__ uint32_t phase2(const uint4 *buf, uint64_t per_wg16, uint32_t wg, uint32_t G,
                                           uint32_t tag) {
  const uint32_t src = (wg + 17) % G;
  const uint4 *p = buf + (uint64_t)src * per_wg16;
  uint32_t bad = 0;
  for (uint64_t i = threadIdx.x; i < per_wg16; i += kBlock) {
    const uint4 v = p[i];
    bad += (v.x != (uint32_t)i) | (v.y != src) | (v.z != tag);
  }
  return bad;
}

__global__ __launch_bounds__(kBlock) void k1(uint4 *buf, uint64_t per_wg16, uint32_t tag) {
  extern __shared__ uint32_t lds[];
  phase1(buf, per_wg16, blockIdx.x, lds, tag);
}

__global__ __launch_bounds__(kBlock) void k2(const uint4 *buf, uint64_t per_wg16, uint32_t tag, uint32_t *bad) {
  const uint32_t b = phase2(buf, per_wg16, blockIdx.x, gridDim.x, tag);
  if (b) atomicAdd(bad, b);
}

// flags[0..G) arrival, flags[G] release; epoch unique per launch.
__device__ void grid_barrier(uint32_t *flags, uint32_t epoch, uint32_t *err) {
  __threadfence();  // every wave: its stores acknowledged and written back for agent scope
  __syncthreads();
  const uint32_t G = gridDim.x;
  if (threadIdx.x == 0) {
    __hip_atomic_store(&flags[blockIdx.x], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    uint32_t spins = 0;
    for (;;) {
      bool all = true;
      for (uint32_t i = threadIdx.x; i < G; i += 64)
        all &= __hip_atomic_load(&flags[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == epoch;
      if (__all(all)) break;
      if (++spins > kSpinLimit) { if (threadIdx.x == 0) atomicOr(err, 1u); break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (threadIdx.x == 0) __hip_atomic_store(&flags[G], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  } else if (threadIdx.x == 0) {
    uint32_t spins = 0;
    while (__hip_atomic_load(&flags[G], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
      if (++spins > kSpinLimit) { atomicOr(err, 2u); break; }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __threadfence();  // every wave: acquire (no stale lines from before the barrier)
}

__global__ __launch_bounds__(kBlock) void fused(uint4 *buf, uint64_t per_wg16, uint32_t *flags, uint32_t epoch,
                                                uint32_t *err, uint32_t *bad) {
  extern __shared__ uint32_t lds[];
  phase1(buf, per_wg16, blockIdx.x, lds, epoch);
  grid_barrier(flags, epoch, err);
  const uint32_t b = phase2(buf, per_wg16, blockIdx.x, gridDim.x, epoch);
  if (b) atomicAdd(bad, b);
}

int main() {
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int coop = 0;
  CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, 0));
  const uint32_t G = cus, lds = 150 * 1024;
  CK(hipFuncSetAttribute((const void *)k1, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void *)fused, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  int per_cu = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)fused, kBlock, lds));
  printf("CUs %d, cooperative launch %d, fused blocks per CU %d\n", cus, coop, per_cu);
  if (!coop || per_cu < 1) return 1;
  const uint64_t maxb = 256ull << 20;
  uint4 *buf;
  uint32_t *flags, *err, *sink;
  CK(hipMalloc(&buf, maxb));
  CK(hipMalloc(&flags, 4096));
  CK(hipMemset(flags, 0, 4096));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(err, 0, 4));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(sink, 0, 4096));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t epoch = 1;
  const int iters = 50;
  printf("%12s %10s %10s %10s\n", "bytes", "two_us", "fused_us", "saved_us");
  for (uint64_t bytes : {0ull, 1ull << 20, 32ull << 20, 256ull << 20}) {
    const uint64_t per_wg16 = bytes / 16 / G;
    float t[2];
    for (int v = 0; v < 2; ++v) {
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int it = 0; it < iters; ++it) {
          uint32_t ep = ++epoch;
          if (v == 0) {
            hipLaunchKernelGGL(k1, dim3(G), dim3(kBlock), lds, 0, buf, per_wg16, ep);
            hipLaunchKernelGGL(k2, dim3(G), dim3(kBlock), 0, 0, (const uint4 *)buf, per_wg16, ep, sink);
          } else {
            void *args[] = {&buf, (void *)&per_wg16, &flags, &ep, &err, &sink};
            CK(hipLaunchCooperativeKernel((const void *)fused, dim3(G), dim3(kBlock), args, lds, 0));
          }
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = fminf(best, ms * 1e3f / iters);
      }
      t[v] = best;
    }
    printf("%12llu %10.2f %10.2f %10.2f\n", (unsigned long long)bytes, t[0], t[1], t[0] - t[1]);
  }
  uint32_t herr = 0, hbad = 0;
  CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&hbad, sink, 4, hipMemcpyDeviceToHost));
  printf("barrier errors: %u, stale words read after the barrier / launch boundary: %u\n", herr, hbad);
  return (herr || hbad) ? 2 : 0;
}
