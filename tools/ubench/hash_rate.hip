// tools/ubench/hash_rate.hip -- VALU cost of hashing 16-byte keys in
// registers (no memory traffic): the production hash16 against variants,
// KPT independent keys per thread, 1024 threads per CU.  Prints cycles per
// key per CU (s_memtime) and per-instruction issue rates of v_mad_u64_u32.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../adlsm-tree_amd/csrc/murmur3_device.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

using namespace adl_dev;

template <int V, int KPT>
__global__ __launch_bounds__(1024) void k(uint32_t *out, uint32_t iters, uint64_t *cyc) {
  uint4 raw[KPT];
#pragma unroll
  for (int i = 0; i < KPT; ++i) raw[i] = make_uint4(threadIdx.x * 77 + i, blockIdx.x, i * 3, 0x80808080u ^ i);
  uint32_t acc = 0;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      uint32_t h1, h2;
      if constexpr (V == 0) hash16(raw[i], h1, h2);
      
      raw[i].x ^= h1;
      raw[i].y += h2;
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < KPT; ++i) acc ^= raw[i].x ^ raw[i].y;
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V, int KPT>
static int run(const char *name, uint32_t *out, uint64_t *cyc, int cus) {
  const uint32_t iters = 512;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL((k<V, KPT>), dim3(cus), dim3(1024), 0, 0, out, iters, cyc);
    CK(hipDeviceSynchronize());
  }
  uint64_t h[1024];
  CK(hipMemcpy(h, cyc, cus * 8, hipMemcpyDeviceToHost));
  double mean = 0;
  for (int i = 0; i < cus; ++i) mean += h[i];
  mean /= cus;
  const double keys = (double)iters * KPT * 1024;
  printf("%-12s KPT %d: %.3f cycles per key per CU -> %.1f Gkeys/s chip at 2.0 GHz\n", name, KPT, mean / keys,
         keys / mean * 2.0 * cus);
  return 0;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t *out;
  uint64_t *cyc;
  CK(hipMalloc(&out, 4096 * 4));
  CK(hipMalloc(&cyc, 4096 * 8));
  run<0, 2>("hash16", out, cyc, cus);
  run<0, 6>("hash16", out, cyc, cus);
  
  
  return 0;
}
