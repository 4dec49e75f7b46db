// tools/ubench/valu_rate.hip -- issue rate of the integer VALU ops the
// murmur3 + fastmod hot loop is made of (v_mul_lo_u32, v_mul_hi_u32,
// v_add_u32, v_lshl_or_b32, v_xor_b32, v_mul_u32_u24, v_cvt_f32_u32), at 4 or
// 8 waves per SIMD, 8 independent chains per lane.  Prints wave-instructions
// per cycle per CU (clock from s_memtime), so 4.0 = one per SIMD per cycle.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int OP>
__device__ __forceinline__ uint32_t op(uint32_t x, uint32_t y) {
  uint32_t r;
  if constexpr (OP == 0) asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  if constexpr (OP == 1) asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  if constexpr (OP == 2) asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  if constexpr (OP == 3) asm volatile("v_lshl_or_b32 %0, %1, 13, %2" : "=v"(r) : "v"(x), "v"(y));
  if constexpr (OP == 4) asm volatile("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  if constexpr (OP == 5) asm volatile("v_cvt_f32_u32 %0, %1" : "=v"(r) : "v"(x));
  if constexpr (OP == 6) asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  if constexpr (OP == 7) asm volatile("v_alignbyte_b32 %0, %1, %2, 3" : "=v"(r) : "v"(x), "v"(y));
  return r;
}

template <int OP>
__global__ __launch_bounds__(1024) void k(uint32_t *out, uint32_t iters, uint64_t *cyc) {
  uint32_t a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  const uint32_t y = blockIdx.x | 1;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = op<OP>(a[i], y);
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= a[i];
  if (s == 0x12345678u) out[blockIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
static int run(const char *name, uint32_t *out, uint64_t *cyc, int cus, int threads) {
  const uint32_t iters = 4096;
  hipLaunchKernelGGL(k<OP>, dim3(cus), dim3(threads), 0, 0, out, iters, cyc);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(k<OP>, dim3(cus), dim3(threads), 0, 0, out, iters, cyc);
  CK(hipDeviceSynchronize());
  uint64_t h[1024];
  CK(hipMemcpy(h, cyc, cus * 8, hipMemcpyDeviceToHost));
  double mean = 0;
  for (int i = 0; i < cus; ++i) mean += h[i];
  mean /= cus;
  const double winstr = (double)iters * 64 * (threads / 64);
  printf("%-16s threads/CU %4d: %.2f wave-instr/cycle/CU (%.2f cycles per wave-instr per SIMD)\n", name, threads,
         winstr / mean, mean * 4 / winstr);
  return 0;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t *out;
  uint64_t *cyc;
  CK(hipMalloc(&out, 4096 * 4));
  CK(hipMalloc(&cyc, 4096 * 8));
  for (int threads : {256, 1024}) {
    run<0>("v_add_u32", out, cyc, cus, threads);
    run<1>("v_mul_lo_u32", out, cyc, cus, threads);
    run<2>("v_mul_hi_u32", out, cyc, cus, threads);
    run<3>("v_lshl_or_b32", out, cyc, cus, threads);
    run<4>("v_mul_u32_u24", out, cyc, cus, threads);
    run<5>("v_cvt_f32_u32", out, cyc, cus, threads);
    run<6>("v_xor_b32", out, cyc, cus, threads);
    run<7>("v_alignbyte_b32", out, cyc, cus, threads);
  }
  return 0;
}
