// tools/ubench/lds_ops.hip -- cycles per wave-instruction of the LDS ops the
// bloom build leans on (ds_or_b32, ds_add_u32, ds_add_rtn_u32, ds_write_b32)
// at random addresses in a 128 KiB LDS array, 1024-thread workgroups, one per
// CU, every CU busy.  Prints ns per wave-instruction per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16; return x;
}

template <int OP>
__global__ __launch_bounds__(1024) void k(uint32_t *out, int iters, uint32_t words_mask, int spread) {
  extern __shared__ uint32_t lds[];
  for (uint32_t i = threadIdx.x; i <= words_mask; i += 1024) lds[i] = 0;
  __syncthreads();
  uint32_t x = mix(threadIdx.x * 7919u + blockIdx.x * 104729u);
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      x = x * 1664525u + 1013904223u;
      uint32_t addr;
      if (spread) addr = (x >> 8) & words_mask;          // random word
      else addr = (threadIdx.x * 16 + u) & words_mask;  // conflict-free
      if (OP == 0) atomicOr(&lds[addr], 1u << (x & 31));
      if (OP == 1) atomicAdd(&lds[addr], 1u);
      if (OP == 2) acc += atomicAdd(&lds[addr], 1u);
      if (OP == 3) lds[addr] = x;
      if (OP == 4) acc += lds[addr];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = lds[0] + acc;
  if (acc == 0x12345) out[blockIdx.x + 1] = acc;
}

template <int OP>
float run(const char *name, int spread, uint32_t words = 32768) {
  uint32_t *out;
  (void)hipMalloc(&out, 1 << 20);
  const int iters = 256, cus = 256;
  hipFuncSetAttribute((const void *)k<OP>, hipFuncAttributeMaxDynamicSharedMemorySize, words * 4);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL(k<OP>, dim3(cus), dim3(1024), words * 4, 0, out, iters, words - 1, spread);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL(k<OP>, dim3(cus), dim3(1024), words * 4, 0, out, iters, words - 1, spread);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  ms /= 5;
  const double instr_per_cu = 16.0 * 16 * iters;  // 16 waves x 16 unroll x iters
  const double ns = ms * 1e6 / instr_per_cu;
  printf("%-16s words=%6u spread=%d  %.3f ms  %.2f ns/wave-instr/CU  (%.1f cycles @2.4GHz)  %.2f Gops/s chip\n", name,
         words, spread, ms, ns, ns * 2.4, 64.0 * instr_per_cu * cus / (ms * 1e-3) / 1e9);
  (void)hipFree(out);
  return ms;
}

int main() {
  // random over 1024 words: the pass-A tile histogram (T+1 = 764 counters at 10 M keys)
  run<1>("ds_add_u32", 1, 1024);
  run<2>("ds_add_rtn_u32", 1, 1024);
  run<4>("ds_read_b32", 1, 1024);
  for (int s = 1; s >= 0; --s) {
    run<0>("ds_or_b32", s);
    run<1>("ds_add_u32", s);
    run<2>("ds_add_rtn_u32", s);
    run<3>("ds_write_b32", s);
    run<4>("ds_read_b32", s);
  }
  return 0;
}
