// tools/ubench/tile_lists.hip -- feasibility of a tile-list layout for the
// build's position workspace (10 M keys, k = 6, 763 tiles of 2^20 bits):
//   append: 256 persistent workgroups, each 7 chunks of 33,504 positions
//           sorted by tile in LDS; per chunk one returning device-scope
//           atomicAdd per tile reserves the chunk's piece of that tile's list,
//           then the chunk is written piece-wise (dword per lane, lanes in
//           sorted order).  Measures the reservation + scattered-store cost.
//   stream: one workgroup per tile reads the tile's whole list contiguously
//           (dwordx4 per lane) and ds_or_b32s every position into a 128 KiB
//           LDS tile, then writes the tile out.  Measures pass B as a stream.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr uint32_t T = 763, CH = 1791, PC = 33504;  // tiles, chunks, positions per chunk
constexpr uint32_t CAP = 90000;                      // per-tile list capacity (mean 78.6 K)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16; return x;
}

template <bool SCATTER, bool ATOM = true>
__global__ __launch_bounds__(1024) void append(uint32_t *lists, uint32_t *ctr, uint32_t salt) {
  __shared__ uint32_t hist[T + 1];
  __shared__ uint32_t tb[T];
  extern __shared__ uint32_t lpos[];
  for (uint32_t c = blockIdx.x; c < CH; c += gridDim.x) {
    for (uint32_t t = threadIdx.x; t <= T; t += 1024) hist[t] = 0;
    __syncthreads();
    // synthetic sorted chunk: positions with random tiles, counted then laid out by tile
    for (uint32_t i = threadIdx.x; i < PC; i += 1024) atomicAdd(&hist[mix(c * PC + i + salt) % T], 1u);
    __syncthreads();
    {  // block exclusive scan of hist[0..T], one entry per thread
      __shared__ uint32_t ws[17];
      const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
      const uint32_t v = threadIdx.x <= T ? hist[threadIdx.x] : 0u;
      uint32_t x = v;
      for (int o = 1; o < 64; o <<= 1) { const uint32_t y = __shfl_up(x, o, 64); if (lane >= (uint32_t)o) x += y; }
      if (lane == 63) ws[w] = x;
      __syncthreads();
      if (threadIdx.x == 0) { uint32_t r = 0; for (int i = 0; i < 16; ++i) { const uint32_t q = ws[i]; ws[i] = r; r += q; } }
      __syncthreads();
      if (threadIdx.x <= T) hist[threadIdx.x] = ws[w] + x - v;
      __syncthreads();
    }
    for (uint32_t t = threadIdx.x; t < T; t += 1024) {
      const uint32_t cnt = hist[t + 1] - hist[t];
      const uint32_t off = ATOM ? atomicAdd(&ctr[t], cnt) : (c / gridDim.x) * 110u;
      tb[t] = t * CAP + min(off, CAP - cnt) - hist[t];
    }
    for (uint32_t i = threadIdx.x; i < PC; i += 1024) {
      const uint32_t v = mix(c * PC + i + salt);
      lpos[atomicAdd(&hist[v % T], 1u)] = ((v % T) << 20) | (v & 0xfffff);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < PC; i += 1024) {
      const uint32_t v = lpos[i];
      if (SCATTER) lists[tb[v >> 20] + i] = v & 0xfffff;
      else lists[(uint64_t)c * PC + i] = v & 0xfffff;
    }
    __syncthreads();
  }
}

template <int U>
__global__ __launch_bounds__(1024) void stream(const uint32_t *lists, const uint32_t *ctr, uint4 *bitmap) {
  extern __shared__ uint32_t tile[];
  for (uint32_t t = blockIdx.x; t < T; t += gridDim.x) {
    for (uint32_t i = threadIdx.x; i < 32768; i += 1024) tile[i] = 0;
    __syncthreads();
    const uint32_t n = min(ctr[t], CAP);
    const uint4 *l4 = reinterpret_cast<const uint4 *>(lists + (uint64_t)t * CAP);
    const uint32_t n4 = n / 4;
    for (uint32_t i0 = 0; i0 < n4; i0 += 1024 * U) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = min(i0 + u * 1024 + threadIdx.x, n4 - 1);
        v[u] = l4[i];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        asm volatile("" : "+v"(v[u].x), "+v"(v[u].y), "+v"(v[u].z), "+v"(v[u].w));
        if (i0 + u * 1024 + threadIdx.x < n4) {
          atomicOr(&tile[(v[u].x >> 5) & 32767], 1u << (v[u].x & 31));
          atomicOr(&tile[(v[u].y >> 5) & 32767], 1u << (v[u].y & 31));
          atomicOr(&tile[(v[u].z >> 5) & 32767], 1u << (v[u].z & 31));
          atomicOr(&tile[(v[u].w >> 5) & 32767], 1u << (v[u].w & 31));
        }
      }
    }
    __syncthreads();
    const uint4 *t4 = reinterpret_cast<const uint4 *>(tile);
    for (uint32_t i = threadIdx.x; i < 8192; i += 1024) bitmap[(uint64_t)t * 8192 + i] = t4[i];
    __syncthreads();
  }
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t *lists, *ctr;
  uint4 *bitmap;
  CK(hipMalloc(&lists, (uint64_t)T * CAP * 4));
  CK(hipMalloc(&ctr, T * 4));
  CK(hipMalloc(&bitmap, (uint64_t)T * 131072));
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
  CK(hipFuncSetAttribute((const void *)append<true>, hipFuncAttributeMaxDynamicSharedMemorySize, PC * 4));
  CK(hipFuncSetAttribute((const void *)append<false>, hipFuncAttributeMaxDynamicSharedMemorySize, PC * 4));
  CK(hipFuncSetAttribute((const void *)append<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, PC * 4));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemset(ctr, 0, T * 4));
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((append<true, false>), dim3(cus), dim3(1024), PC * 4, 0, lists, ctr, (uint32_t)rep);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float a;
    CK(hipEventElapsedTime(&a, e0, e1));
    printf("append(scatter, no atomics) %.1f us\n", a * 1e3);
  }
  CK(hipFuncSetAttribute((const void *)stream<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void *)stream<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void *)stream<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  for (int rep = 0; rep < 9; ++rep) {
    CK(hipMemset(ctr, 0, T * 4));
    CK(hipEventRecord(e0, 0));
    if (rep % 3 == 2) hipLaunchKernelGGL(append<false>, dim3(cus), dim3(1024), PC * 4, 0, lists, ctr, (uint32_t)rep);
    else hipLaunchKernelGGL(append<true>, dim3(cus), dim3(1024), PC * 4, 0, lists, ctr, (uint32_t)rep);
    CK(hipEventRecord(e1, 0));
    if (rep % 3 == 0) hipLaunchKernelGGL(stream<1>, dim3(cus), dim3(1024), 131072, 0, lists, ctr, bitmap);
    else if (rep % 3 == 1) hipLaunchKernelGGL(stream<4>, dim3(cus), dim3(1024), 131072, 0, lists, ctr, bitmap);
    else hipLaunchKernelGGL(stream<8>, dim3(cus), dim3(1024), 131072, 0, lists, ctr, bitmap);
    CK(hipEventRecord(e2, 0));
    CK(hipEventSynchronize(e2));
    float a, b;
    CK(hipEventElapsedTime(&a, e0, e1));
    CK(hipEventElapsedTime(&b, e1, e2));
    uint32_t c0;
    CK(hipMemcpy(&c0, ctr, 4, hipMemcpyDeviceToHost));
    printf("append(%s) %.1f us  stream<U=%d> %.1f us  (tile 0 list %u positions)\n", rep % 3 == 2 ? "contig" : "scatter",
           a * 1e3, rep % 3 == 0 ? 1 : rep % 3 == 1 ? 4 : 8, b * 1e3, c0);
  }
  return 0;
}
