// tools/ubench/seg_gather.hip -- pass B's read pattern in isolation: each
// workgroup gathers one short segment (LEN u32 positions) from each of W
// chunk regions for its tile, tiles t..t+G-1 in flight, the segments of
// consecutive tiles adjacent in every region.  Variants:
//   dword   one segment per wave-load (lane i = position i; LEN of 64 lanes live)
//   dwordx4 four segments per wave-load (16 lanes each, 4 positions per lane)
// Prints useful GB/s (segment bytes only) for several segment lengths.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int kBlock = 1024, kWaves = kBlock / 64, kInFlight = 8;

// X4: 0 dword loads, 1 dwordx4 loads, 2 dword loads + ds_or_b32 of each
// position into a 128 KiB LDS tile (pass B's full inner loop)
template <int X4>
__global__ __launch_bounds__(kBlock) void gather(const uint32_t *__restrict__ pos, uint32_t W, uint32_t cap,
                                                 uint32_t len, uint32_t tiles, uint32_t remap,
                                                 uint32_t *__restrict__ sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  extern __shared__ uint32_t tile[];
  uint32_t acc = 0;
  const uint32_t G = gridDim.x;
  const uint32_t t0 = remap ? (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8 : blockIdx.x;  // XCD-consecutive tiles
  for (uint32_t t = t0; t < tiles; t += G) {
    if (X4 != 1) {
      // wave w: regions c = w, w+16, ...; kInFlight loads in flight
      for (uint32_t c0 = wave; c0 < W; c0 += kWaves * kInFlight) {
        uint32_t v[kInFlight];
#pragma unroll
        for (int u = 0; u < kInFlight; ++u) {
          const uint32_t c = c0 + u * kWaves;
          const uint32_t cc = c < W ? c : W - 1;
          const uint32_t *sp = pos + (uint64_t)cc * cap + (uint64_t)t * len;
          if (X4 == 3) {
            v[u] = sp[lane];  // every lane loads (the real pass B's first stage)
          } else if (X4 == 4) {
            // bounds-checked buffer load: lanes past len return 0 with no memory access
            const __amdgpu_buffer_rsrc_t r =
                __builtin_amdgcn_make_buffer_rsrc((void *)sp, 0, c < W ? len * 4 : 0, 0x00020000);
            v[u] = __builtin_amdgcn_raw_buffer_load_b32(r, lane * 4, 0, 0);
          } else {
            v[u] = (c < W && (uint32_t)lane < len) ? sp[lane] : 0u;
          }
        }
#pragma unroll
        for (int u = 0; u < kInFlight; ++u) {
          if (X4 >= 2) {
            if (c0 + u * kWaves < W && (uint32_t)lane < len) atomicOr(&tile[(v[u] >> 5) & 32767], 1u << (v[u] & 31));
          } else {
            acc += v[u];
          }
        }
      }
    } else {
      // lane group g (16 lanes) of wave w: regions c = 4*(w + 16*q) + g
      const int g = lane >> 4, l = lane & 15;
      for (uint32_t q0 = 0; 4 * (wave + kWaves * q0) < W; q0 += kInFlight) {
        uint4 v[kInFlight];
#pragma unroll
        for (int u = 0; u < kInFlight; ++u) {
          const uint32_t c = 4 * (wave + kWaves * (q0 + u)) + g;
          const uint32_t *sp = pos + (uint64_t)c * cap + (uint64_t)t * len;
          v[u] = (c < W && (uint32_t)(4 * l) < len) ? *reinterpret_cast<const uint4 *>(sp + 4 * l)
                                                    : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < kInFlight; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
      }
    }
  }
  if (X4 >= 2) {
    __syncthreads();
    acc = tile[threadIdx.x * 31];
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;
}

int main() {
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t W = 1792, tiles = 763;
  const uint32_t maxlen = 64;
  const uint32_t cap = tiles * maxlen;  // words per region
  uint32_t *pos, *sink;
  CK(hipMalloc(&pos, (uint64_t)W * cap * 4 + 4096));
  {  // random positions inside a 2^20-bit tile
    const uint64_t nw = (uint64_t)W * cap + 1024;
    uint32_t *h = (uint32_t *)malloc(nw * 4);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < nw; ++i) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      h[i] = (uint32_t)x & 0xfffffu;
    }
    CK(hipMemcpy(pos, h, nw * 4, hipMemcpyHostToDevice));
    free(h);
  }
  CK(hipFuncSetAttribute((const void *)gather<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void *)gather<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void *)gather<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipMalloc(&sink, 1 << 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("%5s %6s %12s %12s %12s %12s %12s  (useful GB/s; %u regions x %u tiles)\n", "len", "remap", "dword",
         "dwordx4", "dword+ds_or", "all64+ds_or", "buf+ds_or", W, tiles);
  for (uint32_t remap : {1u})
  for (uint32_t len : {32u, 44u, 53u, 64u}) {
    float gbs[5];
    for (int v = 0; v < 5; ++v) {
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(e0, 0));
        if (v == 0) hipLaunchKernelGGL(gather<0>, dim3(cus), dim3(kBlock), 0, 0, pos, W, cap, len, tiles, remap, sink);
        else if (v == 1) hipLaunchKernelGGL(gather<1>, dim3(cus), dim3(kBlock), 0, 0, pos, W, cap, len, tiles, remap, sink);
        else if (v == 2) hipLaunchKernelGGL(gather<2>, dim3(cus), dim3(kBlock), 131072, 0, pos, W, cap, len, tiles, remap, sink);
        else if (v == 3) hipLaunchKernelGGL(gather<3>, dim3(cus), dim3(kBlock), 131072, 0, pos, W, cap, len, tiles, remap, sink);
        else hipLaunchKernelGGL(gather<4>, dim3(cus), dim3(kBlock), 131072, 0, pos, W, cap, len, tiles, remap, sink);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = fminf(best, ms);
      }
      gbs[v] = (float)((double)W * tiles * len * 4 / (best * 1e-3) / 1e9);
    }
    printf("%5u %6u %12.0f %12.0f %12.0f %12.0f %12.0f\n", len, remap, gbs[0], gbs[1], gbs[2], gbs[3], gbs[4]);
  }
  return 0;
}
