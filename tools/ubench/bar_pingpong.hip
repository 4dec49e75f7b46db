// tools/ubench/bar_pingpong.hip -- host <-> resident-kernel round trip, by
// where the request lives.  One single-wave kernel polls a bell word; the host
// writes a 512-byte request and then the bell, the wave reads the request
// (one 8-byte load per lane) and writes the answer into coherent host memory,
// where the host spins.  The probe server (csrc/probe_server.hip) keeps its
// bells and slots in host memory (mode host): every poll and the request read
// cross PCIe.  Modes fine / uncached put bell and request in device memory
// that the host writes through the BAR, so the wave polls local memory and
// only the host's posted writes and the answer cross the bus.
//
// usage: bar_pingpong host|fine|uncached|nopayload|wide|pipe2|pipe4 [calls]
//   pipe2 / pipe4: host memory, no request read, the wave keeps 2 / 4 bell
//         polls in flight (a new one issued as the oldest returns)
//   nopayload: host memory, the wave answers without reading the request
//   wide: host memory, the wave polls 64 bell lines of 64 B (4 KiB) per poll,
//         as if each request sat inline in its bell line (one round trip)
// prints one JSON line: round-trip percentiles in microseconds
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                                \
    }                                                                          \
  } while (0)

constexpr uint32_t kReqWords = 128;  // 512 B

__global__ void pingpong(const uint32_t *bell, const uint64_t *req, uint32_t *ans, uint32_t n,
                         uint64_t timeout_ticks, int wide) {
  const int lane = threadIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t i = 1; i <= n; ++i) {
    uint32_t b = 0;
    for (;;) {
      if (wide) {
        // 64 lines of 64 B: lane l loads 16 B of each of 4 lines per instruction
        uint32_t w[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          w[u] = __hip_atomic_load(bell + 256 * u + (lane / 4) * 16 + (lane % 4) * 4, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
        b = __shfl(w[0], 0);
      } else {
        if (lane == 0) b = __hip_atomic_load(bell, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        b = __shfl(b, 0);
      }
      if (b == i) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) return;  // the host is gone: end
      __builtin_amdgcn_s_sleep(1);
    }
    const uint64_t v = req ? __hip_atomic_load(req + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull;
    // every lane's word takes part in the answer, so the loads are waited for
    uint32_t x = (uint32_t)v ^ (uint32_t)(v >> 32);
    for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o);
    if (lane == 0) __hip_atomic_store(ans, i | ((x & 1u) << 31), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// bell polls kept D deep: each iteration waits for the oldest poll only
template <int D>
__global__ void pingpong_pipe(const uint32_t *bell, uint32_t *ans, uint32_t n, uint64_t timeout_ticks) {
  const int lane = threadIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t b[D];
#pragma unroll
  for (int d = 0; d < D; ++d) b[d] = __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  uint32_t i = 1;
  while (i <= n) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const uint32_t v = __shfl(b[d], 0);
      b[d] = __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (v == i) {
        if (lane == 0) __hip_atomic_store(ans, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        ++i;
      }
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) return;
  }
}

int main(int argc, char **argv) {
  const char *mode = argc > 1 ? argv[1] : "host";
  const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 20000;
  void *area = nullptr;  // bell (word 0) + request (from byte 256)
  const int pipe = !strcmp(mode, "pipe2") ? 2 : !strcmp(mode, "pipe4") ? 4 : 0;
  const bool nopayload = !strcmp(mode, "nopayload") || pipe, wide = !strcmp(mode, "wide");
  if (!strcmp(mode, "host") || nopayload || wide) {
    CHECK(hipHostMalloc(&area, 8192, hipHostMallocCoherent | hipHostMallocMapped));
  } else if (!strcmp(mode, "fine")) {
    CHECK(hipExtMallocWithFlags(&area, 4096, hipDeviceMallocFinegrained));
  } else if (!strcmp(mode, "uncached")) {
    CHECK(hipExtMallocWithFlags(&area, 4096, hipDeviceMallocUncached));
  } else {
    fprintf(stderr, "mode: host|fine|uncached|nopayload|wide\n");
    return 2;
  }
  hipPointerAttribute_t at{};
  CHECK(hipPointerGetAttributes(&at, area));
  volatile uint32_t *hbell = reinterpret_cast<volatile uint32_t *>(at.hostPointer ? at.hostPointer : area);
  if (!at.hostPointer && strcmp(mode, "host") && !nopayload && !wide) {
    printf("{\"mode\": \"%s\", \"host_mapped\": false}\n", mode);
    return 0;
  }
  // the host writes through its mapping, and the device sees the same bytes
  hbell[1] = 0x5a5a5a5au;
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  uint32_t back = 0;
  CHECK(hipMemcpy(&back, (uint32_t *)area + 1, 4, hipMemcpyDefault));
  if (back != 0x5a5a5a5au) {
    printf("{\"mode\": \"%s\", \"host_write_visible\": false}\n", mode);
    return 0;
  }
  hbell[0] = 0;
  uint32_t *ans = nullptr;
  CHECK(hipHostMalloc((void **)&ans, 256, hipHostMallocCoherent | hipHostMallocMapped));
  *(volatile uint32_t *)ans = 0;
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  volatile uint64_t *hreq = reinterpret_cast<volatile uint64_t *>((uint8_t *)hbell + 256);
  const uint32_t *dbell = reinterpret_cast<const uint32_t *>(area);
  const uint64_t *dreq = reinterpret_cast<const uint64_t *>((const uint8_t *)area + 256);
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  if (pipe == 2)
    hipLaunchKernelGGL(pingpong_pipe<2>, dim3(1), dim3(64), 0, st, dbell, ans, n, (uint64_t)100000000 * 5);
  else if (pipe == 4)
    hipLaunchKernelGGL(pingpong_pipe<4>, dim3(1), dim3(64), 0, st, dbell, ans, n, (uint64_t)100000000 * 5);
  else
    hipLaunchKernelGGL(pingpong, dim3(1), dim3(64), 0, st, dbell, wide || nopayload ? nullptr : dreq, ans, n,
                       (uint64_t)100000000 * 5, (int)wide);  // 5 s
  CHECK(hipGetLastError());
  std::vector<double> us;
  us.reserve(n);
  bool lost = false;
  for (uint32_t i = 1; i <= n && !lost; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t w = 0; w < kReqWords / 2; ++w) hreq[w] = ((uint64_t)i << 32) | w;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    hbell[0] = i;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    for (;;) {
      const uint32_t a = *(volatile uint32_t *)ans;
      if ((a & 0x7fffffffu) == i) break;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        lost = true;
        break;
      }
    }
    us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  CHECK(hipStreamSynchronize(st));
  if (lost) {
    printf("{\"mode\": \"%s\", \"lost_at\": %zu}\n", mode, us.size());
    return 1;
  }
  std::vector<double> s = us;
  std::sort(s.begin(), s.end());
  auto pct = [&](double p) { return s[std::min(s.size() - 1, (size_t)(p * (double)s.size()))]; };
  printf("{\"mode\": \"%s\", \"calls\": %u, \"p50_us\": %.2f, \"p90_us\": %.2f, \"p99_us\": %.2f, \"max_us\": %.2f}\n",
         mode, n, pct(0.5), pct(0.9), pct(0.99), s.back());
  return 0;
}
