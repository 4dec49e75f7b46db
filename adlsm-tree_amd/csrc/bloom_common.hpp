// adlsm-tree_amd/csrc/bloom_common.hpp -- shared host/device plumbing of
// libadlbloom.so: status handling, key-set views, block scans.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/adl_bloom.h"
#include "murmur3_device.hpp"

// ADL_BLOOM_DEBUG=1: the HIP error behind a failed call goes to stderr
#define ADL_HIP_TRY(expr)                                                                    \
  do {                                                                                       \
    hipError_t adl_e_ = (expr);                                                              \
    if (adl_e_ != hipSuccess) {                                                              \
      if (getenv("ADL_BLOOM_DEBUG"))                                                         \
        fprintf(stderr, "adl_bloom: %s:%d: %s\n", __FILE__, __LINE__, hipGetErrorString(adl_e_)); \
      return adl_e_ == hipErrorOutOfMemory ? ADL_ERR_OUT_OF_MEMORY : ADL_ERR_DEVICE;         \
    }                                                                                        \
  } while (0)

namespace adl_dev {

constexpr int kWave = 64;

// ---------------------------------------------------------------- key views
// Fixed 16-byte keys, 16-byte aligned: one global_load_dwordx4 per key, so a
// wave reads 1 KiB contiguous.
struct Keys16 {
  const uint4 *keys;
  __device__ __forceinline__ void hash(uint64_t i, uint32_t &h1, uint32_t &h2) const {
    hash16(keys[i], h1, h2);
  }
  // key i == key i-1 (i > 0)
  __device__ __forceinline__ bool same_as_prev(uint64_t i) const {
    const uint4 a = keys[i], b = keys[i - 1];
    return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w;
  }
};

// Fixed stride (any stride, any alignment).
struct KeysStride {
  const uint8_t *keys;
  uint32_t stride;
  __device__ __forceinline__ void hash(uint64_t i, uint32_t &h1, uint32_t &h2) const {
    hash_bytes(keys + i * stride, stride, kSeed1, kSeed2, h1, h2);
  }
  __device__ __forceinline__ bool same_as_prev(uint64_t i) const {
    const uint8_t *a = keys + i * stride, *b = a - stride;
    for (uint32_t j = 0; j < stride; ++j)
      if (a[j] != b[j]) return false;
    return true;
  }
};

// Variable length: key i = keys[offs[i] .. offs[i+1]).
struct KeysVar {
  const uint8_t *keys;
  const uint64_t *offs;
  __device__ __forceinline__ void hash(uint64_t i, uint32_t &h1, uint32_t &h2) const {
    const uint64_t o0 = offs[i], o1 = offs[i + 1];
    hash_bytes(keys + o0, (uint32_t)(o1 - o0), kSeed1, kSeed2, h1, h2);
  }
  __device__ __forceinline__ bool same_as_prev(uint64_t i) const {
    const uint64_t p0 = offs[i - 1], o0 = offs[i], o1 = offs[i + 1];
    if (o1 - o0 != o0 - p0) return false;
    for (uint64_t j = 0; j < o1 - o0; ++j)
      if (keys[o0 + j] != keys[p0 + j]) return false;
    return true;
  }
};

// ---------------------------------------------------------------- nt access
// Non-temporal 16-byte load/store (global_*_dwordx4 ... nt): streamed data that
// should not displace what the next kernel re-reads from L2 / Infinity Cache.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 load_nt(const uint4 *p) {
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t *>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ void store_nt(uint4 *p, uint4 v) {
  const u32x4_t x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4_t *>(p));
}

// ---------------------------------------------------------------- scans
// Inclusive wave64 scan by DPP (row shifts inside 16-lane rows, then the
// row broadcasts 15 and 31): about 6 VALU steps instead of 6 ds_bpermute round
// trips through the LDS.  Lanes a DPP source does not cover read 0.
__device__ __forceinline__ uint32_t row16_incl_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  return v;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int /*lane*/) {
  v = row16_incl_scan(v);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// Exclusive scan of one value per thread over the block.  `scratch` holds
// BLOCK/64 + 1 words of LDS.  Returns the exclusive prefix; *total = sum.
template <int BLOCK>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *scratch, uint32_t *total) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  constexpr int NW = BLOCK / kWave;
  const uint32_t incl = wave_incl_scan(v, lane);
  if (lane == kWave - 1) scratch[wave] = incl;
  __syncthreads();
  if (wave == 0) {
    uint32_t w = lane < NW ? scratch[lane] : 0u;
    uint32_t wi = wave_incl_scan(w, lane);
    if (lane < NW) scratch[lane] = wi - w;
    if (lane == NW - 1) scratch[NW] = wi;
  }
  __syncthreads();
  const uint32_t r = scratch[wave] + incl - v;
  *total = scratch[NW];
  __syncthreads();  // scratch may be reused right after
  return r;
}

// In-place exclusive scan of an LDS array a[0..N), N <= BLOCK * 4 entries per
// thread; returns the total.  Each thread owns a contiguous run.
template <int BLOCK>
__device__ __forceinline__ uint32_t block_excl_scan_array(uint32_t *a, uint32_t N, uint32_t *scratch) {
  const uint32_t per = (N + BLOCK - 1) / BLOCK;
  const uint32_t beg = threadIdx.x * per;
  const uint32_t end = beg + per < N ? beg + per : N;
  uint32_t s = 0;
  for (uint32_t i = beg; i < end; ++i) s += a[i];
  uint32_t total;
  uint32_t run = block_excl_scan<BLOCK>(s, scratch, &total);
  for (uint32_t i = beg; i < end; ++i) {
    const uint32_t v = a[i];
    a[i] = run;
    run += v;
  }
  __syncthreads();
  return total;
}

// The same in-place exclusive scan with one barrier instead of four: every
// wave scans its threads' run sums, publishes its total, and after the one
// barrier each wave adds up the totals of the waves before it itself.  When
// each thread owns at most one entry (N <= BLOCK), entry i is written and
// later read back by thread i only, so no barrier follows; otherwise one does.
template <int BLOCK>
__device__ __forceinline__ uint32_t block_excl_scan_array_1b(uint32_t *a, uint32_t N, uint32_t *scratch) {
  constexpr int NW = BLOCK / kWave;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const uint32_t per = (N + BLOCK - 1) / BLOCK;
  const uint32_t beg = tid * per;
  const uint32_t end = beg + per < N ? beg + per : N;
  uint32_t v = 0;
  for (uint32_t i = beg; i < end; ++i) v += a[i];
  const uint32_t incl = wave_incl_scan(v, lane);
  if (lane == kWave - 1) scratch[wave] = incl;
  __syncthreads();
  // the totals of waves 0..wave-1: lane i < NW <= 16 holds wave i's, scanned
  // inside the first 16-lane row; wave w reads lane w-1, the total lane NW-1
  static_assert(NW <= 16, "wave totals scanned inside one DPP row");
  const uint32_t wt = lane < NW ? scratch[lane] : 0u;
  const uint32_t wi = row16_incl_scan(wt);
  const uint32_t before = wave ? __builtin_amdgcn_readlane(wi, wave - 1) : 0u;
  const uint32_t all = __builtin_amdgcn_readlane(wi, NW - 1);
  uint32_t run = before + incl - v;
  for (uint32_t i = beg; i < end; ++i) {
    const uint32_t x = a[i];
    a[i] = run;
    run += x;
  }
  if (per > 1) __syncthreads();
  return all;
}

}  // namespace adl_dev

namespace adl_host {

// Tuning and test switches, read from the environment once per
// process.  adl_bloom_reload_knobs() reads them again (tests, between calls:
// no call of the library may be running).
struct Knobs {
  uint32_t tile_log2 = 0;         // ADL_BLOOM_TILE_LOG2: pass-B tile bits (10..20; 0: the plan's choice)
  uint32_t claim = 3;             // ADL_BLOOM_CLAIM: 0 off, 1 wherever the share test passes, 2 forced, 3 auto
  uint32_t claim_cap = 0;         // ADL_BLOOM_CLAIM_CAP: claim region cap, percent of k*C (0: the LDS left)
  bool hash_dedup = true;         // ADL_BLOOM_HASH_DEDUP: pass A skips repeated hash pairs
  bool spin = true;               // ADL_BLOOM_SPIN: small cache probes watch their mapped answers
  bool probe_server = true;       // ADL_BLOOM_PROBE_SERVER: cache batches of <= 8 queries go to the server
  uint64_t server_idle_us = 2000;   // ADL_BLOOM_SERVER_IDLE_US
  uint64_t server_life_us = 1000000;  // ADL_BLOOM_SERVER_LIFE_US
  uint64_t pipe_mb = 128;         // ADL_BLOOM_PIPE_MB: keys per group of the pipelined host build
  // ADL_BLOOM_BUILD_QUEUES: when the build passes take their items from work
  // queues instead of the static order: 0 never, 1 while a probe server
  // exists, 2 while a server kernel is resident (its alive word), 3 always.
  // ADL_BLOOM_BUILD_QUEUE_PASSES: which passes (bit 0 pass A, bit 1 pass B).
  uint32_t build_queues = 2;
  uint32_t build_queue_passes = 3;
  bool server_invalidate = false;  // ADL_BLOOM_SERVER_INVALIDATE: the server invalidates its caches at every request
  bool debug = false;             // ADL_BLOOM_DEBUG: the plan and failing HIP calls to stderr
  uint32_t exp = 0, pb_exp = 0;   // ADL_BLOOM_EXP / ADL_PB_EXP: diagnostics build (make stamps) only

  void load() {
    auto u64 = [](const char *name, uint64_t dflt) -> uint64_t {
      const char *e = getenv(name);
      return e && *e ? strtoull(e, nullptr, 10) : dflt;
    };
    *this = Knobs{};
    tile_log2 = (uint32_t)u64("ADL_BLOOM_TILE_LOG2", 0);
    claim = (uint32_t)u64("ADL_BLOOM_CLAIM", 3);
    claim_cap = (uint32_t)u64("ADL_BLOOM_CLAIM_CAP", 0);
    hash_dedup = u64("ADL_BLOOM_HASH_DEDUP", 1) != 0;
    spin = u64("ADL_BLOOM_SPIN", 1) != 0;
    probe_server = u64("ADL_BLOOM_PROBE_SERVER", 1) != 0;
    server_idle_us = u64("ADL_BLOOM_SERVER_IDLE_US", 2000);
    server_life_us = u64("ADL_BLOOM_SERVER_LIFE_US", 1000000);
    pipe_mb = u64("ADL_BLOOM_PIPE_MB", 128);
    build_queues = (uint32_t)u64("ADL_BLOOM_BUILD_QUEUES", 2);
    build_queue_passes = (uint32_t)u64("ADL_BLOOM_BUILD_QUEUE_PASSES", 3);
    server_invalidate = u64("ADL_BLOOM_SERVER_INVALIDATE", 0) != 0;
    debug = u64("ADL_BLOOM_DEBUG", 0) != 0;
#ifdef ADL_BLOOM_STAMPS
    exp = (uint32_t)u64("ADL_BLOOM_EXP", 0);
    pb_exp = (uint32_t)u64("ADL_PB_EXP", 0);
#endif
  }
};

inline Knobs g_knobs;
inline std::once_flag g_knobs_once;

inline const Knobs &knobs() {
  std::call_once(g_knobs_once, [] { g_knobs.load(); });
  return g_knobs;
}

inline void reload_knobs() {
  (void)knobs();
  g_knobs.load();
}

// Host-side magic numbers for adl_dev::fastmod (see murmur3_device.hpp).
inline adl_dev::FastMod make_fastmod(uint32_t m) {
  adl_dev::FastMod f{};
  f.m = m;
  uint32_t l = 0;
  while ((1ull << l) < m) ++l;  // ceil(log2 m); m >= 2 (m = 8 * bitmap bytes >= 56)
  f.magic = (uint32_t)((((1ull << 32) * ((1ull << l) - m)) / m) + 1ull);
  f.shift = l - 1;
  return f;
}

// Compute units of the current device (256 on MI355X), queried once.
inline uint32_t device_cus() {
  static std::once_flag once;
  static uint32_t cus = 256;
  std::call_once(once, [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      cus = (uint32_t)v;
  });
  return cus;
}

inline int num_probes(int32_t bpk) {
  int k = (int)(bpk * 0.69);  // src/filter_block.cpp:44
  if (k < 1) k = 1;
  if (k > 30) k = 30;
  return k;
}

inline uint64_t bitmap_bytes(uint64_t n, int32_t bpk) {
  if (bpk < 0) return 0;
  const uint64_t bytes = n * (uint64_t)bpk + 7;
  if (n > 0x7fffffffull || bytes * 8 > 0x7fffffffull) return 0;
  return bytes;
}

inline uint64_t round_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

// Per-thread staging for the synchronous host-pointer entry points: a pinned
// host buffer (so every copy is a stream-ordered DMA; pageable hipMemcpyAsync
// is not used anywhere) and a device buffer, both grown on demand and reused.
// One per thread keeps the C-ABI re-entrant without locks.
struct Staging {
  uint8_t *host = nullptr;
  uint64_t hcap = 0;
  uint8_t *dev = nullptr;
  uint64_t dcap = 0;
  ~Staging() {
    if (host) (void)hipHostFree(host);
    if (dev) (void)hipFree(dev);
  }
  int reserve(uint64_t hbytes, uint64_t dbytes) {
    if (hbytes > hcap) {
      if (host) (void)hipHostFree(host);
      host = nullptr;
      hcap = 0;
      const uint64_t want = round_up(hbytes + (hbytes >> 3), 1 << 16);
      if (hipHostMalloc((void **)&host, want, hipHostMallocDefault) != hipSuccess) return ADL_ERR_OUT_OF_MEMORY;
      hcap = want;
    }
    if (dbytes > dcap) {
      if (dev) (void)hipFree(dev);
      dev = nullptr;
      dcap = 0;
      const uint64_t want = round_up(dbytes + (dbytes >> 3), 1 << 16);
      if (hipMalloc((void **)&dev, want) != hipSuccess) return ADL_ERR_OUT_OF_MEMORY;
      dcap = want;
    }
    return ADL_OK;
  }
};

inline thread_local Staging t_stage;

// Per-thread small pinned buffer mapped into the device's address space
// (coherent): a small synchronous probe hands the kernel its keys and table
// ids where they are and has it write the answers back there, so a lookup is
// one launch and one stream sync, with no H2D / D2H copy commands.
struct MappedStage {
  static constexpr uint64_t kMax = 64 << 10;
  uint8_t *host = nullptr;
  uint8_t *dev = nullptr;
  bool tried = false;
  ~MappedStage() {
    if (host) (void)hipHostFree(host);
  }
  // nullptr if unavailable or bytes > kMax (the caller then stages and copies)
  uint8_t *get(uint64_t bytes) {
    if (bytes > kMax) return nullptr;
    if (!tried) {
      tried = true;
      void *d = nullptr;
      if (hipHostMalloc((void **)&host, kMax, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
          hipHostGetDevicePointer(&d, host, 0) != hipSuccess) {
        if (host) (void)hipHostFree(host);
        host = nullptr;
        (void)hipGetLastError();
        return nullptr;
      }
      dev = static_cast<uint8_t *>(d);
    }
    return host;
  }
};

inline thread_local MappedStage t_mapped;

// The stream a synchronous host-pointer entry point runs on: the caller's, or
// for stream == NULL a non-blocking stream of the calling thread (created on
// first use).  The legacy null stream would order every thread's calls one
// after the other on the device; these calls only touch their own staging
// buffers, so nothing is lost by not ordering them with the null stream.
struct ThreadStream {
  hipStream_t s = nullptr;
  bool tried = false;
  ~ThreadStream() {
    if (s) (void)hipStreamDestroy(s);
  }
  hipStream_t get() {
    if (!tried) {
      tried = true;
      if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) s = nullptr;
    }
    return s;
  }
};

inline thread_local ThreadStream t_stream;

inline hipStream_t sync_stream(void *stream) { return stream ? (hipStream_t)stream : t_stream.get(); }

// Small host -> device uploads in stream order from pinned memory (a build's
// filter descriptors): a ring of slots per thread, each reused only after its
// previous copy has completed.
struct UploadRing {
  static constexpr int kSlots = 4;
  uint8_t *host[kSlots] = {};
  uint64_t cap[kSlots] = {};
  hipEvent_t ev[kSlots] = {};
  bool used[kSlots] = {};
  int next = 0;
  ~UploadRing() {
    for (int s = 0; s < kSlots; ++s) {
      if (used[s]) (void)hipEventSynchronize(ev[s]);
      if (ev[s]) (void)hipEventDestroy(ev[s]);
      if (host[s]) (void)hipHostFree(host[s]);
    }
  }
  int upload(void *dst, const void *src, uint64_t bytes, hipStream_t st) {
    const int s = next;
    next = (next + 1) % kSlots;
    if (!ev[s]) ADL_HIP_TRY(hipEventCreateWithFlags(&ev[s], hipEventDisableTiming));
    if (used[s]) ADL_HIP_TRY(hipEventSynchronize(ev[s]));
    used[s] = false;
    if (bytes > cap[s]) {
      if (host[s]) (void)hipHostFree(host[s]);
      host[s] = nullptr;
      cap[s] = 0;
      const uint64_t want = round_up(bytes, 1 << 16);
      ADL_HIP_TRY(hipHostMalloc((void **)&host[s], want, hipHostMallocDefault));
      cap[s] = want;
    }
    memcpy(host[s], src, bytes);
    ADL_HIP_TRY(hipMemcpyAsync(dst, host[s], bytes, hipMemcpyHostToDevice, st));
    ADL_HIP_TRY(hipEventRecord(ev[s], st));
    used[s] = true;
    return ADL_OK;
  }
};

inline thread_local UploadRing t_upload;

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per kernel and device
// (the whole 160 KiB of a CU; each launch asks for what it uses), not on every
// launch.
template <auto Kern>
int lds_limit() {
  static std::atomic<uint64_t> done{0};
  int dev = 0;
  ADL_HIP_TRY(hipGetDevice(&dev));
  const uint64_t bit = 1ull << (dev & 63);
  if (done.load(std::memory_order_acquire) & bit) return ADL_OK;
  ADL_HIP_TRY(hipFuncSetAttribute((const void *)Kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  done.fetch_or(bit, std::memory_order_acq_rel);
  return ADL_OK;
}

// Library-internal (bloom_probe.hip): adl_bloom_probe_ranges_device whose
// kernel launch also completes `done`.
__attribute__((visibility("hidden"))) int adl_probe_ranges_device_ev(
    const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n, uint32_t key_stride, const uint32_t *d_filter_id,
    uint32_t num_filters, const uint8_t *d_bitmaps, const uint64_t *d_begin, const uint64_t *d_end,
    const uint8_t *d_k, uint8_t *d_out, hipStream_t st, hipEvent_t done);

// adl_bloom_test_fault's armed sites (-1: off).  take() disarms and returns the
// argument, so an armed fault fires once.
struct TestFaults {
  std::atomic<int64_t> site[3] = {-1, -1, -1};
  int64_t take(int s) {
    if (site[s].load(std::memory_order_relaxed) < 0) return -1;
    return site[s].exchange(-1);
  }
};
inline TestFaults g_test_faults;

}  // namespace adl_host
