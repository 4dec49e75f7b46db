// adlsm-tree_amd/csrc/bloom_probe.hip -- MI355X (gfx950) batched bloom probe,
// batched murmur3 and the device-side synthetic key generators.
//
// Probe replaces BloomFilter::IsKeyExists (reference src/filter_block.cpp:49-62)
// for a batch: m = bitmap_bytes*8 (:50), the same h1 + j*h2 positions as the
// build, "absent" at the first clear bit (:54-59).  One query per lane; the key
// load is coalesced, the k bitmap reads are random byte loads that stop at the
// first clear bit (the same early exit as the reference), issued a few at a
// time so that independent reads overlap.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <new>

#include "bloom_common.hpp"

using namespace adl_dev;

namespace {

constexpr int kBlockP = 256;

constexpr uint32_t kLdsFilters = 4096;   // per-filter divisor table kept in LDS up to this many

// The k bitmap reads of one query, one at a time with the reference's stop at
// the first clear bit (src/filter_block.cpp:54-59).  Issuing 2-8 reads per
// round (so they overlap) measured slower: the probe is bound by random HBM
// reads, so the fewest reads win.
__device__ __forceinline__ uint8_t probe_bits(const uint8_t *__restrict__ bm, uint32_t h1, uint32_t h2,
                                              uint32_t k, const FastMod &mod) {
  for (uint32_t j = 0; j < k; ++j) {
    const uint32_t p = fastmod(h1 + j * h2, mod);
    if (!((bm[p >> 3] >> (p & 7)) & 1u)) return 0;
  }
  return 1;
}

template <class Keys>
__global__ __launch_bounds__(kBlockP) void bloom_probe_kernel(Keys keys, uint64_t n, uint32_t k,
                                                              FastMod mod,
                                                              const uint8_t *__restrict__ bitmap,
                                                              uint8_t *__restrict__ out) {
  for (uint64_t i = blockIdx.x * (uint64_t)kBlockP + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kBlockP) {
    uint32_t h1, h2;
    keys.hash(i, h1, h2);
    out[i] = probe_bits(bitmap, h1, h2, k, mod);
  }
}

// Multi-filter probe: query i against filter fid[i] (or uniform_f).  Each
// filter has its own divisor m = 8 * bitmap bytes, and -- when kf is given --
// its own probe count kf[f] (blocks written with different bits_per_key: the
// reference reads bpk per block, src/filter_block.cpp:158-170).  The
// magic-multiply constants and k of up to kLdsFilters filters are built once
// per workgroup into LDS (dynamic, 8 B per filter), beyond that per query.
struct ModLds {
  uint32_t magic, shift_k;  // shift | k << 8
};

template <class Keys>
__global__ __launch_bounds__(kBlockP) void bloom_probe_multi_kernel(
    Keys keys, uint64_t n, uint32_t k, const uint8_t *__restrict__ kf, const uint32_t *__restrict__ fid,
    uint32_t uniform_f, uint32_t nf, const uint8_t *__restrict__ bitmaps, const uint64_t *__restrict__ boff,
    const uint64_t *__restrict__ bend, uint8_t *__restrict__ out) {
  // filter f = bitmaps[boff[f], bend[f]), or [boff[f], boff[f+1]) when bend is null
  extern __shared__ ModLds lmod[];
  const bool lds_tab = nf <= kLdsFilters;
  if (lds_tab) {
    for (uint32_t f = threadIdx.x; f < nf; f += kBlockP) {
      // an empty range (m = 0: a filter the table does not have) and a filter
      // of 2^31 bits or more answer 0 below and need no divisor
      const uint64_t bytes = (bend ? bend[f] : boff[f + 1]) - boff[f];
      const uint32_t m = bytes <= 0x0fffffffull ? (uint32_t)(bytes * 8) : 0u;
      const FastMod fm = m ? fastmod_for(m) : FastMod{};
      lmod[f] = ModLds{fm.magic, fm.shift | (kf ? (uint32_t)kf[f] : k) << 8};
    }
    __syncthreads();
  }
  for (uint64_t i = blockIdx.x * (uint64_t)kBlockP + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kBlockP) {
    const uint32_t f = fid ? fid[i] : uniform_f;  // fid == nullptr: every query -> uniform_f
    uint8_t hit = 0;
    if (f < nf) {
      const uint64_t b0 = boff[f], b1 = bend ? bend[f] : boff[f + 1];
      // 0 for an empty filter or one of 2^31 bits or more (outside the
      // reference's int m, src/filter_block.cpp:50)
      const uint32_t m = b1 - b0 <= 0x0fffffffull ? (uint32_t)((b1 - b0) * 8) : 0u;
      if (m != 0) {
        FastMod mod;
        uint32_t kq;
        if (lds_tab) {
          const ModLds e = lmod[f];
          mod = FastMod{m, e.magic, e.shift_k & 0xFFu, 0u};
          kq = e.shift_k >> 8;
        } else {
          mod = fastmod_for(m);
          kq = kf ? (uint32_t)kf[f] : k;
        }
        uint32_t h1, h2;
        keys.hash(i, h1, h2);
        hit = probe_bits(bitmaps + b0, h1, h2, kq, mod);
      }
    }
    out[i] = hit;
  }
}

template <class Keys>
__global__ __launch_bounds__(kBlockP) void murmur3_batch_kernel(Keys keys, uint64_t n,
                                                                uint32_t *__restrict__ out) {
  for (uint64_t i = blockIdx.x * (uint64_t)kBlockP + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kBlockP) {
    uint32_t a, b;
    keys.hash(i, a, b);
    out[2 * i] = a;
    out[2 * i + 1] = b;
  }
}

// Arbitrary seeds (the key views hash with the filter's two seeds).
__global__ __launch_bounds__(kBlockP) void murmur3_seeded_kernel(const uint8_t *__restrict__ keys,
                                                                 const uint64_t *__restrict__ offs,
                                                                 uint32_t stride, uint64_t n,
                                                                 uint32_t sa, uint32_t sb,
                                                                 uint32_t *__restrict__ out) {
  for (uint64_t i = blockIdx.x * (uint64_t)kBlockP + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kBlockP) {
    const uint64_t o0 = offs ? offs[i] : i * stride;
    const uint32_t len = offs ? (uint32_t)(offs[i + 1] - o0) : stride;
    uint32_t a, b;
    hash_bytes(keys + o0, len, sa, sb, a, b);
    out[2 * i] = a;
    out[2 * i + 1] = b;
  }
}

// ---------------------------------------------------------------- synthetic data
__device__ __forceinline__ uint64_t splitmix_at(uint64_t seed, uint64_t call /* 1-based */) {
  uint64_t z = seed + call * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void synth_keys16_kernel(uint4 *__restrict__ out, uint64_t seed,
                                                           uint64_t skip, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t c = 2 * (skip + i);
    const uint64_t a = splitmix_at(seed, c + 1), b = splitmix_at(seed, c + 2);
    out[i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
  }
}

__global__ __launch_bounds__(256) void synth_probe_kernel(uint4 *__restrict__ keys, uint32_t *__restrict__ fid,
                                                          uint8_t *__restrict__ member, uint64_t seed, uint64_t q0,
                                                          uint64_t n, uint32_t tables, uint64_t tseed0,
                                                          uint64_t per_table) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t c = 4 * (q0 + i);
    const uint64_t r0 = splitmix_at(seed, c + 1), r1 = splitmix_at(seed, c + 2);
    const uint32_t t = (uint32_t)(r0 % tables);
    uint64_t a, b;
    const bool ins = (r1 & 1) && per_table;
    if (ins) {
      const uint64_t j = (r1 >> 1) % per_table;
      a = splitmix_at(tseed0 + t, 2 * j + 1);
      b = splitmix_at(tseed0 + t, 2 * j + 2);
    } else {
      a = splitmix_at(seed, c + 3);
      b = splitmix_at(seed, c + 4);
    }
    keys[i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    fid[i] = t;
    if (member) member[i] = ins;
  }
}

constexpr int kZipfR = 249;  // lengths 8 .. 256

// Inverse-CDF table of Zipf(s) on [1, kZipfR] in 53-bit fixed point: r is the
// first rank with x < thr[r-1], x = a SplitMix64 output >> 11.  Built on the
// host (zipf_table), so the device and the oracle's restatement
// (oracle_synth_varlen_lengths) draw identical lengths from the same stream.
struct ZipfTable {
  uint64_t thr[kZipfR];
};

__global__ __launch_bounds__(256) void synth_lengths_kernel(uint32_t *__restrict__ len, uint64_t seed,
                                                            uint64_t n, ZipfTable zt) {
  const uint64_t lseed = seed ^ 0xD1B54A32D192ED03ull;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t x = splitmix_at(lseed, i + 1) >> 11;
    int lo = 0, hi = kZipfR - 1;  // first r with x < thr[r]
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (x < zt.thr[mid]) hi = mid; else lo = mid + 1;
    }
    len[i] = 8u + (uint32_t)lo;
  }
}

// cdf(r) = sum_{i<=r} i^-s / sum_{i<=R} i^-s in double; thr = ceil(cdf * 2^53),
// so x < thr  <=>  x * 2^-53 < cdf  for every 53-bit integer x
ZipfTable zipf_table(double s) {
  ZipfTable z{};
  double cdf[kZipfR], acc = 0;
  for (int r = 1; r <= kZipfR; ++r) {
    acc += pow((double)r, -s);
    cdf[r - 1] = acc;
  }
  for (int r = 0; r < kZipfR; ++r) z.thr[r] = (uint64_t)ceil(cdf[r] / acc * 9007199254740992.0);
  return z;
}

__global__ __launch_bounds__(256) void synth_fill_kernel(uint64_t *__restrict__ out, uint64_t seed,
                                                         uint64_t words) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < words; i += (uint64_t)gridDim.x * 256)
    out[i] = splitmix_at(seed, i + 1);
}

// Grid-stride launches: enough workgroups to cover n, at most blocks_per_cu
// per CU (the multi-filter probe amortises a per-workgroup table over many
// queries, so it asks for a persistent-sized grid).
inline uint32_t grid_for(uint64_t n, int block, uint32_t blocks_per_cu = 64) {
  return (uint32_t)std::max<uint64_t>(
      1, std::min<uint64_t>((n + block - 1) / block, (uint64_t)adl_host::device_cus() * blocks_per_cu));
}

template <class F>
int dispatch_keys(const uint8_t *d_keys, const uint64_t *d_offsets, uint32_t key_stride, F &&fn) {
  if (d_offsets) return fn(KeysVar{d_keys, d_offsets});
  if (key_stride == 16 && reinterpret_cast<uintptr_t>(d_keys) % 16 == 0)
    return fn(Keys16{reinterpret_cast<const uint4 *>(d_keys)});
  return fn(KeysStride{d_keys, key_stride});
}

}  // namespace

extern "C" {

int adl_bloom_probe_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n,
                           uint32_t key_stride, int32_t bits_per_key, const uint8_t *d_bitmap,
                           uint64_t bitmap_bytes, uint8_t *d_out, void *stream) {
  if (n == 0) return ADL_OK;
  if (!d_keys || !d_bitmap || !d_out || bits_per_key < 0) return ADL_ERR_INVALID_ARG;
  if (!d_offsets && key_stride == 0) return ADL_ERR_INVALID_ARG;
  if (bitmap_bytes == 0) return ADL_ERR_INVALID_ARG;  // h % 0 is undefined in the reference
  if (bitmap_bytes * 8 > 0x7fffffffull) return ADL_ERR_TOO_LARGE;
  const uint32_t k = (uint32_t)adl_host::num_probes(bits_per_key);
  const FastMod mod = adl_host::make_fastmod((uint32_t)(bitmap_bytes * 8));
  hipStream_t st = (hipStream_t)stream;
  return dispatch_keys(d_keys, d_offsets, key_stride, [&](auto keys) -> int {
    hipLaunchKernelGGL(bloom_probe_kernel<decltype(keys)>, dim3(grid_for(n, kBlockP)), dim3(kBlockP), 0,
                       st, keys, n, k, mod, d_bitmap, d_out);
    ADL_HIP_TRY(hipGetLastError());
    return ADL_OK;
  });
}

}  // extern "C"

namespace {
// fid == nullptr sends every query to filter `uniform_f`.
int probe_multi(const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n, uint32_t key_stride,
                const uint32_t *d_filter_id, uint32_t uniform_f, uint32_t num_filters,
                const uint8_t *d_bitmaps, const uint64_t *d_bitmap_off, int32_t bits_per_key,
                uint8_t *d_out, hipStream_t st, const uint64_t *d_bitmap_end = nullptr,
                hipEvent_t done = nullptr, const uint8_t *d_k = nullptr) {
  if (num_filters && (!d_bitmaps || !d_bitmap_off)) return ADL_ERR_INVALID_ARG;
  if (!d_offsets && key_stride == 0) return ADL_ERR_INVALID_ARG;
  const uint32_t k = (uint32_t)adl_host::num_probes(bits_per_key);
  return dispatch_keys(d_keys, d_offsets, key_stride, [&](auto keys) -> int {
    const size_t lds = num_filters <= kLdsFilters ? (size_t)num_filters * sizeof(ModLds) : 0;
    // `done` rides on the dispatch packet itself (no marker packet after it)
    hipExtLaunchKernelGGL(bloom_probe_multi_kernel<decltype(keys)>, dim3(grid_for(n, kBlockP, 8)),
                          dim3(kBlockP), lds, st, nullptr, done, 0, keys, n, k, d_k, d_filter_id,
                          uniform_f, num_filters, d_bitmaps, d_bitmap_off, d_bitmap_end, d_out);
    ADL_HIP_TRY(hipGetLastError());
    return ADL_OK;
  });
}
}  // namespace

// adl_bloom_probe_ranges_device with a probe count per filter (d_k[f]), whose
// launch also completes `done` (the filter cache's small batches wait on it;
// see filter_cache.hip).
int adl_host::adl_probe_ranges_device_ev(const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n, uint32_t key_stride,
                               const uint32_t *d_filter_id, uint32_t num_filters, const uint8_t *d_bitmaps,
                               const uint64_t *d_begin, const uint64_t *d_end, const uint8_t *d_k, uint8_t *d_out,
                               hipStream_t st, hipEvent_t done) {
  if (n == 0) return ADL_OK;
  if (!d_keys || !d_filter_id || !d_out || (num_filters && !d_k)) return ADL_ERR_INVALID_ARG;
  if (num_filters && !d_end) return ADL_ERR_INVALID_ARG;
  return probe_multi(d_keys, d_offsets, n, key_stride, d_filter_id, 0, num_filters, d_bitmaps, d_begin, 10, d_out,
                     st, d_end, done, d_k);
}

extern "C" int adl_bloom_probe_ranges_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n,
                                             uint32_t key_stride, const uint32_t *d_filter_id,
                                             uint32_t num_filters, const uint8_t *d_bitmaps,
                                             const uint64_t *d_begin, const uint64_t *d_end,
                                             int32_t bits_per_key, uint8_t *d_out, void *stream) {
  if (n == 0) return ADL_OK;
  if (!d_keys || !d_filter_id || !d_out || bits_per_key < 0) return ADL_ERR_INVALID_ARG;
  if (num_filters && !d_end) return ADL_ERR_INVALID_ARG;
  return probe_multi(d_keys, d_offsets, n, key_stride, d_filter_id, 0, num_filters, d_bitmaps, d_begin,
                     bits_per_key, d_out, (hipStream_t)stream, d_end);
}

extern "C" {

int adl_bloom_probe_multi_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n,
                                 uint32_t key_stride, const uint32_t *d_filter_id,
                                 uint32_t num_filters, const uint8_t *d_bitmaps,
                                 const uint64_t *d_bitmap_off, int32_t bits_per_key,
                                 uint8_t *d_out, void *stream) {
  if (n == 0) return ADL_OK;
  if (!d_keys || !d_filter_id || !d_out || bits_per_key < 0) return ADL_ERR_INVALID_ARG;
  return probe_multi(d_keys, d_offsets, n, key_stride, d_filter_id, 0, num_filters, d_bitmaps,
                     d_bitmap_off, bits_per_key, d_out, (hipStream_t)stream);
}

int adl_bloom_probe(const uint8_t *h_keys, const uint64_t *h_offsets, uint64_t n,
                    uint32_t key_stride, int32_t bits_per_key, const uint8_t *h_bitmap,
                    uint64_t bitmap_bytes, uint8_t *h_out, void *stream) {
  if (n == 0) return ADL_OK;
  if (!h_keys || !h_bitmap || !h_out) return ADL_ERR_INVALID_ARG;
  if (!h_offsets && key_stride == 0) return ADL_ERR_INVALID_ARG;
  hipStream_t st = adl_host::sync_stream(stream);
  const uint64_t key_bytes = h_offsets ? h_offsets[n] : n * (uint64_t)key_stride;
  const uint64_t off_bytes = h_offsets ? (n + 1) * 8 : 0;
  const uint64_t o_offs = adl_host::round_up(key_bytes + 16, 256);
  const uint64_t o_bm = o_offs + adl_host::round_up(off_bytes, 256);
  const uint64_t o_out = o_bm + adl_host::round_up(bitmap_bytes, 256);
  const uint64_t total = o_out + adl_host::round_up(n, 256);
  adl_host::Staging &sg = adl_host::t_stage;
  int rc = sg.reserve(o_out, total);
  if (rc) return rc;
  if (key_bytes) memcpy(sg.host, h_keys, key_bytes);
  if (off_bytes) memcpy(sg.host + o_offs, h_offsets, off_bytes);
  memcpy(sg.host + o_bm, h_bitmap, bitmap_bytes);
  if (hipMemcpyAsync(sg.dev, sg.host, o_out, hipMemcpyHostToDevice, st) != hipSuccess) return ADL_ERR_DEVICE;
  rc = adl_bloom_probe_device(sg.dev, h_offsets ? reinterpret_cast<uint64_t *>(sg.dev + o_offs) : nullptr, n,
                              key_stride, bits_per_key, sg.dev + o_bm, bitmap_bytes, sg.dev + o_out, st);
  if (rc) {
    (void)hipStreamSynchronize(st);
    return rc;
  }
  if (hipMemcpyAsync(sg.host, sg.dev + o_out, n, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return ADL_ERR_DEVICE;
  memcpy(h_out, sg.host, n);
  return ADL_OK;
}

int adl_bloom_murmur3_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n,
                             uint32_t key_stride, uint32_t seed_a, uint32_t seed_b,
                             uint32_t *d_out, void *stream) {
  if (n == 0) return ADL_OK;
  if (!d_keys || !d_out || (!d_offsets && key_stride == 0)) return ADL_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (seed_a == kSeed1 && seed_b == kSeed2) {
    return dispatch_keys(d_keys, d_offsets, key_stride, [&](auto keys) -> int {
      hipLaunchKernelGGL(murmur3_batch_kernel<decltype(keys)>, dim3(grid_for(n, kBlockP)),
                         dim3(kBlockP), 0, st, keys, n, d_out);
      ADL_HIP_TRY(hipGetLastError());
      return ADL_OK;
    });
  }
  hipLaunchKernelGGL(murmur3_seeded_kernel, dim3(grid_for(n, kBlockP)), dim3(kBlockP), 0, st, d_keys,
                     d_offsets, key_stride, n, seed_a, seed_b, d_out);
  ADL_HIP_TRY(hipGetLastError());
  return ADL_OK;
}

int adl_bloom_murmur3(uint32_t seed, const void *data, uint64_t len, uint32_t *h_out) {
  if (!h_out || (len && !data) || len > 0xffffffffull) return ADL_ERR_INVALID_ARG;
  const uint64_t o_out = adl_host::round_up(len + 16, 256);
  adl_host::Staging &sg = adl_host::t_stage;
  int rc = sg.reserve(o_out + 16, o_out + 16);
  if (rc) return rc;
  if (len) memcpy(sg.host, data, len);
  hipStream_t st = adl_host::sync_stream(nullptr);
  if (len && hipMemcpyAsync(sg.dev, sg.host, len, hipMemcpyHostToDevice, st) != hipSuccess) return ADL_ERR_DEVICE;
  hipLaunchKernelGGL(murmur3_seeded_kernel, dim3(1), dim3(kBlockP), 0, st, sg.dev, (const uint64_t *)nullptr,
                     (uint32_t)len, 1ull, seed, seed, reinterpret_cast<uint32_t *>(sg.dev + o_out));
  if (hipGetLastError() != hipSuccess ||
      hipMemcpyAsync(sg.host + o_out, sg.dev + o_out, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return ADL_ERR_DEVICE;
  memcpy(h_out, sg.host + o_out, 4);
  return ADL_OK;
}

int adl_synth_keys16_device(uint8_t *d_out, uint64_t seed, uint64_t skip, uint64_t n, void *stream) {
  if (n == 0) return ADL_OK;
  if (!d_out || reinterpret_cast<uintptr_t>(d_out) % 16) return ADL_ERR_INVALID_ARG;
  hipLaunchKernelGGL(synth_keys16_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<uint4 *>(d_out), seed, skip, n);
  ADL_HIP_TRY(hipGetLastError());
  return ADL_OK;
}

int adl_synth_varlen_lengths_device(uint32_t *d_lengths, uint64_t seed, uint64_t n, double zipf_s,
                                    void *stream) {
  if (n == 0) return ADL_OK;
  if (!d_lengths) return ADL_ERR_INVALID_ARG;
  hipLaunchKernelGGL(synth_lengths_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream,
                     d_lengths, seed, n, zipf_table(zipf_s));
  ADL_HIP_TRY(hipGetLastError());
  return ADL_OK;
}

int adl_synth_varlen_fill_device(uint8_t *d_out, uint64_t seed, uint64_t total_bytes, void *stream) {
  if (total_bytes == 0) return ADL_OK;
  if (!d_out || reinterpret_cast<uintptr_t>(d_out) % 8) return ADL_ERR_INVALID_ARG;
  const uint64_t words = (total_bytes + 7) / 8;  // caller allocates round_up(total_bytes, 8)
  hipLaunchKernelGGL(synth_fill_kernel, dim3(grid_for(words, 256)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<uint64_t *>(d_out), seed, words);
  ADL_HIP_TRY(hipGetLastError());
  return ADL_OK;
}

int adl_synth_probe_queries_device(uint8_t *d_keys, uint32_t *d_filter_id, uint8_t *d_member,
                                   uint64_t seed, uint64_t q0, uint64_t n, uint32_t num_tables,
                                   uint64_t table_seed0, uint64_t keys_per_table, void *stream) {
  if (n == 0) return ADL_OK;
  if (!d_keys || !d_filter_id || num_tables == 0 || reinterpret_cast<uintptr_t>(d_keys) % 16)
    return ADL_ERR_INVALID_ARG;
  hipLaunchKernelGGL(synth_probe_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<uint4 *>(d_keys), d_filter_id, d_member, seed, q0, n, num_tables,
                     table_seed0, keys_per_table);
  ADL_HIP_TRY(hipGetLastError());
  return ADL_OK;
}

}  // extern "C"

// ====================================================================== filter sets
struct adl_bloom_filter_set {
  uint8_t *d_bitmaps = nullptr;
  uint64_t *d_off = nullptr;
  uint32_t nf = 0;
  int32_t bpk = 0;
};

extern "C" {

int adl_bloom_filter_set_create(const uint8_t *h_bitmaps, const uint64_t *h_bitmap_off,
                                uint32_t num_filters, int32_t bits_per_key,
                                adl_bloom_filter_set **out) {
  if (!out || !h_bitmap_off || bits_per_key < 0) return ADL_ERR_INVALID_ARG;
  *out = nullptr;
  const uint64_t total = h_bitmap_off[num_filters];
  for (uint32_t f = 0; f < num_filters; ++f) {
    if (h_bitmap_off[f + 1] < h_bitmap_off[f]) return ADL_ERR_INVALID_ARG;
    // m = 8 * bytes must stay a u32 the probe can reduce by (the reference's
    // int m, src/filter_block.cpp:50; adl_bloom_probe_device rejects the same)
    if ((h_bitmap_off[f + 1] - h_bitmap_off[f]) * 8 > 0x7fffffffull) return ADL_ERR_TOO_LARGE;
  }
  if (total && !h_bitmaps) return ADL_ERR_INVALID_ARG;
  auto *s = new (std::nothrow) adl_bloom_filter_set;
  if (!s) return ADL_ERR_OUT_OF_MEMORY;
  s->nf = num_filters;
  s->bpk = bits_per_key;
  int rc = ADL_OK;
  if (hipMalloc((void **)&s->d_bitmaps, total + 16) != hipSuccess ||
      hipMalloc((void **)&s->d_off, (num_filters + 1) * sizeof(uint64_t)) != hipSuccess) {
    rc = ADL_ERR_OUT_OF_MEMORY;
  } else if ((total && hipMemcpy(s->d_bitmaps, h_bitmaps, total, hipMemcpyHostToDevice) != hipSuccess) ||
             hipMemcpy(s->d_off, h_bitmap_off, (num_filters + 1) * sizeof(uint64_t),
                       hipMemcpyHostToDevice) != hipSuccess) {
    rc = ADL_ERR_DEVICE;
  }
  if (rc) {
    adl_bloom_filter_set_destroy(s);
    return rc;
  }
  *out = s;
  return ADL_OK;
}

int adl_bloom_filter_set_probe(const adl_bloom_filter_set *set, const uint8_t *h_keys,
                               const uint64_t *h_offsets, uint64_t n, uint32_t key_stride,
                               const uint32_t *h_filter_id, uint32_t filter, uint8_t *h_out,
                               void *stream) {
  if (!set) return ADL_ERR_INVALID_ARG;
  if (n == 0) return ADL_OK;
  if (!h_keys || !h_out || (!h_offsets && key_stride == 0)) return ADL_ERR_INVALID_ARG;
  hipStream_t st = adl_host::sync_stream(stream);
  const uint64_t key_bytes = h_offsets ? h_offsets[n] : n * (uint64_t)key_stride;
  const uint64_t off_bytes = h_offsets ? (n + 1) * 8 : 0;
  const uint64_t o_offs = adl_host::round_up(key_bytes + 16, 256);
  const uint64_t o_fid = o_offs + adl_host::round_up(off_bytes, 256);
  const uint64_t o_out = o_fid + adl_host::round_up(h_filter_id ? n * 4 : 0, 256);
  const uint64_t total = o_out + adl_host::round_up(n, 256);
  adl_host::Staging &sg = adl_host::t_stage;
  int rc = sg.reserve(o_out, total);
  if (rc) return rc;
  if (key_bytes) memcpy(sg.host, h_keys, key_bytes);
  if (off_bytes) memcpy(sg.host + o_offs, h_offsets, off_bytes);
  if (h_filter_id) memcpy(sg.host + o_fid, h_filter_id, n * 4);
  if (hipMemcpyAsync(sg.dev, sg.host, o_out, hipMemcpyHostToDevice, st) != hipSuccess) return ADL_ERR_DEVICE;
  rc = probe_multi(sg.dev, h_offsets ? reinterpret_cast<uint64_t *>(sg.dev + o_offs) : nullptr, n, key_stride,
                   h_filter_id ? reinterpret_cast<uint32_t *>(sg.dev + o_fid) : nullptr, filter, set->nf,
                   set->d_bitmaps, set->d_off, set->bpk, sg.dev + o_out, st);
  if (rc) {
    (void)hipStreamSynchronize(st);
    return rc;
  }
  if (hipMemcpyAsync(sg.host, sg.dev + o_out, n, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return ADL_ERR_DEVICE;
  memcpy(h_out, sg.host, n);
  return ADL_OK;
}

int adl_bloom_filter_set_device_view(const adl_bloom_filter_set *set, const uint8_t **d_bitmaps,
                                     const uint64_t **d_bitmap_off, uint32_t *num_filters) {
  if (!set) return ADL_ERR_INVALID_ARG;
  if (d_bitmaps) *d_bitmaps = set->d_bitmaps;
  if (d_bitmap_off) *d_bitmap_off = set->d_off;
  if (num_filters) *num_filters = set->nf;
  return ADL_OK;
}

int adl_bloom_filter_set_destroy(adl_bloom_filter_set *set) {
  if (!set) return ADL_OK;
  int rc = ADL_OK;
  if (set->d_bitmaps && hipFree(set->d_bitmaps) != hipSuccess) rc = ADL_ERR_DEVICE;
  if (set->d_off && hipFree(set->d_off) != hipSuccess) rc = ADL_ERR_DEVICE;
  delete set;
  return rc;
}

}  // extern "C"
