// adlsm-tree_amd/csrc/filter_block_device.hip -- the filter-block container
// framed on the device.
//
// FilterBlockWriter::Final (src/filter_block.cpp:77-102) lays a block out as
//   [bitmap_0][bitmap_1]...[i32 off_0 = 0]...[i32 off_{F-1}]
//   [i32 offsets_start][i32 F]["bf:" i32 bpk][i32 7]
// with every bitmap exactly n_f*bpk+7 bytes, back to back, so bitmap f > 0
// starts at an arbitrary byte offset.  The build kernels write 16-byte-aligned
// bitmaps (their tile write-out is 16-byte stores), so this file builds into
// an aligned staging area of the workspace and then packs: one launch per
// group of up to kPackFilters filters moves the bitmaps to their packed
// offsets (16-byte stores for every output word that lies inside one bitmap,
// a byte-shifted pair of 16-byte loads feeding each; byte stores only at the
// two ends of each bitmap) and writes the group's part of the trailer.  The
// finished block is one contiguous device buffer: one D2H (or one direct
// write to the file) instead of F bitmap copies and host repacking.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "bloom_common.hpp"

namespace {

constexpr uint32_t kPackFilters = 64;  // filters per pack launch (descriptors travel in the kernarg segment)
constexpr int kPackBlock = 256;

struct PackArgs {
  uint32_t nf;              // filters in this launch
  uint32_t first;           // index of the first one in the block
  uint32_t total_filters;   // F
  uint32_t last_group;      // this launch writes the fixed trailer fields
  int32_t bits_per_key;
  uint32_t pad_;
  uint64_t offsets_start;   // byte offset of the i32 offsets array (= sum of bitmap bytes)
  uint64_t word_begin;      // first 16-byte output word this launch covers
  uint64_t words;           // number of 16-byte output words
  uint64_t src_off[kPackFilters];  // aligned staging offset of each bitmap
  uint64_t dst_off[kPackFilters];  // packed offset in the block
  uint64_t bytes[kPackFilters];    // n*bpk+7
};

// Bytes [s, s+16) of the 32-byte concatenation lo|hi (s in 0..15).
__device__ __forceinline__ uint4 shift16(uint4 lo, uint4 hi, uint32_t s) {
  uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  const uint32_t q = s >> 2, r = (s & 3u) * 8u;
  uint32_t o[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {  // o[i] = w[q + i], q uniform per filter
    uint32_t v = w[i];
    v = q == 1 ? w[i + 1] : v;
    v = q == 2 ? w[i + 2] : v;
    v = q == 3 ? w[i + 3] : v;
    o[i] = v;
  }
  if (r == 0) return make_uint4(o[0], o[1], o[2], o[3]);
  return make_uint4(__builtin_amdgcn_alignbyte(o[1], o[0], r >> 3), __builtin_amdgcn_alignbyte(o[2], o[1], r >> 3),
                    __builtin_amdgcn_alignbyte(o[3], o[2], r >> 3), __builtin_amdgcn_alignbyte(o[4], o[3], r >> 3));
}

__device__ __forceinline__ void put32(uint8_t *p, uint32_t v) {  // unaligned little-endian i32
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
  p[2] = (uint8_t)(v >> 16);
  p[3] = (uint8_t)(v >> 24);
}

__global__ __launch_bounds__(kPackBlock) void filter_block_pack_kernel(PackArgs a, const uint8_t *__restrict__ src,
                                                                        uint8_t *__restrict__ block) {
  // trailer: this group's offsets, and the fixed fields from the last group
  if (blockIdx.x == 0) {
    const uint32_t t = threadIdx.x;
    if (t < a.nf) put32(block + a.offsets_start + 4ull * (a.first + t), (uint32_t)a.dst_off[t]);
    if (a.last_group && t == 0) {
      uint8_t *p = block + a.offsets_start + 4ull * a.total_filters;
      put32(p, (uint32_t)a.offsets_start);  // offsets_start
      put32(p + 4, a.total_filters);        // F
      p[8] = 'b';
      p[9] = 'f';
      p[10] = ':';
      put32(p + 11, (uint32_t)a.bits_per_key);
      put32(p + 15, 7u);                    // info_len
    }
  }
  uint4 *out4 = reinterpret_cast<uint4 *>(block);
  const uint4 *src4 = reinterpret_cast<const uint4 *>(src);
  const uint64_t stride = (uint64_t)gridDim.x * kPackBlock;
  uint32_t f = 0;  // filters are in increasing dst order; the word index only grows per thread
  for (uint64_t i = (uint64_t)blockIdx.x * kPackBlock + threadIdx.x; i < a.words; i += stride) {
    const uint64_t o = (a.word_begin + i) * 16;
    while (f + 1 < a.nf && a.dst_off[f] + a.bytes[f] <= o) ++f;
    const uint64_t d = a.dst_off[f], n = a.bytes[f];
    if (o >= d && o + 16 <= d + n) {  // the word lies inside bitmap f
      const uint64_t rel = o - d;
      const uint64_t s = a.src_off[f] + rel;  // src_off is 16-aligned
      const uint32_t sh = (uint32_t)(s & 15u);
      const uint4 lo = src4[s >> 4];
      const uint4 hi = sh ? src4[(s >> 4) + 1] : lo;
      out4[o >> 4] = shift16(lo, hi, sh);
      continue;
    }
    // boundary word: byte stores of exactly the bytes owned by this group's
    // bitmaps (bitmaps f, f+1, ... that start before o+16; a bitmap has at
    // least 7 bytes, so at most 4 of them meet one word)
    for (uint32_t j = 0; j < 16; ++j) {
      const uint64_t p = o + j;
      for (uint32_t g = f; g < a.nf && a.dst_off[g] <= p; ++g) {
        if (p < a.dst_off[g] + a.bytes[g]) {
          block[p] = src[a.src_off[g] + (p - a.dst_off[g])];
          break;
        }
      }
    }
  }
}

struct Layout {
  std::vector<uint64_t> bytes, dst, src;
  uint64_t offsets_start = 0, block_bytes = 0, staging_bytes = 0;
};

int layout(const uint64_t *key_begin, uint32_t nf, int32_t bpk, Layout &L) {
  if (!key_begin || bpk < 0) return ADL_ERR_INVALID_ARG;
  L.bytes.resize(nf);
  L.dst.resize(nf);
  L.src.resize(nf);
  uint64_t dst = 0, src = 0;
  for (uint32_t f = 0; f < nf; ++f) {
    if (key_begin[f + 1] < key_begin[f]) return ADL_ERR_INVALID_ARG;
    const uint64_t b = adl_host::bitmap_bytes(key_begin[f + 1] - key_begin[f], bpk);
    if (!b) return ADL_ERR_TOO_LARGE;
    L.bytes[f] = b;
    L.dst[f] = dst;
    L.src[f] = src;
    dst += b;
    src += adl_host::round_up(b, 16);
  }
  L.offsets_start = dst;
  L.block_bytes = dst + 4ull * nf + 4 + 4 + 7 + 4;  // offsets, offsets_start, F, "bf:"+bpk, info_len
  L.staging_bytes = adl_host::round_up(src, 256);
  if (L.block_bytes > 0x7fffffffull) return ADL_ERR_TOO_LARGE;  // the reference's int offsets
  return ADL_OK;
}

uint64_t build_ws(const uint64_t *key_begin, uint32_t nf, int32_t bpk) {
  if (nf == 0) return 0;
  std::vector<uint64_t> counts(nf);
  for (uint32_t f = 0; f < nf; ++f) counts[f] = key_begin[f + 1] - key_begin[f];
  return adl_bloom_build_workspace_bytes(counts.data(), nf, bpk);
}

}  // namespace

extern "C" {

uint64_t adl_bloom_filter_block_bytes(const uint64_t *key_begin, uint32_t num_filters, int32_t bits_per_key) {
  Layout L;
  return layout(key_begin, num_filters, bits_per_key, L) ? 0 : L.block_bytes;
}

uint64_t adl_bloom_filter_block_workspace_bytes(const uint64_t *key_begin, uint32_t num_filters,
                                                int32_t bits_per_key) {
  Layout L;
  if (layout(key_begin, num_filters, bits_per_key, L)) return 0;
  return L.staging_bytes + 256 + build_ws(key_begin, num_filters, bits_per_key);
}

int adl_bloom_filter_block_build_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint32_t key_stride,
                                        const uint64_t *key_begin, uint32_t num_filters, int32_t bits_per_key,
                                        uint8_t *d_block, uint64_t block_bytes, void *d_workspace,
                                        uint64_t workspace_bytes, void *stream) {
  try {
    Layout L;
    if (int rc = layout(key_begin, num_filters, bits_per_key, L)) return rc;
    if (!d_block || reinterpret_cast<uintptr_t>(d_block) % 16 || block_bytes < L.block_bytes)
      return ADL_ERR_INVALID_ARG;
    const uint64_t need = L.staging_bytes + 256 + build_ws(key_begin, num_filters, bits_per_key);
    if (!d_workspace || workspace_bytes < need) return ADL_ERR_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    uint8_t *staging = reinterpret_cast<uint8_t *>(adl_host::round_up(reinterpret_cast<uintptr_t>(d_workspace), 256));
    uint8_t *bws = staging + L.staging_bytes;
    const uint64_t bws_bytes = workspace_bytes - (uint64_t)(bws - reinterpret_cast<uint8_t *>(d_workspace));
    if (num_filters) {
      const int rc = adl_bloom_build_segmented_device(d_keys, d_offsets, key_stride, key_begin, num_filters,
                                                      bits_per_key, staging, L.src.data(), bws, bws_bytes, stream);
      if (rc) return rc;
    }
    const uint32_t cus = adl_host::device_cus();
    for (uint32_t g = 0; g < num_filters || g == 0; g += kPackFilters) {
      PackArgs a;
      memset(&a, 0, sizeof(a));
      a.nf = std::min<uint32_t>(kPackFilters, num_filters - g);
      a.first = g;
      a.total_filters = num_filters;
      a.last_group = g + kPackFilters >= num_filters;
      a.bits_per_key = bits_per_key;
      a.offsets_start = L.offsets_start;
      for (uint32_t f = 0; f < a.nf; ++f) {
        a.src_off[f] = L.src[g + f];
        a.dst_off[f] = L.dst[g + f];
        a.bytes[f] = L.bytes[g + f];
      }
      if (a.nf) {
        const uint64_t lo = a.dst_off[0], hi = a.dst_off[a.nf - 1] + a.bytes[a.nf - 1];
        a.word_begin = lo / 16;
        a.words = (hi + 15) / 16 - a.word_begin;
      }
      const uint64_t want = std::max<uint64_t>(1, (a.words + kPackBlock - 1) / kPackBlock);
      const uint32_t grid = (uint32_t)std::min<uint64_t>(want, (uint64_t)cus * 8);
      hipLaunchKernelGGL(filter_block_pack_kernel, dim3(grid), dim3(kPackBlock), 0, st, a,
                         (const uint8_t *)staging, d_block);
      ADL_HIP_TRY(hipGetLastError());
      if (num_filters == 0) break;
    }
    return ADL_OK;
  } catch (...) {
    return ADL_ERR_DEVICE;
  }
}

}  // extern "C"
