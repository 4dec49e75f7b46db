// adlsm-tree_amd/csrc/probe_binned.hip -- MI355X (gfx950) tile-binned probe
// for large multi-filter batches (BASELINE.json configs[4]: 100M queries
// against 256 device-resident filters).
//
// Same answers as bloom_probe_multi_kernel, i.e. BloomFilter::IsKeyExists
// (reference src/filter_block.cpp:49-62) per query against filter fid[i]:
// 1 iff all k bits (h1 + j*h2) mod 2^32 mod m are set.  The reference stops at
// the first clear bit; the answer is the AND of the k bits either way.
//
// Why: the direct kernel makes ~4.4 random bitmap reads per query, each one
// 64-byte fabric request (PMC, profiles/pmc_traffic.json "probe": 449M
// TCC_EA0_RDREQ per 100M queries), and runs at the fabric's random-request
// rate (~55 G/s).  Here the random reads become streaming traffic plus LDS
// lookups, the way the build's pass B turns its bit-sets into LDS atomics:
//
//   K0  per filter: m, the fastmod magic, its 2^20-bit tiles (one launch of
//       one workgroup, from the device offsets)
//   K1  per block of 16K queries: LDS histogram of the filter ids
//   K2  per filter: its queries' start in filter order, its chunks of C
//       queries and its (tile, chunk) table; the per-block histograms become
//       each block's starting slot in every filter's run
//   K3  per block: each query's slot in filter order (dest), and its two
//       murmur hashes stored there: the batch grouped by filter, 8 B a query
//   P1  per chunk (C queries of one filter): the k positions of every query,
//       counting-sorted in LDS by tile, written as u32 entries
//       qlocal << 20 | offset-in-tile; answers initialised to 1
//   P2  per tile (persistent): the tile's 128 KiB of bitmap into LDS, then
//       every chunk's run of entries for the tile gathered and tested there;
//       a clear bit stores 0 into its query's answer (only zeros are stored,
//       so the racing stores of different tiles agree)
//   K6  per query: out[i] = answer[dest[i]]
// Algorithmic traffic per query: 16 B key + 4 B id + 1 B answer; the
// pipeline moves ~130 B of streaming traffic per query instead of ~4.4
// random 64-B requests.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "bloom_common.hpp"

using namespace adl_dev;

namespace {

constexpr int kBlk = 1024;
constexpr uint32_t kQB = 16384;                 // queries per bucketing block (K1, K3)
constexpr uint32_t kQPT = kQB / kBlk;
constexpr uint32_t kTL = 20;                    // tile = 2^20 bits = 128 KiB of LDS
constexpr uint32_t kTileBytes = 1u << (kTL - 3);
constexpr uint32_t kMaxTiles = 2048;            // m < 2^31
constexpr uint32_t kMaxC = 4096;                // entry = qlocal (12 bits) << 20 | offset
constexpr uint32_t kCPT = kMaxC / kBlk;         // queries per thread in P1
constexpr uint32_t kMaxBucketFilters = 4096;    // LDS histograms of K1 / K3
constexpr uint32_t kSentinel = 0xFFFFFFFFu;
constexpr uint32_t kLdsWords = 40960;           // 160 KiB
constexpr uint64_t kMinBinned = 1ull << 20;     // below this the direct kernel wins

struct PFilter {
  uint32_t m, magic, shift, tiles;
  uint32_t tile_base;   // first global tile (K0)
  uint32_t cnt;         // queries (K2a)
  uint32_t qbase;       // first slot in filter order (K2b)
  uint32_t chunk_base;  // first chunk (K2b)
  uint32_t nchunks;     // (K2b)
  uint32_t pad_[3];
  uint64_t byte_off;    // bitmap start in the arena (K0)
  uint64_t table_base;  // first (tile, chunk) table entry (K2b)
};
static_assert(sizeof(PFilter) == 64, "PFilter is 64 B");

struct Plan {
  uint64_t n = 0;
  uint32_t F = 0, k = 0, C = 0, nb = 0;
  uint64_t maxch = 0;
  // workspace byte offsets
  uint64_t o_desc, o_scal, o_hist, o_cf, o_dest, o_hs, o_ent, o_tab, o_res, total;
};

Plan make_plan(uint64_t n, uint32_t F, int32_t bpk) {
  Plan p;
  p.n = n;
  p.F = F;
  p.k = (uint32_t)adl_host::num_probes(bpk);
  // chunk size: k*C entries + the tile histogram fit one workgroup's LDS
  const uint32_t room = kLdsWords - (kMaxTiles + 4) - 64;
  p.C = std::min<uint32_t>(kMaxC, (room / p.k) & ~63u);
  p.nb = (uint32_t)((n + kQB - 1) / kQB);
  p.maxch = (n + p.C - 1) / p.C + F + 1;
  uint64_t o = 0;
  auto take = [&](uint64_t bytes) {
    const uint64_t at = o;
    o = adl_host::round_up(o + bytes, 256);
    return at;
  };
  p.o_desc = take((uint64_t)(F + 1) * sizeof(PFilter));
  p.o_scal = take(256);
  p.o_hist = take((uint64_t)(F + 1) * p.nb * 4);
  p.o_cf = take(p.maxch * 4);
  p.o_dest = take(n * 4);
  p.o_hs = take(n * 8);
  p.o_ent = take(p.maxch * p.k * p.C * 4);
  p.o_tab = take(p.maxch * (kMaxTiles + 1) * 4);
  p.o_res = take(n + 64);
  p.total = o;
  return p;
}

// ---------------------------------------------------------------- K0
__global__ __launch_bounds__(kBlk) void pb_desc_kernel(const uint64_t *__restrict__ off,
                                                       const uint64_t *__restrict__ end, uint32_t F,
                                                       PFilter *__restrict__ desc, uint32_t *__restrict__ scal) {
  __shared__ uint32_t scratch[kBlk / kWave + 1];
  uint32_t carry = 0;
  for (uint32_t f0 = 0; f0 <= F; f0 += kBlk) {
    const uint32_t f = f0 + threadIdx.x;
    PFilter d{};
    if (f < F) {
      const uint64_t b0 = off[f], b1 = end ? end[f] : off[f + 1];
      const uint64_t bytes = b1 > b0 ? b1 - b0 : 0;
      // an empty filter answers 0 (src/filter_block.cpp:50 would divide by
      // zero); a filter of 2^31 bits or more is outside the reference's int m
      if (bytes && bytes * 8 <= 0x7fffffffull) {
        const FastMod fm = fastmod_for((uint32_t)(bytes * 8));
        d.m = fm.m;
        d.magic = fm.magic;
        d.shift = fm.shift;
        d.tiles = (d.m + (1u << kTL) - 1) >> kTL;
        d.byte_off = b0;
      }
    }
    uint32_t total;
    const uint32_t pre = block_excl_scan<kBlk>(f <= F ? d.tiles : 0u, scratch, &total);
    d.tile_base = carry + pre;
    if (f <= F) desc[f] = d;
    carry += total;
  }
  if (threadIdx.x == 0) scal[0] = carry;  // tiles over all filters
}

// bucket of a query: its filter, or F for an id out of range / an unusable filter
__device__ __forceinline__ uint32_t bucket_of(uint32_t f, uint32_t F, const uint32_t *ltiles) {
  return (f < F && ltiles[f]) ? f : F;
}

// ---------------------------------------------------------------- K1
__global__ __launch_bounds__(kBlk) void pb_hist_kernel(const uint32_t *__restrict__ fid, uint64_t n, uint32_t F,
                                                       uint32_t nb, const PFilter *__restrict__ desc,
                                                       uint32_t *__restrict__ hist) {
  extern __shared__ uint32_t lds[];
  uint32_t *lh = lds, *ltiles = lds + F + 1;
  for (uint32_t f = threadIdx.x; f <= F; f += kBlk) {
    lh[f] = 0;
    if (f < F) ltiles[f] = desc[f].tiles;
  }
  __syncthreads();
  const uint64_t i0 = (uint64_t)blockIdx.x * kQB + threadIdx.x;
#pragma unroll
  for (uint32_t r = 0; r < kQPT; ++r) {
    const uint64_t i = i0 + (uint64_t)r * kBlk;
    if (i < n) atomicAdd(&lh[bucket_of(fid[i], F, ltiles)], 1u);
  }
  __syncthreads();
  for (uint32_t f = threadIdx.x; f <= F; f += kBlk) hist[(uint64_t)f * nb + blockIdx.x] = lh[f];
}

// ---------------------------------------------------------------- K2
__global__ __launch_bounds__(256) void pb_rows_kernel(const uint32_t *__restrict__ hist, uint32_t nb,
                                                      PFilter *__restrict__ desc) {
  __shared__ uint32_t red[256];
  const uint32_t f = blockIdx.x;
  uint32_t s = 0;
  for (uint32_t b = threadIdx.x; b < nb; b += 256) s += hist[(uint64_t)f * nb + b];
  red[threadIdx.x] = s;
  __syncthreads();
  for (uint32_t h = 128; h; h >>= 1) {
    if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) desc[f].cnt = red[0];
}

__device__ __forceinline__ uint64_t block_sum64(uint64_t v, uint64_t *red) {
  const uint32_t lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  for (int o = kWave / 2; o; o >>= 1) v += __shfl_xor(v, o, kWave);
  if (lane == 0) red[wave] = v;
  __syncthreads();
  uint64_t t = 0;
  for (uint32_t w = 0; w < kBlk / kWave; ++w) t += red[w];
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(kBlk) void pb_scan_kernel(uint32_t *__restrict__ hist, uint32_t nb, uint32_t F,
                                                       uint32_t C, uint64_t maxch, PFilter *__restrict__ desc,
                                                       uint32_t *__restrict__ chunk_filter, uint32_t *__restrict__ scal) {
  __shared__ uint64_t red[kBlk / kWave];
  __shared__ uint32_t scratch[kBlk / kWave + 1];
  const uint32_t f = blockIdx.x;
  // sums over the filters before f: queries, chunks, table entries
  uint64_t sq = 0, sc = 0, st = 0;
  for (uint32_t g = threadIdx.x; g < f; g += kBlk) {
    const PFilter d = desc[g];
    const uint32_t nc = (d.cnt + C - 1) / C;
    sq += d.cnt;
    sc += nc;
    st += (uint64_t)(d.tiles + 1) * nc;
  }
  sq = block_sum64(sq, red);
  sc = block_sum64(sc, red);
  st = block_sum64(st, red);
  const uint32_t cnt = desc[f].cnt;
  const uint32_t nc = f < F ? (cnt + C - 1) / C : 0u;  // the out-of-range bucket has no chunks
  if (threadIdx.x == 0) {
    desc[f].qbase = (uint32_t)sq;
    desc[f].chunk_base = (uint32_t)sc;
    desc[f].nchunks = nc;
    desc[f].table_base = st;
    if (f == F) scal[1] = (uint32_t)sc;  // chunks over all filters
  }
  for (uint32_t j = threadIdx.x; j < nc; j += kBlk) chunk_filter[sc + j] = f;
  if (f == F)
    for (uint64_t j = sc + threadIdx.x; j < maxch; j += kBlk) chunk_filter[j] = kSentinel;
  // row f: block b's first slot in filter f's run
  const uint32_t per = (nb + kBlk - 1) / kBlk;
  const uint32_t b0 = threadIdx.x * per, b1 = min(b0 + per, nb);
  uint32_t *row = hist + (uint64_t)f * nb;
  uint32_t s = 0;
  for (uint32_t b = b0; b < b1; ++b) s += row[b];
  uint32_t total;
  uint32_t run = (uint32_t)sq + block_excl_scan<kBlk>(s, scratch, &total);
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t v = row[b];
    row[b] = run;
    run += v;
  }
}

// ---------------------------------------------------------------- K3
__global__ __launch_bounds__(kBlk) void pb_scatter_kernel(const uint4 *__restrict__ keys,
                                                          const uint32_t *__restrict__ fid, uint64_t n, uint32_t F,
                                                          uint32_t nb, const PFilter *__restrict__ desc,
                                                          const uint32_t *__restrict__ hist,
                                                          uint32_t *__restrict__ dest, uint2 *__restrict__ hs) {
  extern __shared__ uint32_t lds[];
  uint32_t *cur = lds, *ltiles = lds + F + 1;
  for (uint32_t f = threadIdx.x; f <= F; f += kBlk) {
    cur[f] = hist[(uint64_t)f * nb + blockIdx.x];
    if (f < F) ltiles[f] = desc[f].tiles;
  }
  __syncthreads();
  const uint64_t i0 = (uint64_t)blockIdx.x * kQB + threadIdx.x;
#pragma unroll 4
  for (uint32_t r = 0; r < kQPT; ++r) {
    const uint64_t i = i0 + (uint64_t)r * kBlk;
    if (i < n) {
      const uint32_t b = bucket_of(fid[i], F, ltiles);
      if (b < F) {
        const uint32_t d = atomicAdd(&cur[b], 1u);
        uint32_t h1, h2;
        hash16(load_nt(keys + i), h1, h2);
        hs[d] = make_uint2(h1, h2);
        dest[i] = d;
      } else {
        dest[i] = kSentinel;
      }
    }
  }
}

// ---------------------------------------------------------------- P1
template <int KFIX>
__global__ __launch_bounds__(kBlk) void pb_bin_kernel(const uint2 *__restrict__ hs, const PFilter *__restrict__ desc,
                                                      const uint32_t *__restrict__ chunk_filter, uint32_t k,
                                                      uint32_t C, uint32_t *__restrict__ ent,
                                                      uint32_t *__restrict__ table, uint8_t *__restrict__ res) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t *hist = lds;                          // kMaxTiles + 1 counters, later cursors
  uint32_t *scratch = lds + kMaxTiles + 4;       // scan scratch (64 words)
  uint32_t *lpos = scratch + 64;                 // k*C sorted entries
  const uint32_t f = chunk_filter[blockIdx.x];
  if (f == kSentinel) return;  // past the last chunk
  const PFilter d = desc[f];
  const uint32_t j = blockIdx.x - d.chunk_base;
  const uint32_t q0 = d.qbase + j * C;
  const uint32_t cnt = min(C, d.cnt - j * C);
  const uint32_t T = d.tiles;
  const FastMod mod{d.m, d.magic, d.shift, 0u};
  const uint32_t kk = KFIX > 0 ? (uint32_t)KFIX : k;
  const int tid = threadIdx.x;
  for (uint32_t t = tid; t <= T; t += kBlk) hist[t] = 0;
  uint32_t h1[kCPT], h2[kCPT];
#pragma unroll
  for (uint32_t r = 0; r < kCPT; ++r) {
    const uint32_t q = tid + r * kBlk;
    h1[r] = h2[r] = 0;
    if (q < cnt) {
      const uint2 h = hs[q0 + q];
      h1[r] = h.x;
      h2[r] = h.y;
      res[q0 + q] = 1;
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < kCPT; ++r) {
    if (tid + r * kBlk < cnt) {
      for (uint32_t jj = 0; jj < kk; ++jj) atomicAdd(&hist[fastmod(h1[r] + jj * h2[r], mod) >> kTL], 1u);
    }
  }
  __syncthreads();
  const uint32_t total = block_excl_scan_array<kBlk>(hist, T + 1, scratch);
  uint32_t *tab = table + d.table_base;
  for (uint32_t t = tid; t <= T; t += kBlk) tab[(uint64_t)t * d.nchunks + j] = hist[t];
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < kCPT; ++r) {
    const uint32_t q = tid + r * kBlk;
    if (q < cnt) {
      for (uint32_t jj = 0; jj < kk; ++jj) {
        const uint32_t p = fastmod(h1[r] + jj * h2[r], mod);
        const uint32_t slot = atomicAdd(&hist[p >> kTL], 1u);
        lpos[slot] = (q << kTL) | (p & ((1u << kTL) - 1u));
      }
    }
  }
  __syncthreads();
  uint32_t *dst = ent + (uint64_t)blockIdx.x * k * C;
  const uint32_t nvec = total >> 2;
  const uint4 *src4 = reinterpret_cast<const uint4 *>(lpos);
  uint4 *dst4 = reinterpret_cast<uint4 *>(dst);
  for (uint32_t v = tid; v < nvec; v += kBlk) dst4[v] = src4[v];
  for (uint32_t v = (nvec << 2) + tid; v < total; v += kBlk) dst[v] = lpos[v];
}

// ---------------------------------------------------------------- P2
__global__ __launch_bounds__(kBlk) void pb_tile_kernel(const uint8_t *__restrict__ bitmaps,
                                                       const PFilter *__restrict__ desc, uint32_t F,
                                                       const uint32_t *__restrict__ scal, uint32_t k, uint32_t C,
                                                       const uint32_t *__restrict__ ent,
                                                       const uint32_t *__restrict__ table,
                                                       uint8_t *__restrict__ res) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t *ltile = lds;  // kTileBytes + 32 bytes: the tile's bitmap bytes from a 16-byte-aligned start
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  constexpr int NW = kBlk / kWave;
  const uint32_t total_tiles = scal[0];
  const uint32_t G = gridDim.x;
  // consecutive tiles (whose runs share cache lines in every chunk region)
  // go to one XCD; speed only
  const uint32_t slot = (G % 8 == 0) ? (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8 : blockIdx.x;
  for (uint32_t g = slot; g < total_tiles; g += G) {
    // the filter holding global tile g: the last f with tile_base <= g
    uint32_t lo = 0, hi = F;  // desc[F].tile_base = total_tiles > g
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (desc[mid].tile_base <= g) lo = mid; else hi = mid;
    }
    const PFilter d = desc[lo];
    const uint32_t t = g - d.tile_base;
    // bitmap bytes [s, e) of the tile, staged from a0 = s rounded down to 16
    const uint64_t s = d.byte_off + (uint64_t)t * kTileBytes;
    const uint64_t e = min(s + kTileBytes, d.byte_off + (uint64_t)(d.m >> 3));
    const uint64_t a0 = s & ~15ull;
    const uint32_t sh = (uint32_t)(s - a0) * 8u;  // bit offset of the tile in ltile
    const uint32_t nvec = (uint32_t)((e - a0) >> 4);
    const uint4 *src = reinterpret_cast<const uint4 *>(bitmaps + a0);
    uint4 *l4 = reinterpret_cast<uint4 *>(ltile);
    __syncthreads();  // the previous tile's lookups are done
    for (uint32_t v = tid; v < nvec; v += kBlk) l4[v] = load_nt(src + v);
    const uint32_t tail = (uint32_t)(e - a0) & 15u;
    if ((uint32_t)tid < tail)
      reinterpret_cast<uint8_t *>(ltile)[nvec * 16 + tid] = bitmaps[a0 + nvec * 16 + tid];
    __syncthreads();
    // every chunk's run for this tile: wave w takes chunks w, w + 16, ...
    const uint32_t nc = d.nchunks;
    const uint32_t *row = table + d.table_base + (uint64_t)t * nc;
    for (uint32_t jc = wave; jc < nc; jc += NW) {
      const uint32_t b0 = __builtin_amdgcn_readfirstlane(row[jc]);
      const uint32_t b1 = __builtin_amdgcn_readfirstlane(row[nc + jc]);
      const uint32_t *run = ent + (uint64_t)(d.chunk_base + jc) * k * C;
      uint8_t *rq = res + d.qbase + (uint64_t)jc * C;
      for (uint32_t o = b0; o < b1; o += 4 * kWave) {
        uint32_t x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t idx = o + u * kWave + lane;
          x[u] = idx < b1 ? run[idx] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (o + u * kWave + lane < b1) {
            const uint32_t bit = (x[u] & ((1u << kTL) - 1u)) + sh;
            if (!((ltile[bit >> 5] >> (bit & 31)) & 1u)) rq[x[u] >> kTL] = 0;
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------- K6
__global__ __launch_bounds__(256) void pb_gather_kernel(const uint32_t *__restrict__ dest,
                                                        const uint8_t *__restrict__ res, uint64_t n,
                                                        uint8_t *__restrict__ out) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint32_t dd = dest[i];
    out[i] = dd == kSentinel ? 0 : res[dd];
  }
}

bool eligible(uint64_t n, uint32_t F, uint32_t key_stride, const uint8_t *d_keys, const uint64_t *d_offsets) {
  return !d_offsets && key_stride == 16 && reinterpret_cast<uintptr_t>(d_keys) % 16 == 0 && n >= kMinBinned &&
         n < 0x7fffffffull && F >= 1 && F <= kMaxBucketFilters;
}

}  // namespace

extern "C" {

uint64_t adl_bloom_probe_batch_workspace_bytes(uint64_t n, uint32_t num_filters, int32_t bits_per_key,
                                               uint32_t key_stride) {
  if (bits_per_key < 0) return 0;
  if (key_stride != 16 || n < kMinBinned || n >= 0x7fffffffull || num_filters == 0 ||
      num_filters > kMaxBucketFilters)
    return 256;  // the direct kernel: no workspace
  return make_plan(n, num_filters, bits_per_key).total + 256;
}

int adl_bloom_probe_batch_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n, uint32_t key_stride,
                                 const uint32_t *d_filter_id, uint32_t num_filters, const uint8_t *d_bitmaps,
                                 const uint64_t *d_bitmap_off, const uint64_t *d_bitmap_end, int32_t bits_per_key,
                                 uint8_t *d_out, void *d_workspace, uint64_t workspace_bytes, void *stream) {
  if (n == 0) return ADL_OK;
  if (!d_keys || !d_filter_id || !d_out || bits_per_key < 0) return ADL_ERR_INVALID_ARG;
  if (num_filters && (!d_bitmaps || !d_bitmap_off)) return ADL_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (!eligible(n, num_filters, key_stride, d_keys, d_offsets)) {
    if (d_bitmap_end)
      return adl_bloom_probe_ranges_device(d_keys, d_offsets, n, key_stride, d_filter_id, num_filters, d_bitmaps,
                                           d_bitmap_off, d_bitmap_end, bits_per_key, d_out, stream);
    return adl_bloom_probe_multi_device(d_keys, d_offsets, n, key_stride, d_filter_id, num_filters, d_bitmaps,
                                        d_bitmap_off, bits_per_key, d_out, stream);
  }
  const Plan p = make_plan(n, num_filters, bits_per_key);
  if (!d_workspace || workspace_bytes < p.total + 256) return ADL_ERR_WORKSPACE;
  uint8_t *ws = reinterpret_cast<uint8_t *>(adl_host::round_up(reinterpret_cast<uintptr_t>(d_workspace), 256));
  PFilter *desc = reinterpret_cast<PFilter *>(ws + p.o_desc);
  uint32_t *scal = reinterpret_cast<uint32_t *>(ws + p.o_scal);
  uint32_t *hist = reinterpret_cast<uint32_t *>(ws + p.o_hist);
  uint32_t *cf = reinterpret_cast<uint32_t *>(ws + p.o_cf);
  uint32_t *dest = reinterpret_cast<uint32_t *>(ws + p.o_dest);
  uint2 *hs = reinterpret_cast<uint2 *>(ws + p.o_hs);
  uint32_t *ent = reinterpret_cast<uint32_t *>(ws + p.o_ent);
  uint32_t *tab = reinterpret_cast<uint32_t *>(ws + p.o_tab);
  uint8_t *res = ws + p.o_res;
  const uint32_t F = num_filters;
  const size_t lds_b = (size_t)(2 * F + 2) * 4;  // K1 / K3: F+1 counters + F tile counts
  try {
    hipLaunchKernelGGL(pb_desc_kernel, dim3(1), dim3(kBlk), 0, st, d_bitmap_off, d_bitmap_end, F, desc, scal);
    ADL_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(pb_hist_kernel, dim3(p.nb), dim3(kBlk), lds_b, st, d_filter_id, n, F, p.nb, desc, hist);
    ADL_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(pb_rows_kernel, dim3(F + 1), dim3(256), 0, st, hist, p.nb, desc);
    ADL_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(pb_scan_kernel, dim3(F + 1), dim3(kBlk), 0, st, hist, p.nb, F, p.C, p.maxch, desc, cf, scal);
    ADL_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(pb_scatter_kernel, dim3(p.nb), dim3(kBlk), lds_b, st, reinterpret_cast<const uint4 *>(d_keys),
                       d_filter_id, n, F, p.nb, desc, hist, dest, hs);
    ADL_HIP_TRY(hipGetLastError());
    const size_t lds_p1 = (size_t)(kMaxTiles + 4 + 64 + p.k * p.C) * 4;
    auto p1 = p.k == 6 ? pb_bin_kernel<6> : pb_bin_kernel<0>;
    ADL_HIP_TRY(hipFuncSetAttribute((const void *)p1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_p1));
    hipLaunchKernelGGL(p1, dim3((uint32_t)p.maxch), dim3(kBlk), lds_p1, st, hs, desc, cf, p.k, p.C, ent, tab, res);
    ADL_HIP_TRY(hipGetLastError());
    const size_t lds_p2 = (size_t)kTileBytes + 64;
    ADL_HIP_TRY(hipFuncSetAttribute((const void *)pb_tile_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds_p2));
    hipLaunchKernelGGL(pb_tile_kernel, dim3(adl_host::device_cus()), dim3(kBlk), lds_p2, st, d_bitmaps, desc, F,
                       scal, p.k, p.C, ent, tab, res);
    ADL_HIP_TRY(hipGetLastError());
    const uint32_t g6 = (uint32_t)std::min<uint64_t>((n + 255) / 256, (uint64_t)adl_host::device_cus() * 16);
    hipLaunchKernelGGL(pb_gather_kernel, dim3(g6), dim3(256), 0, st, dest, res, n, d_out);
    ADL_HIP_TRY(hipGetLastError());
    return ADL_OK;
  } catch (...) {
    return ADL_ERR_DEVICE;
  }
}

}  // extern "C"
