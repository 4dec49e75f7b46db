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
//   K1  per block of 8K queries: LDS histogram of the filter ids
//   K2  per filter: its queries' start in filter order, its chunks of C
//       queries and its (tile, chunk) table; and each block's starting slot
//       in every filter's run
//   K3  per block: both murmur hashes of every query, counting-sorted by
//       filter in LDS and written out run by run (whole lines) to the
//       query's slot in filter order: the batch grouped by filter, 8 B a
//       query; and the query's place in the block's sorted order (2 B)
//   P1  per chunk (C queries of one filter): the k positions of every query,
//       counting-sorted in LDS by tile, written as u32 entries
//       qlocal << 20 | offset-in-tile; answers initialised to 1
//   P2  per tile (persistent): the tile's 128 KiB of bitmap into LDS, then
//       every chunk's run of entries for the tile gathered and tested there;
//       a clear bit stores 0 into its query's answer (only zeros are stored,
//       so the racing stores of different tiles agree)
//   K6  per block: the block's answers gathered run by run into LDS, then
//       out[i] = answer at the query's place (coalesced throughout)
// Algorithmic traffic per query: 16 B key + 4 B id + 1 B answer; the
// pipeline moves ~130 B of streaming traffic per query instead of ~4.4
// random 64-B requests.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "bloom_common.hpp"

using namespace adl_dev;

namespace {

constexpr int kBlk = 1024;
constexpr uint32_t kQB = 8192;                  // queries per bucketing block (K1, K3, K6)
constexpr uint32_t kQPT = kQB / kBlk;
constexpr uint32_t kTL = 20;                    // tile = 2^20 bits = 128 KiB of LDS
constexpr uint32_t kTileBytes = 1u << (kTL - 3);
constexpr uint32_t kMaxTiles = 2048;            // m < 2^31
constexpr uint32_t kMaxC = 4096;                // entry = qlocal (12 bits) << 20 | offset
constexpr uint32_t kCPT = kMaxC / kBlk;         // queries per thread in P1
constexpr uint32_t kMaxBucketFilters = 4096;    // LDS histograms of K1 / K3
constexpr uint32_t kSentinel = 0xFFFFFFFFu;
constexpr uint16_t kNoSlot = 0xFFFF;            // a query that is answered 0 without probing
constexpr uint32_t kLdsWords = 40960;           // 160 KiB
constexpr uint64_t kMinBinned = 1ull << 20;     // below this the direct kernel wins
constexpr uint32_t kMaxSlots = 1024;            // pb_tile workgroups (the tile split's slots)

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
  uint32_t ng = 0;  // groups of kScanGroup blocks (K2)
  uint64_t o_desc, o_scal, o_cnt, o_start, o_gsum, o_cf, o_dest, o_hs, o_ent, o_tab, o_split, o_res, total;
};

constexpr uint32_t kScanGroup = 64;  // blocks per column-sum group (K2)

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
  p.o_cnt = take((uint64_t)(F + 1) * p.nb * 4);
  p.o_start = take((uint64_t)(F + 1) * p.nb * 4);
  p.ng = (p.nb + kScanGroup - 1) / kScanGroup;
  p.o_gsum = take((uint64_t)(F + 1) * p.ng * 4);
  p.o_cf = take(p.maxch * 4);
  p.o_dest = take(n * 2);
  p.o_hs = take(n * 8);
  p.o_ent = take(p.maxch * p.k * p.C * 4);
  p.o_tab = take(p.maxch * (kMaxTiles + 1) * 4);
  p.o_split = take((kMaxSlots + 1) * 4);
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

// The bucketing block a workgroup of a per-block kernel (K3, K6) takes:
// consecutive blocks on one XCD (workgroup i runs on XCD i % 8), so the runs
// of neighbouring blocks -- adjacent in filter order, sharing the cache line
// where one ends and the next begins -- are written (K3) and read (K6)
// through one L2, which merges the two partial-line writes.  A bijection on
// [0, nb) for any nb.
__device__ __forceinline__ uint32_t xcd_block(uint32_t nb) {
  const uint32_t x = blockIdx.x % 8, i = blockIdx.x / 8, q = nb / 8, r = nb % 8;
  return x * q + min(x, r) + i;
}

// ---------------------------------------------------------------- K1
__global__ __launch_bounds__(kBlk) void pb_hist_kernel(const uint32_t *__restrict__ fid, uint64_t n, uint32_t F,
                                                       uint32_t nb, const PFilter *__restrict__ desc,
                                                       uint32_t *__restrict__ hist) {
  extern __shared__ uint32_t lds[];
  uint32_t *lh = lds, *ltiles = lds + F + 1;
  const uint64_t i0 = (uint64_t)blockIdx.x * kQB + threadIdx.x;
  uint32_t fq[kQPT];  // in flight while the counters are cleared
#pragma unroll
  for (uint32_t r = 0; r < kQPT; ++r) {
    const uint64_t i = i0 + (uint64_t)r * kBlk;
    fq[r] = i < n ? fid[i] : kSentinel;
  }
  for (uint32_t f = threadIdx.x; f <= F; f += kBlk) {
    lh[f] = 0;
    if (f < F) ltiles[f] = desc[f].tiles;
  }
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < kQPT; ++r)
    if (i0 + (uint64_t)r * kBlk < n) atomicAdd(&lh[bucket_of(fq[r], F, ltiles)], 1u);
  __syncthreads();
  // block-major: this block's F+1 counts are one contiguous row
  for (uint32_t f = threadIdx.x; f <= F; f += kBlk) hist[(uint64_t)blockIdx.x * (F + 1) + f] = lh[f];
}

// ---------------------------------------------------------------- K2
// Three launches, every access to the block-major counts a whole-row
// (coalesced) one:
//   K2a  per group of kScanGroup blocks: each filter's count over the group
//   K2b  one workgroup: per filter, the groups' exclusive prefix (in place) and
//        the total; over the filters, query / chunk / table-entry starts; the
//        chunk -> filter map
//   K2c  per group: each block's first slot in every filter's run
__global__ __launch_bounds__(kBlk) void pb_colsum_kernel(const uint32_t *__restrict__ cnt, uint32_t nb, uint32_t F,
                                                         uint32_t *__restrict__ gsum) {
  const uint32_t b0 = blockIdx.x * kScanGroup, b1 = min(b0 + kScanGroup, nb);
  const uint64_t stride = F + 1;
  for (uint32_t f = threadIdx.x; f <= F; f += kBlk) {
    uint32_t s = 0;
    for (uint32_t b = b0; b < b1; ++b) s += cnt[b * stride + f];
    gsum[(uint64_t)blockIdx.x * stride + f] = s;
  }
}

// The tile split for pb_tile's G workgroups: slot s takes global tiles
// [split[s], split[s+1]), a contiguous range holding about 1/G of the work.  A
// tile's work is its bitmap load plus its entries (kTileWork + k x its
// filter's queries / tiles, in 4-byte units): splitting by tile count would
// put several tiles of a hot filter on one workgroup (64 filters with 90 % of
// the queries on one: 1.0 -> 5.5 ms), splitting by work gives a hot tile a
// workgroup of its own (and the workgroups after it none).
constexpr uint64_t kTileWork = kTileBytes / 4;

__global__ __launch_bounds__(kBlk) void pb_plan_kernel(uint32_t *__restrict__ gsum, uint32_t ng, uint32_t F,
                                                       uint32_t C, uint64_t maxch, PFilter *__restrict__ desc,
                                                       uint32_t *__restrict__ chunk_filter,
                                                       uint32_t *__restrict__ scal, uint32_t k, uint32_t G,
                                                       uint32_t *__restrict__ split) {
  __shared__ uint32_t scratch[kBlk / kWave + 1];
  __shared__ uint64_t red[kBlk / kWave];
  __shared__ uint32_t ltb[kMaxBucketFilters + 1], lq[kMaxBucketFilters + 1];  // tile_base, qbase
  const uint64_t stride = F + 1;
  uint64_t cq = 0, cc = 0, ct = 0;  // running query / chunk / table-entry starts over filter blocks
  for (uint32_t f0 = 0; f0 <= F; f0 += kBlk) {
    const uint32_t f = f0 + threadIdx.x;
    uint32_t tot = 0;
    if (f <= F) {
      // the column's group sums, 16 loads in flight at a time (a store between
      // two loads of one array would serialise them)
      constexpr uint32_t U = 16;
      for (uint32_t g0 = 0; g0 < ng; g0 += U) {
        uint32_t v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) v[u] = g0 + u < ng ? gsum[(g0 + u) * stride + f] : 0u;
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
          if (g0 + u < ng) gsum[(g0 + u) * stride + f] = tot;
          tot += v[u];
        }
      }
    }
    const uint32_t tiles = f < F ? desc[f].tiles : 0u;
    const uint32_t nc = f < F ? (tot + C - 1) / C : 0u;  // the out-of-range bucket has no chunks
    // exclusive prefixes over the filters (64-bit table entries)
    uint32_t all_q, all_c;
    const uint32_t pq = block_excl_scan<kBlk>(f <= F ? tot : 0u, scratch, &all_q);
    const uint32_t pc = block_excl_scan<kBlk>(nc, scratch, &all_c);
    const uint64_t te = (uint64_t)(tiles + 1) * nc;
    // 64-bit exclusive scan of the table entries: wave sums, then the waves before
    const uint32_t lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
    uint64_t incl = te;
    for (int o = 1; o < kWave; o <<= 1) {
      const uint64_t y = __shfl_up(incl, o, kWave);
      if ((int)lane >= o) incl += y;
    }
    if (lane == kWave - 1) red[wave] = incl;
    __syncthreads();
    uint64_t before = 0, all_t = 0;
    for (uint32_t w = 0; w < kBlk / kWave; ++w) {
      if (w < wave) before += red[w];
      all_t += red[w];
    }
    __syncthreads();
    if (f <= F) {
      ltb[f] = desc[f].tile_base;
      lq[f] = (uint32_t)(cq + pq);
      desc[f].cnt = tot;
      desc[f].qbase = (uint32_t)(cq + pq);
      desc[f].chunk_base = (uint32_t)(cc + pc);
      desc[f].nchunks = nc;
      desc[f].table_base = ct + before + incl - te;
      for (uint32_t j = 0; j < nc; ++j) chunk_filter[cc + pc + j] = f;
      if (f == F) scal[1] = (uint32_t)(cc + pc);  // chunks over all filters
    }
    cq += all_q;
    cc += all_c;
    ct += all_t;
  }
  __syncthreads();
  for (uint64_t j = cc + threadIdx.x; j < maxch; j += kBlk) chunk_filter[j] = kSentinel;
  // the work before tile t of filter f (filters in order, a filter's queries
  // spread evenly over its tiles)
  auto work = [&](uint32_t f, uint32_t t) -> uint64_t {
    const uint32_t tiles = ltb[f + 1] - ltb[f], q = lq[f + 1] - lq[f];
    return kTileWork * (ltb[f] + t) + (uint64_t)k * (lq[f] + (tiles ? (uint64_t)t * q / tiles : 0u));
  };
  const uint64_t wtot = work(F, 0);  // (filter F, the out-of-range bucket, has no tiles)
  for (uint32_t s = threadIdx.x; s <= G; s += kBlk) {
    uint32_t g = 0;  // the first tile whose work starts at or after s / G of the total
    if (s == G) {
      g = ltb[F];
    } else if (s && wtot) {
      const uint64_t target = ((uint64_t)s * wtot + G - 1) / G;  // >= 1
      uint32_t lo = 0, hi = F;  // work(lo, 0) < target <= work(hi, 0)
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (work(mid, 0) < target) lo = mid; else hi = mid;
      }
      uint32_t tl = 0, th = ltb[lo + 1] - ltb[lo];  // work(lo, tl) < target <= work(lo, th)
      while (th - tl > 1) {
        const uint32_t mid = (tl + th) >> 1;
        if (work(lo, mid) < target) tl = mid; else th = mid;
      }
      g = ltb[lo] + th;
    }
    split[s] = g;
  }
}

__global__ __launch_bounds__(kBlk) void pb_starts_kernel(const uint32_t *__restrict__ cnt,
                                                         const uint32_t *__restrict__ gsum, uint32_t nb, uint32_t F,
                                                         const PFilter *__restrict__ desc,
                                                         uint32_t *__restrict__ start) {
  const uint32_t b0 = blockIdx.x * kScanGroup, b1 = min(b0 + kScanGroup, nb);
  const uint64_t stride = F + 1;
  for (uint32_t f = threadIdx.x; f <= F; f += kBlk) {
    uint32_t run = desc[f].qbase + gsum[(uint64_t)blockIdx.x * stride + f];
    for (uint32_t b = b0; b < b1; ++b) {
      start[b * stride + f] = run;
      run += cnt[b * stride + f];
    }
  }
}

// A block's runs: filter f's queries of block b go to slots [lstart[f],
// lstart[f] + lcnt[f]) in filter order and to places [lbase[f], ...) of the
// block's own sorted order.  Loads lcnt, lstart (and ltiles) and scans lbase.
template <int BLK = kBlk>
__device__ __forceinline__ void load_runs(const uint32_t *cnt, const uint32_t *start, uint32_t b, uint32_t F,
                                          const PFilter *desc, uint32_t *lcnt, uint32_t *lstart, uint32_t *lbase,
                                          uint32_t *ltiles, uint32_t *scratch) {
  const uint64_t row = (uint64_t)b * (F + 1);  // block-major
  for (uint32_t f = threadIdx.x; f <= F; f += BLK) {
    const uint32_t c = cnt[row + f];
    lcnt[f] = c;
    lbase[f] = c;
    lstart[f] = start[row + f];
    if (ltiles && f < F) ltiles[f] = desc[f].tiles;
  }
  __syncthreads();
  block_excl_scan_array<BLK>(lbase, F + 1, scratch);
}

// ---------------------------------------------------------------- K3
__global__ __launch_bounds__(kBlk) void pb_scatter_kernel(const uint4 *__restrict__ keys,
                                                          const uint32_t *__restrict__ fid, uint64_t n, uint32_t F,
                                                          uint32_t nb, const PFilter *__restrict__ desc,
                                                          const uint32_t *__restrict__ cnt,
                                                          const uint32_t *__restrict__ start,
                                                          uint16_t *__restrict__ dest, uint2 *__restrict__ hs,
                                                          uint32_t exp) {
#ifndef ADL_BLOOM_STAMPS
  exp = 0;  // diagnostics build only (wrong answers): 8 no hashing, 16 no run stores, 32 no place stores
#endif
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint2 *lhs = reinterpret_cast<uint2 *>(lds);  // kQB hashes in the block's filter order
  uint32_t *lcnt = lds + 2 * kQB, *lstart = lcnt + F + 1, *lbase = lstart + F + 1, *lcur = lbase + F + 1;
  uint32_t *ltiles = lcur + F + 1, *scratch = ltiles + F + 1;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  // every query's id and key are requested first (unconditionally: a lane
  // past n loads the last query and discards it), so they land while the
  // block's runs are set up
  const uint32_t blk = xcd_block(nb);
  const uint64_t i0 = (uint64_t)blk * kQB + tid;
  uint32_t fq[kQPT];
  uint4 kq[kQPT];
#pragma unroll
  for (uint32_t r = 0; r < kQPT; ++r) {
    const uint64_t i = min(i0 + (uint64_t)r * kBlk, n - 1);
    fq[r] = fid[i];
    kq[r] = load_nt(keys + i);
  }
  load_runs(cnt, start, blk, F, desc, lcnt, lstart, lbase, ltiles, scratch);
  for (uint32_t f = tid; f <= F; f += kBlk) lcur[f] = lbase[f];
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < kQPT; ++r) {
    const uint64_t i = i0 + (uint64_t)r * kBlk;
    if (i < n) {
      const uint32_t b = bucket_of(fq[r], F, ltiles);
      uint16_t place = kNoSlot;
      if (b < F) {
        place = (uint16_t)atomicAdd(&lcur[b], 1u);
        uint32_t h1, h2;
        if (exp & 8) {
          h1 = kq[r].x;
          h2 = kq[r].y;
        } else {
          hash16(kq[r], h1, h2);
        }
        lhs[place] = make_uint2(h1, h2);
      }
      if (!(exp & 32)) dest[i] = place;
    }
  }
  __syncthreads();
  if (exp & 16) return;
  // run by run: consecutive lanes write consecutive slots (whole lines);
  // place by place (every lane of a store carrying one) measured the same
  // (profiles/r04/probe_flat_k3.log), and pieces of 64 slots dealt to the
  // waves round robin (one search per piece) 61 % slower
  // (profiles/r05/rejected/probe_k3_pieces.log)
  for (uint32_t f = wave; f < F; f += kBlk / kWave) {
    const uint32_t c = lcnt[f], lb = lbase[f], gs = lstart[f];
    for (uint32_t r = lane; r < c; r += kWave) hs[gs + r] = lhs[lb + r];
  }
}

// ---------------------------------------------------------------- P1
// Persistent: workgroup b takes chunks b, b + G, ...; the next chunk's hashes
// are in flight into registers while the current one is sorted and stored.
// All k bits of every query are binned in one round (the reference stops at
// the first clear bit, src/filter_block.cpp:54-59; the answer is the AND
// either way, and a two-round form measured slower: HISTORY.md).  KFIX = 0:
// runtime k.
template <int KFIX>
__global__ __launch_bounds__(kBlk) void pb_bin_kernel(const uint2 *__restrict__ hs, const PFilter *__restrict__ desc,
                                                      const uint32_t *__restrict__ chunk_filter,
                                                      const uint32_t *__restrict__ scal, uint32_t k, uint32_t C,
                                                      uint32_t *__restrict__ ent, uint32_t *__restrict__ table,
                                                      uint8_t *__restrict__ res, uint32_t exp) {
#ifndef ADL_BLOOM_STAMPS
  exp = 0;  // diagnostics build only (wrong answers): 64 no entry stores, 128 no scatter (count only), 256 no count
#endif
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t *hist = lds;                          // kMaxTiles + 1 counters, later cursors
  uint32_t *scratch = lds + kMaxTiles + 4;       // scan scratch (64 words)
  uint32_t *lpos = scratch + 64;                 // k*C sorted entries
  const uint32_t kk = KFIX > 0 ? (uint32_t)KFIX : k;
  constexpr int KR = KFIX > 0 ? KFIX : 1;
  const int tid = threadIdx.x;
  const uint32_t total_chunks = scal[1];
  const uint32_t G = gridDim.x;
  // answers are one "cleared" bit per slot (1: a tested bit was clear, the answer is 0)
  uint32_t *clrw = reinterpret_cast<uint32_t *>(res);
  auto fetch = [&](uint32_t c, uint2 (&h)[kCPT]) {
    if (c >= total_chunks) return;
    const uint32_t f = chunk_filter[c];
    const uint32_t j = c - desc[f].chunk_base;
    const uint32_t q0 = desc[f].qbase + j * C;
    const uint32_t cnt = min(C, desc[f].cnt - j * C);
#pragma unroll
    for (uint32_t r = 0; r < kCPT; ++r) h[r] = hs[q0 + min(tid + r * kBlk, cnt - 1u)];
  };
  uint2 nxt[kCPT];
  fetch(blockIdx.x, nxt);
  for (uint32_t c = blockIdx.x; c < total_chunks; c += G) {
    uint2 cur[kCPT];
    bool live[kCPT];
#pragma unroll
    for (uint32_t r = 0; r < kCPT; ++r) cur[r] = nxt[r], live[r] = true;
    fetch(c + G, nxt);
    const uint32_t f = chunk_filter[c];
    const PFilter d = desc[f];
    const uint32_t j = c - d.chunk_base;
    const uint32_t q0 = d.qbase + j * C;
    const uint32_t cnt = min(C, d.cnt - j * C);
    const uint32_t T = d.tiles;
    const FastMod mod{d.m, d.magic, d.shift, 0u};
    __syncthreads();  // the previous chunk's entries are read out of lpos
    for (uint32_t t = tid; t <= T; t += kBlk) hist[t] = 0;
    // the chunk's cleared bits start at 0 (the words it shares with its
    // neighbours are zeroed by both, before any pb_tile)
    if (cnt)
      for (uint32_t wd = (q0 >> 5) + tid; wd <= ((q0 + cnt - 1u) >> 5); wd += kBlk) clrw[wd] = 0u;
#pragma unroll
    for (uint32_t r = 0; r < kCPT; ++r) live[r] = live[r] && tid + r * kBlk < cnt;
    __syncthreads();
    uint32_t *dst = ent + (uint64_t)c * k * C;
    if (T == 1) {
      // A filter of one tile (under 2^20 bits): the chunk's run is all of its
      // entries, in query order -- no count, scan or atomics (a counting sort
      // into one bucket serialises every wave's 64 atomics on one address).
#pragma unroll
      for (uint32_t r = 0; r < kCPT; ++r) {
        if (live[r]) {
          const uint32_t q = tid + r * kBlk;
          for (uint32_t jj = 0; jj < kk; ++jj)
            lpos[q * kk + jj] = (q << kTL) | (fastmod(cur[r].x + jj * cur[r].y, mod) & ((1u << kTL) - 1u));
        }
      }
      const uint32_t total = cnt * kk;
      if (tid == 0) {
        table[d.table_base + j] = 0u;                 // tile 0 starts at 0
        table[d.table_base + d.nchunks + j] = total;  // the row after the last tile: the total
      }
      __syncthreads();
      const uint32_t nvec = total >> 2;
      const uint4 *src4 = reinterpret_cast<const uint4 *>(lpos);
      uint4 *dst4 = reinterpret_cast<uint4 *>(dst);
      for (uint32_t v = tid; v < nvec; v += kBlk) dst4[v] = src4[v];
      for (uint32_t v = (nvec << 2) + tid; v < total; v += kBlk) dst[v] = lpos[v];
      continue;
    }
    uint32_t pos[kCPT][KR];
#pragma unroll
    for (uint32_t r = 0; r < kCPT; ++r) {
      if (live[r]) {
        if constexpr (KFIX > 0) {
#pragma unroll
          for (int jj = 0; jj < KFIX; ++jj) {
            pos[r][jj] = fastmod(cur[r].x + (uint32_t)jj * cur[r].y, mod);
            if (!(exp & 256)) atomicAdd(&hist[pos[r][jj] >> kTL], 1u);
          }
        } else {
          for (uint32_t jj = 0; jj < kk; ++jj) atomicAdd(&hist[fastmod(cur[r].x + jj * cur[r].y, mod) >> kTL], 1u);
        }
      }
    }
    __syncthreads();
    const uint32_t total = block_excl_scan_array_1b<kBlk>(hist, T + 1, scratch);
    uint32_t *tab = table + d.table_base;
    for (uint32_t t = tid; t <= T; t += kBlk) tab[(uint64_t)t * d.nchunks + j] = hist[t];
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < kCPT; ++r) {
      const uint32_t q = tid + r * kBlk;
      if (live[r] && !(exp & 128)) {
        if constexpr (KFIX > 0) {
          uint32_t sl[KFIX];
#pragma unroll
          for (int jj = 0; jj < KFIX; ++jj) sl[jj] = atomicAdd(&hist[pos[r][jj] >> kTL], 1u);
#pragma unroll
          for (int jj = 0; jj < KFIX; ++jj) lpos[sl[jj]] = (q << kTL) | (pos[r][jj] & ((1u << kTL) - 1u));
        } else {
          for (uint32_t jj = 0; jj < kk; ++jj) {
            const uint32_t p = fastmod(cur[r].x + jj * cur[r].y, mod);
            const uint32_t slot = atomicAdd(&hist[p >> kTL], 1u);
            lpos[slot] = (q << kTL) | (p & ((1u << kTL) - 1u));
          }
        }
      }
    }
    __syncthreads();
    const uint32_t nvec = total >> 2;
    const uint4 *src4 = reinterpret_cast<const uint4 *>(lpos);
    uint4 *dst4 = reinterpret_cast<uint4 *>(dst);
    if (exp & 64) continue;
    for (uint32_t v = tid; v < nvec; v += kBlk) dst4[v] = src4[v];
    for (uint32_t v = (nvec << 2) + tid; v < total; v += kBlk) dst[v] = lpos[v];
  }
}

// ---------------------------------------------------------------- P2
// Persistent: each workgroup takes a contiguous range of tiles of about equal
// work (pb_plan's split; consecutive ranges on one XCD).  The next tile's bitmap
// bytes are in flight into registers while the current tile's runs are
// tested; each wave stages the (start, end) of all its chunks' runs in two
// registers at the tile's start and keeps two runs' loads in flight.
constexpr uint32_t kTileVecPT = kTileBytes / 16 / kBlk;  // 16-byte tile vectors per thread
constexpr int kRunLoads = 6;                             // entries per run per stage: 6 x 64 (runs average ~320)
constexpr uint32_t kMaskW64 = (kMaxC + 63) / 64 + 1;     // a wave's cleared-bit mask of one chunk (+ its shift), u64 words
constexpr int kRegRuns = 8;                               // runs per wave whose masks accumulate over a filter's tiles
constexpr uint32_t kMaskWords = 2 * kMaskW64 + 2 * kRegRuns;  // + word 64 of each accumulated mask

struct TileRef {
  uint32_t f, t, sh, nvec, tail;
  uint64_t a0;
};

// ltb: the filters' tile_base in LDS (F+1 entries)
__device__ __forceinline__ TileRef tile_ref(const PFilter *desc, const uint32_t *ltb, uint32_t F, uint32_t g) {
  uint32_t lo = 0, hi = F;  // the last f with tile_base <= g (tile_base[F] = all tiles > g)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ltb[mid] <= g) lo = mid; else hi = mid;
  }
  TileRef r;
  r.f = lo;
  r.t = g - ltb[lo];
  const uint64_t base = desc[lo].byte_off;
  const uint64_t s = base + (uint64_t)r.t * kTileBytes;
  const uint64_t e = min(s + kTileBytes, base + (uint64_t)(desc[lo].m >> 3));
  r.a0 = s & ~15ull;
  r.sh = (uint32_t)(s - r.a0) * 8u;
  r.nvec = (uint32_t)((e - r.a0) >> 4);
  r.tail = (uint32_t)(e - r.a0) & 15u;
  return r;
}

__global__ __launch_bounds__(kBlk) void pb_tile_kernel(const uint8_t *__restrict__ bitmaps,
                                                       const PFilter *__restrict__ desc, uint32_t F, uint32_t k,
                                                       uint32_t C, const uint32_t *__restrict__ ent,
                                                       const uint32_t *__restrict__ table,
                                                       const uint32_t *__restrict__ split,
                                                       uint8_t *__restrict__ res, uint32_t exp) {
#ifndef ADL_BLOOM_STAMPS
  exp = 0;  // diagnostics build only (wrong answers): 1 no answer stores, 2 no bitmap loads, 4 no entry loads
#endif
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t *ltile = lds;  // the tile's bitmap bytes from a 16-byte-aligned start (+ <= 15 bytes before it)
  uint32_t *ltb = lds + (kTileBytes + 64) / 4;  // the filters' first tiles (F+1), for the tile -> filter search
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  // A clear bit sets its query's "cleared" bit.  Each wave gathers the bits
  // of the run (one chunk) it is testing in a private LDS mask of the chunk's
  // 4 096 slots (shifted by the chunk's first slot mod 64).  When the wave
  // moves to its next run, the mask goes into the wave's registers: lane l
  // holds word l of the masks of the wave's first kRegRuns runs (the same
  // chunks in every tile of a filter, since a workgroup takes a contiguous
  // range of tiles, mostly of one filter).  The registers are ORed into the
  // global bit array with coalesced 64-bit device-scope atomics only when the
  // workgroup moves on to another filter: about one flush per chunk and
  // workgroup instead of one per (tile, chunk) run (round 5: the run-by-run
  // flushes were ~1 GB of memory-side atomic traffic per 100 M queries).
  // Runs past the first kRegRuns of a wave flush at their end as before.
  unsigned long long *clr64 = reinterpret_cast<unsigned long long *>(res);  // (the workspace area is 256-B aligned)
  uint32_t *zmaskw = lds + (kTileBytes + 64) / 4 + ((F + 1 + 3) & ~3u) + (uint32_t)wave * kMaskWords;  // 8-B aligned
  unsigned long long *zmask64 = reinterpret_cast<unsigned long long *>(zmaskw);
  for (uint32_t w = (uint32_t)lane; w < kMaskWords; w += kWave) zmaskw[w] = 0u;
  unsigned long long rmask[kRegRuns];  // lane l: word l of run slot i's mask
  unsigned long long *rmx = zmask64 + kMaskW64;  // word 64 of run slot i's mask (LDS, lane 0)
#pragma unroll
  for (int i = 0; i < kRegRuns; ++i) rmask[i] = 0ull;
  auto flush_run = [&](uint32_t rq) {
#pragma unroll
    for (uint32_t k2 = 0; k2 < 2; ++k2) {
      const uint32_t w = (uint32_t)lane + k2 * kWave;
      if (w < kMaskW64) {
        const unsigned long long v = zmask64[w];
        if (v) {
          atomicOr(&clr64[(rq >> 6) + w], v);
          zmask64[w] = 0ull;
        }
      }
    }
  };
  constexpr int NW = kBlk / kWave;
  for (uint32_t f = tid; f <= F; f += kBlk) ltb[f] = desc[f].tile_base;
  __syncthreads();
  const uint32_t G = gridDim.x;
  const uint32_t slot = (G % 8 == 0) ? (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8 : blockIdx.x;
  uint4 pre[kTileVecPT];
  auto prefetch = [&](const TileRef &r) {
    const uint4 *src = reinterpret_cast<const uint4 *>(bitmaps + r.a0);
#pragma unroll
    for (uint32_t u = 0; u < kTileVecPT; ++u) {
      const uint32_t v = tid + u * kBlk;
      pre[u] = (v < r.nvec && !(exp & 2)) ? load_nt(src + v) : make_uint4(0, 0, 0, 0);
    }
  };
  // The first 64 runs of this wave in a tile: lane q holds run q's (start,
  // end) from the (tile, chunk) table.  They are loaded with the tile's
  // bitmap, one tile ahead, so a tile starts with no table round trip.
  const uint32_t wv = __builtin_amdgcn_readfirstlane((uint32_t)wave);  // (SGPR: the stage cursor below is scalar)
  uint32_t pre_rs = 0, pre_re = 0;
  // A tile of a filter with fewer chunks than waves would leave waves idle
  // while a few process its long runs: each run is then cut into `split`
  // equal parts (virtual runs v = jc * split + part), dealt to the waves like
  // runs.  A wave flushes its mask at the end of each part, so parts of one
  // chunk on several waves OR their cleared bits into the same words.
  auto split_of = [](uint32_t nc) { return nc && nc < (uint32_t)NW ? (uint32_t)NW / nc : 1u; };
  // virtual run v's (start, end) from the (tile, chunk) table row
  // (split == 1, the common case, takes the plain row loads: no division)
  auto vrun = [](const uint32_t *row, uint32_t nc, uint32_t split, uint32_t v, uint32_t &rs, uint32_t &re) {
    if (split == 1) {
      rs = row[v];
      re = row[nc + v];
      return;
    }
    const uint32_t jc = v / split, part = v - jc * split;
    const uint32_t s0 = row[jc], e0 = row[nc + jc], len = e0 - s0;
    rs = s0 + (len * part) / split;  // len < 2^16, part < split <= 16: no overflow
    re = s0 + (len * (part + 1)) / split;
  };
  auto prefetch_rows = [&](const TileRef &r) {
    const PFilter &dn = desc[r.f];
    const uint32_t nc = dn.nchunks, split = split_of(nc), nvr = nc * split;
    const uint32_t nq = nvr > wv ? (nvr - wv + NW - 1) / NW : 0u;
    if (nq) {
      const uint32_t *row = table + dn.table_base + (uint64_t)r.t * nc;
      vrun(row, nc, split, wv + NW * min((uint32_t)lane, min((uint32_t)kWave, nq) - 1u), pre_rs, pre_re);
    }
  };
  // this workgroup's tiles: a contiguous range of about 1/G of the work
  // (pb_plan's split; mostly one filter's tiles, so the register masks above
  // accumulate over all of them)
  const uint32_t gb = split[slot], ge = split[slot + 1];
  // the filter whose chunks the register masks hold, and what locates them
  uint32_t mf = ~0u, m_qbase = 0, m_split = 1, m_nq = 0;
  auto flush_regs = [&]() {
#pragma unroll
    for (int i = 0; i < kRegRuns; ++i) {
      if ((uint32_t)i < m_nq) {
        const uint32_t v = wv + NW * (uint32_t)i;
        const uint32_t jc = m_split == 1 ? v : v / m_split;
        const uint32_t rq = m_qbase + jc * C;
        if (rmask[i]) atomicOr(&clr64[(rq >> 6) + lane], rmask[i]);
        if (lane == 0 && rmx[i]) {
          atomicOr(&clr64[(rq >> 6) + kWave], rmx[i]);
          rmx[i] = 0ull;
        }
      }
      rmask[i] = 0ull;
    }
  };
  // the run in slot qi of this wave ends: its LDS mask into the registers (or,
  // past the register slots, straight to the global array)
  auto retire_run = [&](uint32_t qi, uint32_t rq) {
    if (qi >= (uint32_t)kRegRuns) {
      flush_run(rq);
      return;
    }
    const unsigned long long v = zmask64[lane];
    zmask64[lane] = 0ull;
    if (lane == 0) {
      rmx[qi] |= zmask64[kWave];
      zmask64[kWave] = 0ull;
    }
#pragma unroll
    for (int i = 0; i < kRegRuns; ++i)
      if ((uint32_t)i == qi) rmask[i] |= v;
  };
  static_assert(kMaskW64 == kWave + 1, "a chunk mask is kWave words plus one");
  TileRef cur{};
  if (gb < ge) {
    cur = tile_ref(desc, ltb, F, gb);
    prefetch(cur);
    prefetch_rows(cur);
  }
  for (uint32_t g = gb; g < ge; ++g) {
    __syncthreads();  // the previous tile's lookups are done
    uint4 *l4 = reinterpret_cast<uint4 *>(ltile);
#pragma unroll
    for (uint32_t u = 0; u < kTileVecPT; ++u) {
      const uint32_t v = tid + u * kBlk;
      if (v < cur.nvec) l4[v] = pre[u];
    }
    if ((uint32_t)tid < cur.tail)
      reinterpret_cast<uint8_t *>(ltile)[cur.nvec * 16 + tid] = bitmaps[cur.a0 + cur.nvec * 16 + tid];
    const TileRef now = cur;
    const uint32_t now_rs = pre_rs, now_re = pre_re;
    if (g + 1 < ge) {
      cur = tile_ref(desc, ltb, F, g + 1);
      prefetch(cur);
      prefetch_rows(cur);
    }
    const PFilter d = desc[now.f];
    const uint32_t nc = d.nchunks, split = split_of(nc), nvr = nc * split;
    const uint32_t *row = table + d.table_base + (uint64_t)now.t * nc;
    // this wave's (virtual) runs: wave + NW*q; lane q holds run q's (start, end)
    const uint32_t nq = nvr > wv ? (nvr - wv + NW - 1) / NW : 0u;
    if (now.f != mf) {  // (wave-uniform) a new filter: the previous one's masks out
      flush_regs();
      mf = now.f;
      m_qbase = d.qbase;
      m_split = split;
      m_nq = nq;
    }
    __syncthreads();  // the tile is in LDS
    // Two-stage pipeline over the wave's runs cut into stages of at most
    // kRunLoads x 64 entries (a long run is several stages): stage s+1's loads
    // are in flight while stage s is tested.  Every stage issues all its loads
    // unconditionally -- past the last run an empty stage re-reads a valid
    // entry -- so the compiler can count them and wait for one stage only.
    struct Stage {
      uint32_t x[kRunLoads];
      uint32_t b0, b1, jc, qi;  // qi: the run's slot in this wave's list
      bool live;  // a stage of a run (possibly empty); false past the batch's last run
    };
    auto issue = [&](Stage &sg, uint32_t b0, uint32_t b1, uint32_t jc, uint32_t qi, bool live) {
      sg.live = live;
      sg.b0 = b0;
      sg.b1 = b1;
      sg.jc = jc;
      sg.qi = qi;
      const uint32_t *run = ent + (uint64_t)(d.chunk_base + jc) * k * C;
#pragma unroll
      for (int u = 0; u < kRunLoads; ++u) {
        const uint32_t idx = b0 + u * kWave + lane;
        // an empty stage reads entry b0 - 1 (or entry 0): inside the workspace, unused
        sg.x[u] = (exp & 4) ? (idx * 2654435761u) & 0x7fffffu : run[min(idx, b1 > 0 ? b1 - 1u : 0u)];
      }
    };
    // all kRunLoads LDS words are read before any is tested (the reads are
    // unconditional -- a lane past the stage holds a clamped entry -- so they
    // issue back to back), then the clear bits go to the zero ring
    auto consume = [&](const Stage &sg, const Stage &nx) {
      const uint32_t rq = d.qbase + sg.jc * C;  // the chunk's first answer (n < 2^31)
      const uint32_t rs = rq & 63u;
      uint32_t w[kRunLoads];
#pragma unroll
      for (int u = 0; u < kRunLoads; ++u) w[u] = ltile[((sg.x[u] & ((1u << kTL) - 1u)) + now.sh) >> 5];
#pragma unroll
      for (int u = 0; u < kRunLoads; ++u) {
        const uint32_t bit = (sg.x[u] & ((1u << kTL) - 1u)) + now.sh;
        // bitwise, not short-circuit: no branch per entry
        const bool clr = (sg.b0 + u * kWave + lane < sg.b1) & (((w[u] >> (bit & 31)) & 1u) == 0u) & !(exp & 1);
        if (clr) {
          const uint32_t b = rs + (sg.x[u] >> kTL);
          atomicOr(&zmaskw[b >> 5], 1u << (b & 31));
        }
      }
      // the run ends here: the next stage is another run's, or past the last
      if (sg.live && (!nx.live || nx.qi != sg.qi)) retire_run(sg.qi, rq);
    };
    for (uint32_t q0 = 0; q0 < nq; q0 += kWave) {
      const uint32_t nr = min((uint32_t)kWave, nq - q0);
      uint32_t rs = now_rs, re = now_re;  // the first 64 runs came with the tile
      if (q0) vrun(row, nc, split, wv + NW * (q0 + min((uint32_t)lane, nr - 1u)), rs, re);
      // the stage cursor: run sq of this batch, entries from so
      uint32_t sq = 0, so = __builtin_amdgcn_readlane(rs, 0);
      auto take = [&](Stage &sg) {
        const bool more = sq < nr;  // wave-uniform
        const uint32_t qe = more ? __builtin_amdgcn_readlane(re, sq) : 0u;
        const uint32_t b0 = more ? so : 0u;
        const uint32_t b1 = more ? min(so + (uint32_t)(kRunLoads * kWave), qe) : 0u;
        const uint32_t qi = q0 + (more ? sq : nr - 1u);
        const uint32_t v = wv + NW * qi;
        const uint32_t jc = split == 1 ? v : v / split;  // the virtual run's chunk
        issue(sg, b0, b1, jc, qi, more);
        if (more) {
          so = b1;
          if (so >= qe) {
            ++sq;
            if (sq < nr) so = __builtin_amdgcn_readlane(rs, sq);
          }
        }
      };
      // An empty run (a chunk with no entry in this tile) is a live stage with
      // nothing to test: the loop ends only past the last run, not at the
      // first empty stage.
      Stage A, B;
      take(A);
      while (A.live) {
        take(B);
        consume(A, B);
        take(A);
        consume(B, A);
      }
    }
  }
  flush_regs();
}

// ---------------------------------------------------------------- K6
// Per block: the answers of its runs, gathered run by run into an LDS bit
// array in the block's sorted order, then out[i] = the bit at the query's
// place (coalesced).  A filter's run of cleared bits is a contiguous range of
// the answer array (filter order); the runs are cut into pieces of 32, and a
// thread reads a piece as a funnel of two words and ORs it into the LDS bits
// at the run's place: about two loads per 32 queries instead of one per
// query, and one search per piece instead of one per query.
// Small workgroups (kGatherBlk threads), so several blocks per CU overlap
// their round trips.
constexpr int kGatherBlk = 256;
__global__ __launch_bounds__(kGatherBlk) void pb_gather_kernel(const uint16_t *__restrict__ dest,
                                                               const uint8_t *__restrict__ res, uint64_t n, uint32_t F,
                                                               uint32_t nb, const uint32_t *__restrict__ cnt,
                                                               const uint32_t *__restrict__ start,
                                                               uint8_t *__restrict__ out) {
  constexpr int B = kGatherBlk;
  constexpr uint32_t QPT = kQB / B;  // queries per thread
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t *lbits = lds;  // kQB cleared bits in the block's sorted order
  uint32_t *lcnt = lds + kQB / 32, *lstart = lcnt + F + 1, *lbase = lstart + F + 1, *lpc = lbase + F + 1;
  uint32_t *scratch = lpc + F + 1;
  const int tid = threadIdx.x;
  const uint32_t *clrw = reinterpret_cast<const uint32_t *>(res);
  // this thread's queries' places (coalesced 16-byte loads: 8 places each),
  // in flight while the block's runs are set up
  const uint32_t blk = xcd_block(nb);
  const uint64_t i0 = (uint64_t)blk * kQB;
  const uint32_t nq = (uint32_t)min((uint64_t)kQB, n - i0);
  uint4 pv[QPT / 8];
#pragma unroll
  for (uint32_t r = 0; r < QPT / 8; ++r) {
    const uint32_t q = (tid + r * B) * 8;  // the block's first query of these 8
    pv[r] = q + 8 <= nq ? *reinterpret_cast<const uint4 *>(dest + i0 + q) : make_uint4(~0u, ~0u, ~0u, ~0u);
    if (q < nq && q + 8 > nq) {  // the block's ragged end
      uint16_t t[8];
      for (uint32_t u = 0; u < 8; ++u) t[u] = q + u < nq ? dest[i0 + q + u] : kNoSlot;
      pv[r] = make_uint4(t[0] | (uint32_t)t[1] << 16, t[2] | (uint32_t)t[3] << 16, t[4] | (uint32_t)t[5] << 16,
                         t[6] | (uint32_t)t[7] << 16);
    }
  }
  for (uint32_t w = tid; w < kQB / 32; w += B) lbits[w] = 0u;
  load_runs<B>(cnt, start, blk, F, nullptr, lcnt, lstart, lbase, nullptr, scratch);
  // the runs cut into pieces of 32 queries, numbered over the block (one long
  // run -- a batch with one filter -- spreads over all threads): lpc[f] = the
  // first piece of filter f's run
  for (uint32_t f = tid; f <= F; f += B) lpc[f] = f < F ? (lcnt[f] + 31u) >> 5 : 0u;
  __syncthreads();
  const uint32_t pieces = block_excl_scan_array<B>(lpc, F + 1, scratch);
  for (uint32_t pc = tid; pc < pieces; pc += B) {
    uint32_t lo = 0, hi = F;  // the last f with lpc[f] <= pc: its run holds piece pc
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (lpc[mid] <= pc) lo = mid; else hi = mid;
    }
    const uint32_t o = (pc - lpc[lo]) * 32u;
    const uint32_t s = lstart[lo] + o, p = lbase[lo] + o, len = min(32u, lcnt[lo] - o);
    const uint32_t sh = s & 31u;
    const uint32_t w0 = clrw[s >> 5], w1 = clrw[(s >> 5) + 1];  // (the array has 64 bytes of slack)
    uint32_t v = sh ? (w0 >> sh) | (w1 << (32u - sh)) : w0;
    if (len < 32) v &= (1u << len) - 1u;
    if (!v) continue;
    const uint32_t ps = p & 31u;
    atomicOr(&lbits[p >> 5], v << ps);
    if (ps && ps + len > 32) atomicOr(&lbits[(p >> 5) + 1], v >> (32u - ps));
  }
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < QPT / 8; ++r) {
    const uint32_t q = (tid + r * B) * 8;
    if (q >= nq) continue;
    const uint32_t pw[4] = {pv[r].x, pv[r].y, pv[r].z, pv[r].w};
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (uint32_t u = 0; u < 8; ++u) {
      const uint32_t pl = (pw[u / 2] >> (16 * (u & 1))) & 0xFFFFu;
      // answer 1 iff the query was probed (a place) and none of its bits was clear
      const uint32_t a = pl == kNoSlot ? 0u : ((lbits[pl >> 5] >> (pl & 31u)) & 1u) ^ 1u;
      if (u < 4) lo |= a << (8 * u); else hi |= a << (8 * (u - 4));
    }
    if (q + 8 <= nq && (reinterpret_cast<uintptr_t>(out) & 7u) == 0) {
      *reinterpret_cast<uint2 *>(out + i0 + q) = make_uint2(lo, hi);
    } else {
      for (uint32_t u = 0; u < 8 && q + u < nq; ++u) out[i0 + q + u] = (uint8_t)(((u < 4 ? lo : hi) >> (8 * (u & 3))) & 1u);
    }
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
  uint32_t *cnt = reinterpret_cast<uint32_t *>(ws + p.o_cnt);
  uint32_t *start = reinterpret_cast<uint32_t *>(ws + p.o_start);
  uint32_t *cf = reinterpret_cast<uint32_t *>(ws + p.o_cf);
  uint16_t *dest = reinterpret_cast<uint16_t *>(ws + p.o_dest);
  uint2 *hs = reinterpret_cast<uint2 *>(ws + p.o_hs);
  uint32_t *ent = reinterpret_cast<uint32_t *>(ws + p.o_ent);
  uint32_t *tab = reinterpret_cast<uint32_t *>(ws + p.o_tab);
  uint8_t *res = ws + p.o_res;
  uint32_t *split = reinterpret_cast<uint32_t *>(ws + p.o_split);
  const uint32_t F = num_filters;
  const uint32_t cus = adl_host::device_cus();
  const uint32_t g_tile = std::min(cus, kMaxSlots);  // pb_tile's workgroups
  const size_t lds_k1 = (size_t)(2 * F + 2) * 4;                       // counters + tile counts
  const size_t lds_k3 = (size_t)(2 * kQB + 5 * (F + 1) + 32) * 4;      // hashes + 5 per-filter arrays + scratch
  const size_t lds_k6 = (size_t)(kQB / 32 + 4 * (F + 1) + 32) * 4;     // answer bits + 4 per-filter arrays + scratch
  const size_t lds_p1 = (size_t)(kMaxTiles + 4 + 64 + p.k * p.C) * 4;
  const size_t lds_p2 = (size_t)kTileBytes + 64 + (size_t)((F + 1 + 3) & ~3u) * 4 +
                        (size_t)(kBlk / kWave) * kMaskWords * 4;
#ifdef ADL_BLOOM_STAMPS
  const uint32_t exp = adl_host::knobs().pb_exp;  // diagnostics build only
#else
  constexpr uint32_t exp = 0;
#endif
  try {
    hipLaunchKernelGGL(pb_desc_kernel, dim3(1), dim3(kBlk), 0, st, d_bitmap_off, d_bitmap_end, F, desc, scal);
    ADL_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(pb_hist_kernel, dim3(p.nb), dim3(kBlk), lds_k1, st, d_filter_id, n, F, p.nb, desc, cnt);
    ADL_HIP_TRY(hipGetLastError());
    uint32_t *gsum = reinterpret_cast<uint32_t *>(ws + p.o_gsum);
    hipLaunchKernelGGL(pb_colsum_kernel, dim3(p.ng), dim3(kBlk), 0, st, cnt, p.nb, F, gsum);
    ADL_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(pb_plan_kernel, dim3(1), dim3(kBlk), 0, st, gsum, p.ng, F, p.C, p.maxch, desc, cf, scal, p.k,
                       g_tile, split);
    ADL_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(pb_starts_kernel, dim3(p.ng), dim3(kBlk), 0, st, cnt, gsum, p.nb, F, desc, start);
    ADL_HIP_TRY(hipGetLastError());
    if (int rc = adl_host::lds_limit<pb_scatter_kernel>()) return rc;
    hipLaunchKernelGGL(pb_scatter_kernel, dim3(p.nb), dim3(kBlk), lds_k3, st, reinterpret_cast<const uint4 *>(d_keys),
                       d_filter_id, n, F, p.nb, desc, cnt, start, dest, hs, exp);
    ADL_HIP_TRY(hipGetLastError());
    if (int rc = adl_host::lds_limit<pb_tile_kernel>()) return rc;
    auto bin = [&](auto lim, auto kern) -> int {
      if (int rc = lim()) return rc;
      hipLaunchKernelGGL(kern, dim3(cus), dim3(kBlk), lds_p1, st, hs, desc, cf, scal, p.k, p.C, ent, tab, res, exp);
      ADL_HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(pb_tile_kernel, dim3(g_tile), dim3(kBlk), lds_p2, st, d_bitmaps, desc, F, p.k, p.C, ent, tab,
                         split, res, exp);
      ADL_HIP_TRY(hipGetLastError());
      return ADL_OK;
    };
    const int rc_bin = p.k == 6 ? bin(adl_host::lds_limit<pb_bin_kernel<6>>, pb_bin_kernel<6>)
                                : bin(adl_host::lds_limit<pb_bin_kernel<0>>, pb_bin_kernel<0>);
    if (rc_bin != ADL_OK) return rc_bin;
    if (int rc = adl_host::lds_limit<pb_gather_kernel>()) return rc;
    hipLaunchKernelGGL(pb_gather_kernel, dim3(p.nb), dim3(kGatherBlk), lds_k6, st, dest, res, n, F, p.nb, cnt, start,
                       d_out);
    ADL_HIP_TRY(hipGetLastError());
    return ADL_OK;
  } catch (...) {
    return ADL_ERR_DEVICE;
  }
}

}  // extern "C"
