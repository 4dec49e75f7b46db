// adlsm-tree_amd/csrc/bloom_bucket.hip -- MI355X (gfx950) bucketed bloom-filter
// build, the default for 16-byte keys.
//
// Replaces BloomFilter::Keys2Block (reference src/filter_block.cpp:9-33): for
// every key, h1/h2 = the reference's murmur3 variant with two seeds, then k bits
// (h1 + j*h2) % m are ORed into an (n*bpk+7)-byte bitmap.  The bitmap is an
// order-independent OR, so any routing of the bit-sets gives the reference's
// bitmap bit for bit.
//
// Two passes, each one persistent 1024-thread workgroup per CU:
//
//   pass A  bk_bin16_kernel   a workgroup owns a *slice* of one filter's keys
//           (about n/256 keys) and keeps one LDS bucket of 32 slots per bitmap
//           tile of 2^20 bits.  Per batch of 1024 keys: hash, k positions,
//           claim a slot (one ds_add_rtn on the tile's word) and write the
//           position (one ds_write); barrier; every full 16-entry granule is
//           copied out with one 16-byte store per lane to the slice's own
//           region for that tile.  No count pass, no scan, no table: the
//           workgroup is the only writer of its regions, so nothing needs a
//           global atomic.  A claim that finds its bucket full is retried in
//           the next batch.
//   pass B  bk_tile_kernel    a workgroup owns bitmap tiles held in LDS; a
//           tile's entries are the slices' regions for it (one per slice,
//           ~270 entries each at the headline), read as 64-entry units with
//           several loads in flight per wave and ds_or_b32'd into the tile;
//           then one coalesced write of the tile.
//
// Against the chunk/table build (bloom_build.hip), pass A issues two LDS
// operations per position instead of three plus a read-out, and pass B reads
// 256 long runs per tile instead of ~1 800 segments of ~38 entries.
//
// A region holds `cap` entries (the slice's expected share of a tile plus six
// standard deviations).  Should a slice put more into one tile (a skewed key
// set), the rest goes to 256-entry overflow extents allocated from the slice's
// own pool and chained through a link word; the pool is sized so that every
// entry of the slice fits whatever the distribution, so there is no failure
// path and no atomic outside LDS.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <type_traits>
#include <vector>

#include "bloom_bucket.hpp"
#include "bloom_common.hpp"

using namespace adl_dev;

namespace {

constexpr uint32_t kBlock = 1024;               // threads per workgroup, both passes
constexpr uint32_t kWaves = kBlock / kWave;     // 16
constexpr uint32_t kTL = 20;                    // log2 bits per tile: 128 KiB of LDS in pass B
constexpr uint32_t kTileWords = 1u << (kTL - 5);
constexpr uint32_t kTMask = (1u << kTL) - 1u;
constexpr uint32_t kRing = 32;                  // bucket slots per tile, pass A
constexpr uint32_t kGran = 16;                  // entries per flushed granule (64 B)
constexpr uint32_t kMaxTiles = 1024;            // flush owners: 64 lanes x 16 waves
constexpr uint32_t kListCap = 2 * kWave;        // flush-list entries per wave (<= 2 granules per owner)
constexpr uint32_t kMaxSlices = kBlock;         // pass B stages one slice count per thread
constexpr uint32_t kLdsWords = 40960;           // 160 KiB
constexpr uint32_t kPad = 64;                   // spare words after each area block (unit over-reads)
constexpr int kMaxFilt = 8;                     // filters whose descriptors ride in the kernargs
constexpr uint32_t kLink = 16;                  // words after a region / extent: link word + pad

struct BkDesc {
  uint64_t key_begin;    // first key of the filter in the key set
  uint64_t area_base;    // word offset of slice 0's area in the workspace
  uint64_t count_base;   // word offset of the filter's [T][R] entry-count table
  uint64_t bitmap_off;   // output byte offset
  uint32_t n;            // keys
  uint32_t L;            // keys per slice (the last slice may be shorter)
  uint32_t R;            // slices
  uint32_t slice0;       // first global slice index
  uint32_t T;            // tiles
  uint32_t tile0;        // first global tile index
  uint32_t cap;          // region entries per (slice, tile); a region is cap + kLink words
  uint32_t xo;           // overflow extent entries (0: no pool); an extent is xo + kLink words
  uint32_t stride;       // words per slice area: T * (cap + kLink) + pool
  uint32_t alloc_bytes;  // bitmap bytes rounded up to 16
  uint32_t pad0, pad1;
  FastMod mod;           // m = 8 * bitmap bytes
};
static_assert(sizeof(BkDesc) % 16 == 0, "descriptors load as whole uint4s");

struct BkArgs {
  uint32_t nf, k, total_slices, total_tiles;
  uint32_t tmax;       // pass A LDS tile rows (max T, multiple of 4)
  uint32_t dd_log2;    // pass A: slots (log2) of the table that skips keys whose h1 == h2 repeats (0: off)
  uint32_t nt_bitmap;  // pass B: non-temporal bitmap stores
  uint32_t pad_;
  BkDesc f[kMaxFilt];
};

template <typename T>
using cptr = const __attribute__((address_space(4))) T *;
struct BkTable {  // more than kMaxFilt filters: descriptors and maps in the workspace
  cptr<BkDesc> fd;
  cptr<uint32_t> slice_f, tile_f;
};

template <bool DT>
struct BF;
template <>
struct BF<false> {
  __device__ static const BkDesc &at(const BkArgs &a, const BkTable &, int i) { return a.f[i]; }
  // the last filter whose first slice / tile is <= s: an empty filter (R = 0)
  // shares its slice0 with the next one, which is the one that owns the slice
  __device__ static int of_slice(const BkArgs &a, const BkTable &, uint32_t s) {
    int f = 0;
#pragma unroll
    for (int i = 1; i < kMaxFilt; ++i)
      if ((uint32_t)i < a.nf && s >= a.f[i].slice0) f = i;
    return f;
  }
  __device__ static int of_tile(const BkArgs &a, const BkTable &, uint32_t t) {
    int f = 0;
#pragma unroll
    for (int i = 1; i < kMaxFilt; ++i)
      if ((uint32_t)i < a.nf && t >= a.f[i].tile0) f = i;
    return f;
  }
};
template <>
struct BF<true> {
  __device__ static BkDesc at(const BkArgs &, const BkTable &t, int i) {
    constexpr int NV = sizeof(BkDesc) / 16;
    const cptr<u32x4_t> src = reinterpret_cast<cptr<u32x4_t>>(t.fd) + (uint32_t)i * NV;
    u32x4_t v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = src[j];
    BkDesc d;
    __builtin_memcpy(&d, v, sizeof(d));
    return d;
  }
  __device__ static int of_slice(const BkArgs &, const BkTable &t, uint32_t s) { return (int)t.slice_f[s]; }
  __device__ static int of_tile(const BkArgs &, const BkTable &t, uint32_t x) { return (int)t.tile_f[x]; }
};

__global__ __launch_bounds__(256) void bk_fill_maps_kernel(const BkDesc *__restrict__ fd, uint32_t *__restrict__ slice_f,
                                                           uint32_t *__restrict__ tile_f) {
  const uint32_t f = blockIdx.x;
  const BkDesc d = fd[f];
  for (uint32_t i = threadIdx.x; i < d.R; i += 256) slice_f[d.slice0 + i] = f;
  for (uint32_t i = threadIdx.x; i < d.T; i += 256) tile_f[d.tile0 + i] = f;
}

// Ring slot -> LDS word of tile t's bucket.  The XOR moves whole aligned
// 4-word groups (bits 2..4 of the slot), so a 16-entry granule is still four
// aligned 16-byte groups, while buckets of different tiles start on
// different banks.
__device__ __forceinline__ uint32_t ring_word(uint32_t t, uint32_t slot) {
  return t * kRing + (slot ^ ((t & 7u) << 2));
}

// ---------------------------------------------------------------- pass A
// K > 0: k known at compile time (positions and claims unrolled); K == 0:
// runtime k (a.k), one position at a time.
template <int K, bool DT>
__global__ __launch_bounds__(kBlock) void bk_bin16_kernel(BkArgs a, const uint4 *__restrict__ keys,
                                                          uint32_t *__restrict__ ws, BkTable ft) {
  using F = BF<DT>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const uint32_t TM = a.tmax;
  uint32_t *ring = lds;                  // TM x kRing positions
  uint32_t *word = ring + TM * kRing;    // per tile: (ring start << 16) | entries claimed since the last flush
  uint32_t *flg = word + TM;             // per tile: granules copied out
  uint32_t *cur = flg + TM;              // per tile: current overflow extent (slice-area word offset)
  uint2 *wl = reinterpret_cast<uint2 *>(cur + TM) + wave * kListCap;  // this wave's flush list
  uint32_t *dtab = cur + TM + 2 * kWaves * kListCap;
  const uint32_t dd = a.dd_log2;
  uint32_t *bump = dtab + (dd ? (1u << dd) : 0u);  // overflow pool words used
  // "any thread has work left", one word per batch parity (__syncthreads_or
  // would take static LDS of its own, past the 160 KiB this kernel declares)
  uint32_t *more_flag = bump + 1;
  const uint32_t kk = K > 0 ? (uint32_t)K : a.k;
  const uint32_t all = kk >= 32 ? ~0u : (1u << kk) - 1u;

  int fprev = -1;
  for (uint32_t s = blockIdx.x; s < a.total_slices; s += gridDim.x) {
    const int fi = F::of_slice(a, ft, s);
    const auto &d = F::at(a, ft, fi);
    const uint32_t sl = s - d.slice0;
    const uint32_t first = sl * d.L;
    const uint32_t cnt = first < d.n ? min(d.L, d.n - first) : 0u;
    const uint32_t T = d.T, cap = d.cap, xo = d.xo, tstride = cap + kLink;
    const FastMod mod = d.mod;
    uint32_t *area = ws + d.area_base + (uint64_t)sl * d.stride;
    for (uint32_t t = tid; t < T; t += kBlock) {
      word[t] = 0;
      flg[t] = 0;
    }
    // the pair table holds one filter's keys (positions depend on m)
    if (dd && fi != fprev)
      for (uint32_t i = tid; i < (1u << dd); i += kBlock) dtab[i] = ~0u;
    if (tid == 0) {
      *bump = 0;
      more_flag[0] = more_flag[1] = 0;
    }
    fprev = fi;
    __syncthreads();

    // Copy every full granule out (FINAL: every entry, the last granule
    // partial) -- owner lane `lane` of wave `wave` owns tile wave*tpw + lane.
    // Its granules go to the wave's list; then 4 lanes per granule move it
    // with one ds_read_b128 + one 16-byte global store each.  The list is
    // written and read by the same wave (LDS operations of a wave complete
    // in order), so no barrier is needed inside.
    const uint32_t tpw = (T + kWaves - 1) / kWaves;
    auto flush = [&](auto final_tag) {
      constexpr bool FINAL = decltype(final_tag)::value;
      const uint32_t t = wave * tpw + lane;
      const bool own = lane < tpw && t < T;
      uint32_t g = 0, start = 0, f = 0, fl = 0;
      if (own) {
        const uint32_t w = word[t];
        start = w >> 16;
        f = min(w & 0xffffu, kRing);
        g = FINAL ? (f + kGran - 1) / kGran : f / kGran;
        fl = flg[t];
      }
      const uint64_t b0 = __ballot(g & 1u), b1 = __ballot((g >> 1) & 1u);
      const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(b0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b0, 0u)) +
                           2u * __builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)b1, 0u));
      const uint32_t tot = (uint32_t)__popcll(b0) + 2u * (uint32_t)__popcll(b1);
      if (own) {
        for (uint32_t i = 0; i < g; ++i) {
          const uint32_t e = (fl + i) * kGran;  // entry offset in the (slice, tile) stream
          uint32_t tgt;
          if (e < cap) {
            tgt = t * tstride + e;
          } else {  // past the region: overflow extents from the slice's pool
            const uint32_t eo = e - cap, o = eo % xo;
            if (o == 0) {
              const uint32_t ext = T * tstride + atomicAdd(bump, xo + kLink);
              area[eo == 0 ? t * tstride + cap : cur[t] + xo] = ext;  // link from the region / previous extent
              cur[t] = ext;
            }
            tgt = cur[t] + o;
          }
          wl[pre + i] = make_uint2(t | (((start + i * kGran) & (kRing - 1)) << 16), tgt);
        }
        if (FINAL) {
          ws[d.count_base + (uint64_t)t * d.R + sl] = fl * kGran + f;
        } else {
          word[t] = (((start + g * kGran) & (kRing - 1)) << 16) | (f - g * kGran);
          flg[t] = fl + g;
        }
      }
      for (uint32_t e0 = 0; e0 < tot; e0 += kWave / 4) {
        const uint32_t e = e0 + lane / 4;
        if (e < tot) {
          const uint2 le = wl[e];
          const uint32_t tt = le.x & 0xffffu, ro = le.x >> 16, q = lane & 3u;
          const uint4 v = *reinterpret_cast<const uint4 *>(ring + ring_word(tt, ro + 4u * q));
          *reinterpret_cast<uint4 *>(area + le.y + 4u * q) = v;
        }
      }
    };

    const uint4 *kp = keys + d.key_begin + first;
    const uint32_t last = cnt ? cnt - 1u : 0u;
    uint32_t j = 0;     // keys this thread has taken
    uint32_t pend = 0;  // positions of the current key still to place
    uint32_t h1 = 0, h2 = 0;
    uint4 nxt = make_uint4(0, 0, 0, 0);
    if (cnt) nxt = load_nt(kp + min(tid, last));
    for (uint32_t it = 0;; ++it) {
      if (pend == 0 && tid + j * kBlock < cnt) {
        hash16(nxt, h1, h2);
        ++j;
        pend = all;
        // the reference's murmur variant collapses: 39 % of SplitMix keys have
        // h1 == h2, on few values; a key whose h1 == h2 value this workgroup
        // already placed (same filter) sets no new bit.  Skipped only when the
        // slot holds exactly its value, installed by a key that was placed.
        if (dd && h1 == h2) {
          const uint32_t old = atomicCAS(&dtab[h1 >> (32u - dd)], ~0u, h1);
          if (old != ~0u && old == h1) pend = 0;
        }
        if (cnt) nxt = load_nt(kp + min(tid + j * kBlock, last));
      }
      if (K > 0) {
        uint32_t pos[K > 0 ? K : 1], old[K > 0 ? K : 1];
#pragma unroll
        for (int jj = 0; jj < K; ++jj) pos[jj] = fastmod(h1 + (uint32_t)jj * h2, mod);
#pragma unroll
        for (int jj = 0; jj < K; ++jj)
          old[jj] = ((pend >> jj) & 1u) ? atomicAdd(&word[pos[jj] >> kTL], 1u) : 0xffffu;
#pragma unroll
        for (int jj = 0; jj < K; ++jj) {
          const uint32_t rel = old[jj] & 0xffffu;
          if (rel < kRing) {
            const uint32_t t = pos[jj] >> kTL;
            ring[ring_word(t, ((old[jj] >> 16) + rel) & (kRing - 1))] = pos[jj];
            pend &= ~(1u << jj);
          }
        }
      } else {
        for (uint32_t jj = 0; jj < kk; ++jj) {
          if ((pend >> jj) & 1u) {
            const uint32_t p = fastmod(h1 + jj * h2, mod);
            const uint32_t t = p >> kTL;
            const uint32_t o = atomicAdd(&word[t], 1u), rel = o & 0xffffu;
            if (rel < kRing) {
              ring[ring_word(t, ((o >> 16) + rel) & (kRing - 1))] = p;
              pend &= ~(1u << jj);
            }
          }
        }
      }
      __syncthreads();  // claims and writes of this batch complete
      flush(std::false_type{});
      if (pend != 0 || tid + j * kBlock < cnt) more_flag[it & 1u] = 1u;
      __syncthreads();  // also: the flush has read the ring before new claims
      const bool any = more_flag[it & 1u] != 0;
      // the other word is next written after the next batch's claim barrier
      if (tid == 0) more_flag[(it + 1u) & 1u] = 0;
      if (!any) break;
    }
    flush(std::true_type{});
    __syncthreads();  // LDS reused by the next slice
  }
}

// ---------------------------------------------------------------- pass B
// Per tile: the slices' entry counts are staged in LDS and scanned into
// 64-entry units; wave w takes units [U*w/16, U*(w+1)/16) -- a contiguous
// stretch of long runs -- and gathers them D units per stage, two stages in
// flight (unit descriptors computed per lane, handed out by readlane).
template <int D, bool DT>
__global__ __launch_bounds__(kBlock) void bk_tile_kernel(BkArgs a, const uint32_t *__restrict__ ws,
                                                         uint8_t *__restrict__ bitmaps, BkTable ft) {
  using F = BF<DT>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  uint32_t *tile = lds;                      // 2^20 bits
  uint32_t *pre = tile + kTileWords;         // kMaxSlices: exclusive unit prefix
  uint32_t *cfast = pre + kMaxSlices;        // entries in the slice's region (<= cap)
  uint32_t *cfull = cfast + kMaxSlices;      // all entries
  uint32_t *scratch = cfull + kMaxSlices;    // block scan (kWaves + 1)
  {
    uint4 *t4 = reinterpret_cast<uint4 *>(tile);
    for (uint32_t i = tid; i < kTileWords / 4; i += kBlock) t4[i] = make_uint4(0, 0, 0, 0);
  }
  for (uint32_t tg = blockIdx.x; tg < a.total_tiles; tg += gridDim.x) {
    const auto &d = F::at(a, ft, F::of_tile(a, ft, tg));
    const uint32_t t = tg - d.tile0, R = d.R, cap = d.cap, tstride = cap + kLink, stride = d.stride;
    const uint32_t *abase = ws + d.area_base;
    // (a count can never exceed the slice's k*L positions; clamped so that a
    // corrupted workspace gives a wrong bitmap, never a wild read or a long walk)
    uint32_t c = 0;
    if (tid < R) c = min(ws[d.count_base + (uint64_t)t * R + tid], a.k * d.L);
    const uint32_t cf = min(c, cap);
    uint32_t U;
    const uint32_t ex = block_excl_scan<kBlock>((cf + kWave - 1) / kWave, scratch, &U);  // (barriers inside)
    if (tid < R) {
      pre[tid] = ex;
      cfast[tid] = cf;
      cfull[tid] = c;
    }
    __syncthreads();

    const uint32_t u0 = (uint32_t)(((uint64_t)U * wave) / kWaves);
    const uint32_t u1 = (uint32_t)(((uint64_t)U * (wave + 1)) / kWaves);
    for (uint32_t ub = u0; ub < u1; ub += kWave) {
      const uint32_t nb = min((uint32_t)kWave, u1 - ub);
      // lane l: unit ub + l -> (word offset in the filter's areas, valid entries)
      uint32_t doff = 0, dval = 0;
      if (lane < nb) {
        const uint32_t u = ub + lane;
        uint32_t lo = 0, hi = R;  // the last slice whose units start at or before u
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (pre[mid] <= u) lo = mid;
          else hi = mid;
        }
        const uint32_t q = u - pre[lo];
        doff = lo * stride + t * tstride + q * kWave;
        dval = min(cfast[lo] - q * kWave, (uint32_t)kWave);
      }
      struct Stage {
        uint32_t v[D];
      };
      // A stage's loads are issued unconditionally (a slot past nb reads
      // unit 0 again and is masked out), so the compiler waits vmcnt(D) for
      // the older stage instead of vmcnt(0).
      auto issue = [&](Stage &st, uint32_t q0) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
          const uint32_t i = min(q0 + (uint32_t)u, (uint32_t)kWave - 1u);
          st.v[u] = abase[__builtin_amdgcn_readlane(doff, i) + lane];
        }
      };
      auto consume = [&](const Stage &st, uint32_t q0) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
          const uint32_t i = q0 + (uint32_t)u;
          const uint32_t val = i < nb ? __builtin_amdgcn_readlane(dval, min(i, (uint32_t)kWave - 1u)) : 0u;
          if (lane < val) {
            const uint32_t off = st.v[u] & kTMask;
            atomicOr(&tile[off >> 5], 1u << (off & 31u));
          }
        }
      };
      Stage A, B;
      issue(A, 0);
      for (uint32_t q0 = 0; q0 < nb; q0 += 2 * D) {
        issue(B, q0 + D);
        consume(A, q0);
        issue(A, q0 + 2 * D);
        consume(B, q0 + D);
      }
    }
    // entries past a region (skewed key sets only): follow the extent chain
    for (uint32_t s = wave; s < R; s += kWaves) {
      const uint32_t cs = cfull[s];
      if (cs <= cap) continue;
      const uint32_t sb = s * stride;
      uint32_t lk = sb + t * tstride + cap;
      for (uint32_t e = cap; e < cs; e += d.xo) {
        // an extent lies inside the slice's pool (clamped: see the counts)
        const uint32_t ext =
            min(__builtin_amdgcn_readfirstlane(abase[lk]), stride - d.xo - kLink);
        const uint32_t nn = min(d.xo, cs - e);
        for (uint32_t o = 0; o < nn; o += kWave) {
          if (o + lane < nn) {
            const uint32_t off = abase[sb + ext + o + lane] & kTMask;
            atomicOr(&tile[off >> 5], 1u << (off & 31u));
          }
        }
        lk = sb + ext + d.xo;
      }
    }
    __syncthreads();  // the tile is complete

    // write the tile: bytes [t << (kTL-3), ...) of this filter, up to the
    // 16-byte-rounded bitmap length (pad bytes are zero: no position lands
    // there); each 16-byte word is re-zeroed as it is read out
    const uint64_t tile_bytes = 1ull << (kTL - 3);
    const uint64_t b0 = (uint64_t)t * tile_bytes;
    const uint32_t nvec = (uint32_t)(min(tile_bytes, (uint64_t)d.alloc_bytes - b0) >> 4);
    uint4 *out4 = reinterpret_cast<uint4 *>(bitmaps + d.bitmap_off + b0);
    uint4 *t4 = reinterpret_cast<uint4 *>(tile);
    for (uint32_t i = tid; i < kTileWords / 4; i += kBlock) {
      const uint4 v = t4[i];
      t4[i] = make_uint4(0, 0, 0, 0);
      if (i < nvec) {
        if (a.nt_bitmap) store_nt(out4 + i, v);
        else out4[i] = v;
      }
    }
    __syncthreads();  // read out and zero again; counts staged for the next tile
  }
}

// ---------------------------------------------------------------- host plan
struct BkPlan {
  BkArgs a;
  std::vector<BkDesc> f;
  bool dt = false;
  uint64_t area_words = 0, count_words = 0, ft_bytes = 0, ws_bytes = 0;
  uint32_t grid_a = 0, grid_b = 0;
  size_t lds_a = 0, lds_b = 0;
};

constexpr size_t kLdsB = (size_t)(kTileWords + 3 * kMaxSlices + kWaves + 1) * 4;

int make_plan(const uint64_t *counts, uint32_t nf, int32_t bpk, BkPlan &p) {
  if (nf == 0 || bpk < 0) return ADL_ERR_INVALID_ARG;
  memset(&p.a, 0, sizeof(p.a));
  p.f.assign(nf, BkDesc{});
  p.dt = nf > (uint32_t)kMaxFilt;
  const uint32_t k = (uint32_t)adl_host::num_probes(bpk);
  uint64_t total_n = 0;
  for (uint32_t f = 0; f < nf; ++f) {
    if (adl_host::bitmap_bytes(counts[f], bpk) == 0) return ADL_ERR_TOO_LARGE;
    total_n += counts[f];
  }
  const uint32_t cus = adl_host::device_cus();
  // slice size: one slice per CU for the whole group, at least 1024 keys (one batch)
  const uint64_t Lg = std::max<uint64_t>(1024, (total_n + cus - 1) / cus);
  uint64_t area = 0, cntw = 0;  // words of the slice areas; of the count tables (placed after the areas)
  uint32_t slice = 0, tile = 0, tmax = 0;
  for (uint32_t f = 0; f < nf; ++f) {
    BkDesc &d = p.f[f];
    const uint64_t n = counts[f];
    const uint64_t bytes = adl_host::bitmap_bytes(n, bpk);
    const uint64_t m = bytes * 8;
    const uint64_t T = (m + (1ull << kTL) - 1) >> kTL;
    if (T > kMaxTiles) return ADL_ERR_TOO_LARGE;
    const uint64_t R = n ? (n + Lg - 1) / Lg : 0;
    if (R > kMaxSlices) return ADL_ERR_TOO_LARGE;
    const uint64_t L = R ? (n + R - 1) / R : 0;
    if (R && (R - 1) * L >= n) return ADL_ERR_TOO_LARGE;  // every slice holds a key (cannot happen for L >= R)
    // Region capacity: a position lands in one tile with probability at most
    // 2^20 * ceil(2^32 / m) / 2^32 (positions are (h1 + j*h2) mod 2^32 mod m);
    // the expected count plus six standard deviations.
    const uint64_t kl = (uint64_t)k * L;
    const uint64_t kl16 = adl_host::round_up(std::max<uint64_t>(kl, 1), kGran);
    const double q = (double)(((1ull << 32) + m - 1) / m);
    const double pmax = T == 1 ? 1.0 : std::min(1.0, (double)(1ull << kTL) * q / 4294967296.0);
    const double E = (double)kl * pmax;
    uint64_t cap = adl_host::round_up((uint64_t)(E + 6.0 * sqrt(E) + 32.0), kGran);
    cap = std::max<uint64_t>(cap, 64);
    uint64_t xo = 0, pool = 0;
    if (cap >= kl16) {
      cap = kl16;  // the slice's every entry fits one region: no pool
    } else {
      // extents of xo <= cap - 16 entries: the slice's overflow needs at most
      // ceil(kl / xo) + 2 of them whatever the key distribution
      xo = std::min<uint64_t>(256, (cap - kGran) & ~(uint64_t)(kGran - 1));
      pool = ((kl + xo - 1) / xo + 2) * (xo + kLink);
    }
    const uint64_t stride = T * (cap + kLink) + pool;
    if (R * stride + kPad >= (1ull << 32)) return ADL_ERR_TOO_LARGE;  // u32 offsets inside a filter's areas
    d.n = (uint32_t)n;
    d.L = (uint32_t)L;
    d.R = (uint32_t)R;
    d.slice0 = slice;
    d.T = (uint32_t)T;
    d.tile0 = tile;
    d.cap = (uint32_t)cap;
    d.xo = (uint32_t)xo;
    d.stride = (uint32_t)stride;
    d.alloc_bytes = (uint32_t)adl_host::round_up(bytes, 16);
    d.mod = adl_host::make_fastmod((uint32_t)m);
    d.area_base = area;
    d.count_base = cntw;
    d.key_begin = 0;
    d.bitmap_off = 0;
    area += R * stride + kPad;
    cntw += T * R;
    slice += (uint32_t)R;
    tile += (uint32_t)T;
    tmax = std::max<uint32_t>(tmax, (uint32_t)T);
  }
  tmax = (uint32_t)adl_host::round_up(tmax, 4);
  // pass A LDS: rings + 3 words per tile, the flush lists, the pair table
  const uint32_t fixed = 35 * tmax + 2 * kWaves * kListCap + 4;
  if (fixed > kLdsWords) return ADL_ERR_TOO_LARGE;
  uint32_t dd = 0;
  if (adl_host::env_on("ADL_BLOOM_HASH_DEDUP", true)) {
    const uint32_t lg_max = std::min<uint32_t>(adl_host::env_on("ADL_BLOOM_BK_DD13", false) ? 13 : 12, 13);
    for (uint32_t lg = lg_max; lg >= 8; --lg)
      if (fixed + (1u << lg) <= kLdsWords) {
        dd = lg;
        break;
      }
  }
  p.a.nf = nf;
  p.a.k = k;
  p.a.total_slices = slice;
  p.a.total_tiles = tile;
  p.a.tmax = tmax;
  p.a.dd_log2 = dd;
  p.a.nt_bitmap = adl_host::env_on("ADL_BLOOM_NT_BITMAP", true) ? 1u : 0u;
  p.area_words = adl_host::round_up(area, 64);
  p.count_words = adl_host::round_up(cntw + kPad, 64);
  for (BkDesc &d : p.f) d.count_base += p.area_words;  // the count tables follow the areas
  p.ft_bytes = p.dt ? adl_host::round_up(nf * sizeof(BkDesc), 256) + 4ull * (slice + tile) + 256 : 0;
  p.ws_bytes = (p.area_words + p.count_words) * 4 + p.ft_bytes + 256;
  p.lds_a = (size_t)(fixed + (dd ? (1u << dd) : 0u)) * 4;
  p.lds_b = kLdsB;
  p.grid_a = std::min<uint32_t>(slice, cus);
  p.grid_b = std::min<uint32_t>(tile, cus);
  if (!p.dt) std::copy(p.f.begin(), p.f.end(), p.a.f);
  return ADL_OK;
}

template <bool DT>
int launch(BkPlan &p, const uint4 *keys, uint8_t *bitmaps, void *ws, hipStream_t st, hipEvent_t *ev) {
  uint32_t *w = reinterpret_cast<uint32_t *>(ws);
  BkTable ft{};
  if constexpr (DT) {
    uint8_t *fbase = reinterpret_cast<uint8_t *>(w + p.area_words + p.count_words);
    BkDesc *fd = reinterpret_cast<BkDesc *>(fbase);
    uint32_t *slice_f = reinterpret_cast<uint32_t *>(fbase + adl_host::round_up(p.f.size() * sizeof(BkDesc), 256));
    uint32_t *tile_f = slice_f + p.a.total_slices;
    if (int rc = adl_host::t_upload.upload(fd, p.f.data(), p.f.size() * sizeof(BkDesc), st)) return rc;
    hipLaunchKernelGGL(bk_fill_maps_kernel, dim3((uint32_t)p.f.size()), dim3(256), 0, st, fd, slice_f, tile_f);
    ADL_HIP_TRY(hipGetLastError());
    ft.fd = (cptr<BkDesc>)fd;
    ft.slice_f = (cptr<uint32_t>)slice_f;
    ft.tile_f = (cptr<uint32_t>)tile_f;
  }
  if (p.a.total_slices) {
    auto go = [&](auto lim, auto kern) -> int {
      if (int rc = lim()) return rc;
      hipExtLaunchKernelGGL(kern, dim3(p.grid_a), dim3(kBlock), p.lds_a, st, ev ? ev[0] : nullptr,
                            ev ? ev[1] : nullptr, 0, p.a, keys, w, ft);
      ADL_HIP_TRY(hipGetLastError());
      return ADL_OK;
    };
    const int rc = p.a.k == 6 ? go(adl_host::lds_limit<bk_bin16_kernel<6, DT>>, bk_bin16_kernel<6, DT>)
                              : go(adl_host::lds_limit<bk_bin16_kernel<0, DT>>, bk_bin16_kernel<0, DT>);
    if (rc) return rc;
  } else if (ev) {  // no keys: an empty pass-A interval
    ADL_HIP_TRY(hipEventRecord(ev[0], st));
    ADL_HIP_TRY(hipEventRecord(ev[1], st));
  }
  if (int rc = adl_host::lds_limit<bk_tile_kernel<8, DT>>()) return rc;
  hipExtLaunchKernelGGL(bk_tile_kernel<8, DT>, dim3(p.grid_b), dim3(kBlock), p.lds_b, st, ev ? ev[2] : nullptr,
                        ev ? ev[3] : nullptr, 0, p.a, (const uint32_t *)w, bitmaps, ft);
  ADL_HIP_TRY(hipGetLastError());
  return ADL_OK;
}

std::vector<uint64_t> group_counts(const uint64_t *key_begin, uint32_t nf) {
  std::vector<uint64_t> c(nf);
  for (uint32_t f = 0; f < nf; ++f) c[f] = key_begin[f + 1] - key_begin[f];
  return c;
}

}  // namespace

namespace adl_bk {

uint64_t workspace_bytes(const uint64_t *counts, uint32_t nf, int32_t bpk) {
  BkPlan p;
  if (make_plan(counts, nf, bpk, p)) return 0;
  return p.ws_bytes;
}

int build16(const uint4 *d_keys, const uint64_t *key_begin, uint32_t nf, int32_t bpk, uint8_t *d_bitmaps,
            const uint64_t *bitmap_off, void *ws, uint64_t ws_bytes, hipStream_t st, hipEvent_t *ev) {
  const std::vector<uint64_t> counts = group_counts(key_begin, nf);
  BkPlan p;
  if (int rc = make_plan(counts.data(), nf, bpk, p)) return rc;
  if (!ws || ws_bytes < p.ws_bytes) return ADL_ERR_WORKSPACE;
  for (uint32_t f = 0; f < nf; ++f) {
    if (bitmap_off[f] % 16) return ADL_ERR_INVALID_ARG;
    p.f[f].key_begin = key_begin[f];
    p.f[f].bitmap_off = bitmap_off[f];
    if (!p.dt) p.a.f[f] = p.f[f];
  }
  return p.dt ? launch<true>(p, d_keys, d_bitmaps, ws, st, ev) : launch<false>(p, d_keys, d_bitmaps, ws, st, ev);
}

int positions(const uint64_t *counts, uint32_t nf, int32_t bpk, const void *ws, uint64_t *out, hipStream_t st) {
  BkPlan p;
  if (int rc = make_plan(counts, nf, bpk, p)) return rc;
  std::vector<uint32_t> tab(p.count_words);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(ws) + p.area_words;
  ADL_HIP_TRY(hipMemcpyAsync(tab.data(), w, p.count_words * 4, hipMemcpyDeviceToHost, st));
  ADL_HIP_TRY(hipStreamSynchronize(st));
  uint64_t sum = 0;
  for (const BkDesc &d : p.f)
    for (uint64_t i = 0; i < (uint64_t)d.T * d.R; ++i) sum += tab[d.count_base - p.area_words + i];
  *out = sum;
  return ADL_OK;
}

}  // namespace adl_bk
