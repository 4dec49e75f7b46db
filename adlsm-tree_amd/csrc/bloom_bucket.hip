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
constexpr uint32_t kRingMin = 32, kRingMax = 1024;  // bucket slots per tile, pass A (a power of two)
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
  uint32_t ring;       // pass A bucket slots per tile (power of two, 32 .. 1024)
  uint32_t dd_log2;    // pass A: slots (log2) of the table that skips keys whose h1 == h2 repeats (0: off)
  uint32_t nt_bitmap;  // pass B: non-temporal bitmap stores
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

// ---------------------------------------------------------------- diagnostics
// -DADL_BLOOM_STAMPS only (make stamps): wave 0 of every workgroup sums
// s_memtime cycles per phase; adl_bloom_debug_stamps appends them after the
// chunk/table build's (tools/stamps.py BK=1).  The product library has none.
#ifdef ADL_BLOOM_STAMPS
__device__ uint64_t g_bk_stamps[2][256][16][8];  // pass A, pass B; workgroup < 256, every wave
#define BK_STAMP_DECL                                  \
  uint64_t bst_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}; \
  uint64_t bst_t_ = __builtin_amdgcn_s_memtime();
#define BK_STAMP(i)                                    \
  do {                                                 \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    bst_acc_[i] += t_ - bst_t_;                        \
    bst_t_ = t_;                                       \
  } while (0)
#define BK_STAMP_FLUSH(pass)                                                                          \
  do {                                                                                                \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 256)                                                  \
      for (int i_ = 0; i_ < 8; ++i_) g_bk_stamps[pass][blockIdx.x][threadIdx.x / 64][i_] = bst_acc_[i_]; \
  } while (0)
#else
#define BK_STAMP_DECL
#define BK_STAMP(i) do { } while (0)
#define BK_STAMP_FLUSH(pass) do { } while (0)
#endif

// Ring slot -> LDS word of tile t's bucket.  The XOR moves whole aligned
// 4-word groups (bits 2..4 of the slot), so a 16-entry granule is still four
// aligned 16-byte groups, while buckets of different tiles start on
// different banks.
__device__ __forceinline__ uint32_t ring_word(uint32_t t, uint32_t slot, uint32_t lgS) {
  return (t << lgS) + (slot ^ ((t & 7u) << 2));
}

// Entry layout.  P3 = false: one u32 position per entry.  P3 = true: 24-bit
// entries, 4 to 3 words (a tile offset needs 20 bits), so the round trip
// through HBM moves 3/4 of the bytes; a 16-entry granule is 48 bytes.
// Region, extent and unit starts are multiples of 16 entries.
template <bool P3>
__device__ __forceinline__ uint32_t ent_words(uint32_t e) {
  return P3 ? (e >> 2) * 3u : e;
}
typedef uint32_t u32x3_t __attribute__((ext_vector_type(3)));
__device__ __forceinline__ u32x3_t pack3(uint4 v) {
  const uint32_t a = v.x & kTMask, b = v.y & kTMask, c = v.z & kTMask, e = v.w & kTMask;
  u32x3_t r;
  r.x = a | (b << 24);
  r.y = (b >> 8) | (c << 16);
  r.z = (c >> 16) | (e << 8);
  return r;
}
__device__ __forceinline__ uint4 unpack3(u32x3_t r) {
  return make_uint4(r.x & 0xffffffu, (r.x >> 24) | ((r.y & 0xffffu) << 8), (r.y >> 16) | ((r.z & 0xffu) << 16),
                    r.z >> 8);
}

// ---------------------------------------------------------------- pass A
// K > 0: k known at compile time (positions and claims unrolled); K == 0:
// runtime k (a.k), one position at a time.
// Key sources: 16-byte keys (hashed here), or the (h1, h2) pairs the
// var-len hashing pass wrote (bloom_build.hip, hash_var_kernel), indexed like
// the keys relative to the group's first key.
struct BkSrc16 {
  const uint4 *keys;
  using Raw = uint4;
  __device__ __forceinline__ Raw load(uint64_t i) const { return load_nt(keys + i); }
  __device__ static __forceinline__ void hash(const Raw &r, uint32_t &h1, uint32_t &h2) { hash16(r, h1, h2); }
};
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
struct BkSrcPairs {
  const uint2 *pairs;
  using Raw = uint2;
  __device__ __forceinline__ Raw load(uint64_t i) const {
    const u32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x2_t *>(pairs + i));
    return make_uint2(v.x, v.y);
  }
  __device__ static __forceinline__ void hash(const Raw &r, uint32_t &h1, uint32_t &h2) {
    h1 = r.x;
    h2 = r.y;
  }
};

template <int K, class Src, bool DT, bool P3>
__global__ __launch_bounds__(kBlock) void bk_bin16_kernel(BkArgs a, Src src,
                                                          uint32_t *__restrict__ ws, BkTable ft) {
  using F = BF<DT>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const uint32_t TM = a.tmax;
  const uint32_t S = a.ring;             // slots per tile bucket (a power of two >= 32)
  const uint32_t lgS = 31u - __clz(S);
  uint32_t *ring = lds;                  // TM x S positions
  uint32_t *word = ring + TM * S;        // per tile: (ring start << 16) | entries claimed since the last flush
  uint32_t *flg = word + TM;             // per tile: granules copied out
  uint32_t *cur = flg + TM;              // per tile: current overflow extent (slice-area word offset)
  uint2 *wl = reinterpret_cast<uint2 *>(cur + TM) + wave * kListCap;  // this wave's flush list
  uint32_t *dtab = cur + TM + 2 * kWaves * kListCap;
  const uint32_t dd = a.dd_log2;
  uint32_t *bump = dtab + (dd ? (1u << dd) : 0u);  // overflow pool words used
  // "any thread has work left", one word per batch parity (__syncthreads_or
  // would take static LDS of its own, past the 160 KiB this kernel declares)
  uint32_t *more_flag = bump + 1;
  // a word per lane that a rejected claim writes instead of the ring (the
  // claim phase stores unconditionally); nothing reads it
  uint32_t *sink = bump + 4 + lane;
  const uint32_t kk = K > 0 ? (uint32_t)K : a.k;
  const uint32_t all = kk >= 32 ? ~0u : (1u << kk) - 1u;

  int fprev = -1;
  BK_STAMP_DECL
  for (uint32_t s = blockIdx.x; s < a.total_slices; s += gridDim.x) {
    const int fi = F::of_slice(a, ft, s);
    const auto &d = F::at(a, ft, fi);
    const uint32_t sl = s - d.slice0;
    const uint32_t first = sl * d.L;
    const uint32_t cnt = first < d.n ? min(d.L, d.n - first) : 0u;
    const uint32_t T = d.T, cap = d.cap, xo = d.xo;
    const uint32_t tstride = ent_words<P3>(cap) + kLink, xw = ent_words<P3>(xo) + kLink;
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
    BK_STAMP(5);  // slice set-up

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
        f = min(w & 0xffffu, S);
        g = FINAL ? (f + kGran - 1) / kGran : f / kGran;
        fl = flg[t];
      }
      const uint32_t incl = wave_incl_scan(g, (int)lane);
      const uint32_t pre = incl - g;
      const uint32_t tot = __builtin_amdgcn_readlane(incl, kWave - 1);
      if (own) {
        for (uint32_t i = 0; i < g; ++i) {
          const uint32_t e = (fl + i) * kGran;  // entry offset in the (slice, tile) stream
          uint32_t tgt;
          if (e < cap) {
            tgt = t * tstride + ent_words<P3>(e);
          } else {  // past the region: overflow extents from the slice's pool
            const uint32_t eo = e - cap, o = eo % xo;
            if (o == 0) {
              const uint32_t ext = T * tstride + atomicAdd(bump, xw);
              // link from the region / previous extent
              area[eo == 0 ? t * tstride + ent_words<P3>(cap) : cur[t] + ent_words<P3>(xo)] = ext;
              cur[t] = ext;
            }
            tgt = cur[t] + ent_words<P3>(o);
          }
          wl[pre + i] = make_uint2(t | (((start + i * kGran) & (S - 1)) << 16), tgt);
        }
        if (FINAL) {
          ws[d.count_base + (uint64_t)t * d.R + sl] = fl * kGran + f;
        } else {
          word[t] = (((start + g * kGran) & (S - 1)) << 16) | (f - g * kGran);
          flg[t] = fl + g;
        }
      }
      for (uint32_t e0 = 0; e0 < tot; e0 += kWave / 4) {
        const uint32_t e = e0 + lane / 4;
        if (e < tot) {
          const uint2 le = wl[e];
          const uint32_t tt = le.x & 0xffffu, ro = le.x >> 16, q = lane & 3u;
          const uint4 v = *reinterpret_cast<const uint4 *>(ring + ring_word(tt, ro + 4u * q, lgS));
          if (P3) *reinterpret_cast<u32x3_t *>(area + le.y + 3u * q) = pack3(v);
          else *reinterpret_cast<uint4 *>(area + le.y + 4u * q) = v;
        }
      }
    };

    const uint64_t kp = d.key_begin + first;
    const uint32_t last = cnt ? cnt - 1u : 0u;
    uint32_t j = 0;     // keys this thread has taken
    // Two keys per thread in flight: A is being placed (its positions'
    // claims), B is hashed while A's claims are in flight, so the murmur VALU
    // overlaps the LDS atomics across the waves of a SIMD instead of running
    // in a phase of its own.  A claim rejected by a full bucket keeps its bit
    // in pendA and is retried next batch; B then waits.
    constexpr int KP = K > 0 ? K : 1;
    uint32_t posA[KP], posB[KP];
    uint32_t pendA = 0, pendB = 0;
    bool hasB = false;
    uint32_t h1 = 0, h2 = 0;  // K == 0: the hashes of A
    uint32_t h1B = 0, h2B = 0;
    typename Src::Raw nxt{};
    if (cnt) nxt = src.load(kp + min(tid, last));
    // Hash the loaded key into B and load the one after it.
    auto take = [&]() {
      if (!hasB && tid + j * kBlock < cnt) {
        Src::hash(nxt, h1B, h2B);
        ++j;
        hasB = true;
        pendB = all;
        // the reference's murmur variant collapses: 39 % of SplitMix keys have
        // h1 == h2, on few values; a key whose h1 == h2 value this workgroup
        // already placed (same filter) sets no new bit.  Skipped only when the
        // slot holds exactly its value, installed by a key that was placed.
        if (dd && h1B == h2B) {
          const uint32_t old = atomicCAS(&dtab[h1B >> (32u - dd)], ~0u, h1B);
          if (old != ~0u && old == h1B) pendB = 0;
        }
        if (cnt) nxt = src.load(kp + min(tid + j * kBlock, last));
        if (K > 0) {
#pragma unroll
          for (int jj = 0; jj < KP; ++jj) posB[jj] = fastmod(h1B + (uint32_t)jj * h2B, mod);
        }
      }
    };
    auto promote = [&]() {  // B becomes A once A is placed
      if (pendA == 0 && hasB) {
#pragma unroll
        for (int jj = 0; jj < KP; ++jj) posA[jj] = posB[jj];
        pendA = pendB;
        h1 = h1B;
        h2 = h2B;
        hasB = false;
      }
    };
    take();
    promote();
    for (uint32_t it = 0;; ++it) {
      // Typical wave: every lane's key A has all k positions or none left (a
      // retried claim is rare), so one exec mask covers the k claims and the
      // writes go out unconditionally (a rejected one into the lane's sink).
      const bool whole = (pendA == 0 || pendA == all);
      if (K > 0 && __all(whole)) {
        uint32_t old[KP];
        if (pendA) {
#pragma unroll
          for (int jj = 0; jj < KP; ++jj) old[jj] = atomicAdd(&word[posA[jj] >> kTL], 1u);
        }
        take();  // hash the next key while the atomics are in flight
        if (pendA) {
          uint32_t left = 0;
#pragma unroll
          for (int jj = 0; jj < KP; ++jj) {
            const uint32_t rel = old[jj] & 0xffffu;
            const uint32_t t = posA[jj] >> kTL;
            uint32_t *dst = ring + ring_word(t, ((old[jj] >> 16) + rel) & (S - 1), lgS);
            *(rel < S ? dst : sink) = posA[jj];
            left |= rel < S ? 0u : 1u << jj;
          }
          pendA = left;
        }
      } else if (K > 0) {
        uint32_t old[KP];
#pragma unroll
        for (int jj = 0; jj < KP; ++jj)
          old[jj] = ((pendA >> jj) & 1u) ? atomicAdd(&word[posA[jj] >> kTL], 1u) : 0xffffu;
        take();
#pragma unroll
        for (int jj = 0; jj < KP; ++jj) {
          const uint32_t rel = old[jj] & 0xffffu;
          if (rel < S) {
            const uint32_t t = posA[jj] >> kTL;
            ring[ring_word(t, ((old[jj] >> 16) + rel) & (S - 1), lgS)] = posA[jj];
            pendA &= ~(1u << jj);
          }
        }
      } else {
        for (uint32_t jj = 0; jj < kk; ++jj) {
          if ((pendA >> jj) & 1u) {
            const uint32_t p = fastmod(h1 + jj * h2, mod);
            const uint32_t t = p >> kTL;
            const uint32_t o = atomicAdd(&word[t], 1u), rel = o & 0xffffu;
            if (rel < S) {
              ring[ring_word(t, ((o >> 16) + rel) & (S - 1), lgS)] = p;
              pendA &= ~(1u << jj);
            }
          }
        }
        take();
      }
      promote();
      BK_STAMP(0);  // claims + hash of the next key
      __syncthreads();  // claims and writes of this batch complete
      BK_STAMP(1);  // claim barrier
      flush(std::false_type{});
      BK_STAMP(2);  // flush
      if (pendA != 0 || hasB || tid + j * kBlock < cnt) more_flag[it & 1u] = 1u;
      __syncthreads();  // also: the flush has read the ring before new claims
      const bool any = more_flag[it & 1u] != 0;
      // the other word is next written after the next batch's claim barrier
      if (tid == 0) more_flag[(it + 1u) & 1u] = 0;
      BK_STAMP(3);  // end barrier
      if (!any) break;
    }
    flush(std::true_type{});
    __syncthreads();  // LDS reused by the next slice
    BK_STAMP(4);  // final flush
  }
  BK_STAMP_FLUSH(0);
}

// ---------------------------------------------------------------- pass B
// Per tile: the slices' entry counts are staged in LDS and scanned into
// 64-entry units; wave w takes units [U*w/16, U*(w+1)/16) -- a contiguous
// stretch of long runs -- and gathers them D units per stage, two stages in
// flight (unit descriptors computed per lane, handed out by readlane).
template <int D, bool DT, bool P3>
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
  uint32_t *ovf = scratch + kWaves + 1;      // some slice of this tile overflowed its region
  if (tid == 0) *ovf = 0;
  {
    uint4 *t4 = reinterpret_cast<uint4 *>(tile);
    for (uint32_t i = tid; i < kTileWords / 4; i += kBlock) t4[i] = make_uint4(0, 0, 0, 0);
  }
  BK_STAMP_DECL
  // thread i's slice count of a tile, loaded one tile ahead (unconditionally,
  // at a clamped index: an unconditional load keeps the gather's counted waits)
  auto count_of = [&](uint32_t tg) -> uint32_t {
    const auto &d = F::at(a, ft, F::of_tile(a, ft, tg));
    const uint32_t R = d.R;
    return ws[d.count_base + (uint64_t)(tg - d.tile0) * R + min(tid, R ? R - 1u : 0u)];
  };
  uint32_t c_next = blockIdx.x < a.total_tiles ? count_of(blockIdx.x) : 0u;
  for (uint32_t tg = blockIdx.x; tg < a.total_tiles; tg += gridDim.x) {
    const auto &d = F::at(a, ft, F::of_tile(a, ft, tg));
    const uint32_t t = tg - d.tile0, R = d.R, cap = d.cap, stride = d.stride;
    const uint32_t tstride = ent_words<P3>(cap) + kLink, xw = ent_words<P3>(d.xo) + kLink;
    constexpr uint32_t EPU = P3 ? 4 * kWave : kWave;  // entries per unit (one load per lane)
    const uint32_t *abase = ws + d.area_base;
    // (a count can never exceed the slice's k*L positions; clamped so that a
    // corrupted workspace gives a wrong bitmap, never a wild read or a long walk)
    const uint32_t c = tid < R ? min(c_next, a.k * d.L) : 0u;
    c_next = count_of(tg + gridDim.x < a.total_tiles ? tg + gridDim.x : tg);
    if (c > cap) *ovf = 1;
    const uint32_t cf = min(c, cap);
    uint32_t U;
    const uint32_t ex = block_excl_scan<kBlock>((cf + EPU - 1) / EPU, scratch, &U);  // (barriers inside)
    if (tid < R) {
      pre[tid] = ex;
      cfast[tid] = cf;
      cfull[tid] = c;
    }
    __syncthreads();
    BK_STAMP(0);  // counts staged and scanned

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
        doff = lo * stride + t * tstride + ent_words<P3>(q * EPU);
        dval = min(cfast[lo] - q * EPU, EPU);
      }
      struct Stage {
        uint32_t v[D][P3 ? 3 : 1];
        uint32_t val[D];  // valid entries of each slot's unit (wave-uniform)
      };
      // A stage's loads are issued unconditionally (a slot past nb reads
      // unit 0 again and is masked out), so the compiler waits vmcnt(D) for
      // the older stage instead of vmcnt(0).  Lanes past a unit's valid
      // entries read the unit's first word, so they fetch no extra line.
      auto issue = [&](Stage &st, uint32_t q0) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
          const uint32_t i = min(q0 + (uint32_t)u, (uint32_t)kWave - 1u);
          st.val[u] = q0 + (uint32_t)u < nb ? __builtin_amdgcn_readlane(dval, i) : 0u;
          if (P3) {
            const u32x3_t r = *reinterpret_cast<const u32x3_t *>(
                abase + __builtin_amdgcn_readlane(doff, i) + (4u * lane < st.val[u] ? 3u * lane : 0u));
            st.v[u][0] = r.x;
            st.v[u][P3 ? 1 : 0] = r.y;
            st.v[u][P3 ? 2 : 0] = r.z;
          } else {
            st.v[u][0] = abase[__builtin_amdgcn_readlane(doff, i) + (lane < st.val[u] ? lane : 0u)];
          }
        }
      };
      auto consume = [&](const Stage &st, uint32_t) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
          if (P3) {
            u32x3_t r;
            r.x = st.v[u][0];
            r.y = st.v[u][P3 ? 1 : 0];
            r.z = st.v[u][P3 ? 2 : 0];
            const uint4 e = unpack3(r);
            const uint32_t ev[4] = {e.x, e.y, e.z, e.w};
#pragma unroll
            for (int v = 0; v < 4; ++v)
              if (4u * lane + (uint32_t)v < st.val[u]) {
                const uint32_t off = ev[v] & kTMask;
                atomicOr(&tile[off >> 5], 1u << (off & 31u));
              }
          } else if (lane < st.val[u]) {
            const uint32_t off = st.v[u][0] & kTMask;
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
    BK_STAMP(1);  // gather + or (this wave's units)
    // entries past a region (skewed key sets only): follow the extent chain
    for (uint32_t s = wave; *ovf && s < R; s += kWaves) {
      const uint32_t cs = cfull[s];
      if (cs <= cap) continue;
      const uint32_t sb = s * stride;
      uint32_t lk = sb + t * tstride + ent_words<P3>(cap);
      for (uint32_t e = cap; e < cs; e += d.xo) {
        // an extent lies inside the slice's pool (clamped: see the counts)
        const uint32_t ext = min(__builtin_amdgcn_readfirstlane(abase[lk]), stride - xw);
        const uint32_t nn = min(d.xo, cs - e);
        if (P3) {
          for (uint32_t o = 0; o < nn; o += 4 * kWave) {
            if (o + 4u * lane < nn) {
              const uint4 ev = unpack3(*reinterpret_cast<const u32x3_t *>(abase + sb + ext + ent_words<P3>(o) + 3u * lane));
              const uint32_t e4[4] = {ev.x, ev.y, ev.z, ev.w};
#pragma unroll
              for (int v = 0; v < 4; ++v)
                if (o + 4u * lane + (uint32_t)v < nn) {
                  const uint32_t off = e4[v] & kTMask;
                  atomicOr(&tile[off >> 5], 1u << (off & 31u));
                }
            }
          }
        } else {
          for (uint32_t o = 0; o < nn; o += kWave) {
            if (o + lane < nn) {
              const uint32_t off = abase[sb + ext + o + lane] & kTMask;
              atomicOr(&tile[off >> 5], 1u << (off & 31u));
            }
          }
        }
        lk = sb + ext + ent_words<P3>(d.xo);
      }
    }
    BK_STAMP(2);  // overflow chains
    __syncthreads();  // the tile is complete
    BK_STAMP(3);  // tile barrier

    // write the tile: bytes [t << (kTL-3), ...) of this filter, up to the
    // 16-byte-rounded bitmap length (pad bytes are zero: no position lands
    // there); each 16-byte word is re-zeroed as it is read out
    const uint64_t tile_bytes = 1ull << (kTL - 3);
    const uint64_t b0 = (uint64_t)t * tile_bytes;
    const uint32_t nvec = (uint32_t)(min(tile_bytes, (uint64_t)d.alloc_bytes - b0) >> 4);
    uint4 *out4 = reinterpret_cast<uint4 *>(bitmaps + d.bitmap_off + b0);
    uint4 *t4 = reinterpret_cast<uint4 *>(tile);
    if (tid == 0) *ovf = 0;  // next set after the barrier below
    for (uint32_t i = tid; i < kTileWords / 4; i += kBlock) {
      const uint4 v = t4[i];
      t4[i] = make_uint4(0, 0, 0, 0);
      if (i < nvec) {
        if (a.nt_bitmap) store_nt(out4 + i, v);
        else out4[i] = v;
      }
    }
    __syncthreads();  // read out and zero again; counts staged for the next tile
    BK_STAMP(4);  // write + zero tile
  }
  BK_STAMP_FLUSH(1);
}

// ---------------------------------------------------------------- host plan
struct BkPlan {
  BkArgs a;
  std::vector<BkDesc> f;
  bool dt = false;
  uint64_t area_words = 0, count_words = 0, ft_bytes = 0, ws_bytes = 0;
  uint64_t pair_off = 0, scratch_off = 0;  // var-len keys: (h1, h2) pairs, then the hashing pass's table
  uint32_t grid_a = 0, grid_b = 0;
  uint32_t depth_b = 8;
  bool p3 = false;  // 24-bit entries (ADL_BLOOM_BK_P3)
  size_t lds_a = 0, lds_b = 0;
};

constexpr size_t kLdsB = (size_t)(kTileWords + 3 * kMaxSlices + kWaves + 2) * 4;

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
  p.p3 = k == 6 && adl_host::env_on("ADL_BLOOM_BK_P3", false);  // (the runtime-k pass A writes u32 entries)
  auto words = [&](uint64_t e) { return p.p3 ? e / 4 * 3 : e; };  // entries (multiple of 16) -> words
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
      pool = ((kl + xo - 1) / xo + 2) * (words(xo) + kLink);
    }
    const uint64_t stride = T * (words(cap) + kLink) + pool;
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
  const uint32_t tpw = (tmax + kWaves - 1) / kWaves;  // flush owners per wave
  tmax = (uint32_t)adl_host::round_up(tmax, 4);
  // pass A LDS: TM x S ring slots and 3 words per tile, the flush lists, the
  // pair table.  S: the largest power of two whose rings fit beside a
  // 256-slot pair table and whose full flush (S/16 granules per owner) fits a
  // wave's list; the pair table then takes what is left, up to 2^12 slots.
  const uint32_t lists = 2 * kWaves * kListCap + 4 + kWave;  // + pool word, 2 flags, pad; the sink words
  uint32_t S = 0;
  for (uint32_t r = kRingMax; r >= kRingMin; r /= 2)
    if (tmax * (r + 3) + lists + 256 <= kLdsWords && tpw * (r / kGran) <= kListCap) {
      S = r;
      break;
    }
  if (!S) return ADL_ERR_TOO_LARGE;
  const uint32_t fixed = tmax * (S + 3) + lists;
  uint32_t dd = 0;
  if (adl_host::env_on("ADL_BLOOM_HASH_DEDUP", true))
    for (uint32_t lg = 12; lg >= 8; --lg)
      if (fixed + (1u << lg) <= kLdsWords) {
        dd = lg;
        break;
      }
  p.a.nf = nf;
  p.a.k = k;
  p.a.total_slices = slice;
  p.a.total_tiles = tile;
  p.a.tmax = tmax;
  p.a.ring = S;
  p.a.dd_log2 = dd;
  p.a.nt_bitmap = adl_host::env_on("ADL_BLOOM_NT_BITMAP", true) ? 1u : 0u;
  p.area_words = adl_host::round_up(area, 64);
  p.count_words = adl_host::round_up(cntw + kPad, 64);
  for (BkDesc &d : p.f) d.count_base += p.area_words;  // the count tables follow the areas
  p.ft_bytes = p.dt ? adl_host::round_up(nf * sizeof(BkDesc), 256) + 4ull * (slice + tile) + 256 : 0;
  // Every key shape is sized for (the workspace query does not carry it): var-len
  // keys add their (h1, h2) pairs and, past kMaxFilt filters, the hashing pass's
  // descriptor table (bloom_build.hip: at most 128 B per filter and one word
  // per run of >= 256 keys).
  p.pair_off = adl_host::round_up((p.area_words + p.count_words) * 4 + p.ft_bytes, 256);
  p.scratch_off = p.pair_off + adl_host::round_up(8 * total_n + 16, 256);
  const uint64_t scratch = nf > (uint32_t)kMaxFilt ? adl_host::round_up(128ull * nf, 256) + 4 * (total_n / 256 + nf + 1) + 512
                                                   : 0;
  p.ws_bytes = p.scratch_off + scratch + 256;
  p.lds_a = (size_t)(fixed + (dd ? (1u << dd) : 0u)) * 4;
  p.lds_b = kLdsB;
  {
    const char *e = getenv("ADL_BLOOM_BK_DEPTH");
    p.depth_b = e ? (uint32_t)atoi(e) : 8u;
  }
  p.grid_a = std::min<uint32_t>(slice, cus);
  p.grid_b = std::min<uint32_t>(tile, cus);
  if (!p.dt) std::copy(p.f.begin(), p.f.end(), p.a.f);
  return ADL_OK;
}

template <bool DT, class Src>
int launch(BkPlan &p, Src keys, uint8_t *bitmaps, void *ws, hipStream_t st, hipEvent_t *ev) {
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
    const int rc =
        p.a.k != 6 ? go(adl_host::lds_limit<bk_bin16_kernel<0, Src, DT, false>>, bk_bin16_kernel<0, Src, DT, false>)
        : p.p3     ? go(adl_host::lds_limit<bk_bin16_kernel<6, Src, DT, true>>, bk_bin16_kernel<6, Src, DT, true>)
                   : go(adl_host::lds_limit<bk_bin16_kernel<6, Src, DT, false>>, bk_bin16_kernel<6, Src, DT, false>);
    if (rc) return rc;
  } else if (ev) {  // no keys: an empty pass-A interval
    if (ev[0]) ADL_HIP_TRY(hipEventRecord(ev[0], st));
    if (ev[1]) ADL_HIP_TRY(hipEventRecord(ev[1], st));
  }
  auto go_b = [&](auto lim, auto kern) -> int {
    if (int rc = lim()) return rc;
    hipExtLaunchKernelGGL(kern, dim3(p.grid_b), dim3(kBlock), p.lds_b, st, ev ? ev[2] : nullptr,
                          ev ? ev[3] : nullptr, 0, p.a, (const uint32_t *)w, bitmaps, ft);
    ADL_HIP_TRY(hipGetLastError());
    return ADL_OK;
  };
  // pass-B units per pipeline stage (ADL_BLOOM_BK_DEPTH, tuning)
  const bool p3 = p.p3;
  if (p3) return go_b(adl_host::lds_limit<bk_tile_kernel<8, DT, true>>, bk_tile_kernel<8, DT, true>);
  if (p.depth_b >= 16) return go_b(adl_host::lds_limit<bk_tile_kernel<16, DT, false>>, bk_tile_kernel<16, DT, false>);
  if (p.depth_b <= 4) return go_b(adl_host::lds_limit<bk_tile_kernel<4, DT, false>>, bk_tile_kernel<4, DT, false>);
  return go_b(adl_host::lds_limit<bk_tile_kernel<8, DT, false>>, bk_tile_kernel<8, DT, false>);
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

namespace {
template <class Src>
int build_src(Src src, const uint64_t *key_begin, uint64_t key0, uint32_t nf, int32_t bpk, uint8_t *d_bitmaps,
              const uint64_t *bitmap_off, void *ws, uint64_t ws_bytes, hipStream_t st, hipEvent_t *ev) {
  const std::vector<uint64_t> counts = group_counts(key_begin, nf);
  BkPlan p;
  if (int rc = make_plan(counts.data(), nf, bpk, p)) return rc;
  if (!ws || ws_bytes < p.ws_bytes) return ADL_ERR_WORKSPACE;
  for (uint32_t f = 0; f < nf; ++f) {
    if (bitmap_off[f] % 16) return ADL_ERR_INVALID_ARG;
    p.f[f].key_begin = key_begin[f] - key0;
    p.f[f].bitmap_off = bitmap_off[f];
    if (!p.dt) p.a.f[f] = p.f[f];
  }
  return p.dt ? launch<true>(p, src, d_bitmaps, ws, st, ev) : launch<false>(p, src, d_bitmaps, ws, st, ev);
}
}  // namespace

int build16(const uint4 *d_keys, const uint64_t *key_begin, uint32_t nf, int32_t bpk, uint8_t *d_bitmaps,
            const uint64_t *bitmap_off, void *ws, uint64_t ws_bytes, hipStream_t st, hipEvent_t *ev) {
  return build_src(BkSrc16{d_keys}, key_begin, 0, nf, bpk, d_bitmaps, bitmap_off, ws, ws_bytes, st, ev);
}

int var_layout(const uint64_t *counts, uint32_t nf, int32_t bpk, uint64_t *pair_off, uint64_t *scratch_off) {
  BkPlan p;
  if (int rc = make_plan(counts, nf, bpk, p)) return rc;
  *pair_off = p.pair_off;
  *scratch_off = p.scratch_off;
  return ADL_OK;
}

int build_pairs(const uint2 *d_pairs, const uint64_t *key_begin, uint32_t nf, int32_t bpk, uint8_t *d_bitmaps,
                const uint64_t *bitmap_off, void *ws, uint64_t ws_bytes, hipStream_t st, hipEvent_t *ev) {
  return build_src(BkSrcPairs{d_pairs}, key_begin, key_begin[0], nf, bpk, d_bitmaps, bitmap_off, ws, ws_bytes, st,
                   ev);
}

#ifdef ADL_BLOOM_STAMPS
int debug_stamps(uint64_t *out, uint64_t n) {
  const uint64_t bytes = std::min<uint64_t>(n, 2 * 256 * 16 * 8) * 8;
  ADL_HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bk_stamps), bytes, 0, hipMemcpyDeviceToHost));
  return ADL_OK;
}
#endif

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
