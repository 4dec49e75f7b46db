// adlsm-tree_amd/csrc/bloom_build.hip -- MI355X (gfx950) bloom-filter build.
//
// Replaces BloomFilter::Keys2Block (reference src/filter_block.cpp:9-33): for
// every key, h1/h2 = murmur3 with two seeds, then k bits (h1 + j*h2) % m are
// ORed into an (n*bpk+7)-byte bitmap.  The result is an order-independent OR,
// so any decomposition gives the reference's bitmap bit for bit.
//
// Design (DESIGN.md "Build kernels"): random single-bit RMW into a 100 MB
// bitmap cannot go through device-scope global atomics (they execute at the
// memory side at ~20 G lanes/s chip-wide, ~3 ms for 60 M bit-sets), so the
// bit-sets are routed through LDS in two passes:
//
//   pass A  bloom_bin_kernel   one workgroup per chunk of C keys: coalesced
//           key loads, both hashes, k positions per key, an LDS counting sort
//           of the chunk's k*C positions by bitmap tile, one coalesced write of
//           the sorted chunk to its workspace region and of the per-tile start
//           offsets to the (tile, chunk) table.
//   pass B  bloom_tile_kernel  one workgroup per bitmap tile of 2^TL bits held
//           in LDS: gathers that tile's segment from every chunk region,
//           ds_or_b32 of every position into LDS, then one coalesced write of
//           the finished tile.  Every bitmap byte is written exactly once, so
//           the bitmap needs no zero-fill.
//
// Pass A skips a key whose hash pair its workgroup already counted (the
// reference's murmur variant repeats pairs heavily; see bloom_bin16_kernel).
// Variable-length keys are hashed first, in length-sorted runs staged in LDS
// (hash_var_kernel), and pass A then bins the (h1, h2) pairs.
//
// Designs measured slower (a direct atomicOr build, collapsed-key stamping,
// live-key compaction, a bucketed pass A, split-seed hashing, dynamic tile
// queues, ...) are not in this library; HISTORY.md keeps their numbers and
// git history their code.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <mutex>
#include <type_traits>
#include <vector>

#include "bloom_common.hpp"
#include "probe_server.hpp"

using namespace adl_dev;

namespace {

constexpr uint32_t kLdsWordsPerCu = 40960;  // 160 KiB of LDS per CU
constexpr int kKptMax = 8;          // keys per thread, pass A
constexpr int kBlockB = 1024;       // pass B threads per workgroup
constexpr int kDepthB = 8;          // segments per pipeline stage per wave, pass B (ADL_BLOOM_DEPTH)
constexpr int kSegBatch = 2048;     // segment descriptors staged in LDS per batch, pass B
constexpr uint32_t kTablePad = 64;  // spare words after the table
constexpr int kMaxFilters = 8;      // filters whose descriptors ride in the kernargs (more: a device table)
constexpr uint32_t kHistMax = 2049; // tiles per filter + 1 (m < 2^31, TL >= ... keeps T <= 2048)
constexpr uint32_t kMinTileLog2 = 10;
constexpr uint32_t kMaxTileLog2 = 20;     // 128 KiB LDS tile
constexpr uint32_t kTargetWorkgroups = 512;
constexpr uint32_t kFewTiles = 256;       // tiles per filter below which smaller tiles are taken
constexpr uint32_t kMinRun = 64;          // ... while a chunk's run per tile stays this long (positions)
constexpr uint32_t kChunkEst = 5500;      // keys per pass-A chunk (k = 6), for that estimate
constexpr uint32_t kClaimTiles = 10;      // claim layout by default only up to this many tiles per filter
constexpr uint32_t kClaimSlack = 125;     // claim layout: region = k*C positions * 125 %
constexpr uint32_t kClaimSigma = 4;       // ... kept when a tile's share clears its mean run by 4 sigma
#ifndef ADL_HV_KEYS
#define ADL_HV_KEYS 512
#endif
constexpr uint32_t kHvKeys = ADL_HV_KEYS;  // keys per hash_var_kernel run
constexpr uint32_t kBlockA = 1024;        // pass A threads per workgroup (one workgroup per CU)
constexpr uint32_t kDdLog2Max = 11;       // log2 slots of pass A's repeated-hash table, at most
// LDS pass A leaves free on its CU (3 KiB): the resident probe server's
// workgroup (probe_server.hip, 2.25 KiB) fits beside it, so a Get never waits for
// a build's persistent grid (DB::Get probes while DoCompaction builds,
// src/db.cpp:164-172, 263).  The headline's chunk still fits 7 whole rounds.
constexpr uint32_t kLdsReserveWords = 768;

struct FilterDesc {
  uint64_t key_begin;   // first key (index into the key set)
  uint64_t pos_base;    // word offset of this filter's chunk-0 region
  uint64_t table_base;  // u32-word offset of this filter's (tile, chunk) table
  uint64_t bitmap_off;  // output byte offset
  uint32_t n;           // keys
  uint32_t alloc_bytes; // bitmap bytes rounded up to 16
  uint32_t chunk_base;  // first pass-A workgroup
  uint32_t tile_base;   // first pass-B workgroup
  uint32_t chunks;      // W
  uint32_t tiles;       // T
  FastMod mod;          // m = 8 * bitmap bytes
  uint32_t sc_base;     // first hash_var_kernel workgroup (variable-length keys)
  uint32_t pad_;
};

struct BuildArgs {
  uint32_t nf;     // filters in this launch
  uint32_t k;      // probes per key
  uint32_t C;      // keys per chunk
  uint32_t TL;     // log2 tile bits
  uint32_t cap;    // positions per chunk region (k*C; C % 4 == 0 keeps regions 16-byte aligned)
  uint32_t hist_words;  // pass A LDS tile counters (max tiles per filter + 1, rounded to 4)
  uint32_t stage_keys; // pass A: LDS-staged variable-length keys (16-byte-aligned key buffers only)
  uint32_t dedup;      // skip a key equal to its predecessor in the same filter (ADL_BLOOM_SKIP_ADJACENT_DUPLICATES)
  // Claim layout (bloom_bin16_kernel<..., CL> and the pass B after it): a chunk
  // region gives each of a filter's T tiles tcap = (cap / T) & ~3 fixed slots,
  // a position takes its slot with one ds_add_rtn (no count pass, no scan), and
  // a (tile, chunk) table entry is (start << 16) | length.
  uint32_t claim;
  uint32_t dd_log2;    // bloom_bin16_kernel: log2 slots of the table that skips repeated hashes
                       // (0: off; ADL_BLOOM_HASH_DEDUP)
  uint32_t exp;        // diagnostics build only (ADL_BLOOM_EXP bits, wrong results): pass A 1 no hash,
                       // 2 no position stores, 32 no reduction; pass B 4 no ds_or, 8 no bitmap stores;
                       // hashing pass 16 no hashing
  uint32_t pad_;
  FilterDesc f[kMaxFilters];
};

__device__ __forceinline__ int find_filter_by_chunk(const BuildArgs &a, uint32_t wg) {
  int f = 0;
#pragma unroll
  for (int i = 1; i < kMaxFilters; ++i)
    if ((uint32_t)i < a.nf && wg >= a.f[i].chunk_base) f = i;
  return f;
}

__device__ __forceinline__ int find_filter_by_tile(const BuildArgs &a, uint32_t wg) {
  int f = 0;
#pragma unroll
  for (int i = 1; i < kMaxFilters; ++i)
    if ((uint32_t)i < a.nf && wg >= a.f[i].tile_base) f = i;
  return f;
}

__device__ __forceinline__ int find_filter_by_run(const BuildArgs &a, uint32_t sc) {
  int f = 0;
#pragma unroll
  for (int i = 1; i < kMaxFilters; ++i)
    if ((uint32_t)i < a.nf && sc >= a.f[i].sc_base) f = i;
  return f;
}

// A launch of more than kMaxFilters filters (a compaction's tables in one
// launch pair) finds its descriptors in the workspace: the descriptor array
// and, filled on the device by fill_maps_kernel, one filter index per pass-A
// chunk, per pass-B tile and per hashing run.  Constant address space, so a
// lookup is one scalar load.
template <typename T>
using cptr = const __attribute__((address_space(4))) T *;
struct FilterTable {
  cptr<FilterDesc> fd;
  cptr<uint32_t> chunk_f, tile_f, sc_f;
};

template <bool DT>
struct Filt;
template <>
struct Filt<false> {  // descriptors in BuildArgs::f
  // a reference into the kernarg segment: fields load from it as needed (a
  // copy of a dynamically indexed kernarg element goes through scratch)
  __device__ static const FilterDesc &at(const BuildArgs &a, const FilterTable &, int i) { return a.f[i]; }
  __device__ static int of_chunk(const BuildArgs &a, const FilterTable &, uint32_t wg) {
    return find_filter_by_chunk(a, wg);
  }
  __device__ static int of_tile(const BuildArgs &a, const FilterTable &, uint32_t wg) {
    return find_filter_by_tile(a, wg);
  }
  __device__ static int of_run(const BuildArgs &a, const FilterTable &, uint32_t sc) { return find_filter_by_run(a, sc); }
};
template <>
struct Filt<true> {  // descriptors in the workspace's FilterTable
  __device__ static FilterDesc at(const BuildArgs &, const FilterTable &t, int i) {
    static_assert(sizeof(FilterDesc) % 16 == 0, "descriptors load as whole uint4s");
    constexpr int NV = sizeof(FilterDesc) / 16;
    const cptr<u32x4_t> src = reinterpret_cast<cptr<u32x4_t>>(t.fd) + (uint32_t)i * NV;
    u32x4_t v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = src[j];
    FilterDesc d;
    __builtin_memcpy(&d, v, sizeof(d));
    return d;
  }
  __device__ static int of_chunk(const BuildArgs &, const FilterTable &t, uint32_t wg) { return (int)t.chunk_f[wg]; }
  __device__ static int of_tile(const BuildArgs &, const FilterTable &t, uint32_t wg) { return (int)t.tile_f[wg]; }
  __device__ static int of_run(const BuildArgs &, const FilterTable &t, uint32_t sc) { return (int)t.sc_f[sc]; }
};

// FilterTable maps: block f writes filter f's chunk, tile and run ranges.
__global__ __launch_bounds__(256) void fill_maps_kernel(const FilterDesc *__restrict__ fd, uint32_t *__restrict__ chunk_f,
                                                        uint32_t *__restrict__ tile_f, uint32_t *__restrict__ sc_f) {
  const uint32_t f = blockIdx.x;
  const FilterDesc d = fd[f];
  for (uint32_t i = threadIdx.x; i < d.chunks; i += 256) chunk_f[d.chunk_base + i] = f;
  for (uint32_t i = threadIdx.x; i < d.tiles; i += 256) tile_f[d.tile_base + i] = f;
  const uint32_t runs = (d.n + kHvKeys - 1) / kHvKeys;
  for (uint32_t i = threadIdx.x; i < runs; i += 256) sc_f[d.sc_base + i] = f;
}

// ---------------------------------------------------------------- work queues
// A persistent grid's static order assigns workgroup b the items of stripe b,
// so a workgroup that starts late or runs slow -- one sharing its CU with the
// resident probe server's wave (probe_server.hip) -- makes the whole pass
// wait for its stripe.  While a server exists the build passes take their
// items from these queues instead: XCD group h = blockIdx % 8 (workgroups
// that share an L2) hands out the items of the static order's group h (item
// i of round r is r*G + h*(G/8) + i % (G/8)) through counter q[16h], and a
// workgroup whose group has run dry takes from the next groups.  A slow
// workgroup then just takes fewer items.  The counters start at 0 (the host
// clears them before pass A).  Called by one thread; G % 8 == 0.
constexpr uint32_t kQueueWords = 256;  // pass A's 8 counters, then pass B's, 64 B apart
constexpr uint32_t kQueueMinItems = 16;  // items per workgroup below which a pass keeps the static order
struct GroupQueue {
  uint32_t *q;
  uint32_t G, total, g;
  uint32_t dry;  // bit h: group h ran dry (this thread's view)
  __device__ GroupQueue(uint32_t *q_, uint32_t G_, uint32_t total_)
      : q(q_), G(G_), total(total_), g(blockIdx.x % 8), dry(0) {}
  __device__ uint32_t next() {
    const uint32_t per = G / 8;
    for (uint32_t s = 0; s < 8; ++s) {
      const uint32_t h = (g + s) & 7u;
      if ((dry >> h) & 1u) continue;
      const uint32_t i = atomicAdd(q + 16 * h, 1u);
      const uint32_t t = (i / per) * G + h * per + i % per;
      if (t < total) return t;
      dry |= 1u << h;
    }
    return total;
  }
};

// ---------------------------------------------------------------- diagnostics
// Built only with -DADL_BLOOM_STAMPS (make stamps): wave 0 of every
// workgroup accumulates s_memtime cycles per kernel phase; read back with
// adl_bloom_debug_stamps() (tools/stamps.py).  The product library has none
// of this.
#ifdef ADL_BLOOM_STAMPS
__device__ uint64_t g_stamps[3][2048][8];  // pass A, pass B, hashing pass
#define STAMP_DECL                                  \
  uint64_t st_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}; \
  uint64_t st_t_ = __builtin_amdgcn_s_memtime();
#define STAMP(i)                                      \
  do {                                                \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    st_acc_[i] += t_ - st_t_;                         \
    st_t_ = t_;                                       \
  } while (0)
#define STAMP_FLUSH(pass)                                                         \
  do {                                                                            \
    if (threadIdx.x == 0 && blockIdx.x < 2048)                                    \
      for (int i_ = 0; i_ < 8; ++i_) g_stamps[pass][blockIdx.x][i_] = st_acc_[i_]; \
  } while (0)
#else
#define STAMP_DECL
#define STAMP(i) do { } while (0)
#define STAMP_FLUSH(pass) do { } while (0)
#endif

// ---------------------------------------------------------------- pass A
// At most 120 VGPRs per lane (the attribute counts arch VGPRs and is doubled
// for gfx950's unified file): four pass-A waves per SIMD then leave 32, the
// resident probe server's wave (probe_server.hip), so a Get is served on the
// same CU while a build runs.
#define kPassARegs __attribute__((amdgpu_num_vgpr(60)))
// Register prefetch of a chunk's keys.  Only the fixed 16-byte view has raw
// words worth holding (4 VGPRs per key); the other views hash straight from
// memory.
template <class Keys>
struct KeyRegs {
  static constexpr bool kPrefetch = false;
  uint32_t dummy;
};
template <>
struct KeyRegs<Keys16> {
  static constexpr bool kPrefetch = true;
  uint4 raw;
};

// The generic pass A (any key shape, any k, adjacent-duplicate skipping).
// Persistent, one workgroup per CU.  A workgroup processes one chunk per round
// of the grid; the keys of its next chunk are already in flight into
// registers while the current one is hashed, sorted and stored.
//
// KFIX > 0: k known at compile time, positions kept in registers between the
// count and the scatter; KFIX == 0: runtime k, positions recomputed.
template <int BLOCK, int KFIX, int KPT, class Keys, bool DT>
__global__ __launch_bounds__(BLOCK) kPassARegs void bloom_bin_kernel(BuildArgs a, Keys keys,
                                                            uint32_t *__restrict__ pos_ws,
                                                            uint32_t *__restrict__ table_ws,
                                                            uint32_t total_chunks, FilterTable ft) {
  using FT = Filt<DT>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int tid = threadIdx.x;
  const uint32_t C = a.C;
  const uint32_t k = KFIX > 0 ? (uint32_t)KFIX : a.k;
  const uint32_t TL = a.TL;
  const uint32_t tmask = (1u << TL) - 1u;
  uint32_t *hist = lds;                        // T+1 counters, later cursors
  uint32_t *scratch = lds + a.hist_words;      // scan scratch (BLOCK/64 + 1, padded to 32)
  uint32_t *lpos = lds + a.hist_words + 32;    // k*C sorted tile offsets
  constexpr bool PF = KeyRegs<Keys>::kPrefetch;
  // Variable-length keys are hashed in length order: a counting sort of the
  // chunk's keys by length (LDS perm[]), then slot i of wave w takes the 64
  // keys at sorted positions (i*NW + w)*64 .. +63 -- lanes of a wave hash keys
  // of nearly equal length and every wave gets an even share of long keys.
  constexpr bool SORT = std::is_same<Keys, KeysVar>::value;
  constexpr int NW = BLOCK / kWave;
  uint32_t *perm = lpos + k * C;   // C key indices (SORT)
  uint32_t *lbin = perm + C;       // 256 length-class counters (SORT)
  const int lane = tid & (kWave - 1), wave = tid / kWave;

  auto fetch = [&](uint32_t chunk, KeyRegs<Keys> (&r)[KPT]) {
    if constexpr (PF) {
      const auto &d = FT::at(a, ft, FT::of_chunk(a, ft, chunk));
      const uint32_t first = (chunk - d.chunk_base) * C;
      const uint32_t cnt = min(C, d.n - first);
#pragma unroll
      for (int i = 0; i < KPT; ++i) {
        const uint32_t idx = tid + i * BLOCK;
        if (idx < cnt) {
          r[i].raw = load_nt(keys.keys + d.key_begin + first + idx);
        }
      }
    }
  };

  // Round r of the persistent grid covers chunks [r*G, (r+1)*G).  Inside a
  // round, the 8 XCDs (blocks b, b+8, ... share one under round-robin
  // dispatch) each take G/8 consecutive chunks, so the 4-byte (tile, chunk)
  // table entries of neighbouring chunks -- one 64-byte line holds 16 -- are
  // written from one L2.  Speed only: any placement gives the same result.
  const uint32_t G = gridDim.x;
  const uint32_t slot = G % 8 == 0 ? (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8 : blockIdx.x;
  const uint32_t rounds = (total_chunks + G - 1) / G;
  KeyRegs<Keys> cur[KPT];
  if (slot < total_chunks) fetch(slot, cur);
  for (uint32_t i = tid; i < a.hist_words; i += BLOCK) hist[i] = 0;
  STAMP_DECL

  for (uint32_t r = 0; r < rounds; ++r) {
    const uint32_t wg = r * G + slot;
    if (wg >= total_chunks) break;  // only the last round is partial
    const auto &d = FT::at(a, ft, FT::of_chunk(a, ft, wg));
    const uint32_t w = wg - d.chunk_base;
    const uint32_t first = w * C;
    const uint32_t cnt = min(C, d.n - first);
    const uint32_t T = d.tiles;
    const FastMod mod = d.mod;

    KeyRegs<Keys> nxt[KPT];
    if (wg + G < total_chunks) fetch(wg + G, nxt);

    // slot i of this thread: valid[i] and the key index it hashes
    auto slot_pos = [&](int i) -> uint32_t {
      return SORT ? (uint32_t)((i * NW + wave) * kWave + lane) : (uint32_t)(tid + i * BLOCK);
    };
    uint32_t kidx[KPT];
    // Variable-length keys are staged through LDS in windows of wcap bytes at
    // a fixed stride S = wcap - M (keys of at most M bytes starting in window
    // w lie wholly inside it; longer keys, and keys past kNWin windows, are
    // hashed from global memory).  The counting sort orders the chunk's keys
    // by (window, length class), so the 64 keys of a wave slot share a window
    // and nearly share a length: each window pass hashes only its own slots,
    // with lanes of one slot running equally long loops.
    constexpr uint32_t kNWin = 4;
    uint64_t A0 = 0, B1 = 0;
    uint32_t wcap = 0, S = 0, M = 0;
    FastMod divS{};
    bool staged = false;
    if constexpr (SORT) {
      const uint64_t kb = d.key_begin + first;
      A0 = keys.offs[kb] & ~15ull;
      B1 = keys.offs[kb + cnt];
      wcap = (4u * k * C - 16u) & ~15u;
      M = min(4096u, wcap / 2);
      S = wcap - M;
      staged = a.stage_keys && wcap >= 64 && B1 - A0 < (1ull << 31);
      if (staged) divS = fastmod_for(S);
    }
    auto sort_bin = [&](uint64_t o0, uint32_t len) -> uint32_t {
      if (!staged) return min(len >> 2, 255u);
      const uint32_t w = fastdiv((uint32_t)(o0 - A0), divS);
      return (len > M || w >= kNWin) ? 255u : w * 64u + min(len >> 2, 62u);
    };
    if constexpr (SORT) {
      for (uint32_t i = tid; i < 256; i += BLOCK) lbin[i] = 0;
      __syncthreads();
      uint32_t lb[KPT], lr[KPT];
#pragma unroll
      for (int i = 0; i < KPT; ++i) {
        const uint32_t idx = tid + i * BLOCK;
        if (idx < cnt) {
          const uint64_t ki = d.key_begin + first + idx;
          const uint64_t o0 = keys.offs[ki];
          lb[i] = sort_bin(o0, (uint32_t)(keys.offs[ki + 1] - o0));
          lr[i] = atomicAdd(&lbin[lb[i]], 1u);
        }
      }
      __syncthreads();
      block_excl_scan_array<BLOCK>(lbin, 256, scratch);
#pragma unroll
      for (int i = 0; i < KPT; ++i) {
        const uint32_t idx = tid + i * BLOCK;
        if (idx < cnt) perm[lbin[lb[i]] + lr[i]] = idx;
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < KPT; ++i) kidx[i] = slot_pos(i) < cnt ? perm[slot_pos(i)] : 0u;
      STAMP(0);
    } else {
#pragma unroll
      for (int i = 0; i < KPT; ++i) kidx[i] = tid + i * BLOCK;
    }

    uint32_t h1[KPT], h2[KPT];
    if constexpr (SORT) {
      const uint64_t kb = d.key_begin + first;
      if (staged) {
        uint4 *stage4 = reinterpret_cast<uint4 *>(lpos);
        uint32_t ks0[KPT], klen[KPT];  // key start (relative to A0; ~0 if the slot is
                                       // empty or hashed from global) and length
        uint32_t pending = 0;          // bit i: slot i still to hash
#pragma unroll
        for (int i = 0; i < KPT; ++i) {
          h1[i] = h2[i] = 0;
          ks0[i] = ~0u;
          klen[i] = 0;
          if (slot_pos(i) < cnt) {
            const uint64_t o0 = keys.offs[kb + kidx[i]];
            const uint32_t rel = (uint32_t)(o0 - A0);
            klen[i] = (uint32_t)(keys.offs[kb + kidx[i] + 1] - o0);
            if (klen[i] <= M && rel < kNWin * S) ks0[i] = rel;
            pending |= 1u << i;
          }
        }
        STAMP(1);  // setup: key starts and lengths
        const uint32_t nwin = min(kNWin, (uint32_t)((B1 - A0 + S - 1) / S));
        for (uint32_t win = 0; win < nwin; ++win) {
          const uint64_t wb = A0 + (uint64_t)win * S;
          const uint64_t we = min(wb + wcap, B1);
          const uint32_t nv = (uint32_t)((we - wb) >> 4);
          const uint4 *src = reinterpret_cast<const uint4 *>(keys.keys + wb);
          for (uint32_t v = tid; v < nv; v += BLOCK) stage4[v] = src[v];
          const uint32_t rem = (uint32_t)(we - wb) & 15u;  // last partial vector, bytewise
          if (rem && (uint32_t)tid < rem)
            reinterpret_cast<uint8_t *>(lpos)[nv * 16 + tid] = keys.keys[wb + nv * 16 + tid];
          __syncthreads();  // window staged
          STAMP(6);
          const uint32_t wlo = win * S;
#pragma unroll
          for (int i = 0; i < KPT; ++i) {
            if (ks0[i] - wlo < S) {  // starts in this window (unsigned wrap for earlier keys)
              hash_lds(lpos, ks0[i] - wlo, klen[i], h1[i], h2[i]);
              pending &= ~(1u << i);
            }
          }
          __syncthreads();  // window consumed before the next one overwrites it
          STAMP(7);
        }
#pragma unroll
        for (int i = 0; i < KPT; ++i)
          if (pending & (1u << i)) keys.hash(kb + kidx[i], h1[i], h2[i]);
      } else {
#pragma unroll
        for (int i = 0; i < KPT; ++i) {
          h1[i] = h2[i] = 0;
          if (slot_pos(i) < cnt) keys.hash(d.key_begin + first + kidx[i], h1[i], h2[i]);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < KPT; ++i) {
        h1[i] = h2[i] = 0;
        if (slot_pos(i) < cnt) {
          if constexpr (PF) hash16(cur[i].raw, h1[i], h2[i]);
          else keys.hash(d.key_begin + first + kidx[i], h1[i], h2[i]);
        }
      }
    }
    // live slots: valid, and (dedup) not equal to the previous key of the
    // filter -- a repeated key sets the same bits, so skipping it leaves the
    // bitmap unchanged (src/keys.cpp:61-74 feeds versions of a user key in a row)
    uint32_t live = 0;
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      if (slot_pos(i) < cnt) {
        const uint32_t ki = first + kidx[i];
        if (!(a.dedup && ki > 0 && keys.same_as_prev(d.key_begin + ki))) live |= 1u << i;
      }
    }
    __syncthreads();  // hist cleared (previous iteration / prologue); staging area free
    STAMP(1);

    constexpr int KR = KFIX > 0 ? KFIX : 1;
    uint32_t pos[KPT][KR];
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      if (live & (1u << i)) {
        if constexpr (KFIX > 0) {
#pragma unroll
          for (int j = 0; j < KFIX; ++j) {
            pos[i][j] = fastmod(h1[i] + (uint32_t)j * h2[i], mod);
            atomicAdd(&hist[pos[i][j] >> TL], 1u);
          }
        } else {
          for (uint32_t j = 0; j < k; ++j) {
            const uint32_t p = fastmod(h1[i] + j * h2[i], mod);
            atomicAdd(&hist[p >> TL], 1u);
          }
        }
      }
    }
    __syncthreads();
    STAMP(2);

    // Exclusive scan: hist[t] = start of tile t's run; hist[T] = k * live keys.
    // the table rows below are written by the thread that scanned them
    const uint32_t total = block_excl_scan_array_1b<BLOCK>(hist, T + 1, scratch);

    // (tile, chunk) table, T+1 rows of W entries: row t = start of tile t.
    uint32_t *tab = table_ws + d.table_base;
    for (uint32_t t = tid; t <= T; t += BLOCK) tab[(uint64_t)t * d.chunks + w] = hist[t];
    __syncthreads();
    STAMP(3);

    // Scatter tile offsets into LDS by tile (hist now serves as the cursor).
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      if (live & (1u << i)) {
        if constexpr (KFIX > 0) {
          // all k cursor bumps in flight before the first dependent write
          uint32_t slot_l[KFIX];
#pragma unroll
          for (int j = 0; j < KFIX; ++j) slot_l[j] = atomicAdd(&hist[pos[i][j] >> TL], 1u);
#pragma unroll
          for (int j = 0; j < KFIX; ++j) lpos[slot_l[j]] = pos[i][j] & tmask;
        } else {
          for (uint32_t j = 0; j < k; ++j) {
            const uint32_t p = fastmod(h1[i] + j * h2[i], mod);
            const uint32_t slot_l = atomicAdd(&hist[p >> TL], 1u);
            lpos[slot_l] = p & tmask;
          }
        }
      }
    }
    __syncthreads();
    STAMP(4);

    // Stream the sorted chunk out to region w (a.cap positions, 16-byte
    // aligned).  The hist is cleared for the next chunk meanwhile.
    for (uint32_t i = tid; i <= T; i += BLOCK) hist[i] = 0;
    uint32_t *dst = pos_ws + d.pos_base + (uint64_t)w * a.cap;
    const uint32_t nvec = total >> 2;
    const uint4 *src4 = reinterpret_cast<const uint4 *>(lpos);
    uint4 *dst4 = reinterpret_cast<uint4 *>(dst);
    for (uint32_t i = tid; i < nvec; i += BLOCK) dst4[i] = src4[i];
    for (uint32_t i = (nvec << 2) + tid; i < total; i += BLOCK) dst[i] = lpos[i];
    STAMP(5);

    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < KPT; ++i) cur[i] = nxt[i];
    }
  }
  STAMP_FLUSH(0);
}

// ---------------------------------------------------------------- var-len hashing
// Variable-length keys (Zipf lengths) hashed before pass A, in length order.
// A wave hashes 64 keys in lockstep, so it costs as much as its longest key;
// keys sorted by exact length within runs of S keys give waves of nearly
// equal keys.  One workgroup per run of a filter:
//   sort   key lengths counted into kHvBins exact-length bins in LDS, each
//          key's (start, length) scattered to its sorted slot;
//   stage  the run's key bytes copied into LDS with coalesced 16-byte loads
//          (each byte read from HBM once, in memory order);
//   hash   wave w takes groups of 64 sorted slots, each lane one key, hashed
//          from LDS (hash_lds: both seeds, alignbyte words); a key that lies
//          past the staging buffer is hashed from global memory;
//   out    (h1, h2) of sorted slot s to hp[chunk_base * C + first + s].
// The bitmap is an OR over the filter's keys, so pass A may take them in this
// order.  Pass A then reads 8 bytes per key (bloom_bin16_kernel over SrcH).
// Workgroups are small (256 threads), two per CU, so one workgroup's sort and
// staging overlap the other's hashing; no barrier waits for the slowest group
// (a workgroup ends when its last wave does).
// Measured against hashing in sorted order straight from global memory (lanes
// reading scattered keys): L2 missed each key line ~3.7 times, 1.4 GB fetched
// for 0.4 GB of keys.
#ifndef ADL_HV_BLOCK
#define ADL_HV_BLOCK 256
#endif
constexpr int kHvBlock = ADL_HV_BLOCK;
constexpr uint32_t kHvBins = 512;          // exact key length 0..510; 511 = longer
// LDS staging of a run's key bytes: 48 bytes per key (mean key ~40 B)
template <uint32_t S>
constexpr uint32_t hv_stage_bytes() {
  return S * 48;
}

template <uint32_t S>
constexpr size_t hv_lds_bytes() {
  return kHvBins * 4 + S * 4 + S * 2 + hv_stage_bytes<S>() + 16;  // + hash_lds's read slack
}

template <uint32_t S, bool DT>
__global__ __launch_bounds__(kHvBlock) void hash_var_kernel(BuildArgs a, KeysVar keys, uint2 *__restrict__ hp,
                                                            uint32_t total_sc, FilterTable ft) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t *bins = lds;                                             // kHvBins
  uint32_t *s_rel = lds + kHvBins;                                  // key start - base16, by sorted slot
  uint16_t *s_len = reinterpret_cast<uint16_t *>(s_rel + S);        // length (0xffff: >= 64 KiB)
  uint32_t *stage = reinterpret_cast<uint32_t *>(s_len + S);        // 16-byte aligned (S % 8 == 0)
  constexpr int KPT = S / kHvBlock;
  constexpr uint32_t NW = kHvBlock / kWave;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const uint32_t sc = blockIdx.x;
  if (sc >= total_sc) return;
  STAMP_DECL
  const auto &d = Filt<DT>::at(a, ft, Filt<DT>::of_run(a, ft, sc));
  const uint32_t first = (sc - d.sc_base) * S;
  const uint32_t cnt = min(S, d.n - first);
  const uint64_t kb = d.key_begin + first;
  const uint64_t base16 = keys.offs[kb] & ~15ull;
  const uint64_t end = keys.offs[kb + cnt];
  // staged: bytes [base16, base16 + sbytes), whole 16-byte blocks of the
  // (16-byte-aligned) key buffer, each holding at least one byte of the run:
  // up to 15 bytes past the run's last key are read, never a block the key
  // bytes do not touch (include/adl_bloom.h)
  constexpr uint32_t kStage = hv_stage_bytes<S>();
  static_assert(kStage % (16 * kHvBlock) == 0, "the staging loads cover kStage in whole rounds of 16 B per thread");
  const uint32_t sbytes = (uint32_t)min((end - base16 + 15) & ~15ull, (uint64_t)kStage);

  // ---- load the run's offsets and key bytes: every load in flight before
  // the first is used (clamped indices: unconditional, countable waits), so
  // the run costs one memory round trip
  constexpr int VPT = kStage / 16 / kHvBlock;
  const uint32_t nv = sbytes / 16;
  for (uint32_t i = tid; i < kHvBins; i += kHvBlock) bins[i] = 0;
  uint64_t o0[KPT], o1[KPT];
#pragma unroll
  for (int i = 0; i < KPT; ++i) {
    const uint32_t idx = min((uint32_t)(tid + i * kHvBlock), cnt - 1u);
    o0[i] = keys.offs[kb + idx];
    o1[i] = keys.offs[kb + idx + 1];
  }
  u32x4_t v[VPT];  // (the ext-vector type: an array of uint4 held across the barrier goes to scratch)
  if (nv) {  // a run of empty keys has no byte to stage (and maybe none to read)
    const u32x4_t *src = reinterpret_cast<const u32x4_t *>(keys.keys + base16);
#pragma unroll
    for (int i = 0; i < VPT; ++i) v[i] = src[min((uint32_t)(tid + i * kHvBlock), nv - 1u)];
  }
  __syncthreads();
  STAMP(0);  // offsets and key bytes loaded
  // ---- sort the run's keys by length
  uint32_t rk[KPT];
#pragma unroll
  for (int i = 0; i < KPT; ++i) {
    rk[i] = ~0u;
    if (tid + i * kHvBlock < cnt) {
      const uint32_t c = (uint32_t)min(o1[i] - o0[i], (uint64_t)(kHvBins - 1));
      rk[i] = (atomicAdd(&bins[c], 1u) << 9) | c;
    }
  }
  {
    u32x4_t *dst = reinterpret_cast<u32x4_t *>(stage);
#pragma unroll
    for (int i = 0; i < VPT; ++i)
      if (tid + i * kHvBlock < nv) dst[tid + i * kHvBlock] = v[i];
  }
  __syncthreads();
  STAMP(1);  // lengths counted, bytes staged
  if (wave == 0) {  // exclusive scan of the bins, 8 per lane
    constexpr int PER = kHvBins / kWave;
    uint32_t bv[PER], t = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) bv[j] = bins[lane * PER + j], t += bv[j];
    uint32_t run = wave_incl_scan(t, lane) - t;
#pragma unroll
    for (int j = 0; j < PER; ++j) bins[lane * PER + j] = run, run += bv[j];
  }
  __syncthreads();
  STAMP(2);  // bins scanned
#pragma unroll
  for (int i = 0; i < KPT; ++i) {
    if (rk[i] != ~0u) {
      const uint32_t slot = bins[rk[i] & (kHvBins - 1)] + (rk[i] >> 9);
      const uint64_t len = o1[i] - o0[i];
      // a key of 64 KiB or more, or one starting 4 GiB or more past the run's
      // first key, keeps its index in the run instead of its start (and is
      // hashed from global memory)
      const bool near = len < 0xffffu && o0[i] - base16 < 0xffffffffull;
      s_rel[slot] = near ? (uint32_t)(o0[i] - base16) : tid + i * kHvBlock;
      s_len[slot] = near ? (uint16_t)len : (uint16_t)0xffffu;
    }
  }
  __syncthreads();
  STAMP(3);  // slots scattered

  // ---- hash, group g = 64 sorted slots
  const uint32_t groups = (cnt + kWave - 1) / kWave;
  uint2 *out = hp + (uint64_t)d.chunk_base * a.C + first;
  // longest groups first (slots are sorted by length): the waves start on the
  // groups that set the workgroup's end, and the short ones fill in behind.
  // (A queue handing each free wave the next group measured the same: the
  // longest group alone sets the end; so did splitting the longest groups
  // between two waves by seed, which was slower.)
  for (uint32_t gi = wave; gi < groups; gi += NW) {
    const uint32_t g = groups - 1 - gi;
    const uint32_t s = g * kWave + lane;
    if (s >= cnt) continue;
    uint32_t len = s_len[s];
    const uint32_t r = s_rel[s];
    uint32_t h1, h2;
#ifdef ADL_BLOOM_STAMPS
    if (a.exp & 16) {  // diagnostics: no hashing (wrong pairs)
      out[s] = make_uint2(r, len | 1u);
      continue;
    }
#endif
    if (len < 0xffffu && (uint64_t)r + len <= sbytes) {
      hash_lds(stage, r, len, h1, h2);
    } else {
      uint64_t k0 = base16 + r;
      if (len == 0xffffu) {
        k0 = keys.offs[kb + r];
        len = (uint32_t)(keys.offs[kb + r + 1] - k0);
      }
      hash_bytes(keys.keys + k0, len, kSeed1, kSeed2, h1, h2);
    }
    out[s] = make_uint2(h1, h2);
  }
  STAMP(4);  // this wave's groups hashed and stored
  STAMP_FLUSH(2);
}

// Key sources of bloom_bin16_kernel: raw 16-byte keys (hashed in pass A), or
// the (h1, h2) pairs hash_var_kernel wrote in pass A's chunk grid.
struct Src16 {
  const uint4 *keys;
  using Raw = uint4;
  __device__ __forceinline__ Raw load(const FilterDesc &d, uint32_t chunk, uint32_t first, uint32_t idx) const {
    return load_nt(keys + d.key_begin + first + idx);
  }
  __device__ static __forceinline__ void hash(const Raw &r, uint32_t &h1, uint32_t &h2) { hash16(r, h1, h2); }
};

typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
struct SrcH {
  const uint2 *h;
  uint32_t C;
  using Raw = uint2;
  __device__ __forceinline__ Raw load(const FilterDesc &, uint32_t chunk, uint32_t, uint32_t idx) const {
    const u32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x2_t *>(h + (uint64_t)chunk * C + idx));
    return make_uint2(v.x, v.y);
  }
  __device__ static __forceinline__ void hash(const Raw &r, uint32_t &h1, uint32_t &h2) {
    h1 = r.x;
    h2 = r.y;
  }
};

// Pass A for the hot path (16-byte keys, compile-time k).  Same output as
// bloom_bin_kernel, with the chunk loop software-pipelined so VALU, LDS and
// memory overlap inside one workgroup:
//   count(c)   [fastmod + ds_add]          interleaved with  store(c-1)  [ds_read_b128 + global stores]
//   scan(c), table(c)
//   scatter(c) [ds_add_rtn + ds_write]     interleaved with  hash(c+1)   [murmur VALU]
//   prefetch keys of c+2
// so the murmur work hides under the scatter's LDS latency and the position
// stores drain under the next count.
//
// CL (claim layout, a.claim): every position claims a slot of its tile's
// fixed share of the chunk region with one ds_add_rtn, so the count pass, the
// scan and two barriers go; two counter arrays alternate by chunk parity (the
// store phase zeroes the other one).  A chunk in which some tile overflows its
// share (rare: the share is the mean plus several standard deviations) is
// counting-sorted exactly as above from the positions still in registers,
// and its table entries describe the dense runs instead.
template <int BLOCK, int K, class Src, bool DT, bool CL = false, bool DYN = false>
__global__ __launch_bounds__(BLOCK) kPassARegs void bloom_bin16_kernel(BuildArgs a, Src keys,
                                                              uint32_t *__restrict__ pos_ws,
                                                              uint32_t *__restrict__ table_ws,
                                                              uint32_t total_chunks, uint32_t *__restrict__ scratch_ws,
                                                              FilterTable ft) {
  using FT = Filt<DT>;
  constexpr int KPT = 6;                    // keys per thread (C <= 6 * BLOCK)
  constexpr int VPT = (K * KPT + 3) / 4;    // 16-byte stores per thread per chunk, at most (CL: cap <= 4 * VPT * BLOCK)
  constexpr int SPI = (VPT + KPT - 1) / KPT;  // of those, per count iteration
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int tid = threadIdx.x;
  const uint32_t C = a.C;
  const uint32_t TL = a.TL;
  const uint32_t tmask = (1u << TL) - 1u;
  uint32_t *hist = lds;                        // T+1 counters, later cursors
  uint32_t *scratch = lds + a.hist_words;      // scan scratch
  uint32_t *lpos = lds + a.hist_words + 32;    // K*C sorted tile offsets (CL: the cap-word region)
  const uint4 *src4 = reinterpret_cast<const uint4 *>(lpos);
  // CL: the second counter array and the two overflow flags follow the region
  uint32_t *hist2 = lpos + a.cap;
  uint32_t *oflag = hist2 + a.hist_words;
  uint32_t *after = CL ? oflag + 4 : lpos + K * C;  // the repeated-hash table

  const uint32_t G = gridDim.x;
  const uint32_t slot = G % 8 == 0 ? (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8 : blockIdx.x;

  // Every global load and store of the chunk loop below is issued
  // unconditionally (out-of-range lanes load a clamped key, and store to
  // their wave's scratch line), so the compiler can count them: the hash of
  // chunk c+1 waits only for its own keys (vmcnt(stores issued since)), not
  // for every outstanding store of chunk c-1 and the table (vmcnt(0)).
  const int wave = tid / kWave;
  uint32_t *dummy = scratch_ws + kQueueWords + ((uint64_t)blockIdx.x * (BLOCK / kWave) + wave) * 4;
  uint4 *dummy4 = reinterpret_cast<uint4 *>(dummy);
  constexpr int TPT = (int)((kHistMax + BLOCK - 1) / BLOCK);  // table entries per thread, at most

  using Raw = typename Src::Raw;
  auto fetch = [&](uint32_t chunk, Raw (&raw)[KPT]) {
    const auto &d = FT::at(a, ft, FT::of_chunk(a, ft, chunk));
    const uint32_t first = (chunk - d.chunk_base) * C;
    const uint32_t last = min(C, d.n - first) - 1u;
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const uint32_t idx = min((uint32_t)(tid + i * BLOCK), last);
      raw[i] = keys.load(d, chunk, first, idx);
    }
  };

  // The keys of chunk c+2 load at the end of step c (two chunks ahead) and
  // are hashed in step c+1.  Measured against loading chunk c+1's keys at the
  // top of step c (no load in flight across the back-edge): 111 vs 127 us.
  Raw raw[KPT];
  uint32_t h1[KPT], h2[KPT];
  // this workgroup's chunks c (wg), c+1 (n1) and c+2 (n2); DYN: from the
  // queue, three ahead (thread 0 takes c+3 at the top of step c and publishes
  // it in qa[] at the step's last barrier, so the atomic's latency is hidden)
  uint32_t wg0 = slot, n1 = slot + G, n2 = slot + 2 * G;
  uint32_t *qa = lds + (a.hist_words + 28);  // 2 words of the scan scratch's tail (scans use <= 17)
  [[maybe_unused]] GroupQueue gq(scratch_ws, G, total_chunks);
  if constexpr (DYN) {
    if (tid == 0) {
      qa[0] = gq.next();
      qa[1] = gq.next();
      qa[2] = gq.next();
    }
    __syncthreads();
    wg0 = qa[0];
    n1 = qa[1];
    n2 = qa[2];
    __syncthreads();  // read before qa is written again
  }
  if (wg0 >= total_chunks) return;
  fetch(wg0, raw);
#pragma unroll
  for (int i = 0; i < KPT; ++i) Src::hash(raw[i], h1[i], h2[i]);
  fetch(min(n1, total_chunks - 1), raw);
  for (uint32_t i = tid; i < a.hist_words; i += BLOCK) hist[i] = 0;
  if constexpr (CL)
    for (uint32_t i = tid; i < a.hist_words + 4; i += BLOCK) hist2[i] = 0;  // and the flags

  // Repeated hashes.  The reference's murmur variant collapses: rotations with
  // an arithmetic shift and sign-extended bytes leave SplitMix keys only ~69 %
  // distinct (h1, h2) pairs at 10M keys, one pair 14 723 times.  A key whose
  // pair another key of this workgroup (same filter) already counted sets no
  // new bit, so it is skipped.  Only keys whose seeds converged (h1 == h2: 39 %
  // of the keys, 90 % of the repeats) take part: each claims slot h1 >> (31 -
  // dd) of a 2^(dd+1)-entry table with a 32-bit compare-and-swap (EMPTY ->
  // h1), and a key is skipped only when its slot holds exactly its own h1,
  // installed by a key that was counted.  (Every key claiming its 64-bit pair
  // measured slower: DESIGN.md §4.)
  const uint32_t dd = a.dd_log2;
  uint32_t *dtab32 = after;
  if (dd)
    for (uint32_t i = tid; i < (2u << dd); i += BLOCK) dtab32[i] = ~0u;

  uint4 *pdst = dummy4;  // deferred store of the previous chunk
  uint32_t ptotal = 0;
  uint32_t par = 0;  // CL: counter array / overflow flag of this chunk
  uint32_t qpar = 0;  // DYN: qa slot of this step
  STAMP_DECL
  for (uint32_t wg = wg0; wg < total_chunks;) {
    [[maybe_unused]] uint32_t n3 = 0;
    if (DYN && tid == 0) n3 = gq.next();  // used at this step's last barrier
    const int fcur = FT::of_chunk(a, ft, wg);
    const auto &d = FT::at(a, ft, fcur);
    const uint32_t w = wg - d.chunk_base;
    const uint32_t cnt = min(C, d.n - w * C);
    const uint32_t T = d.tiles;
    const FastMod mod = d.mod;
    uint32_t *hcur = hist, *hoth = hist2;
    if (CL && par) hcur = hist2, hoth = hist;
    const uint32_t tcap = CL ? (a.cap / T) & ~3u : 0u;  // slots per tile (the plan keeps it >= 4)
    __syncthreads();  // hist cleared; the previous scatter is complete in lpos
    STAMP(0);

    // count(c) + store(c-1)
    const uint32_t pvec = ptotal >> 2;
    uint32_t live = 0;  // bit i: key slot i is counted
#pragma unroll
    for (int i = 0; i < KPT; ++i)
      if (tid + i * BLOCK < cnt) live |= 1u << i;
    if (dd) {
      uint32_t old[KPT];
#pragma unroll
      for (int i = 0; i < KPT; ++i) {
        const uint32_t sl = h1[i] >> (31 - dd);
        old[i] = ((live >> i) & 1u) && h1[i] == h2[i] ? atomicCAS(&dtab32[sl], ~0u, h1[i]) : ~0u;
      }
#pragma unroll
      for (int i = 0; i < KPT; ++i)
        if (old[i] != ~0u && old[i] == h1[i] && h1[i] == h2[i]) live &= ~(1u << i);
    }
    uint32_t pos[KPT][K];
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      if ((live >> i) & 1u) {
#pragma unroll
        for (int j = 0; j < K; ++j) pos[i][j] = fastmod(h1[i] + (uint32_t)j * h2[i], mod);
#ifdef ADL_BLOOM_STAMPS
        if (a.exp & 32)  // diagnostics: no reduction (wrong positions, inside m for m >= 2^29)
#pragma unroll
          for (int j = 0; j < K; ++j) pos[i][j] = (h1[i] + (uint32_t)j * h2[i]) >> 3;
#endif
#ifdef ADL_BLOOM_STAMPS
        // diagnostics: conflict-free LDS sort (wrong tiles, needs T >= 128 and
        // no hash dedup).  Lane l counts into counter l, except that key slot 0
        // of wave 0 puts its first position into counter 64 + l: a full chunk
        // gives counters 0-63 an odd count each (16 waves x 6 keys x 6 - 1), so
        // the scatter's 32 lanes of a group write 32 different banks too.
        if (a.exp & 64)
#pragma unroll
          for (int j = 0; j < K; ++j)
            pos[i][j] = (((uint32_t)(tid & 63) + (i == 0 && j == 0 && tid < 64 ? 64u : 0u)) << TL) | (pos[i][j] & tmask);
#endif
        if constexpr (!CL)
#pragma unroll
          for (int j = 0; j < K; ++j) atomicAdd(&hist[pos[i][j] >> TL], 1u);
      }
      if constexpr (!CL) {
#pragma unroll
        for (int sv = i * SPI; sv < (i + 1) * SPI && sv < VPT; ++sv) {
          const uint32_t v = tid + sv * BLOCK;
          bool ok = v < pvec;
#ifdef ADL_BLOOM_STAMPS
          if (a.exp & 2) ok = false;
#endif
          *(ok ? pdst + v : dummy4) = src4[ok ? v : 0u];
        }
      }
    }
    if constexpr (!CL) {
      const bool ok = (uint32_t)tid < (ptotal & 3u);
      *(ok ? reinterpret_cast<uint32_t *>(pdst) + pvec * 4 + tid : dummy) = lpos[ok ? pvec * 4 + tid : 0u];
    }
    uint32_t *tab = table_ws + d.table_base;
    uint32_t total = 0;
    if constexpr (!CL) {
      __syncthreads();  // counts complete; the previous chunk's LDS copy is read out
      STAMP(1);

      total = block_excl_scan_array_1b<BLOCK>(hist, T + 1, scratch);
      STAMP(2);
#pragma unroll
      for (int r = 0; r < TPT; ++r) {
        const uint32_t t = tid + r * BLOCK;
        const bool ok = t <= T;
        *(ok ? tab + (uint64_t)t * d.chunks + w : dummy) = hist[ok ? t : 0u];
      }
      __syncthreads();
      STAMP(3);
    }

    // scatter(c) + hash(c+1) (its keys arrived during the previous chunk;
    // lanes past the end hash a clamped key and never use the result)
    bool ovf = false;  // CL: a position found its tile's slots taken
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      if ((live >> i) & 1u) {
        uint32_t sl[K];
        if constexpr (CL) {
#pragma unroll
          for (int j = 0; j < K; ++j) sl[j] = atomicAdd(&hcur[pos[i][j] >> TL], 1u);
#pragma unroll
          for (int j = 0; j < K; ++j) {
            if (sl[j] < tcap) lpos[(pos[i][j] >> TL) * tcap + sl[j]] = pos[i][j] & tmask;
            else ovf = true;
          }
        } else {
#pragma unroll
          for (int j = 0; j < K; ++j) sl[j] = atomicAdd(&hist[pos[i][j] >> TL], 1u);
#pragma unroll
          for (int j = 0; j < K; ++j) lpos[sl[j]] = pos[i][j] & tmask;
        }
      }
#ifdef ADL_BLOOM_STAMPS
      if (a.exp & 1) {
        h1[i] = raw[i].x;
        h2[i] = raw[i].y | 1u;
      } else
#endif
        Src::hash(raw[i], h1[i], h2[i]);
    }
    fetch(min(n2, total_chunks - 1), raw);
    // the repeated-hash table holds one filter's keys (positions depend on m)
    const bool last_of_filter = n1 >= total_chunks || FT::of_chunk(a, ft, n1) != fcur;
    if (CL && ovf) oflag[par] = 1u;
    if (DYN && tid == 0) qa[qpar] = n3;
    __syncthreads();  // lpos holds chunk c sorted; hist is free
    STAMP(4);
    if constexpr (CL) {
      // the other counter array and flag were last read before this chunk's
      // first barrier, and are next used after the next one
      for (uint32_t i = tid; i < a.hist_words; i += BLOCK) hoth[i] = 0;
      if (tid == 0) oflag[par ^ 1u] = 0;
    } else {
      for (uint32_t i = tid; i <= T; i += BLOCK) hist[i] = 0;
    }
    if (dd && last_of_filter && n1 < total_chunks)
      for (uint32_t i = tid; i < (2u << dd); i += BLOCK) dtab32[i] = ~0u;
    if constexpr (CL) {
      uint4 *dst = reinterpret_cast<uint4 *>(pos_ws + d.pos_base + (uint64_t)w * a.cap);
      if (oflag[par] == 0u) {
        // table entries (start << 16) | count for tiles t < T
#pragma unroll
        for (int r = 0; r < TPT; ++r) {
          const uint32_t t = tid + r * BLOCK;
          const bool ok = t < T;
          *(ok ? tab + (uint64_t)t * d.chunks + w : dummy) = ((t * tcap) << 16) | hcur[ok ? t : 0u];
        }
        // the region's 16-byte words that hold positions (tile t's slots are
        // words [t * tcap, t * tcap + count)); v / tq = umulhi(v, mg), exact
        // for v, tq < 2^16
        const uint32_t tq = tcap >> 2, nvec = T * tq;
        const uint32_t mg = 0xffffffffu / tq + 1u;
#pragma unroll
        for (int sv = 0; sv < VPT; ++sv) {
          const uint32_t v = tid + sv * BLOCK;
          const uint32_t t = __umulhi(v, mg);
          const bool ok = v < nvec && 4u * (v - t * tq) < hcur[min(t, T - 1u)];
          *(ok ? dst + v : dummy4) = src4[ok ? v : 0u];
        }
      } else {
        // some tile overflowed its slots: counting-sort this chunk exactly
        // from the positions still in registers; the entries describe the
        // dense runs
        total = block_excl_scan_array<BLOCK>(hcur, T + 1, scratch);
#pragma unroll
        for (int r = 0; r < TPT; ++r) {
          const uint32_t t = tid + r * BLOCK;
          const bool ok = t < T;
          const uint32_t s0 = hcur[ok ? t : 0u], s1 = hcur[ok ? t + 1 : 0u];
          *(ok ? tab + (uint64_t)t * d.chunks + w : dummy) = (s0 << 16) | (s1 - s0);
        }
        __syncthreads();  // the starts are read before the cursors move
#pragma unroll
        for (int i = 0; i < KPT; ++i) {
          if ((live >> i) & 1u) {
            uint32_t sl[K];
#pragma unroll
            for (int j = 0; j < K; ++j) sl[j] = atomicAdd(&hcur[pos[i][j] >> TL], 1u);
#pragma unroll
            for (int j = 0; j < K; ++j) lpos[sl[j]] = pos[i][j] & tmask;
          }
        }
        __syncthreads();  // the chunk is sorted in lpos
        const uint32_t tv = total >> 2;
#pragma unroll
        for (int sv = 0; sv < VPT; ++sv) {
          const uint32_t v = tid + sv * BLOCK;
          const bool ok = v < tv;
          *(ok ? dst + v : dummy4) = src4[ok ? v : 0u];
        }
        const bool ok = (uint32_t)tid < (total & 3u);
        *(ok ? reinterpret_cast<uint32_t *>(dst) + tv * 4 + tid : dummy) = lpos[ok ? tv * 4 + tid : 0u];
      }
      par ^= 1u;
    } else {
      pdst = reinterpret_cast<uint4 *>(pos_ws + d.pos_base + (uint64_t)w * a.cap);
      ptotal = total;
    }
    // the next step: (qa[qpar] was published at this step's last barrier and
    // is rewritten two steps on, after two more barriers)
    wg = n1;
    n1 = n2;
    if constexpr (DYN) {
      n2 = qa[qpar];
      qpar ^= 1u;
    } else {
      n2 += G;
    }
  }
  // epilogue: the last chunk's store
  const uint32_t pvec = ptotal >> 2;
  for (uint32_t v = tid; v < pvec; v += BLOCK) pdst[v] = src4[v];
  if ((uint32_t)tid < (ptotal & 3u))
    reinterpret_cast<uint32_t *>(pdst)[pvec * 4 + tid] = lpos[pvec * 4 + tid];
  STAMP(5);
  STAMP_FLUSH(0);
}

// ---------------------------------------------------------------- pass B
// Persistent: workgroup b owns the tiles of slot(b) in every round.  For a
// tile, the (tile, chunk) table rows give one segment per chunk region.  The
// segment list {start, length} is staged in LDS (its rows for the next tile
// are prefetched into registers during the current tile's gather).  A wave
// takes segments j = wave + 16q and runs a two-stage register pipeline over
// them: a stage's D descriptors are read with one ds_read_b64 per lane and
// handed to the slots by readlane (no load waits on LDS); every slot gathers
// positions 0..63 of its segment with one wave-load and 64..127 with a second
// when the segment is that long, so the loads of the next stage are in flight
// while the current stage is ds_or_b32'd into the LDS tile.  The rare longer
// segments (hot tiles) finish in a 4-deep unrolled loop.  The finished tile's
// 16-byte stores drain while the next tile is zeroed.
// OCC: workgroups per CU the kernel is compiled for (2: at most 64 VGPRs, for
// tiles whose LDS leaves room for two).  DYN: tiles from the work queues (while
// a resident probe server exists; two 1024-thread workgroups fill a CU's 32
// wave slots, so on the server's CU one of them starts only at the end and
// then finds the queues empty).
template <int D, bool DT, int OCC = 1, bool DYN = false, int BLK = kBlockB>
__global__ __launch_bounds__(BLK, 4 * OCC) void bloom_tile_kernel(BuildArgs a,
                                                             const uint32_t *__restrict__ pos_ws,
                                                             const uint32_t *__restrict__ table_ws,
                                                             uint8_t *__restrict__ bitmaps,
                                                             uint32_t total_tiles, uint32_t *__restrict__ scratch_ws,
                                                             FilterTable ft) {
  using FT = Filt<DT>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  constexpr int NWAVES = BLK / kWave;
  // segment descriptors staged per batch (half at two workgroups per CU, so
  // a 2^19-bit tile and its batch fit twice in a CU's LDS)
  constexpr int SEGB = OCC == 2 ? BLK : 2 * BLK;
  static_assert(SEGB <= kSegBatch, "the plan's LDS holds kSegBatch descriptors");
  constexpr int RPT = SEGB / BLK;  // table entries per thread per batch
  const uint32_t TL = a.TL;
  const uint32_t tile_words = 1u << (TL - 5);
  uint32_t *tile = lds;                                      // 2^TL bits
  uint2 *seg = reinterpret_cast<uint2 *>(lds + tile_words);  // SEGB {start word, length}
  uint32_t *qb = lds + tile_words + 2 * SEGB;                // DYN: 2 words, the tile after next

  auto fetch_rows = [&](uint32_t wg, uint32_t wb, uint32_t (&rs)[RPT], uint32_t (&re)[RPT]) {
    const auto &d = FT::at(a, ft, FT::of_tile(a, ft, wg));
    const uint32_t lt = wg - d.tile_base, W = d.chunks;
    const uint32_t *row0 = table_ws + d.table_base + (uint64_t)lt * W;
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      const uint32_t i = wb + tid + r * BLK;
      rs[r] = re[r] = 0;
      if (i < W) {
        if (a.claim) {  // (start << 16) | length
          const uint32_t v = row0[i];
          rs[r] = v >> 16;
          re[r] = rs[r] + (v & 0xffffu);
        } else {
          rs[r] = row0[i];
          re[r] = row0[i + W];
        }
      }
    }
  };
#ifdef ADL_BLOOM_STAMPS
  // diagnostics (ADL_BLOOM_EXP, wrong bitmaps): 4 = no ds_or (plain sum), 8 = no bitmap stores
  uint32_t exp_sink = 0;
  auto or_pos = [&](uint32_t off) {
    if (a.exp & 4) exp_sink += off;
    else atomicOr(&tile[off >> 5], 1u << (off & 31));
  };
#else
  auto or_pos = [&](uint32_t off) { atomicOr(&tile[off >> 5], 1u << (off & 31)); };
#endif

  // Round r covers tiles [r*G, (r+1)*G); inside a round each XCD takes G/8
  // consecutive tiles, so the line a tile's segment shares with its
  // neighbour's (segments of consecutive tiles are adjacent in every chunk
  // region) is fetched into one L2 once.  Speed only.  (A work queue of tiles,
  // global or per XCD, measured slower than this static order.)
  const uint32_t G = gridDim.x;
  uint32_t wg = G % 8 == 0 ? (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8 : blockIdx.x;
  uint32_t nxt = wg + G;  // the tile after this one
  // DYN: tiles from the queue (work queues above), two ahead: thread 0 takes
  // the tile after next at the top of a tile and publishes it at its last barrier
  [[maybe_unused]] GroupQueue gq(scratch_ws + 8 * 16, G, total_tiles);
  uint32_t qpar = 0;
  if constexpr (DYN) {
    if (tid == 0) {
      qb[0] = gq.next();
      qb[1] = gq.next();
    }
    __syncthreads();
    wg = qb[0];
    nxt = qb[1];
    __syncthreads();  // read before qb is written again
  }
  uint32_t pre_s[RPT], pre_e[RPT];
  if (wg < total_tiles) fetch_rows(wg, 0, pre_s, pre_e);
  {  // the tile starts zeroed; every write-out re-zeroes it
    uint4 *t4w = reinterpret_cast<uint4 *>(tile);
    for (uint32_t i = tid; i < tile_words / 4; i += BLK) t4w[i] = make_uint4(0, 0, 0, 0);
  }
  STAMP_DECL

  while (wg < total_tiles) {
    const int fi = FT::of_tile(a, ft, wg);
    const auto &d = FT::at(a, ft, fi);
    const uint32_t lt = wg - d.tile_base;
    const uint32_t W = d.chunks;
    const uint32_t pos_base = (uint32_t)d.pos_base;
    STAMP(0);
    const uint32_t next = nxt;
    [[maybe_unused]] uint32_t nn = 0;
    if (DYN && tid == 0) nn = gq.next();  // the tile after next, published at this tile's last barrier
    // an empty filter (no chunks) has no batch to prefetch the next tile from
    if (W == 0 && next < total_tiles) fetch_rows(next, 0, pre_s, pre_e);

    for (uint32_t wb = 0; wb < W; wb += SEGB) {
      const uint32_t nw = min((uint32_t)SEGB, W - wb);
      uint32_t rs[RPT], re[RPT];
      if (wb == 0) {
#pragma unroll
        for (int r = 0; r < RPT; ++r) rs[r] = pre_s[r], re[r] = pre_e[r];
      } else {
        fetch_rows(wg, wb, rs, re);
      }
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        const uint32_t i = tid + r * BLK;
        if (i < nw) seg[i] = make_uint2(pos_base + (wb + i) * a.cap + rs[r], re[r] - rs[r]);
      }
      __syncthreads();  // segment list ready
      STAMP(1);
      if (wb + SEGB >= W && next < total_tiles) fetch_rows(next, 0, pre_s, pre_e);

      const uint32_t Q = nw > (uint32_t)wave ? (nw - wave + NWAVES - 1) / NWAVES : 0;
      struct Stage {
        uint32_t v0[D], v1[D];
        uint32_t base, len;  // lane u: descriptor of slot u
      };
      auto issue = [&](Stage &st, uint32_t q0) {
        const uint32_t q = q0 + lane;
        uint2 dsc = make_uint2(0, 0);
        if (lane < D && q < Q) dsc = seg[wave + NWAVES * q];
        st.base = dsc.x;
        st.len = dsc.y;
        // The segment base is wave-uniform: an SGPR pointer plus the lane's
        // constant byte offset, so a gather needs no per-slot address VALU.
        // Positions 0-63 are loaded by every lane, unconditionally (lanes past
        // the segment read the next segment's words, inside the workspace's
        // slack, and are masked in consume): with no branch around them the
        // compiler can wait for one stage's loads (vmcnt(D)) instead of all.
        uint32_t len[D];
        const uint32_t *sp[D];
#pragma unroll
        for (int u = 0; u < D; ++u) {
          len[u] = __builtin_amdgcn_readlane(st.len, u);
          sp[u] = pos_ws + __builtin_amdgcn_readlane(st.base, u);
        }
#pragma unroll
        for (int u = 0; u < D; ++u)
          if (len[u] > (uint32_t)kWave && (uint32_t)lane + kWave < len[u]) st.v1[u] = sp[u][kWave + lane];
#pragma unroll
        for (int u = 0; u < D; ++u) st.v0[u] = sp[u][lane];
      };
      auto consume = [&](const Stage &st) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
          const uint32_t len = __builtin_amdgcn_readlane(st.len, u);
          if ((uint32_t)lane < len) or_pos(st.v0[u]);
          if (len > (uint32_t)kWave) {
            if ((uint32_t)lane + kWave < len) or_pos(st.v1[u]);
            if (len > 2u * kWave) {  // long segments (hot tiles): 4 loads in flight
              const uint32_t b = __builtin_amdgcn_readlane(st.base, u);
              for (uint32_t o = 2 * kWave; o < len; o += 4 * kWave) {
                uint32_t x[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                  const uint32_t e = o + t * kWave + lane;
                  x[t] = e < len ? pos_ws[b + e] : 0u;
                }
#pragma unroll
                for (int t = 0; t < 4; ++t)
                  if (o + t * kWave + lane < len) or_pos(x[t]);
              }
            }
          }
        }
      };
      Stage A, B;
      issue(A, 0);
      for (uint32_t q0 = 0; q0 < Q; q0 += 2 * D) {
        issue(B, q0 + D);
        consume(A);
        issue(A, q0 + 2 * D);
        consume(B);
      }
      __syncthreads();  // segment list reused by the next batch; tile complete after the last
      STAMP(2);
    }

    // Write the finished tile: bytes [lt << (TL-3), ...) of this filter, up to
    // the 16-byte-rounded bitmap length (pad bytes are zero: no position lands there).
    const uint64_t tile_bytes = 1ull << (TL - 3);
    const uint64_t b0 = (uint64_t)lt * tile_bytes;
    const uint64_t nbytes = min(tile_bytes, (uint64_t)d.alloc_bytes - b0);
    uint4 *out4 = reinterpret_cast<uint4 *>(bitmaps + d.bitmap_off + b0);
    const uint4 *t4 = reinterpret_cast<const uint4 *>(tile);
    // Each 16-byte word is zeroed as it is read out (the whole tile, also past
    // a short last tile), so the next tile needs no separate zeroing sweep.
    uint4 *t4z = reinterpret_cast<uint4 *>(tile);
    const uint32_t nvec = (uint32_t)(nbytes >> 4);
    for (uint32_t i = tid; i < tile_words / 4; i += BLK) {
      const uint4 v = t4[i];
      t4z[i] = make_uint4(0, 0, 0, 0);
      if (i < nvec) {
#ifdef ADL_BLOOM_STAMPS
        if (a.exp & 8) continue;
#endif
        store_nt(out4 + i, v);
      }
    }
    if (DYN && tid == 0) qb[qpar] = nn;
    __syncthreads();  // the tile is read out and zero again
    STAMP(3);
    wg = next;
    if constexpr (DYN) {
      nxt = qb[qpar];
      qpar ^= 1u;
    } else {
      nxt = next + G;
    }
  }
#ifdef ADL_BLOOM_STAMPS
  if (exp_sink == 0x9e3779b9u) scratch_ws[kQueueWords] = exp_sink;  // keeps the diagnostic sum alive
#endif
  STAMP_FLUSH(1);
}

// ---------------------------------------------------------------- host plan
struct Plan {
  BuildArgs a;
  std::vector<FilterDesc> f;  // every filter's descriptor (a.f holds them too when nf <= kMaxFilters)
  bool dt = false;            // more than kMaxFilters: descriptors in the workspace's FilterTable
  uint64_t pos_words = 0, table_words = 0, scratch_words = 0, hash_words = 0, ft_bytes = 0, ws_bytes = 0;
  bool claim = false;      // claim layout sizes: bloom_bin16_kernel<..., CL> runs
  uint32_t total_chunks = 0, total_tiles = 0, total_sc = 0;
  uint32_t grid_a = 0, grid_b = 0;  // persistent grids
  uint32_t occ_b = 1;               // pass-B workgroups per CU
  size_t lds_a = 0, lds_b = 0;
};

int make_plan(const uint64_t *counts, uint32_t nf, int32_t bpk, Plan &p) {
  if (nf == 0 || bpk < 0) return ADL_ERR_INVALID_ARG;
  const adl_host::Knobs &kn = adl_host::knobs();
  memset(&p.a, 0, sizeof(p.a));
  p.f.assign(nf, FilterDesc{});
  p.dt = nf > (uint32_t)kMaxFilters;
  const uint32_t k = (uint32_t)adl_host::num_probes(bpk);
  uint64_t total_n = 0;
  for (uint32_t f = 0; f < nf; ++f) {
    if (adl_host::bitmap_bytes(counts[f], bpk) == 0) return ADL_ERR_TOO_LARGE;
    total_n += counts[f];
  }
  // Tile size: the largest (fewest, longest segments) that still yields
  // enough pass-B workgroups; every filter's tile histogram must fit the
  // pass-A counters (T + 1 <= kHistMax).
  uint32_t TL = kMaxTileLog2;
  auto tiles_at = [&](uint32_t tl, bool max_only) {
    uint64_t t = 0;
    for (uint32_t f = 0; f < nf; ++f) {
      const uint64_t m = adl_host::bitmap_bytes(counts[f], bpk) * 8;
      const uint64_t tf = (m + (1ull << tl) - 1) >> tl;
      t = max_only ? std::max<uint64_t>(t, tf) : t + tf;
    }
    return t;
  };
  while (TL > kMinTileLog2 && tiles_at(TL, false) < kTargetWorkgroups) --TL;
  // Filters of a few tiles each (configs[3]'s 1 M-key tables: 77 tiles of
  // 2^20 bits): smaller tiles, down to 2^18 bits, while a filter has fewer
  // than kFewTiles and a chunk's run per tile stays long (about k*C / tiles
  // positions >= kMinRun).  More tile counters take the contention off pass
  // A's atomics, and such tiles leave LDS for two pass-B workgroups per CU
  // (below).  Measured on configs[3]: 3.66-3.68 ms at 2^18 bits with two
  // per CU, 4.06-4.11 at 2^20 (profiles/r04/ab_tile_size_occ.log).
  const bool tl_set = kn.tile_log2 >= kMinTileLog2 && kn.tile_log2 <= kMaxTileLog2;  // test / tuning override
  if (tl_set) TL = kn.tile_log2;
  if (!tl_set && k == 6)
    while (TL > 18 && tiles_at(TL, true) < kFewTiles && (uint64_t)k * kChunkEst >= kMinRun * tiles_at(TL - 1, true))
      --TL;
  while (TL < kMaxTileLog2 && tiles_at(TL, true) + 1 > kHistMax) ++TL;
  const uint32_t hist_words = (uint32_t)adl_host::round_up(tiles_at(TL, true) + 1, 4);

  // Keys per chunk: as many as the rest of the pass-A LDS holds, then evened
  // out so the chunks split into whole rounds of the persistent grid (one
  // 1024-thread workgroup per CU: measured against two 512-thread ones, the
  // longer chunks halve pass B's segments).
  const uint32_t cus = adl_host::device_cus();
  const uint32_t grid_a_max = cus;
  const uint32_t kpt = k == 6 ? 6 : kKptMax;
  const uint32_t lds_words_a = kLdsWordsPerCu - kLdsReserveWords;
  // LDS: tile counters + scan scratch + k*C positions + C key indices and 256
  // length classes (the length sort of variable-length keys; reserved for every
  // key shape so the workspace size does not depend on it)
  const uint32_t cmax =
      std::min<uint32_t>(kBlockA * kpt, (lds_words_a - hist_words - 32 - 256) / (k + 1)) & ~3u;
  if (cmax < 4) return ADL_ERR_TOO_LARGE;
  // chunks of C keys over all filters (each filter's last chunk is partial)
  auto nchunks = [&](uint64_t c) {
    uint64_t w = 0;
    for (uint32_t f = 0; f < nf; ++f) w += (counts[f] + c - 1) / c;
    return w;
  };
  auto pick_c = [&](uint32_t cm) -> uint32_t {
    const uint64_t wmin = nchunks(cm);
    uint32_t c;
    if (wmin >= grid_a_max) {
      const uint64_t rounds = (wmin + grid_a_max - 1) / grid_a_max;
      c = (uint32_t)std::min<uint64_t>(
          cm, adl_host::round_up((total_n + rounds * grid_a_max - 1) / (rounds * grid_a_max), 4));
      // the smallest C whose chunks, rounded up per filter, still fill no more rounds
      while (c + 4 <= cm && nchunks(c) > rounds * grid_a_max) c += 4;
    } else {
      c = (uint32_t)std::min<uint64_t>(
          cm, std::max<uint64_t>(256, adl_host::round_up((total_n + grid_a_max - 1) / grid_a_max, 4)));
    }
    return c;
  };
  // Claim layout (16-byte keys and hashed pairs with k = 6): the region of cap
  // words gives each tile of a filter cap / T slots.  C shrinks so the region
  // holds k*C positions times kClaimSlack percent; the layout is kept only if
  // the largest filter's share per tile clears its mean run by kClaimSigma
  // standard deviations (Poisson), so overflowing chunks (sorted exactly, more
  // slowly) stay rare.  The region takes all the LDS left over (fewer
  // overflows); ADL_BLOOM_CLAIM_CAP (percent of k*C) caps it and
  // ADL_BLOOM_CLAIM=2 skips the share test: the tests force overflowing
  // chunks that way.  Default (3): only filters of at most kClaimTiles tiles,
  // where it measured faster (pass A + B: 512 x 5 K keys 119 against 164 us,
  // 256 x 10 K 92 / 109, 256 x 20 K 124 / 143, 128 x 30 K 94 / 101; 128 x 60 K
  // and 32 x 100 K equal; 256 x 40 K and 64 x 300 K 4-11 % slower;
  // profiles/r04/ab_claim_shapes.log, ab_claim_threshold.log).
  const uint32_t claim_mode = kn.claim;
  bool claim = k == 6 && claim_mode != 0;
  const int64_t room_cl = (int64_t)lds_words_a - 2 * hist_words - 36 - 256;  // region + C
  uint32_t cap_cl = 0;
  uint32_t C = 0;
  if (claim && room_cl > 64) {
    const uint32_t cm = std::min<uint32_t>(kBlockA * kpt, (uint32_t)(room_cl * 100 / (kClaimSlack * k + 100))) & ~3u;
    if (cm >= 4) {
      C = pick_c(cm);
      int64_t cw = std::min<int64_t>(room_cl - C, 36ll * kBlockA);  // <= 4 * VPT * BLOCK
      if (kn.claim_cap) cw = std::min<int64_t>(cw, (int64_t)k * C * std::max<uint32_t>(kn.claim_cap, 100) / 100 + 3);
      cap_cl = (uint32_t)cw & ~3u;
      const uint32_t tmax = (uint32_t)tiles_at(TL, true);
      const uint32_t tcap = (cap_cl / tmax) & ~3u;
      const double mu = (double)k * C / tmax;
      claim = cap_cl >= k * C && tcap >= 16 &&
              (claim_mode == 2 || tcap >= mu + kClaimSigma * std::sqrt(mu) + 8) &&
              (claim_mode != 3 || tmax <= kClaimTiles);
    } else {
      claim = false;
    }
  } else {
    claim = false;
  }
  if (!claim) C = pick_c(cmax);
  p.a.nf = nf;
  p.a.stage_keys = 1;
  {
    // the repeated-hash table sits in the C + 256 words pass A reserves past
    // the positions (the var-len length sort's area; bloom_bin16_kernel does
    // not use it there): 2^(lg+1) u32 slots
    uint32_t lg = 0;
    while (lg < kDdLog2Max && (2u << (lg + 1)) <= C + 256) ++lg;
    p.a.dd_log2 = (kn.hash_dedup && lg >= 4) ? lg : 0;
  }
#ifdef ADL_BLOOM_STAMPS
  p.a.exp = kn.exp;  // diagnostics build only
#endif
  p.a.k = k;
  p.a.C = C;
  p.a.TL = TL;
  const uint32_t cap = claim ? cap_cl : k * C;
  p.a.cap = cap;
  p.claim = claim;
  p.a.hist_words = hist_words;
  uint64_t pos = 0, tab = 0, boff = 0;
  uint32_t chunk = 0, tile = 0, sc = 0;
  for (uint32_t f = 0; f < nf; ++f) {
    FilterDesc &d = p.f[f];
    const uint64_t bytes = adl_host::bitmap_bytes(counts[f], bpk);
    const uint32_t m = (uint32_t)(bytes * 8);
    d.n = (uint32_t)counts[f];
    d.alloc_bytes = (uint32_t)adl_host::round_up(bytes, 16);
    d.chunks = (uint32_t)((counts[f] + C - 1) / C);
    d.tiles = (uint32_t)(((uint64_t)m + (1ull << TL) - 1) >> TL);
    if (d.tiles + 1 > kHistMax) return ADL_ERR_TOO_LARGE;
    d.mod = adl_host::make_fastmod(m);
    d.chunk_base = chunk;
    d.tile_base = tile;
    d.sc_base = sc;
    sc += (uint32_t)((counts[f] + kHvKeys - 1) / kHvKeys);
    d.pos_base = pos;
    d.table_base = tab;
    d.bitmap_off = boff;  // overwritten by the caller
    d.key_begin = 0;      // overwritten by the caller
    chunk += d.chunks;
    tile += d.tiles;
    pos += (uint64_t)d.chunks * cap;
    tab += (uint64_t)(d.tiles + 1) * d.chunks;
  }
  if (pos + 64 >= (1ull << 32)) return ADL_ERR_TOO_LARGE;  // u32 position indices
  if (!p.dt) std::copy(p.f.begin(), p.f.end(), p.a.f);
  p.total_chunks = chunk;
  p.total_tiles = tile;
  p.total_sc = sc;
  p.pos_words = adl_host::round_up(pos, 64);
  p.table_words = adl_host::round_up(tab + kTablePad, 64);
  // after the table: the work-queue counters (GroupQueue), then one 16-byte
  // scratch line per pass-A wave (bloom_bin16_kernel's masked-off stores)
  p.scratch_words = adl_host::round_up(kQueueWords + (uint64_t)grid_a_max * (kBlockA / kWave) * 4 + 4, 64);
  // then (h1, h2) per key in the chunk grid: hash_var_kernel -> pass A
  // (variable-length keys; reserved for every key shape so the workspace size
  // does not depend on it)
  p.hash_words = adl_host::round_up(2ull * chunk * C, 64);
  // then (more than kMaxFilters) the FilterTable: descriptors, chunk / tile / run maps
  p.ft_bytes = p.dt ? adl_host::round_up(nf * sizeof(FilterDesc), 256) + 4ull * (chunk + tile + sc) + 256 : 0;
  p.ws_bytes = (p.pos_words + p.table_words + p.scratch_words + p.hash_words) * 4 + p.ft_bytes + 256;
  p.lds_a = claim ? (size_t)(2 * hist_words + 36 + cap + C + 256) * 4 : (size_t)(hist_words + 32 + (k + 1) * C + 256) * 4;
  p.lds_b = (size_t)((1u << (TL - 5)) + 2 * kSegBatch + 4) * 4;
  p.grid_a = std::min<uint32_t>(p.total_chunks, grid_a_max);
  // Two pass-B workgroups per CU (64-VGPR kernels, half the segment batch,
  // pipeline depth 4) when the tile leaves room for two in LDS and the runs per
  // tile are long: more waves to hide the gathers.  On the headline's
  // 2^20-bit tiles it does not fit; forced at 2^19 there it is slower (short
  // runs: 101 vs 68 us).
  {
    const size_t lds2 = (size_t)((1u << (TL - 5)) + kSegBatch + 4) * 4;
    const bool long_runs = (uint64_t)k * C >= (uint64_t)kMinRun * tiles_at(TL, true);
    p.occ_b = long_runs && lds2 <= 78 * 1024 ? 2 : 1;
    if (p.occ_b == 2) p.lds_b = lds2;
  }
  p.grid_b = std::min<uint32_t>(p.total_tiles, p.occ_b * cus);
  if (kn.debug)
    fprintf(stderr, "adl_bloom plan: filters %u, tile 2^%u bits, tiles %u, C %u, chunks %u, region %u words%s, pass B %u per CU\n",
            nf, TL, p.total_tiles, C, p.total_chunks, cap, claim ? " (claim)" : "", p.occ_b);
  return ADL_OK;
}

// ---------------------------------------------------------------- instrumentation
// Thread-local event quadruples: start/stop of pass A and of pass B, taken
// from the kernels' own dispatch packets (hipExtLaunchKernel), so profiling
// adds no marker packets -- and no gaps -- between the launches.
struct Profile {
  bool on = false;
  uint32_t used = 0;
  std::vector<hipEvent_t> ev;  // 4 per build
  ~Profile() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  }
};
thread_local Profile t_prof;

inline hipEvent_t *prof_slot() {
  if (!t_prof.on || 4 * (t_prof.used + 1) > t_prof.ev.size()) return nullptr;
  return &t_prof.ev[4 * t_prof.used++];
}

// pass A of this thread's last launch pair wrote the claim layout's table
// (adl_bloom_build_positions reads it)
thread_local bool t_last_claim = false;

template <bool DT, class Keys>
int launch_binned_dt(const Plan &p, Keys keys, uint8_t *d_bitmaps, void *ws, hipStream_t st) {
  BuildArgs aa = p.a;
  aa.claim = 0;
  uint32_t claim_used = 0;  // pass A wrote the claim layout's table entries
  uint32_t *pos_ws = reinterpret_cast<uint32_t *>(ws);
  uint32_t *tab_ws = pos_ws + p.pos_words;
  uint32_t *scr = tab_ws + p.table_words;  // the work-queue counters, pass A's per-wave scratch lines
  uint2 *hp = reinterpret_cast<uint2 *>(scr + p.scratch_words);
  // While a probe server's kernel is resident (Gets are being served), a
  // pass with many items per workgroup takes them from the work queues: a
  // workgroup slowed or held back by the server's wave on its CU then takes
  // less work instead of holding up the pass (reads beside
  // builds).  The counters start at 0.  A pass of a few items per workgroup
  // keeps the static order: a queue cannot even out less than one item, and
  // costs its atomics (round 6, profiles/r06/: headline with Gets 0.184 ms
  // static against 0.203 queued -- 7 chunks and 3 tiles per workgroup;
  // configs[3] with Gets 4.82 ms static against 3.63 queued -- 180 chunks and
  // 150 tiles, and pass B's two workgroups per CU leave no room for the
  // server's wave beside both).  Round 5 queued whenever a server object
  // existed, so every build of a process that had served one Get paid +12 %.
  const adl_host::Knobs &kn = adl_host::knobs();
  const bool live = kn.build_queues == 3 || (kn.build_queues == 1 && adl_srv::live_servers() > 0) ||
                    (kn.build_queues == 2 && adl_srv::resident_servers() > 0);
  const bool many_a = kn.build_queues != 2 || p.total_chunks >= kQueueMinItems * p.grid_a;
  const bool many_b = kn.build_queues != 2 || p.total_tiles >= kQueueMinItems * p.grid_b || p.occ_b == 2;
  const bool dyn_a = live && many_a && (kn.build_queue_passes & 1) && p.grid_a % 8 == 0;
  const bool dyn_b = live && many_b && (kn.build_queue_passes & 2) && p.grid_b % 8 == 0;
  if (dyn_a || dyn_b) ADL_HIP_TRY(hipMemsetAsync(scr, 0, kQueueWords * 4, st));
  FilterTable ft{};
  if constexpr (DT) {
    // the descriptors go up in stream order; the maps are filled on the device
    uint8_t *fbase = reinterpret_cast<uint8_t *>(scr + p.scratch_words + p.hash_words);
    FilterDesc *fd = reinterpret_cast<FilterDesc *>(fbase);
    uint32_t *chunk_f = reinterpret_cast<uint32_t *>(fbase + adl_host::round_up(p.f.size() * sizeof(FilterDesc), 256));
    uint32_t *tile_f = chunk_f + p.total_chunks, *sc_f = tile_f + p.total_tiles;
    if (int rc = adl_host::t_upload.upload(fd, p.f.data(), p.f.size() * sizeof(FilterDesc), st)) return rc;
    hipLaunchKernelGGL(fill_maps_kernel, dim3((uint32_t)p.f.size()), dim3(256), 0, st, fd, chunk_f, tile_f, sc_f);
    ADL_HIP_TRY(hipGetLastError());
    ft.fd = (cptr<FilterDesc>)fd;
    ft.chunk_f = (cptr<uint32_t>)chunk_f;
    ft.tile_f = (cptr<uint32_t>)tile_f;
    ft.sc_f = (cptr<uint32_t>)sc_f;
  }
  hipEvent_t *ev = prof_slot();
  if (ev && !p.total_chunks) {  // no pass A: an empty interval
    ADL_HIP_TRY(hipEventRecord(ev[0], st));
    ADL_HIP_TRY(hipEventRecord(ev[1], st));
  }
  if (p.total_chunks) {
    // lim: lds_limit<kern>; the hashing pass (var-len keys) before pass A opens
    // the profiled pass-A interval instead of it
    auto go16 = [&](auto lim, auto kern, const BuildArgs &args, auto src, bool hashed) -> int {
      if (int rc = lim()) return rc;
      hipExtLaunchKernelGGL(kern, dim3(p.grid_a), dim3(kBlockA), p.lds_a, st, ev && !hashed ? ev[0] : nullptr,
                            ev ? ev[1] : nullptr, 0, args, src, pos_ws, tab_ws, p.total_chunks, scr, ft);
      ADL_HIP_TRY(hipGetLastError());
      return ADL_OK;
    };
    auto go = [&](auto lim, auto kern) -> int {
      if (int rc = lim()) return rc;
      hipExtLaunchKernelGGL(kern, dim3(p.grid_a), dim3(kBlockA), p.lds_a, st, ev ? ev[0] : nullptr,
                            ev ? ev[1] : nullptr, 0, aa, keys, pos_ws, tab_ws, p.total_chunks, ft);
      ADL_HIP_TRY(hipGetLastError());
      return ADL_OK;
    };
    constexpr int B = (int)kBlockA;
    // bloom_bin16_kernel in the claim layout or not, its chunks from the work
    // queues or in the static order
    auto bin16 = [&](auto src, BuildArgs args, bool hashed) -> int {
      using S = decltype(src);
      if (p.claim) {
        args.claim = claim_used = 1;
        if (dyn_a)
          return go16(adl_host::lds_limit<bloom_bin16_kernel<B, 6, S, DT, true, true>>,
                      bloom_bin16_kernel<B, 6, S, DT, true, true>, args, src, hashed);
        return go16(adl_host::lds_limit<bloom_bin16_kernel<B, 6, S, DT, true>>, bloom_bin16_kernel<B, 6, S, DT, true>,
                    args, src, hashed);
      }
      if (dyn_a)
        return go16(adl_host::lds_limit<bloom_bin16_kernel<B, 6, S, DT, false, true>>,
                    bloom_bin16_kernel<B, 6, S, DT, false, true>, args, src, hashed);
      return go16(adl_host::lds_limit<bloom_bin16_kernel<B, 6, S, DT>>, bloom_bin16_kernel<B, 6, S, DT>, args, src,
                  hashed);
    };
    int rc = -1;
    if constexpr (std::is_same<Keys, Keys16>::value) {
      if (p.a.k == 6 && !p.a.dedup) rc = bin16(Src16{keys.keys}, aa, false);
    }
    if constexpr (std::is_same<Keys, KeysVar>::value) {
      // length-sorted hashing pass, then pass A over the (h1, h2) pairs; the
      // profiled pass-A interval spans both launches.  (Adjacent-duplicate
      // skipping needs the keys in order: the generic pass A below.)
      if (p.a.k == 6 && p.a.stage_keys && !p.a.dedup) {
        if (int r = adl_host::lds_limit<hash_var_kernel<kHvKeys, DT>>()) return r;
        hipExtLaunchKernelGGL(hash_var_kernel<kHvKeys, DT>, dim3(p.total_sc), dim3(kHvBlock), hv_lds_bytes<kHvKeys>(),
                              st, ev ? ev[0] : nullptr, nullptr, 0, aa, keys, hp, p.total_sc, ft);
        ADL_HIP_TRY(hipGetLastError());
        // the repeated-hash table pays for 16-byte keys only (configs[2]'s keys
        // repeat few pairs: pass B 64 -> 70 us with it)
        BuildArgs av = aa;
        av.dd_log2 = 0;
        rc = bin16(SrcH{hp, p.a.C}, av, true);
      }
    }
    if (rc < 0)
      rc = p.a.k == 6 ? go(adl_host::lds_limit<bloom_bin_kernel<B, 6, 6, Keys, DT>>, bloom_bin_kernel<B, 6, 6, Keys, DT>)
                      : go(adl_host::lds_limit<bloom_bin_kernel<B, 0, kKptMax, Keys, DT>>,
                           bloom_bin_kernel<B, 0, kKptMax, Keys, DT>);
    if (rc) return rc;
  }
  BuildArgs ab = aa;
  ab.claim = claim_used;
  t_last_claim = claim_used != 0;
  auto go_b = [&](auto lim, auto kern) -> int {
    if (int rc = lim()) return rc;
    hipExtLaunchKernelGGL(kern, dim3(p.grid_b), dim3(kBlockB), p.lds_b, st, ev ? ev[2] : nullptr,
                          ev ? ev[3] : nullptr, 0, ab, (const uint32_t *)pos_ws, (const uint32_t *)tab_ws,
                          d_bitmaps, p.total_tiles, scr, ft);
    ADL_HIP_TRY(hipGetLastError());
    return ADL_OK;
  };
  if (p.occ_b == 2 && dyn_b)
    return go_b(adl_host::lds_limit<bloom_tile_kernel<4, DT, 2, true>>, bloom_tile_kernel<4, DT, 2, true>);
  if (dyn_b && p.occ_b == 1)
    return go_b(adl_host::lds_limit<bloom_tile_kernel<kDepthB, DT, 1, true>>, bloom_tile_kernel<kDepthB, DT, 1, true>);
  if (p.occ_b == 2)
    return go_b(adl_host::lds_limit<bloom_tile_kernel<4, DT, 2>>, bloom_tile_kernel<4, DT, 2>);
  return go_b(adl_host::lds_limit<bloom_tile_kernel<kDepthB, DT>>, bloom_tile_kernel<kDepthB, DT>);
}

template <class Keys>
int launch_binned(const Plan &p, Keys keys, uint8_t *d_bitmaps, void *ws, hipStream_t st) {
  return p.dt ? launch_binned_dt<true>(p, keys, d_bitmaps, ws, st) : launch_binned_dt<false>(p, keys, d_bitmaps, ws, st);
}

}  // namespace

namespace {
// Runs the filters through the plan/launch pair: all in one launch pair (a
// compaction's tables; smaller launch groups measured slower), split only
// where the u32 position indices of one launch's workspace would overflow
// (groups of at most 2^31 / k keys).
uint64_t group_keys_max(int32_t bpk) { return (1ull << 31) / (uint64_t)adl_host::num_probes(bpk); }

int build_groups(const uint8_t *d_keys, const uint64_t *d_offsets, uint32_t key_stride,
                 const uint64_t *key_begin, uint32_t num_filters, int32_t bpk, uint8_t *d_bitmaps,
                 const uint64_t *bitmap_off, void *d_workspace, uint64_t workspace_bytes,
                 hipStream_t st, uint32_t flags = 0) {
  if (flags & ~(uint32_t)ADL_BLOOM_SKIP_ADJACENT_DUPLICATES) return ADL_ERR_INVALID_ARG;
  if (!d_keys && key_begin[num_filters] > key_begin[0]) return ADL_ERR_INVALID_ARG;
  if (!d_offsets && key_stride == 0 && key_begin[num_filters] > key_begin[0]) return ADL_ERR_INVALID_ARG;
  if (bpk < 0) return ADL_ERR_INVALID_ARG;
  const uint64_t gmax = group_keys_max(bpk);
  std::vector<uint64_t> counts;
  for (uint32_t g = 0; g < num_filters;) {
    counts.clear();
    uint64_t keys_in = 0;
    uint32_t e = g;
    for (; e < num_filters; ++e) {
      if (key_begin[e + 1] < key_begin[e]) return ADL_ERR_INVALID_ARG;
      const uint64_t c = key_begin[e + 1] - key_begin[e];
      if (e > g && keys_in + c > gmax) break;
      counts.push_back(c);
      keys_in += c;
    }
    const uint32_t nf = e - g;
    Plan p;
    int rc = make_plan(counts.data(), nf, bpk, p);
    if (rc) return rc;
    p.a.dedup = (flags & ADL_BLOOM_SKIP_ADJACENT_DUPLICATES) ? 1u : 0u;
    for (uint32_t f = 0; f < nf; ++f) {
      if (bitmap_off[g + f] % 16) return ADL_ERR_INVALID_ARG;
      p.f[f].key_begin = key_begin[g + f];
      p.f[f].bitmap_off = bitmap_off[g + f];
      if (!p.dt) p.a.f[f] = p.f[f];
    }
    if (!d_workspace || workspace_bytes < p.ws_bytes) return ADL_ERR_WORKSPACE;
    void *ws = reinterpret_cast<void *>(adl_host::round_up(reinterpret_cast<uintptr_t>(d_workspace), 256));
    if (d_offsets) {
      KeysVar keys{d_keys, d_offsets};
      // staging loads (pass A's windows and the hashing pass) read whole aligned
      // 16-byte blocks: only of a 16-byte-aligned key buffer
      if (reinterpret_cast<uintptr_t>(d_keys) % 16) p.a.stage_keys = 0;
      rc = launch_binned(p, keys, d_bitmaps, ws, st);
    } else if (key_stride == 16 && (reinterpret_cast<uintptr_t>(d_keys) % 16) == 0) {
      rc = launch_binned(p, Keys16{reinterpret_cast<const uint4 *>(d_keys)}, d_bitmaps, ws, st);
    } else {
      rc = launch_binned(p, KeysStride{d_keys, key_stride}, d_bitmaps, ws, st);
    }
    if (rc) return rc;
    g = e;
  }
  return ADL_OK;
}
}  // namespace

// ====================================================================== C-ABI
extern "C" {

const char *adl_bloom_strerror(int status) {
  switch (status) {
    case ADL_OK: return "ok";
    case ADL_FILTER_BLOCK_ERROR: return "filter block error";
    case ADL_ERR_INVALID_ARG: return "invalid argument";
    case ADL_ERR_TOO_LARGE: return "filter too large for the reference's int arithmetic";
    case ADL_ERR_DEVICE: return "HIP device error";
    case ADL_ERR_OUT_OF_MEMORY: return "device out of memory";
    case ADL_ERR_WORKSPACE: return "workspace too small";
    default: return "unknown error";
  }
}

int adl_bloom_abi_version(void) { return ADL_BLOOM_ABI_VERSION; }

int adl_bloom_test_fault(int site, int64_t arg) {
  if (site != ADL_TEST_FAULT_PIPELINE_GROUP && site != ADL_TEST_FAULT_CACHE_COMPLETION) return ADL_ERR_INVALID_ARG;
  adl_host::g_test_faults.site[site].store(arg < 0 ? -1 : arg);
  return ADL_OK;
}

int adl_bloom_reload_knobs(void) {
  adl_host::reload_knobs();
  return ADL_OK;
}

#ifdef ADL_BLOOM_STAMPS
// Diagnostics build only: copies g_stamps ([pass][workgroup][phase] cycles).
int adl_bloom_debug_stamps(uint64_t *out, uint64_t n) {
  constexpr uint64_t kOwn = 3 * 2048 * 8;
  const uint64_t bytes = std::min<uint64_t>(n, kOwn) * 8;
  ADL_HIP_TRY(hipDeviceSynchronize());
  ADL_HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), bytes, 0, hipMemcpyDeviceToHost));
  return ADL_OK;
}
#endif

int32_t adl_bloom_num_probes(int32_t bits_per_key) { return adl_host::num_probes(bits_per_key); }

int adl_bloom_get_device(int32_t *device) {
  if (!device) return ADL_ERR_INVALID_ARG;
  int d = 0;
  ADL_HIP_TRY(hipGetDevice(&d));
  *device = d;
  return ADL_OK;
}

int adl_bloom_set_device(int32_t device) {
  if (device < 0) return ADL_ERR_INVALID_ARG;
  ADL_HIP_TRY(hipSetDevice(device));
  return ADL_OK;
}

uint64_t adl_bloom_bitmap_bytes(uint64_t n, int32_t bits_per_key) {
  return adl_host::bitmap_bytes(n, bits_per_key);
}

uint64_t adl_bloom_bitmap_alloc_bytes(uint64_t n, int32_t bits_per_key) {
  const uint64_t b = adl_host::bitmap_bytes(n, bits_per_key);
  return b ? adl_host::round_up(b, 16) : 0;
}

uint64_t adl_bloom_build_workspace_bytes(const uint64_t *key_counts, uint32_t num_filters,
                                         int32_t bits_per_key) {
  if (!key_counts) return 0;
  if (bits_per_key < 0) return 0;
  // the same grouping as build_groups
  const uint64_t gmax = group_keys_max(bits_per_key);
  uint64_t ws = 0;
  for (uint32_t g = 0; g < num_filters;) {
    uint64_t keys_in = 0;
    uint32_t e = g;
    for (; e < num_filters; ++e) {
      if (e > g && keys_in + key_counts[e] > gmax) break;
      keys_in += key_counts[e];
    }
    Plan p;
    if (make_plan(key_counts + g, e - g, bits_per_key, p)) return 0;
    ws = std::max(ws, p.ws_bytes);
    g = e;
  }
  return ws;
}

int adl_bloom_build_positions(const uint64_t *key_counts, uint32_t num_filters, int32_t bits_per_key,
                              const void *d_workspace, uint64_t *positions, void *stream) {
  try {
    if (!key_counts || !d_workspace || !positions || num_filters == 0 || bits_per_key < 0)
      return ADL_ERR_INVALID_ARG;
    // the last group of build_groups' grouping is what the workspace holds
    const uint64_t gmax = group_keys_max(bits_per_key);
    uint32_t g = 0;
    for (uint32_t g0 = 0; g0 < num_filters;) {
      uint64_t keys_in = 0;
      uint32_t e = g0;
      for (; e < num_filters; ++e) {
        if (e > g0 && keys_in + key_counts[e] > gmax) break;
        keys_in += key_counts[e];
      }
      g = g0;
      g0 = e;
    }
    hipStream_t st = adl_host::sync_stream(stream);
    Plan p;
    if (int rc = make_plan(key_counts + g, num_filters - g, bits_per_key, p)) return rc;
    const uint32_t *tab = reinterpret_cast<const uint32_t *>(
                              adl_host::round_up(reinterpret_cast<uintptr_t>(d_workspace), 256)) +
                          p.pos_words;
    uint64_t sum = 0;
    std::vector<uint32_t> row;
    for (const FilterDesc &d : p.f) {  // row T of each filter's table: every chunk's total
      if (t_last_claim) {  // claim layout: the lengths in rows 0..T-1
        row.resize((uint64_t)d.tiles * d.chunks);
        if (row.empty()) continue;
        ADL_HIP_TRY(hipMemcpyAsync(row.data(), tab + d.table_base, row.size() * 4ull, hipMemcpyDeviceToHost, st));
        ADL_HIP_TRY(hipStreamSynchronize(st));
        for (uint32_t v : row) sum += v & 0xffffu;
        continue;
      }
      row.resize(d.chunks);
      if (!d.chunks) continue;
      ADL_HIP_TRY(hipMemcpyAsync(row.data(), tab + d.table_base + (uint64_t)d.tiles * d.chunks, d.chunks * 4ull,
                                 hipMemcpyDeviceToHost, st));
      ADL_HIP_TRY(hipStreamSynchronize(st));
      for (uint32_t v : row) sum += v;
    }
    *positions = sum;
    return ADL_OK;
  } catch (...) {
    return ADL_ERR_DEVICE;
  }
}

int adl_bloom_build_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n,
                           uint32_t key_stride, int32_t bits_per_key, uint8_t *d_bitmap,
                           void *d_workspace, uint64_t workspace_bytes, void *stream) {
  try {
    if (!d_bitmap) return ADL_ERR_INVALID_ARG;
    if (reinterpret_cast<uintptr_t>(d_bitmap) % 16) return ADL_ERR_INVALID_ARG;
    const uint64_t kb[2] = {0, n};
    const uint64_t boff[1] = {0};
    return build_groups(d_keys, d_offsets, key_stride, kb, 1, bits_per_key, d_bitmap, boff,
                        d_workspace, workspace_bytes, (hipStream_t)stream);
  } catch (...) {
    return ADL_ERR_DEVICE;
  }
}

int adl_bloom_build_segmented_device(const uint8_t *d_keys, const uint64_t *d_offsets,
                                     uint32_t key_stride, const uint64_t *key_begin,
                                     uint32_t num_filters, int32_t bits_per_key,
                                     uint8_t *d_bitmaps, const uint64_t *bitmap_off,
                                     void *d_workspace, uint64_t workspace_bytes, void *stream) {
  try {
    if (!key_begin || !bitmap_off || !d_bitmaps || num_filters == 0) return ADL_ERR_INVALID_ARG;
    if (reinterpret_cast<uintptr_t>(d_bitmaps) % 16) return ADL_ERR_INVALID_ARG;
    return build_groups(d_keys, d_offsets, key_stride, key_begin, num_filters, bits_per_key,
                        d_bitmaps, bitmap_off, d_workspace, workspace_bytes, (hipStream_t)stream);
  } catch (...) {
    return ADL_ERR_DEVICE;
  }
}

int adl_bloom_build_segmented_device_ex(const uint8_t *d_keys, const uint64_t *d_offsets,
                                        uint32_t key_stride, const uint64_t *key_begin,
                                        uint32_t num_filters, int32_t bits_per_key,
                                        uint8_t *d_bitmaps, const uint64_t *bitmap_off, uint32_t flags,
                                        void *d_workspace, uint64_t workspace_bytes, void *stream) {
  try {
    if (!key_begin || !bitmap_off || !d_bitmaps || num_filters == 0) return ADL_ERR_INVALID_ARG;
    if (reinterpret_cast<uintptr_t>(d_bitmaps) % 16) return ADL_ERR_INVALID_ARG;
    return build_groups(d_keys, d_offsets, key_stride, key_begin, num_filters, bits_per_key,
                        d_bitmaps, bitmap_off, d_workspace, workspace_bytes, (hipStream_t)stream, flags);
  } catch (...) {
    return ADL_ERR_DEVICE;
  }
}

// One filter from host memory: the pipelined host build with one filter
// (bloom_pipeline.hip), so pinned keys and a pinned bitmap are DMAed directly
// and pageable ones go through one staging copy each way (this
// entry point used to copy every key into staging, then the bitmap out of it).
int adl_bloom_build(const uint8_t *h_keys, const uint64_t *h_offsets, uint64_t n,
                    uint32_t key_stride, int32_t bits_per_key, uint8_t *h_bitmap, void *stream) {
  if (!h_bitmap || (n && !h_keys)) return ADL_ERR_INVALID_ARG;
  if (!h_offsets && n && key_stride == 0) return ADL_ERR_INVALID_ARG;
  if (!adl_host::bitmap_bytes(n, bits_per_key)) return bits_per_key < 0 ? ADL_ERR_INVALID_ARG : ADL_ERR_TOO_LARGE;
  const uint64_t key_begin[2] = {0, n}, bitmap_off[1] = {0};
  return adl_bloom_build_segmented(h_keys, h_offsets, key_stride, key_begin, 1, bits_per_key, h_bitmap, bitmap_off,
                                   stream);
}

int adl_bloom_profile_enable(uint32_t capacity) {
  try {
    while (t_prof.ev.size() < 4ull * capacity) {
      hipEvent_t e;
      ADL_HIP_TRY(hipEventCreate(&e));
      t_prof.ev.push_back(e);
    }
    t_prof.used = 0;
    t_prof.on = true;
    return ADL_OK;
  } catch (...) {
    return ADL_ERR_DEVICE;
  }
}

int adl_bloom_profile_each(double *ms_ab, uint32_t capacity, uint32_t *launch_pairs) {
  if (!ms_ab || !launch_pairs) return ADL_ERR_INVALID_ARG;
  const uint32_t n = std::min(t_prof.used, capacity);
  for (uint32_t i = 0; i < n; ++i) {
    hipEvent_t *e = &t_prof.ev[4 * i];
    float a = 0.f, b = 0.f;
    ADL_HIP_TRY(hipEventSynchronize(e[3]));
    ADL_HIP_TRY(hipEventElapsedTime(&a, e[0], e[1]));
    ADL_HIP_TRY(hipEventElapsedTime(&b, e[2], e[3]));
    ms_ab[2 * i] = a;
    ms_ab[2 * i + 1] = b;
  }
  *launch_pairs = n;
  return ADL_OK;
}

int adl_bloom_profile_collect(double *ms, uint32_t *builds) {
  if (!ms || !builds) return ADL_ERR_INVALID_ARG;
  ms[0] = ms[1] = 0.0;
  for (uint32_t i = 0; i < t_prof.used; ++i) {
    hipEvent_t *e = &t_prof.ev[4 * i];
    float a = 0.f, b = 0.f;
    ADL_HIP_TRY(hipEventSynchronize(e[3]));
    ADL_HIP_TRY(hipEventElapsedTime(&a, e[0], e[1]));
    ADL_HIP_TRY(hipEventElapsedTime(&b, e[2], e[3]));
    ms[0] += a;
    ms[1] += b;
  }
  *builds = t_prof.used;
  t_prof.used = 0;
  t_prof.on = false;
  return ADL_OK;
}

}  // extern "C"
