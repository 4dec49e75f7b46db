// adlsm-tree_amd/csrc/murmur3_device.hpp -- gfx950 device form of the
// reference's MurmurHash3 variant (src/murmur3_hash.cpp:5-65).
//
// The reference is NOT canonical MurmurHash3:
//   * each data byte is a signed char, sign-extended to 32 bits before it is
//     shifted and ORed into the block word (src/murmur3_hash.cpp:26-29), and
//     XORed into the tail word (:43-49);
//   * rotate_left works on a signed int, so its right shift is arithmetic
//     (src/murmur3_hash.cpp:5-9).
// Both quirks are reproduced bit-exactly here.  Block words are produced from
// four raw little-endian bytes in one 32-bit register with a branch-free fill
// instead of four sign-extending byte loads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace adl_dev {

constexpr uint32_t kSeed1 = 0xe2c6928au;  // src/filter_block.cpp:22
constexpr uint32_t kSeed2 = 0xbaea8a8fu;  // src/filter_block.cpp:23

// (uint32_t)d[0] | (uint32_t)d[1] << 8 | ... with signed d[i]: the lowest byte
// whose sign bit is set sign-extends over every byte above it.
__device__ __forceinline__ uint32_t quirk_word(uint32_t raw) {
  uint32_t s = raw & 0x80808080u;
  uint32_t lowest = s & (0u - s);  // sign bit of the lowest negative byte
  // all bits above that byte (0 if none): ~((lowest << 1) - 1) == (0 - lowest) << 1,
  // kept in that form (one v_lshl_or_b32 with raw) by an opaque negation
  uint32_t neg = 0u - lowest;
  asm("" : "+v"(neg));
  return raw | (neg << 1);
}

// rotate_left(int value, 15|13) with arithmetic >> (src/murmur3_hash.cpp:5-9).
template <int C>
__device__ __forceinline__ uint32_t rotl_quirk(uint32_t x) {
  return (x << C) | (uint32_t)((int32_t)x >> (32 - C));
}

// The block word's own mixing (src/murmur3_hash.cpp:31-33).  It does not
// depend on the seed, so the two hashes of a key share it: two quarter-rate
// v_mul_lo_u32 per block instead of four.
__device__ __forceinline__ uint32_t mix_k(uint32_t k) {
  k *= 0xcc9e2d51u;       // :31
  // opaque: otherwise the compiler folds the rotate's k << 15 into a second
  // v_mul_lo_u32 by c1 << 15 (a quarter-rate op for a full-rate shift)
  asm("" : "+v"(k));
  k = rotl_quirk<15>(k);  // :32
  return k * 0x1b873593u; // :33
}

// The rest of the state update once the block word is XORed in
// (src/murmur3_hash.cpp:36): h*5 + c as shift + 3-input add, an opaque shift
// keeping the compiler from fusing it back into a 64-bit v_mad_u64_u32.
__device__ __forceinline__ uint32_t mix_s(uint32_t s) {
  const uint32_t r = rotl_quirk<13>(s);
  uint32_t r4 = r << 2;
  asm("" : "+v"(r4));
  return r4 + r + 0xe6546b64u;
}

// The state update with a mixed block word (src/murmur3_hash.cpp:35-37).
__device__ __forceinline__ uint32_t mix_h(uint32_t h, uint32_t k) { return mix_s(h ^ k); }

__device__ __forceinline__ uint32_t mix_block(uint32_t h, uint32_t k) { return mix_h(h, mix_k(k)); }

// Both seeds' states advanced by one block word.
__device__ __forceinline__ void mix_block2(uint32_t &a, uint32_t &b, uint32_t k) {
  const uint32_t kk = mix_k(k);
  a = mix_h(a, kk);
  b = mix_h(b, kk);
}

// The tail word mixed (src/murmur3_hash.cpp:50-53), also seed-independent;
// the state update is h ^= it.
__device__ __forceinline__ uint32_t mix_tail_k(uint32_t k1) { return mix_k(k1); }

__device__ __forceinline__ uint32_t mix_tail(uint32_t h, uint32_t k1) { return h ^ mix_tail_k(k1); }

__device__ __forceinline__ uint32_t fmix(uint32_t h, uint32_t len) {
  h ^= len;  // :57-62
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ uint32_t sx8(uint32_t byte) { return (uint32_t)(int32_t)(int8_t)byte; }

// Tail word for len & 3 in {1,2,3}: k1 ^= sx(t2)<<16; k1 ^= sx(t1)<<8; k1 ^= sx(t0)
// (src/murmur3_hash.cpp:41-49).  `raw` holds the tail bytes little-endian.
__device__ __forceinline__ uint32_t tail_word(uint32_t raw, uint32_t rem) {
  uint32_t k1 = 0;
  if (rem >= 3) k1 ^= sx8((raw >> 16) & 0xff) << 16;
  if (rem >= 2) k1 ^= sx8((raw >> 8) & 0xff) << 8;
  k1 ^= sx8(raw & 0xff);
  return k1;
}

// Both seeds of a 16-byte key held as four raw little-endian words.
__device__ __forceinline__ void hash16(uint4 raw, uint32_t &h1, uint32_t &h2) {
  const uint32_t w0 = quirk_word(raw.x), w1 = quirk_word(raw.y);
  const uint32_t w2 = quirk_word(raw.z), w3 = quirk_word(raw.w);
  uint32_t a = kSeed1, b = kSeed2;
  mix_block2(a, b, w0);
  mix_block2(a, b, w1);
  mix_block2(a, b, w2);
  mix_block2(a, b, w3);
  h1 = fmix(a, 16u);
  h2 = fmix(b, 16u);
}

// Unaligned little-endian 32-bit read of 4 bytes (global or LDS generic pointer).
__device__ __forceinline__ uint32_t load_u32_unaligned(const uint8_t *p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}

// Both seeds of an arbitrary-length key at byte pointer p (any alignment).
// The block words are independent of the hash state, so they are loaded 8 at
// a time (one memory round trip per 32 key bytes) and then mixed in order.
__device__ __forceinline__ void hash_bytes(const uint8_t *p, uint32_t len, uint32_t seed_a,
                                           uint32_t seed_b, uint32_t &ha, uint32_t &hb) {
  uint32_t a = seed_a, b = seed_b;
  const uint32_t nblk = len >> 2;
  constexpr uint32_t U = 8;
  for (uint32_t i = 0; i < nblk; i += U) {
    uint32_t w[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) w[u] = i + u < nblk ? load_u32_unaligned(p + 4 * (i + u)) : 0u;
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      if (i + u < nblk) mix_block2(a, b, quirk_word(w[u]));
    }
  }
  const uint32_t rem = len & 3u;
  if (rem) {
    const uint8_t *t = p + 4 * nblk;
    uint32_t raw = t[0];
    if (rem >= 2) raw |= (uint32_t)t[1] << 8;
    if (rem >= 3) raw |= (uint32_t)t[2] << 16;
    const uint32_t kk = mix_tail_k(tail_word(raw, rem));
    a ^= kk;
    b ^= kk;
  }
  ha = fmix(a, len);
  hb = fmix(b, len);
}

// Both seeds of a key staged in LDS at byte offset `off` of `stage` (any
// alignment; `stage` 8-byte aligned): aligned LDS words plus v_alignbyte_b32
// with the previous word.  Reads up to 8 bytes past the key's end (callers
// keep slack).
__device__ __forceinline__ void hash_lds(const uint32_t *stage, uint32_t off, uint32_t len,
                                         uint32_t &ha, uint32_t &hb) {
  uint32_t a = kSeed1, b = kSeed2;
  const uint32_t nblk = len >> 2, sh = off & 3u;
  uint32_t wi = off >> 2;
  uint32_t i = 0;
  // Four blocks per step from two 8-byte-aligned ds_read_b64 (the lanes of a
  // wave read keys at scattered offsets, so every LDS access is a random-bank
  // one: half the instructions of four ds_read_b32, at about the same cycles
  // each).  The step's four words are the dword after the carry and the three
  // after that; a key starting in the high dword of its pair takes them one
  // dword later (odd), selected per lane.
  const uint2 *s2 = reinterpret_cast<const uint2 *>(stage);
  const bool odd = (wi & 1u) != 0;
  uint2 p0 = s2[wi >> 1];
  uint32_t lo = odd ? p0.y : p0.x;
  uint32_t pi = wi >> 1;
  for (; i + 4 <= nblk; i += 4) {
    const uint2 p1 = s2[pi + 1], p2 = s2[pi + 2];
    const uint32_t w[4] = {odd ? p1.x : p0.y, odd ? p1.y : p1.x, odd ? p2.x : p1.y, odd ? p2.y : p2.x};
#pragma unroll
    for (int u = 0; u < 4; ++u)
      mix_block2(a, b, quirk_word(__builtin_amdgcn_alignbyte(w[u], u ? w[u - 1] : lo, sh)));
    lo = w[3];
    p0 = p2;
    pi += 2;
    wi += 4;
  }
  for (; i < nblk; ++i) {
    const uint32_t hi = stage[++wi];
    mix_block2(a, b, quirk_word(__builtin_amdgcn_alignbyte(hi, lo, sh)));
    lo = hi;
  }
  const uint32_t rem = len & 3u;
  if (rem) {
    const uint32_t raw = __builtin_amdgcn_alignbyte(stage[wi + 1], lo, sh);
    const uint32_t kk = mix_tail_k(tail_word(raw, rem));
    a ^= kk;
    b ^= kk;
  }
  ha = fmix(a, len);
  hb = fmix(b, len);
}

// h % m for a launch-constant divisor 2 <= m < 2^31 (Granlund-Montgomery
// round-up method, exact for every 32-bit numerator): q = (t + ((h-t)>>1)) >> (l-1),
// t = mulhi(h, magic), l = ceil(log2 m).  A power of two m = 2^l gets magic = 1
// (t = 0, q = h >> l), so one branch-free sequence covers every divisor.
struct FastMod {
  uint32_t m, magic, shift, pad_;
};

// Device-side construction (same values as adl_host::make_fastmod); for
// per-filter divisors that are only known on the device.
__device__ __forceinline__ FastMod fastmod_for(uint32_t m) {
  FastMod f;
  f.m = m;
  f.pad_ = 0;
  const uint32_t l = 32u - __clz(m - 1u);  // ceil(log2 m), m >= 2
  f.magic = (uint32_t)((((1ull << 32) * ((1ull << l) - m)) / m) + 1ull);
  f.shift = l - 1u;
  return f;
}

// h / m with the same magic numbers.
__device__ __forceinline__ uint32_t fastdiv(uint32_t h, const FastMod &d) {
  const uint32_t t = __umulhi(h, d.magic);
  return (t + ((h - t) >> 1)) >> d.shift;
}

__device__ __forceinline__ uint32_t fastmod(uint32_t h, const FastMod &d) {
  const uint32_t t = __umulhi(h, d.magic);
  const uint32_t q = (t + ((h - t) >> 1)) >> d.shift;
  return h - q * d.m;
}

}  // namespace adl_dev
