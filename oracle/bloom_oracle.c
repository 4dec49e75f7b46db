/*
 * oracle/bloom_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker).
 *
 * A plain-C restatement of the reference SSTable bloom-filter path of
 * adlternative/adlsm-tree, used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py -- never by the product path, which runs on the
 * GPU through libadlbloom.so and fails loudly without it.
 *
 * Parity pinning: this file is checked against
 *   (1) the golden vectors of SURVEY.md Appendix B (generated from the compiled
 *       reference src/filter_block.cpp + src/murmur3_hash.cpp),
 *   (2) murmur3 vectors produced by the reference's own src/murmur3_hash.cpp,
 *       compiled unmodified into oracle/_ref/ by oracle/build_ref.sh
 *       (tests/golden/make_golden.py, tests/golden/murmur3_ref.json),
 *   (3) the assertions of the reference's test/filter_block_test.cpp:37-52.
 *
 * Every function cites the reference file:line it restates.  The quirks are
 * kept on purpose: bytes are signed chars that are
 * sign-extended before they are shifted and ORed, and the "rotate" works on a
 * signed int with an arithmetic right shift.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

/* src/murmur3_hash.cpp:5-9 -- rotate_left(int value, int32_t count):
 * (value << count) | (value >> ((-count) & 31)) on a SIGNED int, so the right
 * shift is arithmetic and a negative value fills the vacated bits with 1s. */
static inline uint32_t oracle_rotl_quirk(uint32_t x, int c) {
  int32_t v = (int32_t)x;
  uint32_t lo = (uint32_t)(v >> ((-c) & 31)); /* arithmetic shift (gcc/clang) */
  return (x << c) | lo;
}

/* (uint32_t)data[i] with data a `const char *` (signed on x86-64):
 * src/murmur3_hash.cpp:26-29 and :43-49. */
static inline uint32_t oracle_sx(uint8_t b) { return (uint32_t)(int32_t)(int8_t)b; }

/* src/murmur3_hash.cpp:11-65 -- uint32_t murmur3_hash(seed, data, len). */
uint32_t oracle_murmur3(uint32_t seed, const uint8_t *data, uint64_t len) {
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  const uint32_t m = 5, n = 0xe6546b64u;
  uint32_t h = seed;
  int len4 = (int)(len / 4); /* :21 -- `int len4 = len / sizeof(uint32_t)` */
  for (int i = 0; i < len4; i++) { /* :24-37 */
    uint32_t k = oracle_sx(data[4 * i]) | (oracle_sx(data[4 * i + 1]) << 8) |
                 (oracle_sx(data[4 * i + 2]) << 16) | (oracle_sx(data[4 * i + 3]) << 24);
    k *= c1;
    k = oracle_rotl_quirk(k, 15);
    k *= c2;
    h ^= k;
    h = oracle_rotl_quirk(h, 13) * m + n;
  }
  const uint8_t *tail = data + (uint64_t)len4 * 4; /* :39 */
  uint32_t k1 = 0;
  switch (len & 3) { /* :41-55 (fall-through) */
    case 3:
      k1 ^= oracle_sx(tail[2]) << 16;
      /* fall through */
    case 2:
      k1 ^= oracle_sx(tail[1]) << 8;
      /* fall through */
    case 1:
      k1 ^= oracle_sx(tail[0]);
      k1 *= c1;
      k1 = oracle_rotl_quirk(k1, 15);
      k1 *= c2;
      h ^= k1;
  }
  h ^= (uint32_t)len; /* :57-62 fmix32 */
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

/* src/filter_block.cpp:35-47 -- k = (int)(bits_per_key * 0.69) clamped to [1,30]. */
int oracle_num_probes(int bits_per_key) {
  int k = (int)(bits_per_key * 0.69);
  if (k < 1) k = 1;
  if (k > 30) k = 30;
  return k;
}

/* src/filter_block.cpp:11-14 -- bitmap_bits_len = (n*bpk + 7) * 8 as an `int`,
 * so the bitmap is n*bpk + 7 BYTES.  Returns 0 when the reference's int
 * arithmetic would overflow (the reference is undefined there). */
uint64_t oracle_bitmap_bytes(uint64_t n, int bits_per_key) {
  if (bits_per_key < 0) return 0;
  uint64_t bytes = n * (uint64_t)bits_per_key + 7;
  if (bytes * 8 > 0x7fffffffull) return 0;
  return bytes;
}

static inline const uint8_t *oracle_key(const uint8_t *keys, const uint64_t *offsets,
                                        uint64_t stride, uint64_t i, uint64_t *len) {
  if (offsets) {
    *len = offsets[i + 1] - offsets[i];
    return keys + offsets[i];
  }
  *len = stride;
  return keys + i * stride;
}

/* src/filter_block.cpp:9-33 -- BloomFilter::Keys2Block.
 * keys: packed bytes; offsets (n+1 entries) or NULL for a fixed `stride`.
 * bitmap: bitmap_bytes = oracle_bitmap_bytes(n,bpk) bytes, zeroed here
 * (the reference zero-fills the bytes it appends, :16-17).
 * Returns 0, or -1 on a size the reference cannot represent. */
int oracle_keys2block(const uint8_t *keys, const uint64_t *offsets, uint64_t n,
                      uint64_t stride, int bits_per_key, uint8_t *bitmap) {
  uint64_t bytes = oracle_bitmap_bytes(n, bits_per_key);
  if (bytes == 0) return -1;
  uint32_t m = (uint32_t)(bytes * 8);
  int k = oracle_num_probes(bits_per_key);
  memset(bitmap, 0, bytes);
  for (uint64_t i = 0; i < n; i++) { /* :20-30 */
    uint64_t len;
    const uint8_t *key = oracle_key(keys, offsets, stride, i, &len);
    uint32_t h1 = oracle_murmur3(0xe2c6928au, key, len);
    uint32_t h2 = oracle_murmur3(0xbaea8a8fu, key, len);
    for (int j = 0; j < k; j++) {
      uint32_t h = h1 + (uint32_t)j * h2;
      uint32_t bit = h % m;
      bitmap[bit >> 3] |= (uint8_t)(1u << (bit & 7));
    }
  }
  return 0;
}

/* src/filter_block.cpp:49-62 -- BloomFilter::IsKeyExists, batched over n
 * queries against ONE bitmap: m = (int)bitmap.size() * 8; false at the first
 * clear bit.  out[i] = 1 (maybe present) / 0 (absent).  A zero-byte bitmap is
 * undefined in the reference (h % 0); here it returns -1. */
int oracle_probe(const uint8_t *keys, const uint64_t *offsets, uint64_t n, uint64_t stride,
                 int bits_per_key, const uint8_t *bitmap, uint64_t bitmap_bytes, uint8_t *out) {
  if (bitmap_bytes == 0 || bitmap_bytes * 8 > 0x7fffffffull) return -1;
  uint32_t m = (uint32_t)(bitmap_bytes * 8);
  int k = oracle_num_probes(bits_per_key);
  for (uint64_t i = 0; i < n; i++) {
    uint64_t len;
    const uint8_t *key = oracle_key(keys, offsets, stride, i, &len);
    uint32_t h1 = oracle_murmur3(0xe2c6928au, key, len);
    uint32_t h2 = oracle_murmur3(0xbaea8a8fu, key, len);
    uint8_t hit = 1;
    for (int j = 0; j < k; j++) {
      uint32_t bit = (h1 + (uint32_t)j * h2) % m;
      if (!(bitmap[bit >> 3] & (1u << (bit & 7)))) { hit = 0; break; }
    }
    out[i] = hit;
  }
  return 0;
}

/* Multi-filter probe: query i goes to filter filter_id[i], whose bitmap is
 * bitmaps[bitmap_off[f] .. bitmap_off[f+1]).  Same semantics as
 * oracle_probe per query (an empty filter answers 0); an out-of-range filter id answers 0, as
 * FilterBlockReader::IsKeyExists does for filter_block_num >= filters_nums_
 * (src/filter_block.cpp:174). */
int oracle_probe_multi(const uint8_t *keys, const uint64_t *offsets, uint64_t n, uint64_t stride,
                       const uint32_t *filter_id, uint32_t num_filters, const uint8_t *bitmaps,
                       const uint64_t *bitmap_off, int bits_per_key, uint8_t *out) {
  int k = oracle_num_probes(bits_per_key);
  for (uint64_t i = 0; i < n; i++) {
    uint32_t f = filter_id[i];
    if (f >= num_filters) { out[i] = 0; continue; }
    uint64_t bytes = bitmap_off[f + 1] - bitmap_off[f];
    /* an empty filter: the reference divides by zero (h % 0); the GPU path
     * answers 0, and so does this */
    if (bytes == 0) { out[i] = 0; continue; }
    if (bytes * 8 > 0x7fffffffull) return -1;
    uint32_t m = (uint32_t)(bytes * 8);
    const uint8_t *bm = bitmaps + bitmap_off[f];
    uint64_t len;
    const uint8_t *key = oracle_key(keys, offsets, stride, i, &len);
    uint32_t h1 = oracle_murmur3(0xe2c6928au, key, len);
    uint32_t h2 = oracle_murmur3(0xbaea8a8fu, key, len);
    uint8_t hit = 1;
    for (int j = 0; j < k; j++) {
      uint32_t bit = (h1 + (uint32_t)j * h2) % m;
      if (!(bm[bit >> 3] & (1u << (bit & 7)))) { hit = 0; break; }
    }
    out[i] = hit;
  }
  return 0;
}

/* Batched murmur3 for the parity tests: out[2i] = h(seed_a), out[2i+1] = h(seed_b). */
void oracle_murmur3_batch(const uint8_t *keys, const uint64_t *offsets, uint64_t n,
                          uint64_t stride, uint32_t seed_a, uint32_t seed_b, uint32_t *out) {
  for (uint64_t i = 0; i < n; i++) {
    uint64_t len;
    const uint8_t *key = oracle_key(keys, offsets, stride, i, &len);
    out[2 * i] = oracle_murmur3(seed_a, key, len);
    out[2 * i + 1] = oracle_murmur3(seed_b, key, len);
  }
}

/* SplitMix64 16-byte keys exactly as SURVEY.md §8d specifies them (and as the
 * Appendix B golden bitmaps were generated): state = seed; next():
 * z = (state += 0x9E3779B97F4A7C15); z = (z^(z>>30))*0xBF58476D1CE4E5B9;
 * z = (z^(z>>27))*0x94D049BB133111EB; return z^(z>>31).
 * key i = LE64(next()) || LE64(next()), starting after `skip` keys. */
void oracle_splitmix_keys16(uint64_t seed, uint64_t skip, uint64_t n, uint8_t *out) {
  uint64_t state = seed + 2 * skip * 0x9E3779B97F4A7C15ull;
  for (uint64_t i = 0; i < 2 * n; i++) {
    uint64_t z = (state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    memcpy(out + 8 * i, &z, 8); /* little-endian host */
  }
}

/* SplitMix64 output number `call` (1-based) of the stream seeded `seed`. */
static uint64_t oracle_splitmix_at(uint64_t seed, uint64_t call) {
  uint64_t z = seed + call * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* Probe queries of BASELINE.json configs[4] (probe config):
 * query q draws outputs 4q+1..4q+4 of the stream seeded `seed`: r0 picks the
 * filter (r0 % num_tables), r1 odd picks inserted key (r1>>1) % keys_per_table
 * of that table's oracle_splitmix_keys16(table_seed0 + t) stream, r1 even a
 * fresh key LE64(r2) || LE64(r3).  member[q] = 1 for inserted keys. */
void oracle_synth_probe_queries(uint64_t seed, uint64_t q0, uint64_t n, uint32_t num_tables,
                                uint64_t table_seed0, uint64_t keys_per_table, uint8_t *keys,
                                uint32_t *filter_id, uint8_t *member) {
  for (uint64_t i = 0; i < n; i++) {
    uint64_t c = 4 * (q0 + i);
    uint64_t r0 = oracle_splitmix_at(seed, c + 1), r1 = oracle_splitmix_at(seed, c + 2);
    uint32_t t = (uint32_t)(r0 % num_tables);
    int ins = (r1 & 1) && keys_per_table;
    uint64_t kv[2];
    if (ins) {
      uint64_t j = (r1 >> 1) % keys_per_table;
      oracle_splitmix_keys16(table_seed0 + t, j, 1, keys + 16 * i);
    } else {
      kv[0] = oracle_splitmix_at(seed, c + 3);
      kv[1] = oracle_splitmix_at(seed, c + 4);
      memcpy(keys + 16 * i, kv, 16);
    }
    filter_id[i] = t;
    if (member) member[i] = (uint8_t)ins;
  }
}

/* Variable-length synthetic keys of BASELINE.json configs[2], restating the
 * device generator (adlsm-tree_amd/csrc/bloom_probe.hip synth_lengths_kernel /
 * synth_fill_kernel, DESIGN.md "Synthetic inputs"): key i has length
 * 8 + (r - 1), r ~ Zipf(s) on [1, 249] by inverse CDF -- the first r with
 * x < ceil(cdf(r) * 2^53), x = output i+1 of the SplitMix64 stream seeded
 * seed ^ 0xD1B54A32D192ED03, shifted right by 11 -- and byte j of the packed
 * key buffer is byte j % 8 (little-endian) of output j/8 + 1 of the stream
 * seeded `seed`.  These are synthetic inputs of the survey's shape (§8d), not
 * a reference algorithm: the bitmaps built from them are pinned by the
 * oracle's Keys2Block, which is pinned to the reference. */
#include <math.h>
void oracle_synth_varlen_lengths(uint64_t seed, uint64_t n, double s, uint32_t *len) {
  enum { R = 249 };
  double cdf[R], acc = 0;
  uint64_t thr[R];
  for (int r = 1; r <= R; r++) {
    acc += pow((double)r, -s);
    cdf[r - 1] = acc;
  }
  for (int r = 0; r < R; r++) thr[r] = (uint64_t)ceil(cdf[r] / acc * 9007199254740992.0);
  const uint64_t lseed = seed ^ 0xD1B54A32D192ED03ull;
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t x = oracle_splitmix_at(lseed, i + 1) >> 11;
    int lo = 0, hi = R - 1;
    while (lo < hi) {
      int mid = (lo + hi) >> 1;
      if (x < thr[mid]) hi = mid; else lo = mid + 1;
    }
    len[i] = 8u + (uint32_t)lo;
  }
}

void oracle_synth_varlen_fill(uint64_t seed, uint64_t total_bytes, uint8_t *out) {
  for (uint64_t w = 0; 8 * w < total_bytes; w++) {
    const uint64_t z = oracle_splitmix_at(seed, w + 1);
    for (uint64_t b = 0; b < 8 && 8 * w + b < total_bytes; b++) out[8 * w + b] = (uint8_t)(z >> (8 * b));
  }
}
