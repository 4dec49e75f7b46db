// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.
// C-ABI shim over the reference's own, unmodified src/murmur3_hash.cpp and
// src/encode.cpp (compiled in place from /root/reference by oracle/Makefile),
// so tests can ask the real reference for murmur3 values.
#include <cstddef>
#include <cstdint>
#include "encode.hpp"        // reference src/encode.hpp
#include "murmur3_hash.hpp"  // reference src/murmur3_hash.hpp:9

extern "C" uint32_t ref_murmur3(uint32_t seed, const char *data, size_t len) {
  return adl::murmur3_hash(seed, data, len);
}

extern "C" void ref_murmur3_batch(const char *keys, const uint64_t *offsets, uint64_t n,
                                  uint64_t stride, uint32_t seed_a, uint32_t seed_b,
                                  uint32_t *out) {
  for (uint64_t i = 0; i < n; i++) {
    const char *k = offsets ? keys + offsets[i] : keys + i * stride;
    size_t len = offsets ? (size_t)(offsets[i + 1] - offsets[i]) : (size_t)stride;
    out[2 * i] = adl::murmur3_hash(seed_a, k, len);
    out[2 * i + 1] = adl::murmur3_hash(seed_b, k, len);
  }
}

extern "C" int ref_decode32(const char *src) {
  int v = 0;
  adl::Decode32(src, &v);
  return v;
}
