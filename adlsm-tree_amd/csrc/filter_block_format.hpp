// adlsm-tree_amd/csrc/filter_block_format.hpp -- the filter-block trailer walk
// of FilterBlockReader::Init (reference src/filter_block.cpp:113-170), shared
// by the C++ reader mirror (filter_block.cpp) and the device filter cache
// (filter_cache.hip).  Pure host C++: no HIP, so the host ASan build
// (make asan) checks exactly the code that bounds-checks untrusted file bytes.
//
// Block layout (FilterBlockWriter::Final, src/filter_block.cpp:77-102):
//   [bitmap_0 .. bitmap_{F-1}][i32 off_0 = 0 .. i32 off_{F-1}][i32 offsets_start]
//   [i32 F][info: "bf:" + i32 bits_per_key][i32 info_len]
// Every check the reference makes returns FILTER_BLOCK_ERROR here too; where
// the reference would read outside the block (an offsets array or an info
// field running past its end, offsets out of order or beyond offsets_start)
// this returns FILTER_BLOCK_ERROR instead, and so it does for a filter of
// more than 2^31 bits, which the reference's `int m` (:50) cannot probe.
#pragma once
#include <stdint.h>
#include <string.h>

#include <vector>

namespace adl_fmt {

constexpr int kFilterBlockError = 13;  // RC::FILTER_BLOCK_ERROR (src/rc.hpp:22)

struct FilterBlockLayout {
  int32_t bits_per_key = 0;
  int32_t num_filters = 0;
  int32_t offsets_start = 0;          // filters_offsets_offset_
  int64_t info_offset = 0, info_len = 0;
  std::vector<uint64_t> off;          // F+1 entries: filter f = [off[f], off[f+1])
};

inline int32_t load32(const uint8_t *p) {  // Decode32, src/encode.cpp:6
  int32_t v;
  memcpy(&v, p, sizeof(v));
  return v;
}

// Returns 0 or kFilterBlockError.  Reads only bytes [0, len) of `b`.
inline int parse_filter_block(const uint8_t *b, uint64_t len, FilterBlockLayout &out) {
  out = FilterBlockLayout{};
  if (!b && len) return kFilterBlockError;
  /* 1. info_len (:116-122) */
  if (len < 4 || len > 0x7fffffffull) return kFilterBlockError;
  const int64_t info_len_offset = (int64_t)len - 4;
  const int32_t info_len = load32(b + info_len_offset);
  if (info_len > info_len_offset || info_len <= 0) return kFilterBlockError;
  /* 2. CreateFilterAlgorithm (:158-170): "bf", bits_per_key at info[3] */
  const int64_t info_offset = info_len_offset - info_len;
  if (info_len < 2 || b[info_offset] != 'b' || b[info_offset + 1] != 'f') return kFilterBlockError;
  if (info_len < 7) return kFilterBlockError;  // the reference reads past the info here
  out.bits_per_key = load32(b + info_offset + 3);
  out.info_offset = info_offset;
  out.info_len = info_len;
  /* 3. filter count (:128-131) */
  if (info_offset < 4) return kFilterBlockError;
  const int64_t nums_offset = info_offset - 4;
  const int32_t nf = load32(b + nums_offset);
  /* 4-5. offsets array start (:133-140) */
  if (nums_offset < 4) return kFilterBlockError;
  const int32_t offsets_start = load32(b + nums_offset - 4);
  if (offsets_start < 0) return kFilterBlockError;
  /* the offsets array must lie inside the block (the reference reads beyond it) */
  if (nf < 0 || (int64_t)offsets_start + 4ll * (nf ? nf : 1) > nums_offset) return kFilterBlockError;
  /* 6. filter 0 starts at 0 (:142-145) */
  if (load32(b + offsets_start) != 0) return kFilterBlockError;
  out.num_filters = nf;
  out.offsets_start = offsets_start;
  out.off.assign((size_t)nf + 1, 0);
  for (int32_t f = 0; f < nf; ++f) {
    const int32_t o = load32(b + offsets_start + 4ll * f);
    if (o < 0 || o > offsets_start || (f && (uint64_t)o < out.off[f - 1])) return kFilterBlockError;
    out.off[f] = (uint64_t)o;
  }
  out.off[nf] = (uint64_t)offsets_start;
  for (int32_t f = 0; f < nf; ++f)
    if ((out.off[f + 1] - out.off[f]) * 8 > 0x7fffffffull) return kFilterBlockError;
  return 0;
}

}  // namespace adl_fmt
