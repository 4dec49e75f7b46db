// adlsm-tree_amd/csrc/filter_block.hpp -- host C++ mirror of the reference's
// filter API (src/filter_block.hpp:13-73, src/murmur3_hash.hpp:9) on top of the
// gfx950 C-ABI in include/adl_bloom.h.
//
// Same class names, signatures and semantics as the reference, so
// src/sstable.cpp and test/filter_block_test.cpp compile against it unchanged.
// What differs underneath:
//   * FilterBlockWriter keeps its pending keys in a packed arena (bytes +
//     uint64 offsets) instead of vector<string>.  Keys2Block() closes a filter;
//     Final() builds every filter of the block in one pipelined segmented GPU
//     build (adl_bloom_build_segmented) straight into the block buffer, at the
//     byte offsets the reference's successive appends would give them.
//   * FilterBlockReader::Init uploads the block's bitmaps once into a
//     device-resident filter set; IsKeyExists probes on the GPU.  Batched
//     IsKeysExist() is the intended read path (one launch per batch).
//   * Device failures surface as RC::DEVICE_ERROR; nothing throws.
#pragma once
#include <stdint.h>

#include <memory>
#include <string>
#include <string_view>
#include <vector>

#include "rc.hpp"

struct adl_bloom_filter_set;

namespace adl {

using namespace std;

/* Packed key batch: key i = bytes[offsets[i] .. offsets[i+1]). */
class KeyArena {
 public:
  KeyArena() : offsets_{0} {}
  void Add(string_view key) {
    bytes_.append(key.data(), key.size());
    offsets_.push_back(bytes_.size());
  }
  void Clear() {
    bytes_.clear();
    offsets_.assign(1, 0);
  }
  size_t size() const { return offsets_.size() - 1; }
  bool empty() const { return size() == 0; }
  const string &bytes() const { return bytes_; }
  const vector<uint64_t> &offsets() const { return offsets_; }

 private:
  string bytes_;
  vector<uint64_t> offsets_;
};

/* src/filter_block.hpp:13-20 */
class FilterAlgorithm {
 public:
  virtual RC Keys2Block(const vector<string> &keys, string &result) = 0;
  virtual bool IsKeyExists(string_view key, string_view bitmap) = 0;
  virtual void FilterInfo(string &/*info*/) { /* NOTHING */ }
  /* batched extensions */
  virtual RC Keys2Block(const KeyArena &keys, string &result) = 0;
  /* Keys2Block for consecutive filters: filter f = keys [key_begin[f],
   * key_begin[f+1]); the bitmaps are appended to result back to back, as
   * successive Keys2Block calls would, filter f starting at starts[f].  The
   * default loops over Keys2Block. */
  virtual RC Keys2Blocks(const KeyArena &keys, const vector<uint64_t> &key_begin, string &result,
                         vector<uint64_t> &starts);
  virtual RC IsKeysExist(const KeyArena &keys, string_view bitmap, vector<uint8_t> &out) = 0;
  virtual ~FilterAlgorithm() = default;
};

/* src/filter_block.hpp:22-34 */
class BloomFilter : public FilterAlgorithm {
 public:
  explicit BloomFilter(int bits_per_key);
  RC Keys2Block(const vector<string> &keys, string &result) override;
  bool IsKeyExists(string_view key, string_view bitmap) override;
  void FilterInfo(string &info) override;
  RC Keys2Block(const KeyArena &keys, string &result) override;
  RC Keys2Blocks(const KeyArena &keys, const vector<uint64_t> &key_begin, string &result,
                 vector<uint64_t> &starts) override;
  RC IsKeysExist(const KeyArena &keys, string_view bitmap, vector<uint8_t> &out) override;
  int bits_per_key() const { return bits_per_key_; }
  int num_probes() const { return k_; }
  ~BloomFilter() = default;

 private:
  int bits_per_key_;
  int k_;
};

/* src/filter_block.hpp:36-52 */
class FilterBlockWriter {
 public:
  explicit FilterBlockWriter(unique_ptr<FilterAlgorithm> &&method);
  RC Update(string_view key);
  RC Final(string &result);
  RC Keys2Block();

 private:
  KeyArena keys_;              /* keys of every filter not yet built */
  vector<uint64_t> bounds_{0}; /* filter f = keys_ [bounds_[f], bounds_[f+1]) */
  string buffer_;
  unique_ptr<FilterAlgorithm> method_;
};

/* src/filter_block.hpp:54-73 */
class FilterBlockReader {
 public:
  FilterBlockReader();
  ~FilterBlockReader();
  FilterBlockReader(const FilterBlockReader &) = delete;
  FilterBlockReader &operator=(const FilterBlockReader &) = delete;
  RC Init(string_view filter_block);
  bool IsKeyExists(int filter_block_num, string_view key);
  /* batched: out[i] = IsKeyExists(filter_block_num, key i) */
  RC IsKeysExist(int filter_block_num, const KeyArena &keys, vector<uint8_t> &out);
  int filters_nums() const { return filters_nums_; }

 private:
  RC CreateFilterAlgorithm();
  RC Upload();

  int filters_nums_;
  int filters_offsets_offset_;
  string_view filters_offsets_;
  string_view filter_info_;
  string_view filter_blocks_;
  unique_ptr<FilterAlgorithm> method_;
  int bits_per_key_ = 0;
  adl_bloom_filter_set *device_set_ = nullptr; /* owned device copy of the bitmaps */
};

/* src/murmur3_hash.hpp:9 -- computed on the GPU (adl_bloom_murmur3). */
uint32_t murmur3_hash(uint32_t seed, const char *data, size_t len);

}  // namespace adl
