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
//     FilterCache arena (keyed by SSTable oid); IsKeyExists probes on the GPU.
//     Batched IsKeysExist() and the level multi-get (level_filter.hpp) are
//     the intended read paths (one launch per batch).
//   * Device failures surface as RC::DEVICE_ERROR; nothing throws.
#pragma once
#include <stdint.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <vector>

#include "rc.hpp"

struct adl_bloom_filter_set;
struct adl_bloom_filter_cache;

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
  /* room for `keys` more keys of `bytes` bytes in all (no reallocation while they are added) */
  void Reserve(size_t keys, size_t bytes) {
    bytes_.reserve(bytes_.size() + bytes);
    offsets_.reserve(offsets_.size() + keys);
  }
  /* keys i < n = base[off[i] .. off[i+1] - trim): a packed run of records
   * whose last `trim` bytes are not part of the key (inner keys' seq + op);
   * every record must be at least `trim` bytes.  Space is reserved once. */
  void AddTrimmed(const char *base, const uint64_t *off, size_t n, size_t trim) {
    if (!n) return;
    bytes_.reserve(bytes_.size() + (size_t)(off[n] - off[0]) - n * trim);
    offsets_.reserve(offsets_.size() + n);
    for (size_t i = 0; i < n; ++i) {
      bytes_.append(base + off[i], (size_t)(off[i + 1] - off[i]) - trim);
      offsets_.push_back(bytes_.size());
    }
  }
  void Clear() {
    bytes_.clear();
    offsets_.assign(1, 0);
  }
  size_t size() const { return offsets_.size() - 1; }
  string_view key(size_t i) const {
    return string_view(bytes_).substr(offsets_[i], offsets_[i + 1] - offsets_[i]);
  }
  bool empty() const { return size() == 0; }
  const string &bytes() const { return bytes_; }
  const vector<uint64_t> &offsets() const { return offsets_; }

 private:
  string bytes_;
  vector<uint64_t> offsets_;
};

/* src/filter_block.hpp:13-20.  The first three members are the reference's;
 * the batched extensions after them have default implementations in terms of
 * those three, so a subclass written against the reference's FilterAlgorithm
 * (overriding only Keys2Block(vector<string>), IsKeyExists and FilterInfo)
 * compiles and works unchanged in FilterBlockWriter / FilterBlockReader.
 * BloomFilter overrides them with the batched GPU path. */
class FilterAlgorithm {
 public:
  virtual RC Keys2Block(const vector<string> &keys, string &result) = 0;
  virtual bool IsKeyExists(string_view key, string_view bitmap) = 0;
  virtual void FilterInfo(string &/*info*/) { /* NOTHING */ }
  /* batched extensions (defaults: unpack and call the reference methods) */
  virtual RC Keys2Block(const KeyArena &keys, string &result);
  /* Keys2Block for consecutive filters: filter f = keys [key_begin[f],
   * key_begin[f+1]); the bitmaps are appended to result back to back, as
   * successive Keys2Block calls would, filter f starting at starts[f].  The
   * default loops over Keys2Block.  adjacent_duplicates: a hint that many keys
   * equal their predecessor (versions of one user key in memtable order); the
   * result is the same either way, an implementation may skip such keys. */
  virtual RC Keys2Blocks(const KeyArena &keys, const vector<uint64_t> &key_begin, string &result,
                         vector<uint64_t> &starts, bool adjacent_duplicates = false);
  /* out[i] = IsKeyExists(key i, bitmap); the default loops over IsKeyExists */
  virtual RC IsKeysExist(const KeyArena &keys, string_view bitmap, vector<uint8_t> &out);
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
                 vector<uint64_t> &starts, bool adjacent_duplicates = false) override;
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
  /* Update for a packed run (KeyArena::AddTrimmed): n keys, one reservation */
  RC UpdateBatch(const char *base, const uint64_t *off, size_t n, size_t trim);
  RC Final(string &result);
  RC Keys2Block();
  /* keys added since the last Final that equal the previous key of their filter */
  uint64_t adjacent_duplicates() const { return dups_; }

 private:
  void CountDuplicates(size_t from);
  KeyArena keys_;              /* keys of every filter not yet built */
  vector<uint64_t> bounds_{0}; /* filter f = keys_ [bounds_[f], bounds_[f+1]) */
  uint64_t dups_ = 0;          /* adjacent duplicates among keys_ (CountDuplicates) */
  string buffer_;
  unique_ptr<FilterAlgorithm> method_;
};

/* Device-resident filter blocks of many SSTables in one HBM arena, keyed by
 * oid (the SSTable's SHA-256 file name), least recently used evicted first:
 * the filter side of DB::table_cache_ (src/db.hpp:96-97, LRUCache
 * src/cache.hpp:23-93).  C++ handle over adl_bloom_filter_cache (C-ABI);
 * thread-safe, and no lock is held while a probe runs on the device. */
class FilterCache {
 public:
  /* bits_per_key: kept for source compatibility; blocks of any bits_per_key
   * are accepted, each probed with the k of its own "bf:" info */
  FilterCache(uint64_t capacity_bytes, uint32_t max_tables, int bits_per_key = 10);
  ~FilterCache();
  FilterCache(const FilterCache &) = delete;
  FilterCache &operator=(const FilterCache &) = delete;
  RC status() const { return status_; } /* creation result */
  int bits_per_key() const { return bits_per_key_; }
  /* FilterBlockReader::Init's checks (FILTER_BLOCK_ERROR), then one upload */
  RC Put(string_view oid, string_view filter_block);
  bool Contains(string_view oid);
  bool Remove(string_view oid);
  /* One launch for the batch: out[i] = filter `filter` of table
   * oids[table[i]] may contain keys[i] (a table that is not cached answers 1,
   * "may be present"; *uncached counts those queries). */
  RC Probe(const vector<string_view> &oids, const vector<uint32_t> &table, const KeyArena &keys, int filter,
           vector<uint8_t> &out, uint64_t *uncached = nullptr);
  /* The process-wide cache FilterBlockReader::Init(string_view) keeps its
   * bitmaps in, for blocks of every bits_per_key (arena
   * ADL_BLOOM_READER_CACHE_BYTES, default 1 GiB); created on first use and
   * kept until exit.  (Shared(int) is the round-5 spelling: the same cache.) */
  static FilterCache *Shared();
  static FilterCache *Shared(int bits_per_key);

 private:
  adl_bloom_filter_cache *h_ = nullptr;
  int bits_per_key_;
  RC status_;
};

/* src/filter_block.hpp:54-73.  The bitmaps live in a FilterCache arena (one
 * upload per block, no allocation per Init); the reader keeps the caller's
 * view of the block, as the reference's does, and re-uploads it if the cache
 * evicted it. */
class FilterBlockReader {
 public:
  FilterBlockReader();
  ~FilterBlockReader();
  FilterBlockReader(const FilterBlockReader &) = delete;
  FilterBlockReader &operator=(const FilterBlockReader &) = delete;
  /* src/filter_block.hpp:57: the bitmaps go into FilterCache::Shared()
   * under an id private to this reader (removed by the destructor) */
  RC Init(string_view filter_block);
  /* the same, with the table's entry in `cache` under `oid`: every reader of
   * one SSTable (and a level multi-get over it) shares one device copy */
  RC Init(string_view filter_block, FilterCache &cache, string_view oid);
  bool IsKeyExists(int filter_block_num, string_view key);
  /* batched: out[i] = IsKeyExists(filter_block_num, key i), one launch */
  RC IsKeysExist(int filter_block_num, const KeyArena &keys, vector<uint8_t> &out);
  int filters_nums() const { return filters_nums_; }

 private:
  RC Parse(string_view filter_block);
  RC CreateFilterAlgorithm();
  RC Upload();
  RC Probe(int filter_block_num, const KeyArena &keys, vector<uint8_t> &out);
  void Release();

  int filters_nums_;
  int filters_offsets_offset_;
  string_view filters_offsets_;
  string_view filter_info_;
  string_view filter_blocks_;
  unique_ptr<FilterAlgorithm> method_;
  int bits_per_key_ = 0;
  FilterCache *cache_ = nullptr;               /* where the bitmaps are resident */
  string oid_;                                 /* their key in cache_ */
  bool own_oid_ = false;                       /* a private id: removed with the reader */
  std::mutex upload_mu_;                       /* guards the move to device_set_ */
  std::atomic<adl_bloom_filter_set *> device_set_{nullptr}; /* a copy of its own: blocks larger than
                                                   the shared arena, or evicted again and again */
};

/* src/murmur3_hash.hpp:9 -- computed on the GPU (adl_bloom_murmur3). */
uint32_t murmur3_hash(uint32_t seed, const char *data, size_t len);

}  // namespace adl
