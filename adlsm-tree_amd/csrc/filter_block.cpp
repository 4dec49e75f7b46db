// adlsm-tree_amd/csrc/filter_block.cpp -- host C++ mirror of the reference's
// filter API over the gfx950 C-ABI (include/adl_bloom.h).  See
// filter_block.hpp for what differs from src/filter_block.cpp underneath.
#include "filter_block.hpp"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <mutex>

#include "adl_bloom.h"
#include "filter_block_format.hpp"

namespace adl {

namespace {

/* FilterBlockWriter::Final skips adjacent duplicate keys on the device when at
 * least Num/Den of its keys are such duplicates (the generic pass A it then
 * runs costs more than the fast paths on keys without them). */
constexpr uint64_t kSkipDuplicatesNum = 1, kSkipDuplicatesDen = 3;

/* Decode32 (reference src/encode.cpp:6): native-endian unaligned int32 load. */
int Load32(const char *src) {
  int v;
  memcpy(&v, src, sizeof(int));
  return v;
}

void Append32(string &dst, int v) { dst.append(reinterpret_cast<const char *>(&v), sizeof(int)); }

RC FromStatus(int status) {
  if (status == ADL_OK) return OK;
  if (status == ADL_FILTER_BLOCK_ERROR) return FILTER_BLOCK_ERROR;
  if (status == ADL_ERR_TOO_LARGE) return OUT_OF_RANGE;
  return DEVICE_ERROR;
}

void Pack(const vector<string> &keys, KeyArena &arena) {
  for (const auto &k : keys) arena.Add(k);
}

}  // namespace

string_view strrc(RC rc) {
  static const char *const kNames[] = {
      "ok", "not found", "is not directory", "create directory failed",
      "destroy directory failed", "destroy file failed", "un implemented", "existed",
      "open file error", "io error", "close file error", "rename file error",
      "make temp error", "filter block error", "footer block error", "unsupported format",
      "db closed", "stat file error", "mmap error", "out of range", "bad level",
      "bad revision", "bad file meta", "bad record", "file eof", "check sum error",
      "noexcept size", "bad file path", "bad current file", "new sstable error",
      "device error"};
  if (rc >= 0 && rc <= DEVICE_ERROR) return kNames[rc];
  return "unknown error";
}

// ------------------------------------------------------------- BloomFilter

/* src/filter_block.cpp:35-47 -- k from bits_per_key (same formula, in the C-ABI). */
BloomFilter::BloomFilter(int bits_per_key)
    : bits_per_key_(bits_per_key), k_(adl_bloom_num_probes(bits_per_key)) {}

/* src/filter_block.cpp:9-33 -- appends n*bpk+7 bytes of bitmap to `result`. */
RC BloomFilter::Keys2Block(const vector<string> &keys, string &result) {
  KeyArena arena;
  Pack(keys, arena);
  return Keys2Block(arena, result);
}

RC BloomFilter::Keys2Block(const KeyArena &keys, string &result) {
  const uint64_t n = keys.size();
  const uint64_t bytes = adl_bloom_bitmap_bytes(n, bits_per_key_);
  if (bytes == 0) return OUT_OF_RANGE;
  const size_t init_len = result.size();
  result.resize(init_len + bytes);
  const int st = adl_bloom_build(reinterpret_cast<const uint8_t *>(keys.bytes().data()),
                                 keys.offsets().data(), n, 0, bits_per_key_,
                                 reinterpret_cast<uint8_t *>(&result[init_len]), nullptr);
  if (st != ADL_OK) {
    result.resize(init_len);
    return FromStatus(st);
  }
  return OK;
}

RC FilterAlgorithm::Keys2Block(const KeyArena &keys, string &result) {
  vector<string> v;
  v.reserve(keys.size());
  for (size_t i = 0; i < keys.size(); ++i) v.emplace_back(keys.key(i));
  return Keys2Block(v, result);
}

RC FilterAlgorithm::IsKeysExist(const KeyArena &keys, string_view bitmap, vector<uint8_t> &out) {
  out.assign(keys.size(), 0);
  for (size_t i = 0; i < keys.size(); ++i) out[i] = IsKeyExists(keys.key(i), bitmap) ? 1 : 0;
  return OK;
}

RC FilterAlgorithm::Keys2Blocks(const KeyArena &keys, const vector<uint64_t> &key_begin, string &result,
                                vector<uint64_t> &starts, bool /*adjacent_duplicates*/) {
  starts.clear();
  for (size_t f = 0; f + 1 < key_begin.size(); ++f) {
    starts.push_back(result.size());
    KeyArena part;
    for (uint64_t i = key_begin[f]; i < key_begin[f + 1]; ++i)
      part.Add(keys.key(i));
    if (RC rc = Keys2Block(part, result); rc != OK) return rc;
  }
  return OK;
}

/* All filters of a block in one pipelined segmented build, each bitmap written
 * in place at the offset successive Keys2Block appends would give it.  With
 * many adjacent duplicates the build skips them (same bitmaps). */
RC BloomFilter::Keys2Blocks(const KeyArena &keys, const vector<uint64_t> &key_begin, string &result,
                            vector<uint64_t> &off, bool adjacent_duplicates) {
  const size_t nf = key_begin.size() - 1;
  off.assign(nf, 0);
  if (nf == 0) return OK;
  const size_t init_len = result.size();
  uint64_t total = 0;
  for (size_t f = 0; f < nf; ++f) {
    const uint64_t bytes = adl_bloom_bitmap_bytes(key_begin[f + 1] - key_begin[f], bits_per_key_);
    if (bytes == 0) return OUT_OF_RANGE;
    off[f] = init_len + total;
    total += bytes;
  }
  result.resize(init_len + total);
  const int st = adl_bloom_build_segmented_ex(
      reinterpret_cast<const uint8_t *>(keys.bytes().data()), keys.offsets().data(), 0, key_begin.data(),
      (uint32_t)nf, bits_per_key_, reinterpret_cast<uint8_t *>(&result[0]), off.data(),
      adjacent_duplicates ? ADL_BLOOM_SKIP_ADJACENT_DUPLICATES : 0u, nullptr);
  if (st != ADL_OK) {
    result.resize(init_len);
    return FromStatus(st);
  }
  return OK;
}

/* src/filter_block.cpp:49-62 -- one key against a host bitmap view.  The
 * bitmap is not resident, so this uploads it; FilterBlockReader keeps its
 * bitmaps on the device instead.  A device failure answers true ("may be
 * present"), the answer that never loses a key. */
bool BloomFilter::IsKeyExists(string_view key, string_view bitmap) {
  if (bitmap.empty()) return false;
  const uint64_t offs[2] = {0, key.size()};
  const char empty = 0;
  uint8_t hit = 1;
  const int st = adl_bloom_probe(reinterpret_cast<const uint8_t *>(key.empty() ? &empty : key.data()),
                                 offs, 1, 0, bits_per_key_,
                                 reinterpret_cast<const uint8_t *>(bitmap.data()), bitmap.size(),
                                 &hit, nullptr);
  if (st != ADL_OK) {
    fprintf(stderr, "adl::BloomFilter::IsKeyExists: %s\n", adl_bloom_strerror(st));
    return true;
  }
  return hit != 0;
}

RC BloomFilter::IsKeysExist(const KeyArena &keys, string_view bitmap, vector<uint8_t> &out) {
  out.assign(keys.size(), 0);
  if (keys.empty()) return OK;
  if (bitmap.empty()) return OK;
  const int st = adl_bloom_probe(reinterpret_cast<const uint8_t *>(keys.bytes().data()),
                                 keys.offsets().data(), keys.size(), 0, bits_per_key_,
                                 reinterpret_cast<const uint8_t *>(bitmap.data()), bitmap.size(),
                                 out.data(), nullptr);
  return FromStatus(st);
}

/* src/filter_block.cpp:64-67 -- "bf:" + raw native-endian int32 bits_per_key. */
void BloomFilter::FilterInfo(string &info) {
  info.append("bf:");
  Append32(info, bits_per_key_);
}

// ------------------------------------------------------------- FilterBlockWriter

FilterBlockWriter::FilterBlockWriter(unique_ptr<FilterAlgorithm> &&method)
    : method_(std::move(method)) {}

/* src/filter_block.cpp:72-75 */
RC FilterBlockWriter::Update(string_view key) {
  const size_t from = keys_.size();
  keys_.Add(key);
  CountDuplicates(from);
  return OK;
}

RC FilterBlockWriter::UpdateBatch(const char *base, const uint64_t *off, size_t n, size_t trim) {
  const size_t from = keys_.size();
  keys_.AddTrimmed(base, off, n, trim);
  CountDuplicates(from);
  return OK;
}

/* keys [from, size) against their predecessors in the same filter: a user
 * key's versions arrive in a row (memtable order, src/keys.cpp:61-74) */
void FilterBlockWriter::CountDuplicates(size_t from) {
  for (size_t i = std::max<size_t>(from, bounds_.back() + 1); i < keys_.size(); ++i)
    dups_ += keys_.key(i) == keys_.key(i - 1);
}

/* src/filter_block.cpp:104-109 -- closes the current filter; its bitmap is
 * built with all the others in Final(). */
RC FilterBlockWriter::Keys2Block() {
  bounds_.push_back(keys_.size());
  return OK;
}

/* src/filter_block.cpp:77-102 -- [bitmaps][int32 offsets][int32 offsets_start]
 * [int32 num_filters][info]["int32 info_len"], moved out into `result`.
 * Returns the first Keys2Block failure (the reference cannot fail here). */
RC FilterBlockWriter::Final(string &result) {
  if (keys_.size() > bounds_.back()) Keys2Block();
  vector<uint64_t> offsets;
  // Skipping duplicates runs the generic pass A (keys in their order), which
  // only pays when they are frequent (adjacent duplicates).
  const bool skip = dups_ * kSkipDuplicatesDen >= keys_.size() * kSkipDuplicatesNum && dups_ > 0;
  const RC rc = method_->Keys2Blocks(keys_, bounds_, buffer_, offsets, skip);
  keys_.Clear();
  bounds_.assign(1, 0);
  dups_ = 0;
  if (rc != OK) {
    buffer_.clear();
    return rc;
  }
  const int offsets_start = (int)buffer_.size();
  for (uint64_t off : offsets) Append32(buffer_, (int)off);
  Append32(buffer_, offsets_start);
  Append32(buffer_, (int)offsets.size());
  string info;
  method_->FilterInfo(info);
  if (!info.empty()) {
    buffer_.append(info);
    Append32(buffer_, (int)info.size());
  }
  result = std::move(buffer_);
  buffer_.clear();
  return OK;
}

// ------------------------------------------------------------- FilterCache

FilterCache::FilterCache(uint64_t capacity_bytes, uint32_t max_tables, int bits_per_key)
    : bits_per_key_(bits_per_key) {
  status_ = FromStatus(adl_bloom_filter_cache_create(capacity_bytes, max_tables, bits_per_key, &h_));
}

FilterCache::~FilterCache() { adl_bloom_filter_cache_destroy(h_); }

RC FilterCache::Put(string_view oid, string_view filter_block) {
  if (!h_) return status_;
  return FromStatus(adl_bloom_filter_cache_put(h_, oid.data(), oid.size(),
                                               reinterpret_cast<const uint8_t *>(filter_block.data()),
                                               filter_block.size()));
}

bool FilterCache::Contains(string_view oid) {
  return h_ && adl_bloom_filter_cache_contains(h_, oid.data(), oid.size()) == 1;
}

bool FilterCache::Remove(string_view oid) {
  return h_ && adl_bloom_filter_cache_remove(h_, oid.data(), oid.size()) == 1;
}

RC FilterCache::Probe(const vector<string_view> &oids, const vector<uint32_t> &table, const KeyArena &keys,
                      int filter, vector<uint8_t> &out, uint64_t *uncached) {
  out.assign(keys.size(), 0);
  if (uncached) *uncached = 0;
  if (!h_) return status_;
  if (table.size() != keys.size() || filter < 0) return OUT_OF_RANGE;
  if (keys.empty()) return OK;
  vector<const char *> ptr(oids.size());
  vector<uint64_t> len(oids.size());
  for (size_t j = 0; j < oids.size(); ++j) {
    ptr[j] = oids[j].data();
    len[j] = oids[j].size();
  }
  uint64_t unc = 0;
  const int st = adl_bloom_filter_cache_probe(h_, ptr.data(), len.data(), (uint32_t)oids.size(), (uint32_t)filter,
                                              reinterpret_cast<const uint8_t *>(keys.bytes().data()),
                                              keys.offsets().data(), keys.size(), 0, table.data(), out.data(),
                                              &unc, nullptr);
  if (uncached) *uncached = unc;
  return FromStatus(st);
}

FilterCache *FilterCache::Shared(int) { return Shared(); }

FilterCache *FilterCache::Shared() {
  struct Slot {
    FilterCache *cache = nullptr;
    std::chrono::steady_clock::time_point retry_after{};  // after a failed creation
  };
  static std::mutex mu;
  static Slot *slot = new Slot;  // kept until exit
  std::lock_guard<std::mutex> g(mu);
  Slot &s = *slot;
  if (s.cache) return s.cache;  // only created (OK) caches are stored
  // A failed creation is not retried on every reader open (each try holds this
  // lock over up to three arena allocations): not again for a second.
  const auto now = std::chrono::steady_clock::now();
  if (now < s.retry_after) return nullptr;
  const char *e = getenv("ADL_BLOOM_READER_CACHE_BYTES");
  uint64_t bytes = e ? strtoull(e, nullptr, 10) : (1ull << 30);
  // the default size shrinks when device memory is short (other processes on
  // the GPU): a quarter, then a sixteenth; a size the user set is taken as is
  const int tries = e ? 1 : 3;
  for (int i = 0; i < tries; ++i, bytes /= 4) {
    FilterCache *c = new FilterCache(bytes, 1u << 20);
    if (c->status() == OK) {
      s.cache = c;
      return c;
    }
    delete c;
  }
  s.retry_after = now + std::chrono::seconds(1);
  return nullptr;
}

// ------------------------------------------------------------- FilterBlockReader

FilterBlockReader::FilterBlockReader() : filters_nums_(0), filters_offsets_offset_(0) {}

FilterBlockReader::~FilterBlockReader() { Release(); }

void FilterBlockReader::Release() {
  if (cache_ && own_oid_) cache_->Remove(oid_);
  cache_ = nullptr;
  own_oid_ = false;
  oid_.clear();
  adl_bloom_filter_set_destroy(device_set_.exchange(nullptr));
}

/* src/filter_block.cpp:113-155 -- the trailer walk of filter_block_format.hpp
 * (the reference's FILTER_BLOCK_ERROR checks, plus bounds checks where the
 * reference would read outside the block). */
RC FilterBlockReader::Parse(string_view filter_blocks) {
  Release();
  filter_blocks_ = filter_blocks;
  filters_nums_ = 0;
  adl_fmt::FilterBlockLayout lay;
  if (adl_fmt::parse_filter_block(reinterpret_cast<const uint8_t *>(filter_blocks_.data()), filter_blocks_.size(),
                                  lay))
    return FILTER_BLOCK_ERROR;
  filter_info_ = filter_blocks_.substr(lay.info_offset, lay.info_len);
  if (RC rc = CreateFilterAlgorithm(); rc) return rc;
  filters_nums_ = lay.num_filters;
  filters_offsets_offset_ = lay.offsets_start;
  filters_offsets_ = filter_blocks_.substr(filters_offsets_offset_, sizeof(int) * filters_nums_);
  return OK;
}

RC FilterBlockReader::Init(string_view filter_blocks) {
  if (RC rc = Parse(filter_blocks); rc) return rc;
  FilterCache *c = FilterCache::Shared();
  if (!c) return Upload();  // no shared arena: a device copy of its own
  static std::atomic<uint64_t> next_id{0};
  oid_ = "\x01reader:" + std::to_string(next_id.fetch_add(1));
  const RC rc = c->Put(oid_, filter_blocks_);
  if (rc == OK) {
    cache_ = c;
    own_oid_ = true;
    return OK;
  }
  oid_.clear();
  if (rc == FILTER_BLOCK_ERROR) return rc;
  return Upload();  // larger than the shared arena: a device copy of its own
}

RC FilterBlockReader::Init(string_view filter_blocks, FilterCache &cache, string_view oid) {
  if (RC rc = Parse(filter_blocks); rc) return rc;
  // (the cache keeps this block's own bits_per_key with its entry: tables of
  // any bpk share one cache, as Level::Get reads them, src/revision.cpp:265-310)
  oid_.assign(oid.data(), oid.size());
  cache_ = &cache;
  own_oid_ = false;
  if (cache.Contains(oid_)) return OK;  // another reader of this SSTable uploaded it
  return cache.Put(oid_, filter_blocks_);
}

/* src/filter_block.cpp:158-170 -- only "bf" is known; bits_per_key at info[3]. */
RC FilterBlockReader::CreateFilterAlgorithm() {
  if (filter_info_.substr(0, 2) != "bf") return FILTER_BLOCK_ERROR;
  if (filter_info_.size() < 3 + sizeof(int)) return FILTER_BLOCK_ERROR;
  bits_per_key_ = Load32(&filter_info_[3]);
  method_ = std::make_unique<BloomFilter>(bits_per_key_);
  return OK;
}

RC FilterBlockReader::Upload() {
  vector<uint64_t> off(filters_nums_ + 1);
  for (int i = 0; i < filters_nums_; ++i) off[i] = (uint64_t)Load32(&filters_offsets_[i * sizeof(int)]);
  off[filters_nums_] = (uint64_t)filters_offsets_offset_;
  adl_bloom_filter_set *set = nullptr;
  const int st = adl_bloom_filter_set_create(reinterpret_cast<const uint8_t *>(filter_blocks_.data()),
                                             off.data(), (uint32_t)filters_nums_, bits_per_key_, &set);
  if (st == ADL_OK) device_set_.store(set);
  return FromStatus(st);
}

/* One launch over the batch.  The cache may have evicted this block (other
 * tables took its room): then it is uploaded again from the reader's view
 * and the probe repeated.  A block that keeps being evicted before its probe
 * runs (a cache far too small for its working set) moves to a device copy
 * of the reader's own, so the answers stay exact. */
RC FilterBlockReader::Probe(int filter_block_num, const KeyArena &keys, vector<uint8_t> &out) {
  if (!device_set_ && cache_) {
    const vector<string_view> oids{oid_};
    const vector<uint32_t> table(keys.size(), 0);
    for (int attempt = 0; attempt < 4; ++attempt) {
      uint64_t uncached = 0;
      if (RC rc = cache_->Probe(oids, table, keys, filter_block_num, out, &uncached); rc) return rc;
      if (uncached == 0) return OK;
      if (RC rc = cache_->Put(oid_, filter_blocks_); rc) return rc;
    }
    std::lock_guard<std::mutex> g(upload_mu_);
    if (!device_set_)
      if (RC rc = Upload(); rc) return rc;
  }
  if (!device_set_) return FILTER_BLOCK_ERROR;
  out.assign(keys.size(), 0);
  return FromStatus(adl_bloom_filter_set_probe(device_set_.load(), reinterpret_cast<const uint8_t *>(keys.bytes().data()),
                                               keys.offsets().data(), keys.size(), 0, nullptr,
                                               (uint32_t)filter_block_num, out.data(), nullptr));
}

/* src/filter_block.cpp:172-184 -- one key against filter `filter_block_num`.
 * A device failure answers true ("may be present"). */
bool FilterBlockReader::IsKeyExists(int filter_block_num, string_view key) {
  if (filter_block_num < 0 || filter_block_num >= filters_nums_) return false;
  KeyArena one;
  one.Add(key);
  vector<uint8_t> hit;
  if (RC rc = Probe(filter_block_num, one, hit); rc) {
    fprintf(stderr, "adl::FilterBlockReader::IsKeyExists: %s\n", string(strrc(rc)).c_str());
    return true;
  }
  return hit[0] != 0;
}

RC FilterBlockReader::IsKeysExist(int filter_block_num, const KeyArena &keys, vector<uint8_t> &out) {
  out.assign(keys.size(), 0);
  if (filter_block_num < 0 || filter_block_num >= filters_nums_ || keys.empty()) return OK;
  return Probe(filter_block_num, keys, out);
}

/* src/murmur3_hash.cpp:11-65, evaluated on the GPU.  There is no error channel
 * in this signature, so a device failure aborts loudly. */
uint32_t murmur3_hash(uint32_t seed, const char *data, size_t len) {
  uint32_t h = 0;
  const int st = adl_bloom_murmur3(seed, data, len, &h);
  if (st != ADL_OK) {
    fprintf(stderr, "adl::murmur3_hash: %s\n", adl_bloom_strerror(st));
    abort();
  }
  return h;
}

}  // namespace adl
