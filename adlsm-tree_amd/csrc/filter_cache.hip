// adlsm-tree_amd/csrc/filter_cache.hip -- device-resident filter cache keyed by
// SSTable oid, for batched multi-get probes.
//
// The reference keeps open SSTableReaders in an LRU cache keyed by oid
// (DB::table_cache_, src/db.hpp:96-97; LRUCache, src/cache.hpp:23-93); each
// reader holds its filter block as a view into the mmapped file
// (SSTableReader::ReadFilterBlock, src/sstable.cpp:179-209) and Get probes
// filter 0 one key at a time (src/sstable.cpp:238).  Here the filter blocks of
// many tables live in ONE device arena (capacity fixed at creation, sized for
// HBM), so a whole multi-get batch -- keys bound for many tables -- is one
// launch of the range-based multi-filter probe.
//
//  * put(oid, block): parses the trailer as FilterBlockReader::Init does
//    (src/filter_block.cpp:113-155, same FILTER_BLOCK_ERROR cases plus bounds
//    checks), uploads the bitmap region once, and inserts it as most recently
//    used; least recently used blocks are evicted until it fits (arena bytes)
//    and the table count is within max_tables (the reference's maxSize).
//  * probe(oids, per-query table index, keys): every referenced table is
//    looked up (and marked used); a query bound for a table that is not
//    cached answers 1 ("may be present": the caller reads the table), one
//    bound for a filter the block does not have answers 0, as
//    FilterBlockReader::IsKeyExists does (src/filter_block.cpp:174).
//  * One mutex per cache: put/remove/probe are serialised, and a probe holds
//    it until its kernel is done, so no block is evicted under a running probe.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <list>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "bloom_common.hpp"

namespace {

constexpr uint64_t kAlign = 256;
constexpr uint64_t kOnesBytes = 16;  // an all-ones 16-byte filter: every probe hits

int32_t load32(const uint8_t *p) {
  int32_t v;
  memcpy(&v, p, 4);
  return v;
}

// FilterBlockReader::Init's trailer walk (src/filter_block.cpp:113-155):
// bitmaps region [0, offsets_start), filter f = [off_f, off_{f+1} or offsets_start).
int parse_block(const uint8_t *b, uint64_t len, int32_t want_bpk, std::vector<uint64_t> &off) {
  if (len < 4 || len > 0x7fffffffull) return ADL_FILTER_BLOCK_ERROR;
  const int64_t info_len_offset = (int64_t)len - 4;
  const int32_t info_len = load32(b + info_len_offset);
  if (info_len <= 0 || info_len > info_len_offset) return ADL_FILTER_BLOCK_ERROR;
  const int64_t info_offset = info_len_offset - info_len;
  // CreateFilterAlgorithm (:158-170): "bf" and bits_per_key at info[3]
  if (info_len < 7 || b[info_offset] != 'b' || b[info_offset + 1] != 'f') return ADL_FILTER_BLOCK_ERROR;
  const int32_t bpk = load32(b + info_offset + 3);
  if (bpk != want_bpk) return ADL_ERR_INVALID_ARG;  // one k per cache
  if (info_offset < 4) return ADL_FILTER_BLOCK_ERROR;
  const int64_t nums_offset = info_offset - 4;
  const int32_t nf = load32(b + nums_offset);
  if (nums_offset < 4) return ADL_FILTER_BLOCK_ERROR;
  const int32_t offsets_start = load32(b + nums_offset - 4);
  if (offsets_start < 0 || nf < 0) return ADL_FILTER_BLOCK_ERROR;
  if ((int64_t)offsets_start + 4ll * (nf ? nf : 1) > nums_offset) return ADL_FILTER_BLOCK_ERROR;
  if (load32(b + offsets_start) != 0) return ADL_FILTER_BLOCK_ERROR;
  off.assign((size_t)nf + 1, 0);
  for (int32_t f = 0; f < nf; ++f) {
    const int32_t o = load32(b + offsets_start + 4ll * f);
    if (o < 0 || o > offsets_start || (f && (uint64_t)o < off[f - 1])) return ADL_FILTER_BLOCK_ERROR;
    off[f] = (uint64_t)o;
  }
  off[nf] = (uint64_t)offsets_start;
  return ADL_OK;
}

}  // namespace

struct adl_bloom_filter_cache {
  struct Entry {
    std::string oid;
    uint64_t base = 0, size = 0;  // arena range [base, base + size)
    std::vector<uint64_t> off;    // block-relative filter offsets (F+1)
  };
  std::mutex mu;
  uint8_t *arena = nullptr;  // [ones][blocks...]
  uint64_t capacity = 0, used = 0;
  uint32_t max_tables = 0;
  int32_t bpk = 0;
  std::list<Entry> lru;  // front = most recently used
  std::unordered_map<std::string, std::list<Entry>::iterator> index;
  std::map<uint64_t, uint64_t> free_;  // offset -> size, coalesced

  bool alloc(uint64_t size, uint64_t &at) {
    for (auto it = free_.begin(); it != free_.end(); ++it) {
      if (it->second < size) continue;
      at = it->first;
      const uint64_t rest = it->second - size;
      free_.erase(it);
      if (rest) free_[at + size] = rest;
      used += size;
      return true;
    }
    return false;
  }
  void release(uint64_t at, uint64_t size) {
    used -= size;
    auto it = free_.emplace(at, size).first;
    auto nx = std::next(it);
    if (nx != free_.end() && it->first + it->second == nx->first) {
      it->second += nx->second;
      free_.erase(nx);
    }
    if (it != free_.begin()) {
      auto pv = std::prev(it);
      if (pv->first + pv->second == it->first) {
        pv->second += it->second;
        free_.erase(it);
      }
    }
  }
  void evict_back() {
    Entry &e = lru.back();
    release(e.base, e.size);
    index.erase(e.oid);
    lru.pop_back();
  }
};

extern "C" {

int adl_bloom_filter_cache_create(uint64_t capacity_bytes, uint32_t max_tables, int32_t bits_per_key,
                                  adl_bloom_filter_cache **out) {
  if (!out || bits_per_key < 0 || max_tables == 0 || capacity_bytes == 0) return ADL_ERR_INVALID_ARG;
  *out = nullptr;
  try {
    auto *c = new adl_bloom_filter_cache;
    c->capacity = adl_host::round_up(capacity_bytes, kAlign);
    c->max_tables = max_tables;
    c->bpk = bits_per_key;
    if (hipMalloc((void **)&c->arena, c->capacity + kAlign) != hipSuccess) {
      delete c;
      return ADL_ERR_OUT_OF_MEMORY;
    }
    if (hipMemset(c->arena, 0xff, kOnesBytes) != hipSuccess) {
      (void)hipFree(c->arena);
      delete c;
      return ADL_ERR_DEVICE;
    }
    c->free_[kAlign] = c->capacity;  // blocks after the all-ones filter
    *out = c;
    return ADL_OK;
  } catch (...) {
    return ADL_ERR_OUT_OF_MEMORY;
  }
}

int adl_bloom_filter_cache_destroy(adl_bloom_filter_cache *c) {
  if (!c) return ADL_OK;
  (void)hipFree(c->arena);
  delete c;
  return ADL_OK;
}

int adl_bloom_filter_cache_put(adl_bloom_filter_cache *c, const char *oid, uint64_t oid_len,
                               const uint8_t *h_block, uint64_t block_len) {
  if (!c || !oid || !h_block) return ADL_ERR_INVALID_ARG;
  try {
    std::vector<uint64_t> off;
    if (int rc = parse_block(h_block, block_len, c->bpk, off)) return rc;
    const uint64_t bytes = off.back();  // the bitmap region
    const uint64_t size = adl_host::round_up(bytes + 1, kAlign);
    std::lock_guard<std::mutex> g(c->mu);
    if (size > c->capacity) return ADL_ERR_OUT_OF_MEMORY;
    const std::string key(oid, oid_len);
    if (auto it = c->index.find(key); it != c->index.end()) {  // replace, as LRUCache::Put does
      c->release(it->second->base, it->second->size);
      c->lru.erase(it->second);
      c->index.erase(it);
    }
    while (c->lru.size() >= c->max_tables) c->evict_back();
    uint64_t at = 0;
    while (!c->alloc(size, at)) {
      if (c->lru.empty()) return ADL_ERR_OUT_OF_MEMORY;  // fragmentation: cannot happen once empty
      c->evict_back();
    }
    if (bytes && hipMemcpy(c->arena + at, h_block, bytes, hipMemcpyHostToDevice) != hipSuccess) {
      c->release(at, size);
      return ADL_ERR_DEVICE;
    }
    c->lru.push_front(adl_bloom_filter_cache::Entry{key, at, size, std::move(off)});
    c->index[key] = c->lru.begin();
    return ADL_OK;
  } catch (...) {
    return ADL_ERR_OUT_OF_MEMORY;
  }
}

int adl_bloom_filter_cache_contains(adl_bloom_filter_cache *c, const char *oid, uint64_t oid_len) {
  if (!c || !oid) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  auto it = c->index.find(std::string(oid, oid_len));
  if (it == c->index.end()) return 0;
  c->lru.splice(c->lru.begin(), c->lru, it->second);  // LRUCache::Get marks it used
  return 1;
}

int adl_bloom_filter_cache_remove(adl_bloom_filter_cache *c, const char *oid, uint64_t oid_len) {
  if (!c || !oid) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  auto it = c->index.find(std::string(oid, oid_len));
  if (it == c->index.end()) return 0;
  c->release(it->second->base, it->second->size);
  c->lru.erase(it->second);
  c->index.erase(it);
  return 1;
}

int adl_bloom_filter_cache_stats(adl_bloom_filter_cache *c, uint32_t *tables, uint64_t *bytes_used) {
  if (!c) return ADL_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (tables) *tables = (uint32_t)c->lru.size();
  if (bytes_used) *bytes_used = c->used;
  return ADL_OK;
}

int adl_bloom_filter_cache_probe(adl_bloom_filter_cache *c, const char *const *oids, const uint64_t *oid_lens,
                                 uint32_t num_tables, uint32_t filter, const uint8_t *h_keys,
                                 const uint64_t *h_offsets, uint64_t n, uint32_t key_stride,
                                 const uint32_t *h_table, uint8_t *h_out, uint64_t *h_uncached, void *stream) {
  if (!c || (num_tables && (!oids || !oid_lens))) return ADL_ERR_INVALID_ARG;
  if (h_uncached) *h_uncached = 0;
  if (n == 0) return ADL_OK;
  if (!h_keys || !h_table || !h_out || (!h_offsets && key_stride == 0)) return ADL_ERR_INVALID_ARG;
  try {
    hipStream_t st = (hipStream_t)stream;
    std::lock_guard<std::mutex> g(c->mu);
    // per listed table: the arena range of its filter `filter` (the all-ones
    // filter when the table is not cached, an empty range when it has no
    // such filter)
    std::vector<uint64_t> be(2 * (size_t)num_tables);
    std::vector<uint8_t> cached(num_tables);
    for (uint32_t j = 0; j < num_tables; ++j) {
      auto it = c->index.find(std::string(oids[j], oid_lens[j]));
      if (it == c->index.end()) {
        be[j] = 0;
        be[num_tables + j] = kOnesBytes;
        continue;
      }
      cached[j] = 1;
      c->lru.splice(c->lru.begin(), c->lru, it->second);
      const adl_bloom_filter_cache::Entry &e = *it->second;
      const uint64_t nf = e.off.size() - 1;
      be[j] = be[num_tables + j] = e.base;
      if (filter < nf) {
        be[j] = e.base + e.off[filter];
        be[num_tables + j] = e.base + e.off[filter + 1];
      }
    }
    uint64_t uncached = 0;
    for (uint64_t i = 0; i < n; ++i) {
      if (h_table[i] >= num_tables) return ADL_ERR_INVALID_ARG;
      uncached += !cached[h_table[i]];
    }
    // stage keys, offsets, table ids and the range table in one H2D
    const uint64_t key_bytes = h_offsets ? h_offsets[n] : n * (uint64_t)key_stride;
    const uint64_t off_bytes = h_offsets ? (n + 1) * 8 : 0;
    const uint64_t o_offs = adl_host::round_up(key_bytes + 16, 256);
    const uint64_t o_fid = o_offs + adl_host::round_up(off_bytes, 256);
    const uint64_t o_be = o_fid + adl_host::round_up(n * 4, 256);
    const uint64_t o_out = o_be + adl_host::round_up(be.size() * 8, 256);
    const uint64_t total = o_out + adl_host::round_up(n, 256);
    adl_host::Staging &sg = adl_host::t_stage;
    if (int rc = sg.reserve(o_out, total)) return rc;
    if (key_bytes) memcpy(sg.host, h_keys, key_bytes);
    if (off_bytes) memcpy(sg.host + o_offs, h_offsets, off_bytes);
    memcpy(sg.host + o_fid, h_table, n * 4);
    memcpy(sg.host + o_be, be.data(), be.size() * 8);
    if (hipMemcpyAsync(sg.dev, sg.host, o_out, hipMemcpyHostToDevice, st) != hipSuccess) return ADL_ERR_DEVICE;
    const uint64_t *d_be = reinterpret_cast<const uint64_t *>(sg.dev + o_be);
    int rc = adl_bloom_probe_ranges_device(sg.dev, h_offsets ? reinterpret_cast<uint64_t *>(sg.dev + o_offs) : nullptr,
                                           n, key_stride, reinterpret_cast<const uint32_t *>(sg.dev + o_fid),
                                           num_tables, c->arena, d_be, d_be + num_tables, c->bpk, sg.dev + o_out,
                                           stream);
    if (rc) {
      (void)hipStreamSynchronize(st);
      return rc;
    }
    if (hipMemcpyAsync(sg.host, sg.dev + o_out, n, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return ADL_ERR_DEVICE;
    memcpy(h_out, sg.host, n);
    if (h_uncached) *h_uncached = uncached;
    return ADL_OK;
  } catch (...) {
    return ADL_ERR_OUT_OF_MEMORY;
  }
}

}  // extern "C"
