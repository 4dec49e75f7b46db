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
//  * Concurrency: one mutex per cache guards the index, the LRU list and the
//    arena's free list, and is held only for that bookkeeping -- never across
//    a copy or a kernel.  A probe pins the entries it resolved (a count per
//    entry) before it lets go of the lock; an entry evicted, replaced or
//    removed while pinned leaves the index at once but keeps its arena range
//    until the last probe using it unpins it.  A put reserves its range under
//    the lock, uploads without it, and publishes under it again; a put that
//    finds no room while pinned or uploading blocks hold the arena waits for
//    them (condition variable) instead of failing.  So probes never wait for
//    each other, and readers, like the reference's (src/db.cpp:166-172), take
//    no lock for the duration of a lookup.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <stdint.h>
#include <string.h>

#include <condition_variable>
#include <list>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "bloom_common.hpp"
#include "filter_block_format.hpp"
#include "probe_server.hpp"

namespace {

constexpr uint64_t kAlign = 256;
constexpr uint64_t kOnesBytes = 16;  // an all-ones 16-byte filter: every probe hits
constexpr int64_t kServerBackoffNs = 1000000000;  // launched probes for 1 s after a starved server request

// FilterBlockReader::Init's trailer walk (src/filter_block.cpp:113-155, in
// filter_block_format.hpp): bitmaps region [0, offsets_start), filter f =
// [off_f, off_{f+1} or offsets_start).  Each block carries its own
// bits_per_key in its "bf:" info, and the reference builds its BloomFilter
// from it per block (CreateFilterAlgorithm, src/filter_block.cpp:158-170),
// so a level may mix tables written under different DBOptions::bits_per_key
// (src/options.hpp:24): the block's k is kept with its entry.
int parse_block(const uint8_t *b, uint64_t len, std::vector<uint64_t> &off, uint8_t &k) {
  adl_fmt::FilterBlockLayout lay;
  if (adl_fmt::parse_filter_block(b, len, lay)) return ADL_FILTER_BLOCK_ERROR;
  off = std::move(lay.off);
  k = (uint8_t)adl_host::num_probes(lay.bits_per_key);
  return ADL_OK;
}

// The calling thread's completion event of a mapped small-batch probe (timing
// off: it is only queried).
struct DoneEvent {
  hipEvent_t e = nullptr;
  bool tried = false;
  ~DoneEvent() {
    if (e) (void)hipEventDestroy(e);
  }
  hipEvent_t get() {
    if (!tried) {
      tried = true;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
    }
    return e;
  }
};
thread_local DoneEvent t_done;

}  // namespace

struct adl_bloom_filter_cache {
  enum State : uint8_t { kLive, kLoading, kDead };
  struct Entry {
    std::string oid;
    uint64_t base = 0, size = 0;  // arena range [base, base + size)
    std::vector<uint64_t> off;    // block-relative filter offsets (F+1)
    uint8_t k = 1;                // probes per key: from the block's own bits_per_key
    uint32_t pins = 0;            // probes (or the uploading put) using the range
    State state = kLive;
  };
  using Iter = std::list<Entry>::iterator;
  std::mutex mu;
  std::condition_variable freed;  // a dead or loading entry gave back its range
  uint8_t *arena = nullptr;       // [ones][blocks...]
  uint64_t capacity = 0, used = 0;
  uint32_t max_tables = 0;
  std::list<Entry> lru;      // live entries, front = most recently used
  std::list<Entry> limbo;    // loading (pinned by their put) and dead (pinned by probes)
  std::unordered_map<std::string, Iter> index;  // live entries only
  std::map<uint64_t, uint64_t> free_;           // offset -> size, coalesced
  // the resident probe server of this cache's small batches (created on the
  // first one; srv_tried: do not retry a failed creation)
  adl_srv::Server *srv = nullptr;
  bool srv_tried = false;
  // after a kBusy (the server's wave found no room on the GPU for
  // adl_srv::kTimeout), small batches go straight to a launch until this
  // steady-clock time (ns), instead of each waiting out the timeout again
  std::atomic<int64_t> srv_backoff_until{0};
  // published puts so far (the server invalidates its caches before it reads
  // bits of a range that may have been written since it last did)
  std::atomic<uint64_t> epoch{1};

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
  // Take a live entry out of the index: its range is freed now, or -- while
  // probes hold it -- by the last of them (unpin).
  void retire(Iter it) {
    index.erase(it->oid);
    if (it->pins == 0) {
      release(it->base, it->size);
      lru.erase(it);
      freed.notify_all();
    } else {
      it->state = kDead;
      limbo.splice(limbo.end(), lru, it);
    }
  }
  void unpin(Iter it) {
    if (--it->pins == 0 && it->state == kDead) {
      release(it->base, it->size);
      limbo.erase(it);
      freed.notify_all();
    }
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
    if (hipMalloc((void **)&c->arena, c->capacity + kAlign) != hipSuccess) {
      (void)hipGetLastError();
      delete c;
      return ADL_ERR_OUT_OF_MEMORY;
    }
    hipStream_t st = adl_host::sync_stream(nullptr);
    if (hipMemsetAsync(c->arena, 0xff, kOnesBytes, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
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

// No call on the cache may be running or start once this is called.
int adl_bloom_filter_cache_destroy(adl_bloom_filter_cache *c) {
  if (!c) return ADL_OK;
  adl_srv::destroy(c->srv);  // stops its kernel before the arena goes
  (void)hipFree(c->arena);
  delete c;
  return ADL_OK;
}

int adl_bloom_filter_cache_put(adl_bloom_filter_cache *c, const char *oid, uint64_t oid_len,
                               const uint8_t *h_block, uint64_t block_len) {
  if (!c || !oid || !h_block) return ADL_ERR_INVALID_ARG;
  try {
    std::vector<uint64_t> off;
    uint8_t k = 1;
    if (int rc = parse_block(h_block, block_len, off, k)) return rc;
    const uint64_t bytes = off.back();  // the bitmap region
    const uint64_t size = adl_host::round_up(bytes + 1, kAlign);
    const std::string key(oid, oid_len);
    adl_bloom_filter_cache::Iter mine;
    {
      std::unique_lock<std::mutex> g(c->mu);
      if (size > c->capacity) return ADL_ERR_OUT_OF_MEMORY;
      // 1. room: the table count (LRUCache's maxSize) and the arena bytes.  A
      //    block being replaced (LRUCache::Put of a cached key) stays visible to
      //    probes until the new one is published.
      const size_t replacing = c->index.count(key);
      while (c->lru.size() - replacing >= c->max_tables) c->retire(std::prev(c->lru.end()));
      uint64_t at = 0;
      while (!c->alloc(size, at)) {
        if (!c->lru.empty()) {
          c->retire(std::prev(c->lru.end()));
        } else if (!c->limbo.empty()) {
          c->freed.wait(g);  // pinned or uploading blocks hold the rest of the arena
        } else {
          return ADL_ERR_OUT_OF_MEMORY;  // cannot happen: an empty arena fits any size <= capacity
        }
      }
      // 2. reserve the range, pinned by this put while it uploads
      adl_bloom_filter_cache::Entry e;
      e.oid = key;
      e.base = at;
      e.size = size;
      e.off = std::move(off);
      e.k = k;
      e.pins = 1;
      e.state = adl_bloom_filter_cache::kLoading;
      mine = c->limbo.insert(c->limbo.end(), std::move(e));
    }
    // 3. upload without the lock
    hipStream_t st = adl_host::sync_stream(nullptr);
    const bool ok = !bytes || (hipMemcpyAsync(c->arena + mine->base, h_block, bytes, hipMemcpyHostToDevice, st) ==
                                   hipSuccess &&
                               hipStreamSynchronize(st) == hipSuccess);
    // 4. publish as most recently used (or give the range back)
    std::lock_guard<std::mutex> g(c->mu);
    if (!ok) {
      mine->state = adl_bloom_filter_cache::kDead;
      c->unpin(mine);
      return ADL_ERR_DEVICE;
    }
    if (auto it = c->index.find(key); it != c->index.end()) c->retire(it->second);  // the block this one replaces
    mine->pins = 0;
    mine->state = adl_bloom_filter_cache::kLive;
    c->lru.splice(c->lru.begin(), c->limbo, mine);
    c->index[key] = c->lru.begin();
    c->epoch.fetch_add(1, std::memory_order_release);  // (under the lock: before any probe can resolve it)
    while (c->lru.size() > c->max_tables) c->retire(std::prev(c->lru.end()));
    c->freed.notify_all();  // a put waiting for room may evict this entry now
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
  c->retire(it->second);
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
    for (uint64_t i = 0; i < n; ++i)
      if (h_table[i] >= num_tables) return ADL_ERR_INVALID_ARG;
    hipStream_t st = adl_host::sync_stream(stream);
    // 1. under the lock: per listed table, the arena range of its filter
    //    `filter` (the all-ones filter when the table is not cached, an empty
    //    range when it has no such filter) and its block's k, its entry pinned
    //    and marked used
    // (per-thread scratch: a single-key Get allocates nothing here)
    thread_local std::vector<uint64_t> be;
    thread_local std::vector<uint8_t> cached, kt;
    thread_local std::vector<adl_bloom_filter_cache::Iter> pinned;
    thread_local std::string oid_key;
    be.assign(2 * (size_t)num_tables, 0);
    cached.assign(num_tables, 0);
    kt.assign(num_tables, 1);
    pinned.clear();
    {
      std::lock_guard<std::mutex> g(c->mu);
      for (uint32_t j = 0; j < num_tables; ++j) {
        oid_key.assign(oids[j], oid_lens[j]);
        auto it = c->index.find(oid_key);
        if (it == c->index.end()) {
          be[j] = 0;
          be[num_tables + j] = kOnesBytes;
          continue;
        }
        cached[j] = 1;
        adl_bloom_filter_cache::Iter e = it->second;
        kt[j] = e->k;
        c->lru.splice(c->lru.begin(), c->lru, e);
        ++e->pins;
        pinned.push_back(e);
        const uint64_t nf = e->off.size() - 1;
        be[j] = be[num_tables + j] = e->base;
        if (filter < nf) {
          be[j] = e->base + e->off[filter];
          be[num_tables + j] = e->base + e->off[filter + 1];
        }
      }
    }
    auto unpin_all = [&] {
      std::lock_guard<std::mutex> g(c->mu);
      for (auto e : pinned) c->unpin(e);
    };
    uint64_t uncached = 0;
    for (uint64_t i = 0; i < n; ++i) uncached += !cached[h_table[i]];
    // A single-key Get (up to adl_srv::kMaxQ queries): the resident server,
    // no launch.  Its answers arrive after all its reads of the pinned ranges.
    {
      const uint64_t kbytes = h_offsets ? h_offsets[n] - h_offsets[0] : n * (uint64_t)key_stride;
      adl_srv::Server *srv = nullptr;
      const int64_t now_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
                                 std::chrono::steady_clock::now().time_since_epoch())
                                 .count();
      if (adl_srv::eligible(n, kbytes) && adl_host::knobs().probe_server &&
          now_ns >= c->srv_backoff_until.load(std::memory_order_relaxed)) {
        std::lock_guard<std::mutex> g(c->mu);
        if (!c->srv_tried) {
          c->srv_tried = true;
          c->srv = adl_srv::create();
        }
        srv = c->srv;
      }
      if (srv) {
        uint64_t rng[2 * adl_srv::kMaxQ];
        uint8_t kq[adl_srv::kMaxQ];
        const uint64_t a0 = reinterpret_cast<uint64_t>(c->arena);
        for (uint64_t i = 0; i < n; ++i) {
          rng[2 * i] = a0 + be[h_table[i]];
          rng[2 * i + 1] = a0 + be[num_tables + h_table[i]];
          kq[i] = kt[h_table[i]];
        }
        int rc = adl_srv::probe(srv, h_keys, h_offsets, key_stride, n, rng, kq,
                                c->epoch.load(std::memory_order_acquire), h_out);
        if (rc == ADL_OK && adl_host::g_test_faults.take(ADL_TEST_FAULT_CACHE_COMPLETION) >= 0) rc = ADL_ERR_DEVICE;
        // kBusy: no answer in adl_srv::kTimeout (a healthy GPU with no room for
        // the server's wave): probe by a launch below, the ranges still pinned
        if (rc != adl_srv::kBusy) {
          unpin_all();
          if (rc) return rc;
          if (h_uncached) *h_uncached = uncached;
          return ADL_OK;
        }
        c->srv_backoff_until.store(now_ns + kServerBackoffNs, std::memory_order_relaxed);
      }
    }
    // 2. without the lock: stage keys, offsets, table ids and the range table
    //    and the range and k tables in one H2D, one probe launch, one D2H
    const uint64_t key_bytes = h_offsets ? h_offsets[n] : n * (uint64_t)key_stride;
    const uint64_t off_bytes = h_offsets ? (n + 1) * 8 : 0;
    const uint64_t o_offs = adl_host::round_up(key_bytes + 16, 256);
    const uint64_t o_fid = o_offs + adl_host::round_up(off_bytes, 256);
    const uint64_t o_be = o_fid + adl_host::round_up(n * 4, 256);
    const uint64_t o_k = o_be + adl_host::round_up(be.size() * 8, 256);
    const uint64_t o_out = o_k + adl_host::round_up(num_tables, 256);
    const uint64_t total = o_out + adl_host::round_up(n, 256);
    // A small batch (a single-key Get) is handed over in the thread's mapped
    // buffer: the kernel reads it and writes its answers there directly.
    adl_host::Staging &sg = adl_host::t_stage;
    uint8_t *hbuf = adl_host::t_mapped.get(total), *dbuf = hbuf ? adl_host::t_mapped.dev : nullptr;
    int rc = ADL_OK;
    if (!hbuf) {
      rc = sg.reserve(total, total);
      hbuf = sg.host;
      dbuf = sg.dev;
    }
    // A mapped small batch is waited for by watching its answers arrive (each
    // is written once, 0 or 1, over a 0xFF sentinel, by bloom_probe_multi_kernel's
    // one store per query after all its reads) instead of a stream
    // synchronize.  The pinned ranges are released only once the launch's
    // completion event has fired too, so a fault after the answers landed is
    // still this call's error.  Both waits fall back to the synchronize after
    // 2 ms (or with ADL_BLOOM_SPIN=0).
    const bool spin = hbuf != sg.host && n <= 4096 && adl_host::knobs().spin;
    if (rc == ADL_OK) {
      if (key_bytes) memcpy(hbuf, h_keys, key_bytes);
      if (off_bytes) memcpy(hbuf + o_offs, h_offsets, off_bytes);
      memcpy(hbuf + o_fid, h_table, n * 4);
      memcpy(hbuf + o_be, be.data(), be.size() * 8);
      if (num_tables) memcpy(hbuf + o_k, kt.data(), num_tables);
      if (spin) memset(hbuf + o_out, 0xff, n);
      if (hbuf == sg.host && hipMemcpyAsync(dbuf, hbuf, o_out, hipMemcpyHostToDevice, st) != hipSuccess)
        rc = ADL_ERR_DEVICE;
    }
    // a watched batch's completion event rides on the probe's dispatch packet
    hipEvent_t done = spin && rc == ADL_OK ? t_done.get() : nullptr;
    if (rc == ADL_OK) {
      const uint64_t *d_be = reinterpret_cast<const uint64_t *>(dbuf + o_be);
      rc = adl_host::adl_probe_ranges_device_ev(dbuf, h_offsets ? reinterpret_cast<uint64_t *>(dbuf + o_offs) : nullptr, n,
                                      key_stride, reinterpret_cast<const uint32_t *>(dbuf + o_fid), num_tables,
                                      c->arena, d_be, d_be + num_tables, dbuf + o_k, dbuf + o_out, st, done);
    }
    if (rc == ADL_OK && hbuf == sg.host &&
        hipMemcpyAsync(hbuf + o_out, dbuf + o_out, n, hipMemcpyDeviceToHost, st) != hipSuccess)
      rc = ADL_ERR_DEVICE;
    // the kernel and the copies are done before any pinned range can be reused
    bool finished = false;
    if (done) {
      const volatile uint8_t *ans = hbuf + o_out;
      const auto t0 = std::chrono::steady_clock::now();
      auto late = [&] { return std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2); };
      uint64_t i = 0;
      for (;;) {
        while (i < n && ans[i] != 0xff) ++i;
        if (i == n || late()) break;
        __builtin_ia32_pause();
      }
      if (i == n) {  // every answer is in: now the launch itself
        const bool fault = adl_host::g_test_faults.take(ADL_TEST_FAULT_CACHE_COMPLETION) >= 0;
        for (;;) {
          const hipError_t q = fault ? hipErrorLaunchFailure : hipEventQuery(done);
          if (q == hipSuccess) {
            finished = true;
            break;
          }
          if (q != hipErrorNotReady) {
            rc = ADL_ERR_DEVICE;
            break;
          }
          if (late()) break;
          __builtin_ia32_pause();
        }
      }
    }
    if (!finished && hipStreamSynchronize(st) != hipSuccess && rc == ADL_OK) rc = ADL_ERR_DEVICE;
    // 3. unpin (a range retired meanwhile is freed by its last unpin)
    unpin_all();
    if (rc) return rc;
    memcpy(h_out, hbuf + o_out, n);
    if (h_uncached) *h_uncached = uncached;
    return ADL_OK;
  } catch (...) {
    return ADL_ERR_OUT_OF_MEMORY;
  }
}

}  // extern "C"
