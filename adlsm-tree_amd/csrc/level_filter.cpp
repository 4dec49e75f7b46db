// adlsm-tree_amd/csrc/level_filter.cpp -- Level::Get's filter stage, batched
// (see level_filter.hpp).
#include "level_filter.hpp"

#include <string.h>

#include <algorithm>
#include <numeric>

namespace adl {

namespace {

/* An inner key decoded as MemKey::FromKey does (src/keys.cpp:86-91); keys
 * shorter than the 9-byte suffix compare as (whole key, seq 0, op 0). */
struct Decoded {
  string_view user;
  int64_t seq = 0;
  int op = 0;
};

Decoded Decode(string_view k) {
  Decoded d;
  if (k.size() < 9) {
    d.user = k;
    return d;
  }
  d.user = k.substr(0, k.size() - 9);
  memcpy(&d.seq, k.data() + k.size() - 9, 8);
  d.op = (unsigned char)k[k.size() - 1];
  return d;
}

/* MemKey::operator< (src/keys.cpp:61-74) */
bool Less(const Decoded &a, const Decoded &b) {
  const int cmp = a.user.compare(b.user);
  if (cmp < 0) return true;
  if (cmp == 0) {
    if (a.seq > b.seq) return true;
    if (a.seq == b.seq && a.op > b.op) return true;
  }
  return false;
}

}  // namespace

bool InnerKeyLess(string_view a, string_view b) { return Less(Decode(a), Decode(b)); }

bool LookupLess(string_view user_key, int64_t seq, string_view inner_key) {
  return Less(Decoded{user_key, seq, 0 /* OP_PUT */}, Decode(inner_key));
}

bool InnerLessLookup(string_view inner_key, string_view user_key, int64_t seq) {
  return Less(Decode(inner_key), Decoded{user_key, seq, 0});
}

/* src/revision.cpp:281-287:
 *   if ((mk < min_inner_key && mk.user_key_ != min_inner_key.user_key_) ||
 *       max_inner_key < mk) continue; */
bool TableCoversKey(const TableRange &t, string_view user_key, int64_t seq) {
  const Decoded mn = Decode(t.min_inner_key);
  if (LookupLess(user_key, seq, t.min_inner_key) && user_key != mn.user) return false;
  if (InnerLessLookup(t.max_inner_key, user_key, seq)) return false;
  return true;
}

void LevelCandidates(const vector<TableRange> &tables, const vector<string_view> &user_keys, int64_t seq,
                     vector<uint32_t> &begin, vector<uint32_t> &table) {
  const size_t K = user_keys.size(), T = tables.size();
  begin.assign(K + 1, 0);
  table.clear();
  // files_meta_ order (ascending min_inner_key, stable), visited in reverse
  vector<uint32_t> asc(T);
  std::iota(asc.begin(), asc.end(), 0u);
  std::stable_sort(asc.begin(), asc.end(), [&](uint32_t a, uint32_t b) {
    return InnerKeyLess(tables[a].min_inner_key, tables[b].min_inner_key);
  });
  // the ranges decoded once (the inner keys outlive this call)
  vector<Decoded> mn(T), mx(T);
  for (size_t t = 0; t < T; ++t) {
    mn[t] = Decode(tables[t].min_inner_key);
    mx[t] = Decode(tables[t].max_inner_key);
  }
  // Table t is a candidate for lookup mk (src/revision.cpp:281-287) iff
  //   mn[t].user <= mk.user  (not "mk < mn and the user keys differ") and
  //   !(mx[t] < mk).
  // Sweep the lookups in MemKey order: a table enters when the sweep reaches
  // its min user key -- in ascending min order, at the front of the active
  // list, which so stays in Level::Get's visiting order -- and leaves for good
  // once its max is below the lookup.  Each lookup then reads its candidates
  // off the active list: O((K + T) log(K + T) + candidates) instead of K * T
  // range tests.
  vector<uint32_t> order(K);
  std::iota(order.begin(), order.end(), 0u);
  std::stable_sort(order.begin(), order.end(),
                   [&](uint32_t a, uint32_t b) { return user_keys[a].compare(user_keys[b]) < 0; });
  constexpr uint32_t kNil = ~0u;
  vector<uint32_t> nxt(T, kNil), prv(T, kNil);
  uint32_t head = kNil;
  auto unlink = [&](uint32_t t) {
    if (prv[t] != kNil) nxt[prv[t]] = nxt[t];
    else head = nxt[t];
    if (nxt[t] != kNil) prv[nxt[t]] = prv[t];
  };
  auto mx_after = [&](uint32_t a, uint32_t b) { return Less(mx[b], mx[a]); };  // min-heap on mx
  vector<uint32_t> heap;
  vector<uint32_t> cbeg(K + 1, 0), cand;  // candidates by sorted lookup
  size_t ins = 0;
  for (size_t r = 0; r < K; ++r) {
    const Decoded mk{user_keys[order[r]], seq, 0 /* OP_PUT */};
    for (; ins < T && mn[asc[ins]].user.compare(mk.user) <= 0; ++ins) {
      const uint32_t t = asc[ins];
      nxt[t] = head;
      prv[t] = kNil;
      if (head != kNil) prv[head] = t;
      head = t;
      heap.push_back(t);
      std::push_heap(heap.begin(), heap.end(), mx_after);
    }
    while (!heap.empty() && Less(mx[heap.front()], mk)) {
      unlink(heap.front());
      std::pop_heap(heap.begin(), heap.end(), mx_after);
      heap.pop_back();
    }
    for (uint32_t t = head; t != kNil; t = nxt[t]) cand.push_back(t);
    cbeg[r + 1] = (uint32_t)cand.size();
  }
  // back to the caller's key order
  vector<uint32_t> rank(K);
  for (size_t r = 0; r < K; ++r) rank[order[r]] = (uint32_t)r;
  table.reserve(cand.size());
  for (size_t i = 0; i < K; ++i) {
    const uint32_t r = rank[i];
    table.insert(table.end(), cand.begin() + cbeg[r], cand.begin() + cbeg[r + 1]);
    begin[i + 1] = (uint32_t)table.size();
  }
}

RC LevelMultiGetFilter(FilterCache &cache, const vector<TableRange> &tables, const vector<string_view> &user_keys,
                       int64_t seq, MultiGetFilterResult &out) {
  out = MultiGetFilterResult{};
  LevelCandidates(tables, user_keys, seq, out.begin, out.table);
  // the probe batch: pair p = (key, table); SSTableReader::Get probes the user
  // key (src/sstable.cpp:238)
  KeyArena batch;
  for (size_t i = 0; i < user_keys.size(); ++i)
    for (uint32_t c = out.begin[i]; c < out.begin[i + 1]; ++c) batch.Add(user_keys[i]);
  const size_t T = tables.size();
  vector<string_view> oids(T);
  for (size_t t = 0; t < T; ++t) oids[t] = tables[t].oid;
  return cache.Probe(oids, out.table, batch, 0, out.maybe, &out.uncached);
}

}  // namespace adl

/* Test hook (tests/test_level_cpu.py): LevelCandidates over tables and keys
 * handed over as (pointer, length) arrays; begin: K+1 entries, table: up to
 * cap entries.  Returns the number of pairs, or -1 when cap is too small. */
extern "C" int64_t adl_level_candidates(const char *const *mins, const uint64_t *min_lens, const char *const *maxs,
                                        const uint64_t *max_lens, uint32_t T, const char *const *keys,
                                        const uint64_t *key_lens, uint32_t K, int64_t seq, uint32_t *begin,
                                        uint32_t *table, uint64_t cap) {
  std::vector<adl::TableRange> tabs(T);
  for (uint32_t t = 0; t < T; ++t) {
    tabs[t].min_inner_key.assign(mins[t], min_lens[t]);
    tabs[t].max_inner_key.assign(maxs[t], max_lens[t]);
  }
  std::vector<std::string_view> ks(K);
  for (uint32_t i = 0; i < K; ++i) ks[i] = std::string_view(keys[i], key_lens[i]);
  std::vector<uint32_t> b, tb;
  adl::LevelCandidates(tabs, ks, seq, b, tb);
  if (tb.size() > cap) return -1;
  std::copy(b.begin(), b.end(), begin);
  std::copy(tb.begin(), tb.end(), table);
  return (int64_t)tb.size();
}
