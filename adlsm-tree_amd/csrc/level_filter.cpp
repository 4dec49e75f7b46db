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

RC LevelMultiGetFilter(FilterCache &cache, const vector<TableRange> &tables, const vector<string_view> &user_keys,
                       int64_t seq, MultiGetFilterResult &out) {
  out = MultiGetFilterResult{};
  out.begin.assign(user_keys.size() + 1, 0);
  // files_meta_ order (ascending min_inner_key), visited in reverse
  vector<uint32_t> visit(tables.size());
  std::iota(visit.begin(), visit.end(), 0u);
  std::stable_sort(visit.begin(), visit.end(), [&](uint32_t a, uint32_t b) {
    return InnerKeyLess(tables[a].min_inner_key, tables[b].min_inner_key);
  });
  std::reverse(visit.begin(), visit.end());
  // the ranges decoded once (the inner keys outlive this call)
  vector<Decoded> mn(tables.size()), mx(tables.size());
  for (size_t t = 0; t < tables.size(); ++t) {
    mn[t] = Decode(tables[t].min_inner_key);
    mx[t] = Decode(tables[t].max_inner_key);
  }
  // candidates of every key, and the probe batch: pair p = (key, table)
  KeyArena batch;
  for (size_t i = 0; i < user_keys.size(); ++i) {
    const Decoded mk{user_keys[i], seq, 0 /* OP_PUT */};
    for (uint32_t t : visit) {
      // TableCoversKey, on the decoded ranges
      if ((Less(mk, mn[t]) && mk.user != mn[t].user) || Less(mx[t], mk)) continue;
      out.table.push_back(t);
      batch.Add(user_keys[i]);  // SSTableReader::Get probes the user key (src/sstable.cpp:238)
    }
    out.begin[i + 1] = (uint32_t)out.table.size();
  }
  vector<string_view> oids(tables.size());
  for (size_t t = 0; t < tables.size(); ++t) oids[t] = tables[t].oid;
  return cache.Probe(oids, out.table, batch, 0, out.maybe, &out.uncached);
}

}  // namespace adl
