// adlsm-tree_amd/csrc/level_filter.hpp -- the filter stage of the reference's
// point-lookup path, batched: many lookups against every candidate SSTable of
// a level in ONE device launch.
//
// Reference path per key (src/db.cpp:164-197 -> Revision::Get ->
// Level::Get, src/revision.cpp:265-310): walk files_meta_ newest first, skip
// a table whose [min_inner_key, max_inner_key] range does not cover the
// lookup key (:279-287), open its reader from the table cache
// (DB::GetSSTableReader, src/db.cpp:340-364) and call SSTableReader::Get,
// whose first step is the bloom check FilterBlockReader::IsKeyExists(0,
// user_key) (src/sstable.cpp:238): NOT_FOUND without touching the index or
// data blocks when the filter says the key is absent.
//
// Here the same candidate tables are chosen for every key of a batch (same
// comparison, same visiting order), all (key, table) pairs go to the
// FilterCache in one probe launch, and the caller gets, per key, its
// candidates in Level::Get's order with the filter's answer for each -- the
// tables it still has to read.
#pragma once
#include <stdint.h>

#include <string>
#include <string_view>
#include <vector>

#include "filter_block.hpp"
#include "rc.hpp"

namespace adl {

using namespace std;

/* One SSTable of a level as Level::Get sees it: the oid it is cached under
 * (sha256 hex, src/revision.cpp:290) and FileMetaData's key range
 * (src/file_util.hpp:157-158), as inner keys: user_key + LE64 seq + op byte
 * (src/keys.cpp:76-84). */
struct TableRange {
  string oid;
  string min_inner_key;
  string max_inner_key;
};

/* inner key a < inner key b as MemKey::operator< on the decoded keys */
bool InnerKeyLess(string_view a, string_view b);
/* MemKey(user_key, seq, OP_PUT) < inner key k, as MemKey::operator<
 * (src/keys.cpp:61-74): user keys ascending, then seq descending, then op
 * descending. */
bool LookupLess(string_view user_key, int64_t seq, string_view inner_key);
/* inner key k < MemKey(user_key, seq, OP_PUT) */
bool InnerLessLookup(string_view inner_key, string_view user_key, int64_t seq);

/* Level::Get's range test (src/revision.cpp:281-287): true when the table
 * must be visited for (user_key, seq). */
bool TableCoversKey(const TableRange &t, string_view user_key, int64_t seq);

struct MultiGetFilterResult {
  vector<uint32_t> begin;  /* key i's candidates: [begin[i], begin[i+1]) */
  vector<uint32_t> table;  /* index into `tables`, in Level::Get's visiting order */
  vector<uint8_t> maybe;   /* the filter's answer; 0 = NOT_FOUND for that table */
  uint64_t uncached = 0;   /* pairs whose table was not in the cache (answered 1) */
};

/* tables: the level's SSTables, any order; they are visited as Level::Get
 * walks files_meta_ -- a set ordered by min_inner_key (FileMetaData::operator<,
 * src/file_util.hpp:163-165) iterated in reverse (src/revision.cpp:278).
 * user_keys: the batch; seq: the lookup's sequence (DB::Get reads
 * sequence_id_, src/db.cpp:168).  One cache probe for all pairs. */
/* The candidate selection of LevelMultiGetFilter alone (host only): key i's
 * candidate tables are table[begin[i] .. begin[i+1]), in visiting order. */
void LevelCandidates(const vector<TableRange> &tables, const vector<string_view> &user_keys, int64_t seq,
                     vector<uint32_t> &begin, vector<uint32_t> &table);

RC LevelMultiGetFilter(FilterCache &cache, const vector<TableRange> &tables, const vector<string_view> &user_keys,
                       int64_t seq, MultiGetFilterResult &out);

}  // namespace adl
