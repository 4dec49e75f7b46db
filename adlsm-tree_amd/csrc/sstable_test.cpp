// adlsm-tree_amd/csrc/sstable_test.cpp -- the memtables of the reference's
// test/sstable_test.cpp (BuildSSTable :9-27, BuildSSTable2 :29-43) flushed
// through the gfx950-backed SSTableWriter (sstable_writer.hpp).  Needs a GPU.
//
//   sstable_test <which 1|2> <dir>   writes <dir>/<oid>.sst, prints "<oid> <bytes>"
//   sstable_test batch <which> <dir> the same through AddBatch (packed run)
//   sstable_test sha256 <file>       the writer's SHA-256 of a file (CPU only)
//
// tests/test_gpu_parity.py compares the file byte for byte with the oracle
// (oracle/sstable_oracle.py) and the oid with SURVEY.md Appendix B.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "sstable_writer.hpp"

namespace {

struct Entry {
  std::string user_key;
  int64_t seq;
  int op;  // OP_PUT = 0, OP_DELETE = 1 (src/keys.hpp:10-13)
  std::string value;
};

/* MemKey::operator< (src/keys.cpp:61-74) */
bool MemLess(const Entry &a, const Entry &b) {
  const int c = a.user_key.compare(b.user_key);
  if (c) return c < 0;
  if (a.seq != b.seq) return a.seq > b.seq;
  return a.op > b.op;
}

/* MemKey::ToKey (src/keys.cpp:76-84) */
std::string InnerKey(const Entry &e) {
  std::string k = e.user_key;
  k.append(reinterpret_cast<const char *>(&e.seq), 8);
  k.push_back((char)e.op);
  return k;
}

std::vector<Entry> Memtable(int which) {
  std::vector<Entry> v;
  for (int i = 0; i < 10000; ++i) {
    if (which == 1)
      v.push_back({"key" + std::to_string(i), i, 0, "value" + std::to_string(i)});
    else
      v.push_back({"key" + std::to_string(i / 2), i, i % 2 ? 1 : 0, "value" + std::to_string(i / 2)});
  }
  std::sort(v.begin(), v.end(), MemLess);
  return v;
}

}  // namespace

int main(int argc, char **argv) {
  using namespace adl;
  if (argc == 3 && !strcmp(argv[1], "sha256")) {
    std::ifstream in(argv[2], std::ios::binary);
    if (!in) return 1;
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string data = ss.str();
    Sha256 h;
    // odd-sized updates exercise the buffered path
    for (size_t o = 0; o < data.size(); o += 61) h.Update(data.data() + o, std::min<size_t>(61, data.size() - o));
    unsigned char d[32];
    h.Final(d);
    printf("%s\n", Sha256Hex(d).c_str());
    return 0;
  }
  int a = 1;
  bool batch = false;
  if (argc > 1 && !strcmp(argv[1], "batch")) batch = true, a = 2;
  if (argc < a + 2) {
    fprintf(stderr, "usage: %s [batch] <1|2> <dir>\n", argv[0]);
    return 2;
  }
  const int which = atoi(argv[a]);
  if (which != 1 && which != 2) return 2;
  const auto mem = Memtable(which);

  PosixFileSink sink(argv[a + 1]);
  if (RC rc = sink.Open(); rc) {
    fprintf(stderr, "open: %s\n", std::string(strrc(rc)).c_str());
    return 1;
  }
  SSTableWriter w(&sink, 10);
  RC rc = OK;
  if (batch) {
    std::string keys, vals;
    std::vector<uint64_t> ko{0}, vo{0};
    for (const auto &e : mem) {
      keys += InnerKey(e);
      vals += e.value;
      ko.push_back(keys.size());
      vo.push_back(vals.size());
    }
    rc = w.AddBatch(keys.data(), ko.data(), vals.data(), vo.data(), mem.size());
  } else {
    for (const auto &e : mem)
      if ((rc = w.Add(InnerKey(e), e.value))) break;
  }
  unsigned char digest[32];
  if (!rc) rc = w.Final(digest);
  if (rc) {
    fprintf(stderr, "sstable build failed: %s\n", std::string(strrc(rc)).c_str());
    return 1;
  }
  printf("%s %d\n", Sha256Hex(digest).c_str(), w.GetFileSize());
  return 0;
}
