// adlsm-tree_amd/csrc/sstable_test.cpp -- the memtables of the reference's
// test/sstable_test.cpp (BuildSSTable :9-27, BuildSSTable2 :29-43) flushed
// through the gfx950-backed SSTableWriter (sstable_writer.hpp).  Needs a GPU.
//
//   sstable_test <which 1|2|3> <dir> writes <dir>/<oid>.sst, prints "<oid> <bytes> <dups>"
//                                    (3: 1-5 versions per user key; dups = the filter keys
//                                    equal to their predecessor, skipped on the device)
//   sstable_test batch <which> <dir> the same through AddBatch (packed run)
//   sstable_test sha256 <file>       the writer's SHA-256 of a file (CPU only)
//   sstable_test bench <n> <dir>     flush an n-entry memtable ("key%012d" / 100-byte
//                                    values, seq = i): prints one JSON line with the
//                                    time of the Add loop and of Final (GPU filter)
//   sstable_test overlap <dir>       both memtables as two outputs of one compaction:
//                                    table 2 is filled while table 1's filter builds
//                                    (BeginFinal / EndFinal); prints "<oid> <bytes>" twice
//   sstable_test pipebench <n> <t>   t tables of n entries written one after another,
//                                    Final per table vs BeginFinal, fill the next
//                                    table, EndFinal: one JSON line with both times
//
// tests/test_gpu_parity.py compares the file byte for byte with the oracle
// (oracle/sstable_oracle.py) and the oid with SURVEY.md Appendix B.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <fstream>
#include <memory>
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
  if (which == 3) {
    // 1-5 versions of each of 4 000 user keys (puts and deletes): in memtable
    // order a user key's versions are adjacent filter keys
    int64_t seq = 0;
    for (int j = 0; j < 4000; ++j)
      for (int r = 0; r <= (j * 7) % 5; ++r, ++seq)
        v.push_back({"user" + std::to_string(j), seq, seq % 3 == 2 ? 1 : 0, "v" + std::to_string(seq)});
  }
  for (int i = 0; which != 3 && i < 10000; ++i) {
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
  if (argc == 4 && !strcmp(argv[1], "bench")) {
    const long n = atol(argv[2]);
    std::vector<Entry> mem;
    mem.reserve(n);
    char buf[32];
    for (long i = 0; i < n; ++i) {
      snprintf(buf, sizeof buf, "key%012ld", i);
      mem.push_back({buf, (int64_t)i, 0, std::string(100, (char)('a' + i % 26))});
    }
    std::vector<std::string> ikeys;
    ikeys.reserve(n);
    for (const auto &e : mem) ikeys.push_back(InnerKey(e));
    double best_add = 1e30, best_final = 1e30, best_filter = 1e30;
    int size = 0;
    std::string oid;
    for (int rep = 0; rep < 4; ++rep) {  // rep 0 warms the device up
      StringSink sink;
      SSTableWriter w(&sink, 10);
      const auto t0 = std::chrono::steady_clock::now();
      for (long i = 0; i < n; ++i)
        if (w.Add(ikeys[i], mem[i].value)) return 1;
      const auto t1 = std::chrono::steady_clock::now();
      unsigned char d[32];
      if (w.Final(d)) return 1;
      const auto t2 = std::chrono::steady_clock::now();
      if (rep) {
        best_add = std::min(best_add, std::chrono::duration<double>(t1 - t0).count());
        best_final = std::min(best_final, std::chrono::duration<double>(t2 - t1).count());
        best_filter = std::min(best_filter, w.filter_seconds());
      }
      size = w.GetFileSize();
      oid = Sha256Hex(d);
      if (rep == 3) {  // keep one file for the caller's parity check
        std::ofstream(std::string(argv[3]) + "/" + oid + ".sst", std::ios::binary)
            .write(sink.data().data(), (std::streamsize)sink.data().size());
      }
    }
    printf("{\"entries\": %ld, \"bytes\": %d, \"oid\": \"%s\", \"add_s\": %.6f, \"final_s\": %.6f, \"filter_s\": %.6f}\n",
           n, size, oid.c_str(), best_add, best_final, best_filter);
    return 0;
  }
  if (argc == 3 && !strcmp(argv[1], "overlap")) {
    const auto m1 = Memtable(1), m2 = Memtable(2);
    PosixFileSink s1(argv[2]), s2(argv[2]);
    if (s1.Open() || s2.Open()) return 1;
    SSTableWriter w1(&s1, 10), w2(&s2, 10);
    for (const auto &e : m1)
      if (w1.Add(InnerKey(e), e.value)) return 1;
    if (w1.BeginFinal()) return 1;
    if (w1.Add(InnerKey(m1[0]), "x") != BAD_RECORD) return 3;  // no Add while the filter builds
    for (const auto &e : m2)
      if (w2.Add(InnerKey(e), e.value)) return 1;
    unsigned char d1[32], d2[32];
    if (w1.EndFinal(d1) || w2.BeginFinal() || w2.EndFinal(d2)) return 1;
    if (w2.EndFinal(d2) != BAD_RECORD) return 3;  // one EndFinal per BeginFinal
    // a writer dropped with its filter build still pending (an error path of a
    // compaction): ~SSTableWriter waits for the build, whose output lives in
    // the writer; its memory is then reused and scribbled over, and the
    // worker's next build must still be exact
    for (int rep = 0; rep < 3; ++rep) {
      StringSink s3;
      auto w3 = std::make_unique<SSTableWriter>(&s3, 10);
      for (const auto &e : m2)
        if (w3->Add(InnerKey(e), e.value)) return 1;
      if (w3->BeginFinal()) return 1;
      w3.reset();
      auto scribble = std::make_unique<std::vector<char>>(sizeof(SSTableWriter) * 4, (char)0x5A);
      (void)scribble;
    }
    StringSink s4;
    SSTableWriter w4(&s4, 10);
    for (const auto &e : m2)
      if (w4.Add(InnerKey(e), e.value)) return 1;
    unsigned char d4[32];
    if (w4.BeginFinal() || w4.EndFinal(d4)) return 1;
    if (memcmp(d4, d2, 32)) return 4;  // same memtable, same file
    printf("%s %d\n%s %d\n", Sha256Hex(d1).c_str(), w1.GetFileSize(), Sha256Hex(d2).c_str(), w2.GetFileSize());
    return 0;
  }
  if (argc == 4 && !strcmp(argv[1], "pipebench")) {
    const long n = atol(argv[2]);
    const int tables = atoi(argv[3]);
    std::vector<std::vector<std::string>> ikeys(tables), vals(tables);
    char buf[32];
    for (int t = 0; t < tables; ++t)
      for (long i = 0; i < n; ++i) {
        snprintf(buf, sizeof buf, "k%03d%012ld", t, i);
        ikeys[t].push_back(InnerKey({buf, (int64_t)i, 0, ""}));
        vals[t].push_back(std::string(100, (char)('a' + (i + t) % 26)));
      }
    auto fill = [&](SSTableWriter &w, int t) {
      for (long i = 0; i < n; ++i)
        if (w.Add(ikeys[t][i], vals[t][i])) return false;
      return true;
    };
    double best_seq = 1e30, best_pipe = 1e30;
    std::vector<std::string> oid_seq(tables), oid_pipe(tables);
    for (int rep = 0; rep < 4; ++rep) {  // rep 0 warms the device up
      {  // Final per table
        std::vector<StringSink> sinks(tables);
        const auto t0 = std::chrono::steady_clock::now();
        for (int t = 0; t < tables; ++t) {
          SSTableWriter w(&sinks[t], 10);
          unsigned char d[32];
          if (!fill(w, t) || w.Final(d)) return 1;
          oid_seq[t] = Sha256Hex(d);
        }
        if (rep) best_seq = std::min(best_seq, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
      }
      {  // table t+1 filled while table t's filter builds
        std::vector<StringSink> sinks(tables);
        std::vector<std::unique_ptr<SSTableWriter>> ws;
        for (int t = 0; t < tables; ++t) ws.push_back(std::make_unique<SSTableWriter>(&sinks[t], 10));
        const auto t0 = std::chrono::steady_clock::now();
        for (int t = 0; t < tables; ++t) {
          if (!fill(*ws[t], t) || ws[t]->BeginFinal()) return 1;
          if (t) {
            unsigned char d[32];
            if (ws[t - 1]->EndFinal(d)) return 1;
            oid_pipe[t - 1] = Sha256Hex(d);
          }
        }
        unsigned char d[32];
        if (ws[tables - 1]->EndFinal(d)) return 1;
        oid_pipe[tables - 1] = Sha256Hex(d);
        if (rep) best_pipe = std::min(best_pipe, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
      }
      if (oid_seq != oid_pipe) return 4;
    }
    printf("{\"entries_per_table\": %ld, \"tables\": %d, \"final_per_table_s\": %.6f, \"overlapped_s\": %.6f, "
           "\"oids_equal\": true}\n", n, tables, best_seq, best_pipe);
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
  if (which < 1 || which > 3) return 2;
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
  const unsigned long long dups = w.filter_duplicates();
  if (!rc) rc = w.Final(digest);
  if (rc) {
    fprintf(stderr, "sstable build failed: %s\n", std::string(strrc(rc)).c_str());
    return 1;
  }
  printf("%s %d %llu\n", Sha256Hex(digest).c_str(), w.GetFileSize(), dups);
  return 0;
}
