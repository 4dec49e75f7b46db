// adlsm-tree_amd/csrc/asan_test.cpp -- host sanitizer run (make asan) over the
// code that parses and frames untrusted bytes, as the reference builds every
// target with -fsanitize=address (CMakeLists.txt:5,13).  Runs on a CPU: no
// path here reaches the device.
//
//   1. The filter-block trailer walk (filter_block_format.hpp, used by
//      FilterBlockReader::Init and the device filter cache): every truncation
//      of valid blocks, every single-byte change of their trailers, and
//      hand-made hostile trailers (offsets past the end, negative and huge
//      counts, info_len 1..len, filters over 2^31 bits), each parsed from a
//      heap buffer of exactly its length, so any read outside it is caught.
//      Malformed blocks also go through FilterBlockReader::Init, which must
//      answer FILTER_BLOCK_ERROR before touching the device.
//   2. A FilterAlgorithm written against the reference's interface
//      (src/filter_block.hpp:13-20: only Keys2Block(vector<string>),
//      IsKeyExists and FilterInfo) driving FilterBlockWriter and
//      SSTableWriter: the block and the SSTable framing (BlockWriter, footer,
//      SHA-256) end to end, and the block read back.
// Exit 0 = all checks passed and the sanitizers reported nothing.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <memory>
#include <string>
#include <vector>

#include "filter_block.hpp"
#include "filter_block_format.hpp"
#include "sstable_writer.hpp"

namespace {

using namespace adl;

int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                    \
    }                                                              \
  } while (0)

void Put32(std::string &s, int32_t v) { s.append(reinterpret_cast<const char *>(&v), 4); }

// FilterBlockWriter::Final's layout (src/filter_block.cpp:77-102) around
// arbitrary bitmaps
std::string Frame(const std::vector<std::string> &bitmaps, int32_t bpk) {
  std::string b;
  std::vector<int32_t> off;
  for (const auto &m : bitmaps) {
    off.push_back((int32_t)b.size());
    b += m;
  }
  const int32_t start = (int32_t)b.size();
  for (int32_t o : off) Put32(b, o);
  Put32(b, start);
  Put32(b, (int32_t)off.size());
  b += "bf:";
  Put32(b, bpk);
  Put32(b, 7);
  return b;
}

// parse from a heap copy of exactly len bytes
int ParseExact(const std::string &blk, size_t len, adl_fmt::FilterBlockLayout &lay) {
  std::unique_ptr<uint8_t[]> buf(new uint8_t[len ? len : 1]);
  memcpy(buf.get(), blk.data(), len);
  return adl_fmt::parse_filter_block(buf.get(), len, lay);
}

void ReaderRejects(const std::string &blk) {
  std::unique_ptr<char[]> buf(new char[blk.size() ? blk.size() : 1]);
  memcpy(buf.get(), blk.data(), blk.size());
  FilterBlockReader r;
  CHECK(r.Init(std::string_view(buf.get(), blk.size())) == FILTER_BLOCK_ERROR);
  CHECK(!r.IsKeyExists(0, "k"));
}

void ParserChecks() {
  std::vector<std::string> valid = {
      Frame({}, 10),
      Frame({std::string(17, '\x5a')}, 10),
      Frame({std::string(27, '\x01'), std::string(7, '\x00'), std::string(1007, '\xff')}, 10),
      Frame({std::string(7, '\0'), std::string(7, '\0'), std::string(7, '\0'), std::string(7, '\0')}, 0),
  };
  for (const auto &v : valid) {
    adl_fmt::FilterBlockLayout lay;
    CHECK(ParseExact(v, v.size(), lay) == 0);
    CHECK(lay.bits_per_key == 10 || lay.bits_per_key == 0);
    CHECK(lay.off.size() == (size_t)lay.num_filters + 1);
    CHECK(lay.off.back() == (uint64_t)lay.offsets_start);
    // every truncation, from the front and from the back
    for (size_t len = 0; len < v.size(); ++len) {
      ParseExact(v, len, lay);
      std::string tail = v.substr(v.size() - len);
      ParseExact(tail, tail.size(), lay);
    }
    // every single-byte change of the trailer (4F + 19 bytes)
    const size_t trailer = 4 * lay.off.size() + 15;
    for (size_t i = v.size() - std::min(v.size(), trailer); i < v.size(); ++i)
      for (int x : {0x00, 0x01, 0x7f, 0x80, 0xff}) {
        std::string m = v;
        m[i] = (char)x;
        adl_fmt::FilterBlockLayout l2;
        if (ParseExact(m, m.size(), l2) == 0) {
          // accepted: the layout must lie inside the block
          CHECK(l2.offsets_start >= 0 && (uint64_t)l2.offsets_start <= m.size());
          for (size_t f = 0; f + 1 < l2.off.size(); ++f) CHECK(l2.off[f] <= l2.off[f + 1]);
        } else {
          ReaderRejects(m);
        }
      }
  }
  // hostile trailers
  struct Case {
    int32_t start, nf, info_len;
    const char *what;
  } cases[] = {
      {0x7fffffff, 1, 7, "offsets_start past the end"},
      {-4, 1, 7, "negative offsets_start"},
      {0, 0x40000000, 7, "huge filter count"},
      {0, -1, 7, "negative filter count"},
      {0, 1, 0x7ffffff0, "info_len past the front"},
      {0, 1, 0, "zero info_len"},
      {0, 1, 2, "info shorter than bf:<bpk>"},
  };
  for (const auto &c : cases) {
    std::string b(64, '\0');
    Put32(b, c.start);
    Put32(b, c.nf);
    b += "bf:";
    Put32(b, 10);
    Put32(b, c.info_len);
    adl_fmt::FilterBlockLayout lay;
    const int rc = ParseExact(b, b.size(), lay);
    if (rc == 0) fprintf(stderr, "accepted: %s\n", c.what);
    CHECK(rc == adl_fmt::kFilterBlockError);
    ReaderRejects(b);
  }
  // a filter of more than 2^31 bits cannot be probed with the reference's int m
  {
    const std::string b = Frame({std::string((1u << 28) + 1, '\0')}, 10);  // 2^31 + 8 bits
    adl_fmt::FilterBlockLayout lay;
    CHECK(adl_fmt::parse_filter_block(reinterpret_cast<const uint8_t *>(b.data()), b.size(), lay) ==
          adl_fmt::kFilterBlockError);
    const std::string ok = Frame({std::string((1u << 28) - 1, '\0')}, 10);  // 2^31 - 8 bits: accepted
    CHECK(adl_fmt::parse_filter_block(reinterpret_cast<const uint8_t *>(ok.data()), ok.size(), lay) == 0);
  }
  // info_len of every size up to the whole block
  std::string v = Frame({std::string(40, '\x11')}, 10);
  for (int32_t il = -2; il < (int32_t)v.size() + 2; ++il) {
    std::string m = v;
    memcpy(&m[m.size() - 4], &il, 4);
    adl_fmt::FilterBlockLayout lay;
    ParseExact(m, m.size(), lay);
  }
}

// A filter written against the reference's FilterAlgorithm only: one byte
// per key (the key's length), no GPU.  Exercises the default batched
// extensions of the mirror.
class LengthFilter : public FilterAlgorithm {
 public:
  RC Keys2Block(const vector<string> &keys, string &result) override {
    for (const auto &k : keys) result.push_back((char)k.size());
    result.push_back('\x7f');
    return OK;
  }
  bool IsKeyExists(string_view key, string_view bitmap) override {
    return bitmap.find((char)key.size()) != string_view::npos;
  }
  void FilterInfo(string &info) override {
    info.append("bf:");
    Put32(info, 3);
  }
};

void WriterChecks() {
  FilterBlockWriter w(std::make_unique<LengthFilter>());
  for (int f = 0; f < 5; ++f) {
    for (int i = 0; i < 10 * f; ++i) w.Update(std::string(i % 9 + 1, 'k'));
    w.Keys2Block();
  }
  std::string block;
  CHECK(w.Final(block) == OK);
  adl_fmt::FilterBlockLayout lay;
  CHECK(ParseExact(block, block.size(), lay) == 0);
  CHECK(lay.num_filters == 5 && lay.bits_per_key == 3);
  for (int f = 0; f < 5; ++f) CHECK(lay.off[f + 1] - lay.off[f] == (uint64_t)(10 * f + 1));

  // SSTableWriter framing over a memtable-shaped run (sstable.cpp's Add/Final)
  StringSink sink;
  SSTableWriter t(&sink, std::make_unique<LengthFilter>());
  for (int i = 0; i < 5000; ++i) {
    char k[32];
    const int n = snprintf(k, sizeof(k), "key%06d", i);
    std::string inner(k, n);
    const int64_t seq = i;
    inner.append(reinterpret_cast<const char *>(&seq), 8);
    inner.push_back('\0');
    CHECK(t.Add(inner, std::string(i % 300, 'v')) == OK);
  }
  unsigned char sha[32];
  CHECK(t.Final(sha) == OK);
  const std::string &file = sink.data();
  CHECK((int)file.size() == t.GetFileSize());
  CHECK(file.size() > 18 && (unsigned char)file[file.size() - 2] == 0x12 &&
        (unsigned char)file[file.size() - 1] == 0x34);  // footer magic (src/footer_block.cpp:24-25)
}

}  // namespace

int main() {
  ParserChecks();
  WriterChecks();
  printf("asan_test: %d failed checks\n", g_fail);
  return g_fail ? 1 : 0;
}
