// adlsm-tree_amd/csrc/concurrency_test.cpp -- the threading contract of the
// filter path (SURVEY.md §8b "Threading"): the reference builds filters on the
// background worker thread (src/db.cpp:263,294) while user threads probe
// FilterBlockReaders concurrently with no lock (src/db.cpp:166-172).  Needs a
// GPU.  Exit status 0 = every concurrent result equals the sequential one.
//
//   P prober threads share one FilterBlockReader (read-only after Init) and
//   run single-key IsKeyExists and batched IsKeysExist; W builder threads
//   each build their own filter blocks through FilterBlockWriter (the
//   pipelined host-pointer segmented build) at the same time.  Results are
//   compared with the same calls made on one thread beforehand.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "filter_block.hpp"

namespace {

uint64_t splitmix(uint64_t &s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

std::string Key(uint64_t &s) {
  const uint64_t a = splitmix(s);
  std::string k(8 + a % 24, '\0');
  for (size_t i = 0; i < k.size(); i += 8) {
    const uint64_t v = splitmix(s);
    for (size_t j = 0; j < 8 && i + j < k.size(); ++j) k[i + j] = (char)(v >> (8 * j));
  }
  return k;
}

// one block of `nf` filters; filter f holds keys_per * (f + 1) keys from seed
std::string BuildBlock(uint64_t seed, int nf, int keys_per, adl::RC *rc) {
  adl::FilterBlockWriter w(std::make_unique<adl::BloomFilter>(10));
  uint64_t s = seed;
  for (int f = 0; f < nf; ++f) {
    for (int i = 0; i < keys_per * (f + 1); ++i) w.Update(Key(s));
    w.Keys2Block();
  }
  std::string out;
  *rc = w.Final(out);
  return out;
}

}  // namespace

int main(int argc, char **argv) {
  using namespace adl;
  const int P = argc > 1 ? atoi(argv[1]) : 8;   // prober threads
  const int W = argc > 2 ? atoi(argv[2]) : 2;   // builder threads
  const int R = argc > 3 ? atoi(argv[3]) : 20;  // rounds per thread
  std::atomic<int> failures{0};

  RC rc;
  const std::string block = BuildBlock(0x5EED, 3, 20000, &rc);
  if (rc) {
    fprintf(stderr, "build failed: %s\n", std::string(strrc(rc)).c_str());
    return 1;
  }
  FilterBlockReader reader;
  if ((rc = reader.Init(block))) {
    fprintf(stderr, "Init failed: %s\n", std::string(strrc(rc)).c_str());
    return 1;
  }

  // sequential expectations: per prober, a batch of half inserted, half fresh keys
  std::vector<KeyArena> batches(P);
  std::vector<std::vector<std::vector<uint8_t>>> want(P, std::vector<std::vector<uint8_t>>(3));
  for (int t = 0; t < P; ++t) {
    uint64_t ins = 0x5EED, fresh = 0xF00D + t;
    for (int i = 0; i < 4000; ++i) batches[t].Add(i % 2 ? Key(fresh) : Key(ins));
    for (int f = 0; f < 3; ++f)
      if (reader.IsKeysExist(f, batches[t], want[t][f]) != OK) return 1;
  }
  std::vector<std::string> want_blocks(W);
  for (int b = 0; b < W; ++b) {
    want_blocks[b] = BuildBlock(0xB10C + b, 4, 5000, &rc);
    if (rc) return 1;
  }

  std::vector<std::thread> th;
  for (int t = 0; t < P; ++t) {
    th.emplace_back([&, t] {
      std::vector<uint8_t> got;
      for (int r = 0; r < R; ++r) {
        const int f = (t + r) % 3;
        if (reader.IsKeysExist(f, batches[t], got) != OK || got != want[t][f]) ++failures;
        // a few single-key probes (one device round trip each)
        for (int i = r % 7; i < 4000; i += 997) {
          const auto &off = batches[t].offsets();
          std::string_view k(batches[t].bytes().data() + off[i], off[i + 1] - off[i]);
          if (reader.IsKeyExists(f, k) != (want[t][f][i] != 0)) ++failures;
        }
      }
    });
  }
  for (int b = 0; b < W; ++b) {
    th.emplace_back([&, b] {
      for (int r = 0; r < R / 4 + 1; ++r) {
        RC brc;
        const std::string got = BuildBlock(0xB10C + b, 4, 5000, &brc);
        if (brc != OK || got != want_blocks[b]) ++failures;
      }
    });
  }
  for (auto &x : th) x.join();
  printf("%d prober threads x %d rounds, %d builder threads: %d mismatches\n", P, R, W, failures.load());
  return failures.load() ? 1 : 0;
}
