// adlsm-tree_amd/csrc/readpath_test.cpp -- the read side of the filter path
//  under concurrency, and its latency.  Needs a GPU.
//
//   readpath_test <outdir> [threads] [rounds]
//     Builds a level of T SSTable filter blocks (FilterBlockWriter, GPU; the
//     tables' bits_per_key cycle through 10, 3 and 16),
//     caches them in a FilterCache by oid, and runs the level multi-get
//     (LevelMultiGetFilter: Level::Get's candidate tables, src/revision.cpp:
//     265-310, and SSTableReader::Get's filter check, src/sstable.cpp:238,
//     for a whole batch in one launch).  Then `threads` threads repeat
//     multi-gets over slices of the batch and single-key / batched probes
//     through per-table FilterBlockReaders sharing the cache, while another
//     thread puts and removes unrelated tables; a second phase does the same
//     with a cache too small for the level, so tables are evicted (while
//     pinned by running probes) and readers re-upload them.  Every answer
//     must equal the single-threaded one (an evicted table may answer "may be
//     present" in a multi-get, never "absent" where the filter says present).
//     The blocks, the level's key ranges, the queries and the single-threaded
//     multi-get are written to <outdir> for tests/ to check against the
//     oracle.  Exit 0 = no mismatch.
//
//   readpath_test --bench
//     Latency of the read path: a single-key FilterBlockReader::IsKeyExists,
//     and level multi-gets of 1k and 64k keys over 16 cached tables.  One JSON
//     line on stdout.
//
//   readpath_test --tails [calls]
//     The single-key latency distribution (p50 ... max) over many calls, across
//     the probe server's exits and relaunches.
//
//   readpath_test --coexist [reps]
//     Single-key Gets while the headline build and a configs[3]-shaped build
//     run on another thread (Coexist below).
//
//   readpath_test --exit-queued
//     Serves Gets until the probe server has a successor kernel queued behind
//     the running one, then returns from main with both still on the
//     server's stream: the process must exit (the atexit stop path drains the
//     queued successor; ADL_BLOOM_DEBUG=1 logs the state it found).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include <sys/resource.h>

#include <hip/hip_runtime_api.h>

#include "adl_bloom.h"
#include "filter_block.hpp"
#include "level_filter.hpp"
#include "sstable_writer.hpp"

namespace {

using namespace adl;

constexpr int kBpk = 10;

std::string UserKey(uint64_t i) {
  char b[32];
  snprintf(b, sizeof(b), "user%09llu", (unsigned long long)i);
  return b;
}

std::string Inner(const std::string &user, int64_t seq) {
  std::string k = user;
  k.append(reinterpret_cast<const char *>(&seq), 8);
  k.push_back('\0');  // OP_PUT
  return k;
}

struct Level {
  std::vector<TableRange> tables;
  std::vector<std::string> blocks;
};

// table t holds user keys [t * stride, t * stride + span) with seq = key
// index.  mixed: table t is written with bits_per_key {10, 3, 16}[t % 3] (a DB
// reopened with another DBOptions::bits_per_key, src/options.hpp:24, keeps
// its older tables: one level, one cache, several k)
Level BuildLevel(int T, uint64_t stride, uint64_t span, RC *rc, bool mixed = false) {
  Level lv;
  for (int t = 0; t < T; ++t) {
    static const int kMixed[3] = {10, 3, 16};
    FilterBlockWriter w(std::make_unique<BloomFilter>(mixed ? kMixed[t % 3] : kBpk));
    const uint64_t lo = (uint64_t)t * stride, hi = lo + span;
    for (uint64_t i = lo; i < hi; ++i) w.Update(UserKey(i));
    std::string block;
    if ((*rc = w.Final(block))) return lv;
    char oid[80];
    snprintf(oid, sizeof(oid), "%064x", 0xA000 + t);  // stands in for the SHA-256 hex
    lv.tables.push_back(TableRange{oid, Inner(UserKey(lo), (int64_t)lo), Inner(UserKey(hi - 1), (int64_t)hi - 1)});
    lv.blocks.push_back(std::move(block));
  }
  *rc = OK;
  return lv;
}

std::vector<std::string> Queries(size_t n, uint64_t key_space, uint64_t seed) {
  std::vector<std::string> q;
  uint64_t s = seed;
  for (size_t i = 0; i < n; ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    const uint64_t r = s >> 17;
    if (i % 3 == 2) q.push_back(UserKey(r % key_space) + "#");  // absent, inside the ranges
    else if (i % 11 == 10) q.push_back("zzz" + std::to_string(r));  // beyond every table
    else q.push_back(UserKey(r % key_space));
  }
  return q;
}

std::vector<std::string_view> Views(const std::vector<std::string> &v, size_t b, size_t e) {
  std::vector<std::string_view> out;
  for (size_t i = b; i < e; ++i) out.emplace_back(v[i]);
  return out;
}

bool WriteFile(const std::string &path, const std::string &data) {
  FILE *f = fopen(path.c_str(), "wb");
  if (!f) return false;
  const bool ok = fwrite(data.data(), 1, data.size(), f) == data.size();
  return fclose(f) == 0 && ok;
}

std::string Hex(const std::string &s) {
  static const char *d = "0123456789abcdef";
  std::string h;
  for (unsigned char c : s) {
    h.push_back(d[c >> 4]);
    h.push_back(d[c & 15]);
  }
  return h;
}

// the single-threaded multi-get over the slice [b, e) of the queries, read
// off the full result
void Slice(const MultiGetFilterResult &all, size_t b, size_t e, std::vector<uint32_t> &tab,
           std::vector<uint8_t> &maybe) {
  tab.assign(all.table.begin() + all.begin[b], all.table.begin() + all.begin[e]);
  maybe.assign(all.maybe.begin() + all.begin[b], all.maybe.begin() + all.begin[e]);
}

double Now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int Bench() {
  RC rc;
  const int T = 16;
  const uint64_t stride = 50000, span = 200000;
  Level lv = BuildLevel(T, stride, span, &rc);
  if (rc) return 1;
  FilterCache cache(1ull << 30, 1024, kBpk);
  if (cache.status()) return 1;
  for (int t = 0; t < T; ++t)
    if (cache.Put(lv.tables[t].oid, lv.blocks[t])) return 1;
  const uint64_t key_space = stride * (T - 1) + span;
  // single-key IsKeyExists on one SSTable's reader (SSTableReader::Get's check)
  FilterBlockReader reader;
  if (reader.Init(lv.blocks[0], cache, lv.tables[0].oid)) return 1;
  std::vector<std::string> q1 = Queries(3000, span, 7);
  std::vector<double> lat;
  for (size_t i = 0; i < q1.size(); ++i) {
    const double t0 = Now();
    volatile bool hit = reader.IsKeyExists(0, q1[i]);
    (void)hit;
    if (i >= 200) lat.push_back((Now() - t0) * 1e6);
  }
  std::sort(lat.begin(), lat.end());
  printf("{\"single_key_is_key_exists_us\": {\"median\": %.1f, \"p99\": %.1f, \"calls\": %zu}", lat[lat.size() / 2],
         lat[lat.size() * 99 / 100], lat.size());
  for (size_t batch : {(size_t)1000, (size_t)65536}) {
    std::vector<std::string> q = Queries(batch, key_space, 11 + batch);
    std::vector<std::string_view> v = Views(q, 0, q.size());
    MultiGetFilterResult r;
    std::vector<double> ms;
    const int reps = batch > 10000 ? 30 : 200;
    for (int i = 0; i < reps + 5; ++i) {
      const double t0 = Now();
      if (LevelMultiGetFilter(cache, lv.tables, v, INT64_MAX, r)) return 1;
      if (i >= 5) ms.push_back((Now() - t0) * 1e3);
    }
    std::sort(ms.begin(), ms.end());
    uint64_t maybe = 0;
    for (uint8_t m : r.maybe) maybe += m;
    printf(", \"multiget_%zu_keys\": {\"median_ms\": %.4f, \"p90_ms\": %.4f, \"pairs_probed\": %zu, "
           "\"pairs_maybe\": %llu, \"tables\": %d, \"us_per_key\": %.3f}",
           batch, ms[ms.size() / 2], ms[ms.size() * 9 / 10], r.table.size(), (unsigned long long)maybe, T,
           ms[ms.size() / 2] * 1e3 / batch);
  }
  printf("}\n");
  return 0;
}


// ---------------------------------------------------------------- tails
double Pct(std::vector<double> v, double p) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(p * (double)v.size()))];
}

void PrintLat(const char *name, const std::vector<double> &lat) {
  printf("\"%s\": {\"calls\": %zu, \"p50\": %.2f, \"p90\": %.2f, \"p99\": %.2f, \"p99_9\": %.2f, \"max\": %.2f}", name,
         lat.size(), Pct(lat, 0.5), Pct(lat, 0.9), Pct(lat, 0.99), Pct(lat, 0.999),
         lat.empty() ? 0.0 : *std::max_element(lat.begin(), lat.end()));
}

// Context switches of the calling thread so far (voluntary + involuntary).
long CtxSwitches() {
  struct rusage ru;
  if (getrusage(RUSAGE_THREAD, &ru)) return 0;
  return ru.ru_nvcsw + ru.ru_nivcsw;
}

// Single-key IsKeyExists through the resident probe server, `calls` times in a
// row: the latency distribution across the server's idle / life-limit exits
// and relaunches (each relaunch is counted).  Each call is also tagged with
// whether the thread was switched out during it (getrusage around the timed
// window), and a host-only control runs the same number of ~5 us spins, so a
// tail that comes from the operating system is told apart from one that comes
// from the server.
int Tails(size_t calls) {
  RC rc;
  Level lv = BuildLevel(4, 50000, 200000, &rc);
  if (rc) return 1;
  FilterCache cache(1ull << 28, 64, kBpk);
  if (cache.status()) return 1;
  FilterBlockReader reader;
  if (cache.Put(lv.tables[0].oid, lv.blocks[0]) || reader.Init(lv.blocks[0], cache, lv.tables[0].oid)) return 1;
  const std::vector<std::string> q = Queries(4096, 200000, 7);
  std::vector<uint8_t> want(q.size());
  for (size_t i = 0; i < q.size(); ++i) want[i] = reader.IsKeyExists(0, q[i]);
  uint64_t l0 = 0, l1 = 0;
  if (adl_bloom_probe_server_launches(&l0)) return 1;
  (void)adl_bloom_probe_server_phases(nullptr, nullptr, nullptr, 1);
  std::vector<double> lat, lat_relaunch, lat_plain, lat_switched;
  lat.reserve(calls);
  size_t bad = 0;
  const double t_start = Now();
  uint64_t la = l0, lb = l0;
  for (size_t i = 0; i < calls; ++i) {
    const size_t j = i % q.size();
    const long cs0 = CtxSwitches();
    const double t0 = Now();
    const bool hit = reader.IsKeyExists(0, q[j]);
    const double us = (Now() - t0) * 1e6;
    const bool switched = CtxSwitches() != cs0;
    lat.push_back(us);
    (void)adl_bloom_probe_server_launches(&lb);
    if (switched) lat_switched.push_back(us);
    else (lb != la ? lat_relaunch : lat_plain).push_back(us);
    la = lb;
    bad += hit != (want[j] != 0);
    if (i % 2000 == 1999)
      fprintf(stderr, "tails: %zu calls, %.3f s, %llu launches\n", i + 1, Now() - t_start,
              (unsigned long long)(lb - l0));
  }
  const double elapsed = Now() - t_start;
  if (adl_bloom_probe_server_launches(&l1)) return 1;
  uint64_t ph_req = 0, ph_st = 0;
  double ph[7] = {};
  (void)adl_bloom_probe_server_phases(&ph_req, &ph_st, ph, 0);
  // host-only control: spins of the median call's length, timed the same way
  const double spin_us = Pct(lat, 0.5);
  std::vector<double> ctl;
  ctl.reserve(calls);
  for (size_t i = 0; i < calls; ++i) {
    const double t0 = Now();
    while ((Now() - t0) * 1e6 < spin_us) {
    }
    ctl.push_back((Now() - t0) * 1e6);
  }
  std::vector<double> top = lat;
  std::sort(top.rbegin(), top.rend());
  top.resize(std::min<size_t>(top.size(), 12));
  auto over = [](const std::vector<double> &v, double x) {
    size_t c = 0;
    for (double u : v) c += u > x;
    return c;
  };
  printf("{");
  PrintLat("single_key_us", lat);
  printf(", ");
  PrintLat("calls_that_relaunched_us", lat_relaunch);
  printf(", ");
  PrintLat("other_calls_us", lat_plain);
  printf(", ");
  PrintLat("calls_switched_out_us", lat_switched);
  printf(", ");
  PrintLat("host_spin_control_us", ctl);
  printf(", \"over_30us\": %zu, \"over_30us_not_switched_out\": %zu, \"control_over_30us\": %zu, \"top_us\": [",
         over(lat, 30.0), over(lat_plain, 30.0) + over(lat_relaunch, 30.0), over(ctl, 30.0));
  for (size_t i = 0; i < top.size(); ++i) printf("%s%.1f", i ? ", " : "", top[i]);
  printf("], \"server_phases_us\": {\"requests\": %llu, \"stamped\": %llu, \"gap_since_previous_poll\": %.3f, "
         "\"poll_loads_back\": %.3f, \"slot_staged\": %.3f, \"hashed\": %.3f, \"bits_read\": %.3f, "
         "\"answer_stored\": %.3f, \"host_per_request\": %.3f}",
         (unsigned long long)ph_req, (unsigned long long)ph_st, ph[0], ph[1], ph[2], ph[3], ph[4], ph[5], ph[6]);
  printf(", \"elapsed_s\": %.3f, \"server_launches\": %llu, \"mismatches\": %zu}\n", elapsed,
         (unsigned long long)(l1 - l0), bad);
  fflush(stdout);
  fprintf(stderr, "tails: printed, tearing down\n");
  return bad ? 1 : 0;
}

// ---------------------------------------------------------------- coexist
// Reads beside builds (the reference's DB::Get probes filters with no lock
// while DoCompaction builds on the worker thread, src/db.cpp:164-172, 263,
// 294): one thread issues single-key IsKeyExists through the resident probe
// server while another runs the headline build (10 M 16-byte keys, one
// filter) and a configs[3]-shaped segmented build (256 tables x 1 M keys)
// back to back on its own stream.  Phases: builds alone, Gets alone, both.
// Prints one JSON line: build times and Get latencies idle and concurrent
// (calls during which the OS switched the thread out are counted apart, and
// calls that had to launch the server are reported apart),
// the headline bitmap's SHA-256 and the SHA-256 of the 256 tables' SHA-256
// hex digests (idle and concurrent), and the Get mismatches.
struct DevBuf {
  void *p = nullptr;
  explicit DevBuf(size_t n) {
    if (hipMalloc(&p, n) != hipSuccess) p = nullptr;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  uint8_t *u8() const { return static_cast<uint8_t *>(p); }
};

std::string ShaHex(const void *data, size_t n) {
  Sha256 h;
  h.Update(data, n);
  unsigned char d[32];
  h.Final(d);
  return Sha256Hex(d);
}

int Coexist(int reps) {
  RC rc;
  Level lv = BuildLevel(4, 50000, 200000, &rc);
  if (rc) return 1;
  FilterCache cache(1ull << 28, 64, kBpk);
  if (cache.status()) return 1;
  FilterBlockReader reader;
  if (cache.Put(lv.tables[0].oid, lv.blocks[0]) || reader.Init(lv.blocks[0], cache, lv.tables[0].oid)) return 1;
  const std::vector<std::string> q = Queries(4096, 200000, 7);
  std::vector<uint8_t> want(q.size());
  for (size_t i = 0; i < q.size(); ++i) want[i] = reader.IsKeyExists(0, q[i]);

  // build inputs, all device-resident (SURVEY §8d SplitMix keys)
  const uint64_t n1 = 10000000, T = 256, nt = 1000000;
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
  DevBuf k1(n1 * 16), b1(adl_bloom_bitmap_alloc_bytes(n1, kBpk));
  const uint64_t ws1 = adl_bloom_build_workspace_bytes(&n1, 1, kBpk);
  std::vector<uint64_t> counts(T, nt), kb(T + 1), boff(T);
  for (uint64_t t = 0; t <= T; ++t) kb[t] = t * nt;
  const uint64_t tb = adl_bloom_bitmap_bytes(nt, kBpk), tba = adl_bloom_bitmap_alloc_bytes(nt, kBpk);
  for (uint64_t t = 0; t < T; ++t) boff[t] = t * tba;
  const uint64_t wsc = adl_bloom_build_workspace_bytes(counts.data(), (uint32_t)T, kBpk);
  DevBuf kc(T * nt * 16), bc(T * tba), ws(std::max(ws1, wsc));
  if (!k1.p || !b1.p || !kc.p || !bc.p || !ws.p) return 1;
  if (adl_synth_keys16_device(k1.u8(), 0x5EED, 0, n1, st)) return 1;
  for (uint64_t t = 0; t < T; ++t)
    if (adl_synth_keys16_device(kc.u8() + t * nt * 16, 0x5EED + t, 0, nt, st)) return 1;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) || hipEventCreate(&e1) || hipStreamSynchronize(st)) return 1;
  // one build; its pass A / pass B kernel times from their dispatch packets
  // (adl_bloom_profile_*) go to pa / pb
  auto build_ms = [&](bool headline, std::vector<double> &pa, std::vector<double> &pb) -> double {
    if (adl_bloom_profile_enable(4) || hipEventRecord(e0, st)) return -1;
    const int s = headline ? adl_bloom_build_device(k1.u8(), nullptr, n1, 16, kBpk, b1.u8(), ws.p, ws1, st)
                           : adl_bloom_build_segmented_device(kc.u8(), nullptr, 16, kb.data(), (uint32_t)T, kBpk,
                                                              bc.u8(), boff.data(), ws.p, wsc, st);
    float ms = 0;
    if (s || hipEventRecord(e1, st) || hipEventSynchronize(e1) || hipEventElapsedTime(&ms, e0, e1)) return -1;
    double ab[2] = {0, 0};
    uint32_t builds = 0;
    if (adl_bloom_profile_collect(ab, &builds) || builds != 1) return -1;
    pa.push_back(ab[0]);
    pb.push_back(ab[1]);
    return ms;
  };
  auto shas = [&](std::string &h1, std::string &hc) -> bool {
    std::vector<uint8_t> h(std::max(adl_bloom_bitmap_bytes(n1, kBpk), T * tba));
    if (hipMemcpy(h.data(), b1.p, adl_bloom_bitmap_bytes(n1, kBpk), hipMemcpyDeviceToHost)) return false;
    h1 = ShaHex(h.data(), adl_bloom_bitmap_bytes(n1, kBpk));
    if (hipMemcpy(h.data(), bc.p, T * tba, hipMemcpyDeviceToHost)) return false;
    std::string cat;
    for (uint64_t t = 0; t < T; ++t) cat += ShaHex(h.data() + boff[t], tb);
    hc = ShaHex(cat.data(), cat.size());
    return true;
  };
  std::vector<double> idle_h, idle_c, conc_h, conc_c;
  std::vector<double> pa_h[2], pb_h[2], pa_c[2], pb_c[2];  // [idle, with Gets]
  // phase 1: builds alone (one warm-up pair)
  for (int r = 0; r <= reps; ++r) {
    const double a = build_ms(true, pa_h[0], pb_h[0]), b = build_ms(false, pa_c[0], pb_c[0]);
    if (a < 0 || b < 0) return 1;
    if (r) idle_h.push_back(a), idle_c.push_back(b);
  }
  std::string sha1_idle, shac_idle, sha1_conc, shac_conc;
  if (!shas(sha1_idle, shac_idle)) return 1;
  // phase 2: Gets alone
  std::vector<double> get_idle, get_conc;
  std::vector<double> relaunch_idle, relaunch_conc;  // calls that (re)launched the server
  size_t bad = 0, switched_idle = 0, switched_conc = 0;
  auto one_get = [&](size_t i, std::vector<double> &lat, std::vector<double> &relaunched, size_t &switched) {
    const size_t j = i % q.size();
    uint64_t la = 0, lb = 0;
    (void)adl_bloom_probe_server_launches(&la);
    const long cs0 = CtxSwitches();
    const double t0 = Now();
    const bool hit = reader.IsKeyExists(0, q[j]);
    const double us = (Now() - t0) * 1e6;
    (void)adl_bloom_probe_server_launches(&lb);
    if (CtxSwitches() != cs0) ++switched;  // the OS took the thread: not the server's latency
    else (lb != la ? relaunched : lat).push_back(us);
    bad += hit != (want[j] != 0);
  };
  for (size_t i = 0; i < 50000; ++i) one_get(i, get_idle, relaunch_idle, switched_idle);
  // phase 3: both
  std::atomic<bool> building{true};
  std::atomic<int> build_fail{0};
  std::thread builder([&] {
    for (int r = 0; r < reps; ++r) {
      const double a = build_ms(true, pa_h[1], pb_h[1]), b = build_ms(false, pa_c[1], pb_c[1]);
      if (a < 0 || b < 0) ++build_fail;
      conc_h.push_back(a);
      conc_c.push_back(b);
    }
    building = false;
  });
  for (size_t i = 0; building.load(); ++i) one_get(i, get_conc, relaunch_conc, switched_conc);
  builder.join();
  if (build_fail || !shas(sha1_conc, shac_conc)) return 1;
  uint64_t launches = 0;
  (void)adl_bloom_probe_server_launches(&launches);
  printf("{\"reps\": %d, \"build_ms\": {\"headline_idle\": %.4f, \"headline_with_gets\": %.4f, "
         "\"compaction_idle\": %.4f, \"compaction_with_gets\": %.4f}, ",
         reps, Pct(idle_h, 0.5), Pct(conc_h, 0.5), Pct(idle_c, 0.5), Pct(conc_c, 0.5));
  printf("\"pass_ms\": {\"headline_a\": [%.4f, %.4f], \"headline_b\": [%.4f, %.4f], \"compaction_a\": [%.4f, %.4f], "
         "\"compaction_b\": [%.4f, %.4f]}, ",
         Pct(pa_h[0], 0.5), Pct(pa_h[1], 0.5), Pct(pb_h[0], 0.5), Pct(pb_h[1], 0.5), Pct(pa_c[0], 0.5),
         Pct(pa_c[1], 0.5), Pct(pb_c[0], 0.5), Pct(pb_c[1], 0.5));
  PrintLat("get_us_idle", get_idle);
  printf(", ");
  PrintLat("get_us_during_builds", get_conc);
  printf(", ");
  PrintLat("relaunching_gets_us_idle", relaunch_idle);
  printf(", ");
  PrintLat("relaunching_gets_us_during_builds", relaunch_conc);
  printf(", \"gets_switched_out\": [%zu, %zu]", switched_idle, switched_conc);
  printf(", \"get_mismatches\": %zu, \"headline_sha256\": [\"%s\", \"%s\"], \"compaction_sha_of_shas\": [\"%s\", \"%s\"], "
         "\"server_launches\": %llu}\n",
         bad, sha1_idle.c_str(), sha1_conc.c_str(), shac_idle.c_str(), shac_conc.c_str(),
         (unsigned long long)launches);
  return bad ? 1 : 0;
}

// Exit with a successor queued.  The cache and reader are
// leaked on purpose: no destructor runs before exit, so the atexit stop path
// alone must drain the server's stream.
int ExitQueued() {
  RC rc;
  Level lv = BuildLevel(1, 50000, 200000, &rc);
  if (rc) return 1;
  auto *cache = new FilterCache(1ull << 26, 8, kBpk);
  auto *reader = new FilterBlockReader;
  if (cache->status() || cache->Put(lv.tables[0].oid, lv.blocks[0]) ||
      reader->Init(lv.blocks[0], *cache, lv.tables[0].oid))
    return 1;
  const std::vector<std::string> q = Queries(64, 200000, 3);
  uint64_t l0 = 0, l = 0;
  (void)adl_bloom_probe_server_launches(&l0);
  // the first Get launches the server; a later one asks the launcher thread
  // for a successor, which it queues behind the running kernel (1 s life)
  for (int i = 0; i < 2000 && l - l0 < 2; ++i) {
    (void)reader->IsKeyExists(0, q[i % q.size()]);
    std::this_thread::sleep_for(std::chrono::microseconds(20));
    (void)adl_bloom_probe_server_launches(&l);
  }
  printf("{\"server_launches\": %llu, \"exiting\": true}\n", (unsigned long long)(l - l0));
  fflush(stdout);
  return l - l0 >= 2 ? 0 : 3;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc > 1 && strcmp(argv[1], "--bench") == 0) return Bench();
  if (argc > 1 && strcmp(argv[1], "--tails") == 0) {
    const int rc = Tails(argc > 2 ? (size_t)atoll(argv[2]) : 200000);
    fprintf(stderr, "tails: returned %d\n", rc);
    return rc;
  }
  if (argc > 1 && strcmp(argv[1], "--coexist") == 0) return Coexist(argc > 2 ? atoi(argv[2]) : 5);
  if (argc > 1 && strcmp(argv[1], "--exit-queued") == 0) return ExitQueued();
  if (argc < 2) {
    fprintf(stderr, "usage: readpath_test <outdir> [threads] [rounds] | --bench\n");
    return 2;
  }
  const std::string dir = argv[1];
  const int P = argc > 2 ? atoi(argv[2]) : 8;
  const int R = argc > 3 ? atoi(argv[3]) : 10;
  const int T = 24;
  const uint64_t stride = 5000, span = 20000;
  RC rc;
  Level lv = BuildLevel(T, stride, span, &rc, /*mixed=*/true);
  if (rc) {
    fprintf(stderr, "build failed: %s\n", std::string(strrc(rc)).c_str());
    return 1;
  }
  const uint64_t key_space = stride * (T - 1) + span + 1000;
  const std::vector<std::string> q = Queries(12000, key_space, 0xC0FFEE);
  const std::vector<std::string_view> qv = Views(q, 0, q.size());

  // ---- phase 1: the level fits the cache
  FilterCache cache(64ull << 20, 64, kBpk);
  if (cache.status()) return 1;
  for (int t = 0; t < T; ++t)
    if ((rc = cache.Put(lv.tables[t].oid, lv.blocks[t]))) {
      fprintf(stderr, "put failed: %s\n", std::string(strrc(rc)).c_str());
      return 1;
    }
  MultiGetFilterResult want;
  if ((rc = LevelMultiGetFilter(cache, lv.tables, qv, INT64_MAX, want)) || want.uncached) {
    fprintf(stderr, "multi-get failed: %s\n", std::string(strrc(rc)).c_str());
    return 1;
  }
  // for tests/: blocks, ranges, queries, the single-threaded answer
  std::string tables_txt, q_txt, mg_txt;
  for (int t = 0; t < T; ++t) {
    if (!WriteFile(dir + "/table_" + std::to_string(t) + ".blk", lv.blocks[t])) return 1;
    tables_txt += lv.tables[t].oid + " " + Hex(lv.tables[t].min_inner_key) + " " + Hex(lv.tables[t].max_inner_key) +
                  "\n";
  }
  for (const auto &s : q) q_txt += Hex(s) + "\n";
  for (size_t i = 0; i < q.size(); ++i) {
    mg_txt += std::to_string(i);
    for (uint32_t p = want.begin[i]; p < want.begin[i + 1]; ++p)
      mg_txt += " " + std::to_string(want.table[p]) + ":" + std::to_string(want.maybe[p]);
    mg_txt += "\n";
  }
  if (!WriteFile(dir + "/tables.txt", tables_txt) || !WriteFile(dir + "/queries.txt", q_txt) ||
      !WriteFile(dir + "/multiget.txt", mg_txt))
    return 1;

  // per-table readers over the same cache (Init finds the table cached)
  std::vector<std::unique_ptr<FilterBlockReader>> readers(T);
  for (int t = 0; t < T; ++t) {
    readers[t] = std::make_unique<FilterBlockReader>();
    if (readers[t]->Init(lv.blocks[t], cache, lv.tables[t].oid)) return 1;
  }
  // want_reader[t][i]: filter 0 of table t on query i (from the multi-get where
  // t is a candidate of i; every other pair from one batched reader probe)
  std::vector<std::vector<uint8_t>> want_reader(T);
  KeyArena all;
  for (const auto &s : q) all.Add(s);
  for (int t = 0; t < T; ++t)
    if (readers[t]->IsKeysExist(0, all, want_reader[t])) return 1;
  int bad = 0;
  for (size_t i = 0; i < q.size(); ++i)
    for (uint32_t p = want.begin[i]; p < want.begin[i + 1]; ++p)
      bad += want_reader[want.table[p]][i] != want.maybe[p];
  if (bad) {
    fprintf(stderr, "reader and multi-get disagree on %d pairs\n", bad);
    return 1;
  }

  std::atomic<int> failures{0}, evictions_seen{0};
  auto run_phase = [&](FilterCache &c, bool small) {
    std::vector<std::thread> th;
    std::atomic<bool> stop{false};
    for (int p = 0; p < P; ++p) {
      th.emplace_back([&, p] {
        std::vector<uint32_t> wt;
        std::vector<uint8_t> wm;
        for (int r = 0; r < R; ++r) {
          const size_t b = ((size_t)(p * R + r) * 997) % (q.size() - 1500), e = b + 1500;
          MultiGetFilterResult got;
          const std::vector<std::string_view> v = Views(q, b, e);
          if (LevelMultiGetFilter(c, lv.tables, v, INT64_MAX, got)) {
            ++failures;
            continue;
          }
          Slice(want, b, e, wt, wm);
          if (got.table != wt) ++failures;
          if (got.uncached) ++evictions_seen;
          for (size_t k = 0; k < wm.size() && k < got.maybe.size(); ++k) {
            // an uncached table answers "may be present"; a cached one exactly
            if (got.maybe[k] != wm[k] && !(small && got.maybe[k] == 1)) ++failures;
            if (!small && got.maybe[k] != wm[k]) ++failures;
          }
          // a few tables through their own readers: exact even after eviction
          for (int t = (p + r) % T, n = 0; n < 3; ++n, t = (t + 7) % T) {
            std::vector<uint8_t> got_r;
            KeyArena ka;
            for (size_t i = b; i < b + 200; ++i) ka.Add(q[i]);
            if (readers[t]->IsKeysExist(0, ka, got_r) ||
                !std::equal(got_r.begin(), got_r.end(), want_reader[t].begin() + b))
              ++failures;
            if (readers[t]->IsKeyExists(0, q[b + r]) != (want_reader[t][b + r] != 0)) ++failures;
          }
        }
      });
    }
    // churn: unrelated tables come and go (and, in the small cache, push the
    // level's tables out while probes hold them)
    th.emplace_back([&] {
      for (int i = 0; !stop.load(); ++i) {
        const std::string oid = "extra-" + std::to_string(i % 5);
        if (c.Put(oid, lv.blocks[i % T])) ++failures;
        if (i % 3 == 0) c.Remove("extra-" + std::to_string((i + 2) % 5));
        if (small && i % 4 == 1) c.Put(lv.tables[(i * 5) % T].oid, lv.blocks[(i * 5) % T]);
      }
    });
    for (int p = 0; p < P; ++p) th[p].join();
    stop = true;
    th.back().join();
  };
  run_phase(cache, false);
  const int f1 = failures.load();

  // ---- phase 2: a cache that holds about 6 of the level's tables
  FilterCache small(6 * (lv.blocks[0].size() + 4096), 8, kBpk);
  if (small.status()) return 1;
  for (int t = 0; t < T; ++t) {
    readers[t] = std::make_unique<FilterBlockReader>();
    if (readers[t]->Init(lv.blocks[t], small, lv.tables[t].oid)) return 1;
  }
  run_phase(small, true);
  printf("%d threads x %d rounds, %d tables, %zu queries: phase 1 (level cached) %d mismatches, "
         "phase 2 (evicting) %d mismatches, %d multi-gets saw evicted tables\n",
         P, R, T, q.size(), f1, failures.load() - f1, evictions_seen.load());
  return failures.load() ? 1 : 0;
}
