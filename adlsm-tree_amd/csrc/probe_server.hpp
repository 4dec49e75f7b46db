// adlsm-tree_amd/csrc/probe_server.hpp -- library-internal interface of the
// resident single-key probe server (probe_server.hip), used by the filter
// cache's small batches (filter_cache.hip).
#pragma once
#include <stdint.h>

#include <chrono>

namespace adl_srv {

constexpr uint32_t kMaxQ = 8;           // queries per request
constexpr uint32_t kMaxKeyBytes = 320;  // key bytes per request
// probe()'s answer wait before it gives up and returns kBusy (the caller then
// probes by a launch; the request may still be served later, reading only the
// cache arena, and its answer is ignored: each request has its own sequence)
constexpr std::chrono::milliseconds kTimeout{200};
constexpr int kBusy = -1000;

struct Server;

// A server for the calling thread's current device (no kernel runs until the
// first probe), or nullptr.
__attribute__((visibility("hidden"))) Server *create();
// Stops the kernel (if running), waits for it and frees everything.  No probe
// may be running or start.
__attribute__((visibility("hidden"))) void destroy(Server *s);
__attribute__((visibility("hidden"))) bool eligible(uint64_t n, uint64_t key_bytes);
// n queries (keys by offsets or fixed stride), query q against the device
// byte range [range[2q], range[2q+1]) of kq[q]-probe filter bits (each table's
// block carries its own bits_per_key); answers to h_out.  arena_epoch: the
// caller's arena's put count, read after its ranges were resolved (the wave
// invalidates its caches when it has not yet done so since that put).
// Returns ADL_* status, or kBusy when no answer came within kTimeout.
__attribute__((visibility("hidden"))) int probe(Server *s, const uint8_t *h_keys, const uint64_t *h_offsets,
                                                uint32_t key_stride, uint64_t n, const uint64_t *range,
                                                const uint8_t *kq, uint64_t arena_epoch, uint8_t *h_out);

// Servers that exist in this process (created, not destroyed).
__attribute__((visibility("hidden"))) uint32_t live_servers();
// Servers whose kernel is resident or about to start (the alive word: set by
// the host before a launch and by the kernel as it starts, cleared by the
// kernel as it leaves).  The build takes its items from work queues only
// then (bloom_build.hip, ADL_BLOOM_BUILD_QUEUES).
__attribute__((visibility("hidden"))) uint32_t resident_servers();

// Server kernels launched by this process so far (relaunches after the idle
// and life limits included); readpath_test's tail-latency run reports it.
__attribute__((visibility("hidden"))) uint64_t launches();

}  // namespace adl_srv
