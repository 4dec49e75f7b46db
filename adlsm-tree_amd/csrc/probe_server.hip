// adlsm-tree_amd/csrc/probe_server.hip -- resident probe server for single-key
// lookups (SSTableReader::Get's filter check, reference src/sstable.cpp:238,
// BloomFilter::IsKeyExists, src/filter_block.cpp:49-62).
//
// A Get probes one key against one table's filter.  Through a kernel launch
// that costs a dispatch and a completion (about 17 us on MI355X, most of it
// launch latency).  Here one single-wave workgroup stays resident instead and
// serves requests that host threads post into coherent, device-mapped host
// memory:
//
//   slot j (512 B)   queries (<= kMaxQ), k, per query the absolute device range
//                    [begin, end) of its filter in the cache arena, key offsets
//                    and key bytes; written by the host thread holding slot j
//   bell[j] (u32)    request sequence number, written after the slot (release);
//                    the 64 bells share 256 bytes, so one wave-wide load polls
//                    every slot
//   done[j] (64 B)   word 0: the served sequence number (a restarted kernel's
//                    starting point); word 1: the low 24 bits of that number
//                    above the 8 answer bits.  Both in one 8-byte system-scope
//                    store; the host takes its answers from word 1 alone
//
// The wave polls the bells, copies every pending slot into LDS with one load
// per lane per slot (one round trip for all of them), hashes each query's key
// from LDS (hash_bytes), tests its k bits in the arena with all k loads in
// flight at once, writes the answers and then the sequence numbers.  The host
// thread spins on its done line.
//
// Lifetime.  The kernel exits when it has been idle for idle_ticks, when it has
// run for life_ticks, or when the host raises ctl->stop (cache teardown), so
// its wave always finishes.  A host thread whose request is not answered
// checks the server's completion event: if the kernel has exited (idle or
// life limit) it launches a new one, which picks up the pending request; if
// the event reports an error, the call fails with ADL_ERR_DEVICE.  The server
// runs on a stream of its own, created with a CU mask, so no other stream's
// work queues behind it on a shared hardware queue.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <new>
#include <vector>

#include "bloom_common.hpp"
#include "probe_server.hpp"

using namespace adl_dev;

namespace {

constexpr uint32_t kSlots = 64;      // one per lane of the server wave
constexpr uint32_t kSlotBytes = 512;
constexpr uint32_t kHdrBytes = 16;   // seq (unused by the device), n, k, key bytes
constexpr uint32_t kRangeOff = kHdrBytes;                      // u64 begin, end per query
constexpr uint32_t kKoffOff = kRangeOff + 16 * adl_srv::kMaxQ;  // u16 offsets, kMaxQ + 1
constexpr uint32_t kKeyOff = kKoffOff + 2 * (adl_srv::kMaxQ + 8);
static_assert(kKeyOff % 16 == 0 && kKeyOff + adl_srv::kMaxKeyBytes + 16 <= kSlotBytes, "slot layout");

struct Slot {
  uint32_t seq, n, k, key_bytes;
  uint64_t range[2 * adl_srv::kMaxQ];
  uint16_t koff[adl_srv::kMaxQ + 8];
  uint8_t keys[kSlotBytes - kKeyOff];
};
static_assert(sizeof(Slot) == kSlotBytes, "slot size");

struct Done {
  uint32_t seq;
  uint32_t tagged;  // (seq << 8) | answer bits
  uint32_t pad[14];
};
static_assert(sizeof(Done) == 64, "done line");
static_assert(adl_srv::kMaxQ == 8, "a done word holds 8 answer bits");

struct Ctl {
  uint32_t stop[16];  // replicated: lane l reads stop[l % 16] (a per-lane, vector load)
  uint32_t alive;     // host: 1 before a launch; kernel: 0 as it returns
  uint32_t pad[15];
};

// The shared area, one hipHostMalloc (mapped, coherent): bells, control, done
// lines, slots.
struct Area {
  uint32_t bell[kSlots];
  Ctl ctl;
  Done done[kSlots];
  Slot slot[kSlots];
};

__device__ __forceinline__ uint32_t ld_sys(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz

// One wave.  Lane l polls bell l; LDS holds a copy of every pending slot.
__global__ __launch_bounds__(64) void probe_server_kernel(Area *area, uint64_t idle_ticks, uint64_t life_ticks) {
  __shared__ __attribute__((aligned(16))) uint8_t lslot[kSlots][kSlotBytes];
  __shared__ uint8_t lans[kSlots][adl_srv::kMaxQ];
  const uint32_t lane = threadIdx.x;
  uint32_t served = __hip_atomic_load(&area->done[lane].seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t0 = now_ticks();
  uint64_t last = t0;
  for (;;) {
    const uint32_t bell = ld_sys(&area->bell[lane]);
    const bool pend = bell != served;
    const uint64_t pm = __ballot(pend);
    if (pm == 0) {
      const uint64_t t = now_ticks();
      const bool stop = __ballot(ld_sys(&area->ctl.stop[lane & 15]) != 0) != 0;
      if (stop || t - last > idle_ticks || t - t0 > life_ticks) break;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the slots were written before their bells
    // copy every pending slot into LDS: 8 bytes per lane per slot, 8 slots' loads in flight at a time
    for (uint64_t m = pm; m;) {
      uint32_t js[8];
      uint64_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        js[u] = m ? (uint32_t)__builtin_ctzll(m) : kSlots;
        m &= m - 1;  // (m = 0 stays 0)
        const uint64_t *src = reinterpret_cast<const uint64_t *>(&area->slot[js[u] < kSlots ? js[u] : 0]);
        v[u] = __hip_atomic_load(src + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (js[u] < kSlots) reinterpret_cast<uint64_t *>(lslot[js[u]])[lane] = v[u];
    }
    __syncthreads();
    // one lane per (slot, query): slot j's query q is lane (q * 64 + j) % ...;
    // simply: every lane walks the pending slots and takes query `lane % kMaxQ`
    // of slot (8 * r + lane / kMaxQ) in round r
    const uint32_t npend = __popcll(pm);
    for (uint32_t r = 0; r * (64 / adl_srv::kMaxQ) < npend; ++r) {
      const uint32_t which = r * (64 / adl_srv::kMaxQ) + lane / adl_srv::kMaxQ;  // index among pending slots
      const uint32_t q = lane % adl_srv::kMaxQ;
      if (which >= npend) continue;
      uint64_t m = pm;
      for (uint32_t s = 0; s < which; ++s) m &= m - 1;
      const uint32_t j = __builtin_ctzll(m);
      const Slot &sl = *reinterpret_cast<const Slot *>(lslot[j]);
      const uint32_t n = min(sl.n, adl_srv::kMaxQ);
      if (q >= n) continue;
      const uint32_t k = min(sl.k, 30u);
      const uint64_t b0 = sl.range[2 * q], b1 = sl.range[2 * q + 1];
      // 0 for an empty range or a filter of 2^31 bits or more (src/filter_block.cpp:50)
      const uint32_t mbits = b1 > b0 && b1 - b0 <= 0x0fffffffull ? (uint32_t)((b1 - b0) * 8) : 0u;
      uint8_t hit = 0;
      const uint32_t ko = min((uint32_t)sl.koff[q], adl_srv::kMaxKeyBytes);
      const uint32_t ke = min(max((uint32_t)sl.koff[q + 1], ko), adl_srv::kMaxKeyBytes);
      if (mbits) {
        uint32_t h1, h2;
        hash_bytes(sl.keys + ko, ke - ko, kSeed1, kSeed2, h1, h2);
        const FastMod mod = fastmod_for(mbits);
        const uint8_t *bm = reinterpret_cast<const uint8_t *>(b0);
        // all reads in flight together (the answer is the AND of the k bits,
        // src/filter_block.cpp:54-59; the early exit changes no answer); bits
        // past k repeat bit 0
        uint32_t all = 1;
#pragma unroll
        for (uint32_t g = 0; g < 30; ++g) {
          const uint32_t p = fastmod(h1 + (g < k ? g : 0u) * h2, mod);
          all &= (uint32_t)(bm[p >> 3] >> (p & 7));
        }
        hit = (uint8_t)(all & 1u);
      }
      lans[j][q] = hit;
    }
    __syncthreads();
    // the answers: one 8-byte system-scope store (a plain store can sit in the
    // device's write path while the wave keeps polling: the host then sees it
    // only when the kernel ends)
    if (pend) {
      uint32_t bits = 0;
#pragma unroll
      for (uint32_t q = 0; q < adl_srv::kMaxQ; ++q) bits |= (uint32_t)(lans[lane][q] & 1u) << q;
      const uint64_t v = (uint64_t)bell | ((uint64_t)((bell << 8) | bits) << 32);
      __hip_atomic_store(reinterpret_cast<uint64_t *>(&area->done[lane]), v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      served = bell;
    }
    last = now_ticks();
  }
  if (lane == 0) __hip_atomic_store(&area->ctl.alive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

namespace adl_srv {

struct Server {
  Area *host = nullptr;  // mapped, coherent
  Area *dev = nullptr;   // its device address
  hipStream_t stream = nullptr;
  hipEvent_t exited = nullptr;  // completes when the running kernel returns
  bool launched = false;
  int device = 0;
  std::mutex launch_mu;
  std::mutex slot_mu[kSlots];
  uint32_t seq[kSlots] = {};
  std::atomic<uint32_t> next_slot{0};
  uint64_t id = 0;  // unique per server of this process (a thread's slot is per server)
  uint64_t idle_ticks = 0, life_ticks = 0;
};

namespace {

void set_stop(Server *s, uint32_t v) {
  for (uint32_t &w : s->host->ctl.stop) __atomic_store_n(&w, v, __ATOMIC_SEQ_CST);
}

std::mutex g_reg_mu;
std::vector<Server *> *g_reg = nullptr;

void stop_all_at_exit() {
  std::lock_guard<std::mutex> g(g_reg_mu);
  if (!g_reg) return;
  for (Server *s : *g_reg) {
    set_stop(s, 1);
    if (s->launched) (void)hipEventSynchronize(s->exited);
  }
}

uint64_t env_us(const char *name, uint64_t dflt) {
  const char *e = getenv(name);
  return e ? strtoull(e, nullptr, 10) : dflt;
}

// Launch a server kernel unless one is running (caller holds launch_mu).
int ensure_running(Server *s) {
  if (s->launched) {
    const hipError_t q = hipEventQuery(s->exited);
    if (q == hipErrorNotReady) return ADL_OK;
    if (q != hipSuccess) {
      (void)hipGetLastError();
      return ADL_ERR_DEVICE;
    }
  }
  set_stop(s, 0);
  __atomic_store_n(&s->host->ctl.alive, 1u, __ATOMIC_SEQ_CST);
  hipExtLaunchKernelGGL(probe_server_kernel, dim3(1), dim3(64), 0, s->stream, nullptr, s->exited, 0, s->dev,
                        s->idle_ticks, s->life_ticks);
  if (hipGetLastError() != hipSuccess) return ADL_ERR_DEVICE;
  s->launched = true;
  return ADL_OK;
}

}  // namespace

Server *create() {
  auto *s = new (std::nothrow) Server;
  if (!s) return nullptr;
  auto fail = [&]() -> Server * {
    if (s->exited) (void)hipEventDestroy(s->exited);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    if (s->host) (void)hipHostFree(s->host);
    (void)hipGetLastError();
    delete s;
    return nullptr;
  };
  static std::atomic<uint64_t> next_id{1};
  s->id = next_id.fetch_add(1);
  if (hipGetDevice(&s->device) != hipSuccess) return fail();
  void *d = nullptr;
  if (hipHostMalloc((void **)&s->host, sizeof(Area), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer(&d, s->host, 0) != hipSuccess)
    return fail();
  memset(s->host, 0, sizeof(Area));
  s->dev = static_cast<Area *>(d);
  // a CU-masked stream gets a hardware queue of its own (all CUs enabled)
  std::vector<uint32_t> mask((adl_host::device_cus() + 31) / 32, ~0u);
  if (hipExtStreamCreateWithCUMask(&s->stream, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
    (void)hipGetLastError();
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) return fail();
  }
  if (hipEventCreateWithFlags(&s->exited, hipEventDisableTiming) != hipSuccess) return fail();
  // 100 MHz ticks: idle 2 ms, life 20 ms by default
  s->idle_ticks = env_us("ADL_BLOOM_SERVER_IDLE_US", 2000) * 100;
  s->life_ticks = env_us("ADL_BLOOM_SERVER_LIFE_US", 20000) * 100;
  std::lock_guard<std::mutex> g(g_reg_mu);
  if (!g_reg) {
    g_reg = new std::vector<Server *>;
    atexit(stop_all_at_exit);
  }
  g_reg->push_back(s);
  return s;
}

void destroy(Server *s) {
  if (!s) return;
  {
    std::lock_guard<std::mutex> g(g_reg_mu);
    for (auto it = g_reg->begin(); it != g_reg->end(); ++it)
      if (*it == s) {
        g_reg->erase(it);
        break;
      }
  }
  set_stop(s, 1);
  if (s->launched) (void)hipEventSynchronize(s->exited);
  (void)hipEventDestroy(s->exited);
  (void)hipStreamDestroy(s->stream);
  (void)hipHostFree(s->host);
  (void)hipGetLastError();
  delete s;
}

bool eligible(uint64_t n, uint64_t key_bytes) { return n >= 1 && n <= kMaxQ && key_bytes <= kMaxKeyBytes; }

int probe(Server *s, const uint8_t *h_keys, const uint64_t *h_offsets, uint32_t key_stride, uint64_t n,
          const uint64_t *range, uint32_t k, uint8_t *h_out) {
  const uint64_t key_bytes = h_offsets ? h_offsets[n] - h_offsets[0] : n * (uint64_t)key_stride;
  if (!s || !eligible(n, key_bytes)) return ADL_ERR_INVALID_ARG;
  // a slot per thread and server (round-robin); threads beyond kSlots share
  // one in turn.  A thread remembers its slot for the server it used last.
  thread_local uint64_t my_server = 0;
  thread_local uint32_t my = 0;
  if (my_server != s->id) {
    my = s->next_slot.fetch_add(1) % kSlots;
    my_server = s->id;
  }
  std::lock_guard<std::mutex> slot_guard(s->slot_mu[my]);
  Slot &sl = s->host->slot[my];
  sl.n = (uint32_t)n;
  sl.k = k;
  sl.key_bytes = (uint32_t)key_bytes;
  for (uint64_t q = 0; q < n; ++q) {
    sl.range[2 * q] = range[2 * q];
    sl.range[2 * q + 1] = range[2 * q + 1];
    sl.koff[q] = (uint16_t)(h_offsets ? h_offsets[q] - h_offsets[0] : q * key_stride);
  }
  sl.koff[n] = (uint16_t)key_bytes;
  memcpy(sl.keys, h_keys + (h_offsets ? h_offsets[0] : 0), key_bytes);
  const uint32_t seq = ++s->seq[my] == 0 ? ++s->seq[my] : s->seq[my];  // never 0 (the initial done)
  __atomic_store_n(&s->host->bell[my], seq, __ATOMIC_SEQ_CST);
  // a running kernel keeps alive at 1 (cheaper than querying its event every
  // call); one that is just exiting is caught by the 50 us check below
  if (!__atomic_load_n(&s->host->ctl.alive, __ATOMIC_ACQUIRE)) {
    std::lock_guard<std::mutex> g(s->launch_mu);
    if (int rc = ensure_running(s)) return rc;
  }
  volatile Done *dn = &s->host->done[my];
  const auto t0 = std::chrono::steady_clock::now();
  auto since = [&] { return std::chrono::steady_clock::now() - t0; };
  uint32_t spins = 0;
  uint32_t bits = 0;
  for (;;) {
    const uint32_t w = __atomic_load_n(&dn->tagged, __ATOMIC_ACQUIRE);
    if ((w >> 8) == (seq & 0xFFFFFFu)) {
      bits = w & 0xFFu;
      break;
    }
    __builtin_ia32_pause();
    if (++spins % 4096) continue;
    // not answered yet: a server that exited (idle / life limit) before it saw
    // this bell is relaunched; a failed one fails the call
    if (since() > std::chrono::microseconds(50)) {
      std::lock_guard<std::mutex> g(s->launch_mu);
      if (int rc = ensure_running(s)) return rc;
    }
    if (since() > std::chrono::seconds(2)) return ADL_ERR_DEVICE;
  }
  for (uint64_t q = 0; q < n; ++q) h_out[q] = (uint8_t)((bits >> q) & 1u);
  return ADL_OK;
}

}  // namespace adl_srv
