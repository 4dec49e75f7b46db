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
//   slot j (512 B)   queries (<= kMaxQ), per query the absolute device range
//                    [begin, end) of its filter in the cache arena and its k
//                    (the probe count of the block's own bits_per_key), key
//                    offsets and key bytes; written by the host thread holding
//                    slot j
//   bell[j] (u32)    request sequence number (bit 31: the request is inline),
//                    written after the request (release); the 64 bells share
//                    256 bytes, so one wave-wide load polls every slot
//   line[j] (64 B)   slots 0-3 only (the first four threads that probe): a
//                    one-query request with a key of up to 40 bytes sits
//                    here, beside its sequence number and a check word.  The
//                    four lines are read in the same round trip as the bells
//                    (one more 4-byte load per lane), so such a request costs
//                    no second read across PCIe: single-key Gets 7.4-7.8 ->
//                    6.4-6.6 us median (profiles/r05/r05srv_inline_ab.txt;
//                    sixteen lines, four loads per lane, measured 9.0).  A
//                    line read while the host was writing it fails its check
//                    (a position-dependent hash of the other 15 words) and is
//                    read again at the next poll
//   done[j] (64 B)   word 0: the served sequence number (a restarted kernel's
//                    starting point); word 1: the low 24 bits of that number
//                    above the 8 answer bits.  Both in one 8-byte system-scope
//                    store; the host takes its answers from word 1 alone
//
// The wave polls the bells and the inline lines, copies pending slots into LDS
// four at a time (one load per lane per slot, one round trip for the group;
// an inline request is copied from the lines already in LDS), hashes each query's
// key from LDS (hash_lds: 8-byte LDS reads and alignbyte), tests its k bits in
// the arena with six loads in flight at once, and writes the answers with the
// sequence numbers.  The host thread spins on its done line.
//
// Lifetime.  The kernel leaves when it has been idle for idle_ticks, when it
// has run for life_ticks, or when the host raises ctl->stop (cache teardown),
// so its wave always finishes.  Leaving, it clears ctl->alive and then polls
// once more, serving what it finds.  A host thread rings its bell and then
// reads alive: 1 means the kernel's next poll sees the bell; 0 means it waits
// for the kernel to end (that last poll may have answered it) and launches a
// new one if not.  So an exit costs a request one relaunch, never a timeout;
// the unanswered-for-50-us check is left for a kernel that failed (its
// completion event reports the error: ADL_ERR_DEVICE).
//
// Footprint.  2.25 KiB of LDS and 32 VGPRs: the wave fits on a CU beside a
// build's persistent pass-A workgroup, which leaves exactly that free, so a
// Get is served while a compaction builds (reference: DB::Get probes filters
// without a lock while DoCompaction runs, src/db.cpp:164-172, 263, 294).  The
// server runs on a stream of its own at the highest priority, so no other
// stream's work queues behind it on a shared hardware queue (Server::create).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <new>
#include <vector>

#include "bloom_common.hpp"
#include "probe_server.hpp"

using namespace adl_dev;

namespace {

constexpr uint32_t kSlots = 64;      // one per lane of the server wave
constexpr uint32_t kSlotBytes = 512;
constexpr uint32_t kGroup = 4;       // slots staged in LDS at a time (2 KiB)
constexpr uint32_t kHdrBytes = 16;   // seq (unused by the device), n, (unused), key bytes
constexpr uint32_t kInlineSlots = 4;       // slots whose one-query requests can sit in their bell line
constexpr uint32_t kInlineKeyBytes = 40;
constexpr uint32_t kInlineBit = 0x80000000u;  // in a bell: the request is in the slot's line
// In a bell: the cache arena changed since the server last dropped its
// cached copies of it (a put published a block): the wave invalidates its
// caches (a system-scope acquire) before it reads any filter bits of that
// poll.  Round 5 did so after every poll that found a request, which dropped
// the L2 of the server's XCD under a co-running build ~100 000 times a second
// (pass B 10 % slower beside Gets, profiles/r06/).
constexpr uint32_t kInvalidateBit = 0x40000000u;
constexpr uint32_t kSeqMask = 0x3FFFFFFFu;
constexpr uint32_t kLineCheck = 0x5EED5EEDu;  // the XOR of line_word_hash over a line's 16 words
constexpr uint32_t kRangeOff = kHdrBytes;                      // u64 begin, end per query
constexpr uint32_t kKoffOff = kRangeOff + 16 * adl_srv::kMaxQ;  // u16 offsets, kMaxQ + 1
constexpr uint32_t kKeyOff = kKoffOff + 2 * (adl_srv::kMaxQ + 8);
static_assert(kKeyOff % 16 == 0 && kKeyOff + adl_srv::kMaxKeyBytes + 16 <= kSlotBytes, "slot layout");

struct Slot {
  uint32_t seq, n, unused, key_bytes;
  uint64_t range[2 * adl_srv::kMaxQ];
  uint16_t koff[adl_srv::kMaxQ + 1];
  uint8_t kq[adl_srv::kMaxQ];  // per query: k
  uint8_t pad[2 * (adl_srv::kMaxQ + 8) - 2 * (adl_srv::kMaxQ + 1) - adl_srv::kMaxQ];
  uint8_t keys[kSlotBytes - kKeyOff];
};
static_assert(offsetof(Slot, keys) == kKeyOff, "slot layout");
static_assert(sizeof(Slot) == kSlotBytes, "slot size");

struct Done {
  uint32_t seq;
  uint32_t tagged;  // (seq << 8) | answer bits
  uint32_t pad[14];
};
static_assert(sizeof(Done) == 64, "done line");

// A one-query request inline in its slot's bell line: check = kLineCheck ^ the
// XOR of line_word_hash(w_i, i) over the other 15 words (the sequence number
// included).  The hash depends on the word's position and mixes its bits, so
// a line torn between two requests (read while the host wrote it: new words
// beside old ones) fails the check unless a 32-bit hash collides -- a plain
// XOR lets two words that change by the same delta cancel.
struct Line {
  uint32_t seq;    // the bell value of this request
  uint32_t check;
  uint32_t k_klen;  // k | key bytes << 8
  uint32_t len;     // filter range bytes
  uint64_t begin;   // filter range start (device address in the cache arena)
  uint8_t key[kInlineKeyBytes];
};
static_assert(sizeof(Line) == 64, "line size");
static_assert(adl_srv::kMaxQ == 8, "a done word holds 8 answer bits");

struct Ctl {
  uint32_t stop[16];  // replicated: lane l reads stop[l % 16] (a per-lane, vector load)
  uint32_t alive;     // host: 1 before a launch; kernel: 0 as it leaves (before its last poll)
  uint32_t gen_done;  // kernel: its launch generation, after its last poll's answers
  uint32_t gen_started;  // kernel: its launch generation, as it starts (after setting alive)
  uint32_t pad[13];
};

// The shared area, one hipHostMalloc (mapped, coherent): bells, control, done
// lines, slots.
struct Area {
  uint32_t bell[kSlots];
  Line line[kInlineSlots];
  Ctl ctl;
  Done done[kSlots];
  Slot slot[kSlots];
};

// murmur3's finaliser of the word XOR a per-position constant (0 for the
// check word, which is the result): host and device compute the same.
__host__ __device__ __forceinline__ uint32_t line_word_hash(uint32_t w, uint32_t i) {
  if (i == 1) return 0u;
  uint32_t h = w ^ (0x9E3779B9u * (i + 1u));
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ uint32_t ld_sys(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz

// A query staged in LDS, in two phases (timed apart by the kernel): its hash
// pair and divisor, then the k bit reads of its filter range [b0, b1).
struct Prep {
  uint64_t b0;
  uint32_t k, mbits, h1, h2;
};

// The key is at byte `off` of the LDS words `stage` (8-byte aligned, 8 bytes
// of slack after the key): hash_lds reads it with ds_read_b64 + alignbyte
// (round 5 hashed it through a byte pointer: four LDS byte reads per word).
__device__ __forceinline__ Prep prep_query(uint32_t k, uint64_t b0, uint64_t b1, const uint32_t *stage, uint32_t off,
                                           uint32_t klen) {
  Prep p{b0, min(k, 30u), 0u, 0u, 0u};
  // 0 for an empty range or a filter of 2^31 bits or more (src/filter_block.cpp:50)
  p.mbits = b1 > b0 && b1 - b0 <= 0x0fffffffull ? (uint32_t)((b1 - b0) * 8) : 0u;
  if (p.mbits) hash_lds(stage, off, klen, p.h1, p.h2);
  return p;
}

// 1 iff all k bits are set (0 for an empty range).  Six reads in flight: k
// of the default bits_per_key (10) in one round, and five fewer VGPRs spilled
// than with eight (profiles/r06/server/reads_in_flight_8_vs_6.txt: the same
// latency within noise)
constexpr uint32_t kReads = 6;
__device__ __forceinline__ uint32_t read_bits(const Prep &p) {
  if (!p.mbits) return 0;
  const FastMod mod = fastmod_for(p.mbits);
  const uint8_t *bm = reinterpret_cast<const uint8_t *>(p.b0);
  // the answer is the AND of the k bits (src/filter_block.cpp:54-59; the
  // early exit changes no answer): kReads reads in flight at a time
  uint32_t all = 1;
  for (uint32_t g = 0; g < p.k; g += kReads) {
    uint32_t w[kReads];
#pragma unroll
    for (uint32_t u = 0; u < kReads; ++u) {
      const uint32_t q = fastmod(p.h1 + (g + u < p.k ? g + u : 0u) * p.h2, mod);  // past k: bit 0 again
      w[u] = (uint32_t)(bm[q >> 3] >> (q & 7));
    }
#pragma unroll
    for (uint32_t u = 0; u < kReads; ++u) all &= w[u];
  }
  return all & 1u;
}

// Query q of a slot staged in LDS (the slot's keys end 16 bytes before it does).
__device__ __forceinline__ Prep prep_slot_query(const Slot &sl, uint32_t q) {
  const uint32_t ko = min((uint32_t)sl.koff[q], adl_srv::kMaxKeyBytes);
  const uint32_t ke = min(max((uint32_t)sl.koff[q + 1], ko), adl_srv::kMaxKeyBytes);
  return prep_query(sl.kq[q], sl.range[2 * q], sl.range[2 * q + 1], reinterpret_cast<const uint32_t *>(&sl),
                    kKeyOff + ko, ke - ko);
}

// The request of line i staged in LDS (lines: the LDS copy of all of them,
// with slack words after the last).
__device__ __forceinline__ Prep prep_line(const uint32_t *lines, uint32_t i) {
  const Line &ln = *reinterpret_cast<const Line *>(lines + 16 * i);
  return prep_query(ln.k_klen & 0xFFu, ln.begin, ln.begin + ln.len, lines, 64u * i + (uint32_t)offsetof(Line, key),
                    min(ln.k_klen >> 8, kInlineKeyBytes));
}

// One wave.  Lane l polls bell l.  Pending slots are staged kGroup at a time
// in 2 KiB of LDS (one 8-byte load per lane per slot, all in flight at once);
// lane 8u + q then answers query q of the group's slot u.  The small footprint
// (2.25 KiB of LDS, 32 VGPRs) lets the wave run beside a build's persistent
// workgroups, which leave exactly that much of their CU free (bloom_build.hip,
// kLdsReserveWords): a Get does not wait for a build.  amdgpu_num_vgpr(16) is
// doubled for gfx950's unified register file (as kPassARegs' 60 -> 120): the
// code object's .vgpr_count is 32.  Unconstrained the kernel would take 63, so
// 13 VGPRs spill to scratch (52 B per lane, with the phase stamps): kernel arguments and loop state,
// reloaded once per poll and once per served group, from the L1/L2 the wave
// alone uses.  tools/kernel_resources.py prints both from the built library
// and tests/test_kernel_resources.py pins them (no other product kernel on the
// headline, probe or var-len paths spills).
__global__ __launch_bounds__(64) __attribute__((amdgpu_num_vgpr(16))) void probe_server_kernel(
    Area *area, uint64_t idle_ticks, uint64_t life_ticks, uint32_t gen) {
  __shared__ __attribute__((aligned(16))) uint8_t lslot[kGroup][kSlotBytes];
  __shared__ __attribute__((aligned(16))) uint32_t lline[kInlineSlots * 16 + 4];  // the lines of the last poll (+ hash_lds slack)
  const uint32_t lane = threadIdx.x;
  // a successor queued behind a running kernel (Server::launcher) announces
  // itself: alive again, and its generation started
  if (lane == 0) {
    __hip_atomic_store(&area->ctl.alive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&area->ctl.gen_started, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
  uint32_t served = __hip_atomic_load(&area->done[lane].seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t0 = now_ticks();
  uint64_t last = t0, tprev = t0;
  bool closing = false;
  uint32_t closing_polls = 0, idle_polls = 0;
  // (Two polls in flight -- poll i + 2 issued before poll i is examined --
  // would halve the wait for a bell, but the wave has no registers for them:
  // the compiler spilled the in-flight values and waited for each load before
  // its spill store, serialising the polls again.)
  for (;;) {
    const uint64_t tp = now_ticks();  // this poll (diagnostics: the gap since the previous one)
    const uint32_t bell = ld_sys(&area->bell[lane]);
    // the inline lines, in the same round trip: lane l reads word l % 16 of
    // line l / 16
    const uint32_t lw = ld_sys(reinterpret_cast<const uint32_t *>(area->line) + lane);
    bool pend = bell != served;
    if (__ballot(pend && (bell & kInlineBit)) != 0) {
      // some request is inline: the lines into LDS; line i is checked across
      // lanes 16i .. 16i + 15 and judged by lane i
      lline[lane] = lw;
      uint32_t x = line_word_hash(lw, lane & 15);
#pragma unroll
      for (uint32_t o = 1; o < 16; o <<= 1) x ^= (uint32_t)__shfl_xor((int)x, (int)o);
      const uint32_t xi = (uint32_t)__shfl((int)x, (int)(16 * (lane & (kInlineSlots - 1))));
      const uint32_t si = (uint32_t)__shfl((int)lw, (int)(16 * (lane & (kInlineSlots - 1))));
      const uint32_t ci = (uint32_t)__shfl((int)lw, (int)(16 * (lane & (kInlineSlots - 1)) + 1));
      __syncthreads();
      if (pend && (bell & kInlineBit)) pend = lane < kInlineSlots && si == bell && (xi ^ ci) == kLineCheck;
      // (a torn or stale line is read again at the next poll)
    }
    // a rung bell whose line failed its check: read again, also when closing
    // (a bounded number of polls: the host writes the line before its bell)
    const bool torn = __ballot(bell != served && !pend) != 0 && (!closing || ++closing_polls < 4096);
    const uint64_t pm = __ballot(pend);
    const uint64_t t_polled = now_ticks();  // (the poll's loads have returned: pm depends on them)
    const bool last_poll = closing;  // a poll issued after alive was cleared
    if (pm == 0) {
      if (last_poll && !torn) break;
      const uint64_t t = tp;
      tprev = tp;
      // the stop word: a second PCIe read after an empty poll, so only every
      // 8th one (round 5 read it after every empty poll: a poll period of
      // ~3.1 us instead of ~2; reading it with the bells made every poll
      // 1.1 us slower, profiles/r06/)
      const bool stop = !closing && (++idle_polls & 7u) == 0 && __ballot(ld_sys(&area->ctl.stop[lane & 15]) != 0) != 0;
      if (!closing && (stop || t - last > idle_ticks || t - t0 > life_ticks)) {
        // Leaving: alive = 0 first, then one more poll, whose bells are
        // served before the wave ends.  A host thread rings its bell and then
        // reads alive (both sequentially consistent): if it read 1, this
        // poll sees its bell; if it read 0, it waits for this kernel to end
        // and relaunches only if its request is still unanswered.
        if (lane == 0) __hip_atomic_store(&area->ctl.alive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
        closing = true;
        continue;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    // (the slots and their keys are read below with system-scope loads issued
    // after this poll's bells came back, so they are at least as new as the
    // bells; only the arena's bits can be stale in this wave's caches)
    if (__ballot(pend && (bell & kInvalidateBit)) != 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    for (uint64_t m = pm; m;) {
      uint32_t js[kGroup];
      uint64_t v[kGroup];
#pragma unroll
      for (uint32_t u = 0; u < kGroup; ++u) {
        js[u] = m ? (uint32_t)__builtin_ctzll(m) : kSlots;
        m &= m - 1;  // (m = 0 stays 0)
        // (an inline request's slot is not read: its line is in LDS)
        // (js[u] is wave-uniform: a v_readlane, not an LDS permute round trip)
        const uint32_t bj = __builtin_amdgcn_readlane(bell, js[u] < kSlots ? js[u] : 0u);
        const uint64_t *src = reinterpret_cast<const uint64_t *>(&area->slot[js[u] < kSlots ? js[u] : 0]);
        v[u] = js[u] < kSlots && !(bj & kInlineBit) ? __hip_atomic_load(src + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                                     : 0ull;
      }
#pragma unroll
      for (uint32_t u = 0; u < kGroup; ++u) reinterpret_cast<uint64_t *>(lslot[u])[lane] = v[u];
      __syncthreads();
      const uint32_t u = lane / adl_srv::kMaxQ, q = lane % adl_srv::kMaxQ;
      uint32_t j = kSlots;  // the slot lane 8u + q serves (kSlots: none)
#pragma unroll
      for (uint32_t x = 0; x < kGroup; ++x) j = u == x ? js[x] : j;
      const uint64_t t_stage = now_ticks();
      Prep pr{0ull, 0u, 0u, 0u, 0u};
      const uint32_t bj = (uint32_t)__shfl((int)bell, (int)(j < kSlots ? j : 0u));
      if (j < kSlots && (bj & kInlineBit)) {
        if (q == 0) pr = prep_line(lline, j & (kInlineSlots - 1));
      } else if (j < kSlots) {
        const Slot &sl = *reinterpret_cast<const Slot *>(lslot[u]);
        if (q < min(sl.n, adl_srv::kMaxQ)) pr = prep_slot_query(sl, q);
      }
      asm volatile("" ::"v"(pr.h1), "v"(pr.h2));  // the hashes are done before the stamp
      const uint64_t t_hash = now_ticks();
      const uint32_t hit = read_bits(pr);
      asm volatile("" ::"v"(hit));  // the bit reads have returned before the stamp
      const uint64_t t_reads = now_ticks();
      const uint64_t hb = __ballot(hit != 0);
      // lane u < kGroup answers slot js[u]: {seq, (seq << 8) | answer bits} in
      // one 8-byte system-scope store (a plain store can sit in the device's
      // write path while the wave keeps polling)
      uint32_t ju = kSlots;
#pragma unroll
      for (uint32_t x = 0; x < kGroup; ++x) ju = lane == x ? js[x] : ju;
      const uint32_t seq = (uint32_t)__shfl((int)bell, (int)(ju < kSlots ? ju : 0u));
      if (ju < kSlots) {
        const uint32_t bits = (uint32_t)(hb >> (lane * adl_srv::kMaxQ)) & 0xFFu;
        const uint64_t word = (uint64_t)seq | ((uint64_t)((seq << 8) | bits) << 32);
        __hip_atomic_store(reinterpret_cast<uint64_t *>(&area->done[ju]), word, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        // phase stamps (10-ns ticks from the poll that found the request; the
        // host folds them into adl_bloom_probe_server_phases at the slot's
        // next request, and prints them for a slow one under ADL_BLOOM_DEBUG):
        // {seq, gap since the previous poll}, {poll loads back, slot staged},
        // {hashed, bits read}, {answer stored, seq}, {the poll's start and the
        // answer's store on the kernel's clock (low 32 bits), the host
        // relates them to its own clock to place a slow request's delay}
        const uint64_t ta = now_ticks();
        uint64_t *dg = reinterpret_cast<uint64_t *>(&area->done[ju].pad[0]);
        auto w2 = [](uint64_t a, uint64_t b) { return (uint64_t)(uint32_t)a | ((uint64_t)(uint32_t)b << 32); };
        __hip_atomic_store(dg + 0, w2(seq, tp - tprev), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(dg + 1, w2(t_polled - tp, t_stage - tp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(dg + 2, w2(t_hash - tp, t_reads - tp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(dg + 4, w2(tp, ta), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(dg + 3, w2(ta - tp, seq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      __syncthreads();  // the group's LDS copy is read before the next group overwrites it
    }
    if (pend) served = bell;
    last = now_ticks();
    tprev = tp;
    if (last_poll && !torn) break;
  }
  // the last poll's answers are out: the host may launch the next kernel (on
  // the other stream) as soon as it sees this
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (lane == 0) __hip_atomic_store(&area->ctl.gen_done, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

namespace adl_srv {

struct Server {
  Area *host = nullptr;  // mapped, coherent
  Area *dev = nullptr;   // its device address
  hipStream_t stream = nullptr;
  // Completion events of the kernels, by generation mod 3: with a successor
  // queued behind the running kernel, the next launch re-records the event
  // of the kernel two generations back, which completed before the running
  // one started (an event still pending must not be recorded again: that left
  // hipStreamDestroy waiting at teardown now and then).
  static constexpr uint32_t kEvents = 3;
  hipEvent_t exited[kEvents] = {};
  bool launched = false;
  uint32_t gen = 0;  // the latest kernel's launch generation (Ctl::gen_done / gen_started); launch_mu
  std::atomic<uint32_t> gen_pub{0};  // the same, for lock-free readers (probe's successor check)
  int device = 0;
  std::mutex launch_mu;  // launches and gen
  std::mutex slot_mu[kSlots];
  uint32_t seq[kSlots] = {};
  uint32_t last_bell[kSlots] = {};  // the slot's previous request (its phase stamps are read at the next)
  uint32_t last_seen[kSlots] = {};  // ... and the host tick at which its answer was seen
  std::atomic<uint32_t> next_slot{0};
  uint64_t id = 0;  // unique per server of this process (a thread's slot is per server)
  uint64_t idle_ticks = 0, life_ticks = 0;
  bool debug = false;  // ADL_BLOOM_DEBUG at creation (the launcher thread must not read knobs() while a reload runs)
  bool invalidate_always = false;  // ADL_BLOOM_SERVER_INVALIDATE=1 at creation
  // the cache arena's epoch (bumped by each published put) up to which the
  // server's waves have invalidated their caches: raised by a request that
  // carried kInvalidateBit once it is answered.  A launch does not raise it
  // (a fresh wave reads through the same L2, which may hold lines cached
  // before the put).
  std::atomic<uint64_t> inv_epoch{0};
  // The launcher thread keeps one successor queued behind the running kernel
  // while requests come in, so a kernel that reaches its life limit hands
  // over to the next with no host call on any request's path (a launch call
  // stalled 0.5 ms now and then: DESIGN.md §4).  Requests ask for a successor
  // when none is queued; after a quiet period both kernels end on their idle
  // limit and nothing is relaunched until the next request.
  std::thread launcher;
  std::mutex lmu;
  std::condition_variable lcv;
  bool want_successor = false, quit = false;
};

namespace {

std::atomic<uint64_t> g_launches{0};

// adl_bloom_probe_server_phases: the kernel's phase stamps of every request
// whose stamps were read back (ticks of 10 ns), and the host's own time per
// request (ns)
struct PhaseStats {
  std::atomic<uint64_t> requests{0}, stamped{0}, host_ns{0};
  std::atomic<uint64_t> ticks[6] = {};  // gap, polled, staged, hashed, read, answered
};
PhaseStats g_phases;

// The kernel's clock (s_memrealtime, 100 MHz, low 32 bits) against the host's
// steady clock in the same 10-ns ticks: off = min over requests of (host tick
// at which an answer was seen - kernel tick at which it was stored), i.e. the
// clocks' offset plus the fastest answer delivery.  A slow request's bell
// write and answer are then placed on the kernel's clock (ADL_BLOOM_DEBUG).
struct ClockCal {
  std::atomic<uint32_t> ref{0};
  std::atomic<int32_t> best{INT32_MAX};
  std::atomic<bool> init{false}, have{false};  // init: a thread is setting ref; have: ref is set
  void sample(uint32_t host_tick, uint32_t gpu_tick) {
    const uint32_t d = host_tick - gpu_tick;
    if (!have.load(std::memory_order_acquire)) {
      bool expect = false;
      if (!init.compare_exchange_strong(expect, true)) return;  // another thread sets ref: skip this sample
      ref.store(d, std::memory_order_relaxed);
      have.store(true, std::memory_order_release);
    }
    const int32_t rel = (int32_t)(d - ref.load(std::memory_order_relaxed));
    int32_t cur = best.load(std::memory_order_relaxed);
    while (rel < cur && !best.compare_exchange_weak(cur, rel)) {
    }
  }
  bool get(uint32_t *off) const {
    if (!have.load(std::memory_order_acquire) || best.load() == INT32_MAX) return false;
    *off = ref.load() + (uint32_t)best.load();
    return true;
  }
};
ClockCal g_clock;

inline uint32_t host_tick(std::chrono::steady_clock::time_point t) {
  return (uint32_t)(std::chrono::duration_cast<std::chrono::nanoseconds>(t.time_since_epoch()).count() / 10);
}

// Fold the stamps of the slot's previous request into g_phases (they were
// stored after its answer; both copies of its sequence number must match),
// and its answer's kernel and host times into the clock calibration.
void fold_phases(const Area *a, uint32_t my, uint32_t bell, uint32_t seen_tick) {
  if (!bell) return;
  const uint64_t *dg = reinterpret_cast<const uint64_t *>(&a->done[my].pad[0]);
  const uint64_t w4 = __atomic_load_n(dg + 4, __ATOMIC_ACQUIRE);
  const uint64_t w0 = __atomic_load_n(dg + 0, __ATOMIC_ACQUIRE), w1 = __atomic_load_n(dg + 1, __ATOMIC_ACQUIRE);
  const uint64_t w2 = __atomic_load_n(dg + 2, __ATOMIC_ACQUIRE), w3 = __atomic_load_n(dg + 3, __ATOMIC_ACQUIRE);
  if ((uint32_t)w0 != bell || (uint32_t)(w3 >> 32) != bell) return;
  g_clock.sample(seen_tick, (uint32_t)(w4 >> 32));
  const uint64_t v[6] = {w0 >> 32, (uint32_t)w1, w1 >> 32, (uint32_t)w2, w2 >> 32, (uint32_t)w3};
  for (int i = 0; i < 6; ++i) g_phases.ticks[i].fetch_add(v[i], std::memory_order_relaxed);
  g_phases.stamped.fetch_add(1, std::memory_order_relaxed);
}

void set_stop(Server *s, uint32_t v) {
  for (uint32_t &w : s->host->ctl.stop) __atomic_store_n(&w, v, __ATOMIC_SEQ_CST);
}

std::mutex g_reg_mu;
std::vector<Server *> *g_reg = nullptr;

void wait_all(Server *s) {
  if (!s->launched) return;
  for (uint32_t i = 0; i < Server::kEvents && i <= s->gen; ++i) (void)hipEventSynchronize(s->exited[(s->gen - i) % Server::kEvents]);
}

void stop_launcher(Server *s) {
  {
    std::lock_guard<std::mutex> g(s->lmu);
    s->quit = true;
  }
  s->lcv.notify_one();
  if (s->launcher.joinable()) s->launcher.join();
}

// Stop a server whose launcher thread has been joined (no launch can start):
// raise stop, then wait -- on the mapped control words alone, no runtime call
// -- until the last launched generation has published gen_done.  A successor
// queued behind the running kernel (Server::launcher) has then started, seen
// stop at its first poll and left too, so no dispatch of the server's stream
// is pending when its completion events are waited for and the stream is
// torn down (a process that exited with a successor queued is
// the state the CU-masked stream's exit hang left unexplained).  With
// ADL_BLOOM_DEBUG the state found and the wait are logged.
void stop_and_drain(Server *s, const char *why) {
  const uint32_t started0 = __atomic_load_n(&s->host->ctl.gen_started, __ATOMIC_SEQ_CST);
  const uint32_t done0 = __atomic_load_n(&s->host->ctl.gen_done, __ATOMIC_SEQ_CST);
  const uint32_t alive0 = __atomic_load_n(&s->host->ctl.alive, __ATOMIC_SEQ_CST);
  set_stop(s, 1);
  const auto t0 = std::chrono::steady_clock::now();
  bool drained = !s->launched;
  while (!drained && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2)) {
    drained = __atomic_load_n(&s->host->ctl.gen_done, __ATOMIC_ACQUIRE) == s->gen;
    if (!drained) __builtin_ia32_pause();
  }
  if (s->debug)
    fprintf(stderr,
            "adl_bloom server %s: clock calibration %s (samples folded %llu); launched generation %u, started %u, "
            "done %u, alive %u (%s); %s after %.1f us\n",
            why, g_clock.have.load() ? "set" : "unset", (unsigned long long)g_phases.stamped.load(),
            s->gen, started0, done0, alive0,
            !s->launched ? "never launched"
            : started0 != s->gen ? "a successor queued, not started"
            : done0 != s->gen ? "running" : "exited",
            drained ? "drained" : "NOT drained (the runtime's completion events decide)",
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  wait_all(s);
}

void stop_all_at_exit() {
  std::lock_guard<std::mutex> g(g_reg_mu);
  if (!g_reg) return;
  for (Server *s : *g_reg) {
    stop_launcher(s);
    stop_and_drain(s, "at exit");
  }
}

bool answered(const Server *s, uint32_t my, uint32_t seq, uint32_t *bits) {
  const uint32_t w = __atomic_load_n(&s->host->done[my].tagged, __ATOMIC_ACQUIRE);
  if ((w >> 8) != (seq & 0xFFFFFFu)) return false;
  *bits = w & 0xFFu;
  return true;
}

// Launch generation s->gen + 1 behind whatever runs on the server's stream.
// Caller holds launch_mu.
int launch_next(Server *s) {
  const uint32_t gen = s->gen + 1;
  const auto tl0 = std::chrono::steady_clock::now();
  hipLaunchKernelGGL(probe_server_kernel, dim3(1), dim3(64), 0, s->stream, s->dev, s->idle_ticks, s->life_ticks, gen);
  const auto tl1 = std::chrono::steady_clock::now();
  if (hipGetLastError() != hipSuccess || hipEventRecord(s->exited[gen % Server::kEvents], s->stream) != hipSuccess)
    return ADL_ERR_DEVICE;
  if (s->debug) {
    const double us_launch = std::chrono::duration<double, std::micro>(tl1 - tl0).count();
    if (us_launch > 50.0) fprintf(stderr, "adl_bloom server: launch call of generation %u took %.1f us\n", gen, us_launch);
  }
  s->launched = true;
  s->gen = gen;
  s->gen_pub.store(gen, std::memory_order_release);
  g_launches.fetch_add(1, std::memory_order_relaxed);
  return ADL_OK;
}

// The caller saw alive == 0 after ringing bell `my` (or waited long): make
// sure a kernel will answer it.  Caller holds launch_mu.
//  * a launched kernel has not started yet (a queued successor, or a fresh
//    launch): it will poll the bell;
//  * the last launched kernel runs and alive is 1: it will poll the bell,
//    unless it has failed (its completion event says so);
//  * it cleared alive: it is in its last poll or gone: wait until it has
//    published its generation (its last answers are out by then), then
//    launch the next one unless that last poll answered the request.
// *done = answered.
int ensure_running(Server *s, uint32_t my, uint32_t seq, uint32_t *bits, bool *done) {
  *done = false;
  if (s->launched) {
    hipEvent_t ev = s->exited[s->gen % Server::kEvents];
    if (__atomic_load_n(&s->host->ctl.gen_started, __ATOMIC_SEQ_CST) != s->gen) {
      // not started yet, unless it failed (then its completion event says so)
      const hipError_t q = hipEventQuery(ev);
      if (q == hipSuccess || q == hipErrorNotReady) return ADL_OK;
      (void)hipGetLastError();
      return ADL_ERR_DEVICE;
    }
    if (__atomic_load_n(&s->host->ctl.alive, __ATOMIC_SEQ_CST)) {
      const hipError_t q = hipEventQuery(ev);
      if (q == hipErrorNotReady) return ADL_OK;
      if (q != hipSuccess) {
        (void)hipGetLastError();
        return ADL_ERR_DEVICE;
      }
    } else {
      // leaving: its generation word comes a poll later (a kernel that failed
      // in between never writes it: its event reports the error)
      const auto t0 = std::chrono::steady_clock::now();
      for (uint32_t spin = 0; __atomic_load_n(&s->host->ctl.gen_done, __ATOMIC_ACQUIRE) != s->gen; ++spin) {
        __builtin_ia32_pause();
        if (spin % 1024 == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(500)) {
          const hipError_t q = hipEventQuery(ev);
          if (q == hipSuccess) break;
          if (q != hipErrorNotReady) {
            (void)hipGetLastError();
            return ADL_ERR_DEVICE;
          }
        }
      }
    }
    if (answered(s, my, seq, bits)) {
      *done = true;
      return ADL_OK;
    }
  }
  set_stop(s, 0);
  __atomic_store_n(&s->host->ctl.alive, 1u, __ATOMIC_SEQ_CST);
  return launch_next(s);
}

// Launcher thread: on request, queue a successor behind the running kernel
// when none is queued (the last launched kernel has started) and the server
// is not being stopped.
void launcher_main(Server *s) {
  (void)hipSetDevice(s->device);
  std::unique_lock<std::mutex> lk(s->lmu);
  for (;;) {
    s->lcv.wait(lk, [&] { return s->want_successor || s->quit; });
    if (s->quit) return;
    s->want_successor = false;
    lk.unlock();
    {
      std::lock_guard<std::mutex> g(s->launch_mu);
      const bool stopping = __atomic_load_n(&s->host->ctl.stop[0], __ATOMIC_SEQ_CST) != 0;
      if (s->launched && !stopping && __atomic_load_n(&s->host->ctl.gen_started, __ATOMIC_SEQ_CST) == s->gen &&
          __atomic_load_n(&s->host->ctl.gen_done, __ATOMIC_SEQ_CST) != s->gen)
        (void)launch_next(s);  // a failure shows on the request path (its event)
    }
    lk.lock();
  }
}

}  // namespace

Server *create() {
  auto *s = new (std::nothrow) Server;
  if (!s) return nullptr;
  auto fail = [&]() -> Server * {
    for (hipEvent_t e : s->exited)
      if (e) (void)hipEventDestroy(e);
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
  // A stream of the highest priority: its hardware queue is not shared with
  // the process's ordinary streams, so no other stream's work waits behind
  // the resident kernel.  (A CU-masked stream does that too, but after a few
  // relaunches on one the process hung at exit, in the runtime's teardown,
  // every time: profiles/r05/server_stream_exit.log.)
  int lo = 0, hi = 0;
  if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
      hipStreamCreateWithPriority(&s->stream, hipStreamNonBlocking, hi) != hipSuccess) {
    (void)hipGetLastError();
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) return fail();
  }
  for (hipEvent_t &e : s->exited)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail();
  // 100 MHz ticks: idle 2 ms, life 1 s by default.  (Life was 20 ms until
  // round 5: under continuous Gets that relaunched the server 50 times a
  // second, and a relaunch while a build runs waited 0.5-1.3 ms for the new
  // wave to start: profiles/r05/r05m_coexist_life.txt.)
  s->idle_ticks = adl_host::knobs().server_idle_us * 100;
  s->life_ticks = adl_host::knobs().server_life_us * 100;
  s->debug = adl_host::knobs().debug;
  s->invalidate_always = adl_host::knobs().server_invalidate;
  try {
    s->launcher = std::thread(launcher_main, s);
  } catch (...) {
    return fail();
  }
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
  stop_launcher(s);
  stop_and_drain(s, "destroy");
  (void)hipStreamSynchronize(s->stream);
  for (hipEvent_t e : s->exited) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(s->stream);
  (void)hipHostFree(s->host);
  (void)hipGetLastError();
  delete s;
}

bool eligible(uint64_t n, uint64_t key_bytes) { return n >= 1 && n <= kMaxQ && key_bytes <= kMaxKeyBytes; }

uint64_t launches() { return g_launches.load(std::memory_order_relaxed); }

uint32_t resident_servers() {
  std::lock_guard<std::mutex> g(g_reg_mu);
  uint32_t r = 0;
  if (g_reg)
    for (const Server *s : *g_reg) r += __atomic_load_n(&s->host->ctl.alive, __ATOMIC_ACQUIRE) != 0;
  return r;
}

uint32_t live_servers() {
  std::lock_guard<std::mutex> g(g_reg_mu);
  return g_reg ? (uint32_t)g_reg->size() : 0u;
}

int probe(Server *s, const uint8_t *h_keys, const uint64_t *h_offsets, uint32_t key_stride, uint64_t n,
          const uint64_t *range, const uint8_t *kq, uint64_t arena_epoch, uint8_t *h_out) {
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
  fold_phases(s->host, my, s->last_bell[my], s->last_seen[my]);
  // 31-bit sequence numbers, never 0 (the initial done); bit 31 of the bell
  // value says where the request is
  s->seq[my] = (s->seq[my] + 1) & kSeqMask;
  if (s->seq[my] == 0) s->seq[my] = 1;
  const bool inl = my < kInlineSlots && n == 1 && key_bytes <= kInlineKeyBytes && range[1] >= range[0] &&
                   range[1] - range[0] <= 0xFFFFFFFFull;
  // the arena changed since the wave last invalidated its caches (or every
  // request invalidates: ADL_BLOOM_SERVER_INVALIDATE=1, round 5's behaviour)
  const bool inv = s->invalidate_always || arena_epoch > s->inv_epoch.load(std::memory_order_acquire);
  const uint32_t seq = s->seq[my] | (inl ? kInlineBit : 0u) | (inv ? kInvalidateBit : 0u);
  s->last_bell[my] = seq;
  const auto tw0 = std::chrono::steady_clock::now();
  const uint8_t *kp = h_keys + (h_offsets ? h_offsets[0] : 0);
  if (inl) {
    // the whole line, check word last computed, in one copy; then the bell
    Line ln{};
    ln.seq = seq;
    ln.k_klen = kq[0] | (uint32_t)key_bytes << 8;
    ln.len = (uint32_t)(range[1] - range[0]);
    ln.begin = range[0];
    memcpy(ln.key, kp, key_bytes);
    uint32_t w[16];
    memcpy(w, &ln, sizeof(ln));
    uint32_t x = kLineCheck;
    for (uint32_t i = 0; i < 16; ++i) x ^= line_word_hash(w[i], i);
    ln.check = x;
    memcpy(&s->host->line[my], &ln, sizeof(ln));
  } else {
    Slot &sl = s->host->slot[my];
    sl.n = (uint32_t)n;
    sl.key_bytes = (uint32_t)key_bytes;
    for (uint64_t q = 0; q < n; ++q) {
      sl.range[2 * q] = range[2 * q];
      sl.range[2 * q + 1] = range[2 * q + 1];
      sl.kq[q] = kq[q];
      sl.koff[q] = (uint16_t)(h_offsets ? h_offsets[q] - h_offsets[0] : q * key_stride);
    }
    sl.koff[n] = (uint16_t)key_bytes;
    memcpy(sl.keys, kp, key_bytes);
  }
  // bell, then alive, both sequentially consistent (the kernel clears alive
  // and then polls once more: probe_server_kernel)
  __atomic_store_n(&s->host->bell[my], seq, __ATOMIC_SEQ_CST);
  uint32_t bits = 0;
  bool done = false;
  const auto tb = std::chrono::steady_clock::now();
  bool relaunched = false;
  if (!__atomic_load_n(&s->host->ctl.alive, __ATOMIC_SEQ_CST)) {
    // Only if no one else is launching: the holder of launch_mu is the
    // launcher thread queueing a successor (or a thread relaunching), whose
    // kernel polls every bell.  Waiting for the lock made a Get at a hand-over
    // wait out a stalled launch call (one of 50 000 idle Gets took 709 us,
    // profiles/r05/r05f2_coexist.json); a request still unanswered after 50 us
    // takes the lock below in any case.
    std::unique_lock<std::mutex> g(s->launch_mu, std::try_to_lock);
    if (g.owns_lock()) {
      const uint32_t gen0 = s->gen;
      if (int rc = ensure_running(s, my, seq, &bits, &done)) return rc;
      relaunched = s->gen != gen0;
    }
  }
  const auto t0 = std::chrono::steady_clock::now();
  auto since = [&] { return std::chrono::steady_clock::now() - t0; };
  uint32_t spins = 0;
  // ADL_BLOOM_DEBUG: the longest stretch in which this thread did not run its
  // spin loop (an interrupt, an SMI, a stalled core: time the operating
  // system's switch counters do not see), to tell a host stall from an
  // answer that reached host memory late
  std::chrono::steady_clock::time_point tl = t0;
  double max_gap_us = 0;
  while (!done) {
    if (answered(s, my, seq, &bits)) break;
    if (s->debug) {
      const auto tn = std::chrono::steady_clock::now();
      max_gap_us = std::max(max_gap_us, std::chrono::duration<double, std::micro>(tn - tl).count());
      tl = tn;
    }
    __builtin_ia32_pause();
    if (++spins % 4096) continue;
    // unanswered for long (a kernel that failed, or one starved of its CU):
    // check the kernel; past kTimeout the caller probes by a launch instead
    if (since() > std::chrono::microseconds(50)) {
      std::lock_guard<std::mutex> g(s->launch_mu);
      if (int rc = ensure_running(s, my, seq, &bits, &done)) return rc;
    }
    if (since() > kTimeout) return kBusy;
  }
  if (s->debug) {
    // ADL_BLOOM_DEBUG: where a slow request spent its time
    const auto t1 = std::chrono::steady_clock::now();
    const double us_ring = std::chrono::duration<double, std::micro>(t0 - tb).count();
    const double us_wait = std::chrono::duration<double, std::micro>(t1 - t0).count();
    if (us_ring + us_wait > 100.0) {
      // the kernel's own view, stored after the answer: wait for it briefly
      const auto tw = std::chrono::steady_clock::now();
      while (std::chrono::steady_clock::now() - tw < std::chrono::microseconds(50)) __builtin_ia32_pause();
      const uint64_t *dg = reinterpret_cast<const uint64_t *>(&s->host->done[my].pad[0]);
      const uint64_t w0 = __atomic_load_n(dg + 0, __ATOMIC_ACQUIRE), w1 = __atomic_load_n(dg + 1, __ATOMIC_ACQUIRE);
      const uint64_t w2 = __atomic_load_n(dg + 2, __ATOMIC_ACQUIRE), w3 = __atomic_load_n(dg + 3, __ATOMIC_ACQUIRE);
      const uint64_t w4 = __atomic_load_n(dg + 4, __ATOMIC_ACQUIRE);
      // on the kernel's clock: when the bell was written, when the poll that
      // found it started, and how much later than the fastest delivery the
      // answer reached this thread
      uint32_t off = 0;
      if (g_clock.get(&off))
        fprintf(stderr,
                "adl_bloom server: slow request on the kernel's clock: the poll that found it started %.2f us after "
                "the bell was written; the answer reached the host %.2f us later than the fastest answer does; "
                "longest pause of this thread's answer wait: %.1f us\n",
                (double)(int32_t)((uint32_t)w4 + off - host_tick(tb)) / 100.0,
                (double)(int32_t)(host_tick(t1) - ((uint32_t)(w4 >> 32) + off)) / 100.0, max_gap_us);
      fprintf(stderr,
              "adl_bloom server: slow request %.1f us (alive check / relaunch %.1f us%s, answer wait %.1f us; "
              "kernel%s: %.2f us since its previous poll; from the poll that found it: loads back %.2f, "
              "staged %.2f, hashed %.2f, bits read %.2f, answered %.2f us)\n",
              us_ring + us_wait, us_ring, relaunched ? ", relaunched" : "", us_wait,
              (uint32_t)w0 == seq && (uint32_t)(w3 >> 32) == seq ? "" : " (stamps of another request)",
              (double)(w0 >> 32) / 100.0, (double)(uint32_t)w1 / 100.0, (double)(w1 >> 32) / 100.0,
              (double)(uint32_t)w2 / 100.0, (double)(w2 >> 32) / 100.0, (double)(uint32_t)w3 / 100.0);
    }
  }
  // no successor queued behind the running kernel (the last launched one has
  // started and not exited): ask the launcher for one, off this request's path
  const uint32_t g_last = s->gen_pub.load(std::memory_order_acquire);
  if (g_last && __atomic_load_n(&s->host->ctl.gen_started, __ATOMIC_RELAXED) == g_last &&
      __atomic_load_n(&s->host->ctl.gen_done, __ATOMIC_RELAXED) != g_last) {
    {
      std::lock_guard<std::mutex> g(s->lmu);
      s->want_successor = true;
    }
    s->lcv.notify_one();
  }
  s->last_seen[my] = host_tick(std::chrono::steady_clock::now());
  if (inv) {  // answered: the wave invalidated after every put up to arena_epoch
    uint64_t e = s->inv_epoch.load(std::memory_order_relaxed);
    while (e < arena_epoch && !s->inv_epoch.compare_exchange_weak(e, arena_epoch, std::memory_order_release)) {
    }
  }
  g_phases.requests.fetch_add(1, std::memory_order_relaxed);
  g_phases.host_ns.fetch_add(
      (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tw0).count(),
      std::memory_order_relaxed);
  for (uint64_t q = 0; q < n; ++q) h_out[q] = (uint8_t)((bits >> q) & 1u);
  return ADL_OK;
}

}  // namespace adl_srv

extern "C" int adl_bloom_probe_server_phases(uint64_t *requests, uint64_t *stamped, double *avg_us, int reset) {
  using adl_srv::g_phases;
  const uint64_t n = g_phases.requests.load(), ns = g_phases.stamped.load();
  if (requests) *requests = n;
  if (stamped) *stamped = ns;
  if (avg_us) {
    for (int i = 0; i < 6; ++i) avg_us[i] = ns ? (double)g_phases.ticks[i].load() / 100.0 / (double)ns : 0.0;
    avg_us[6] = n ? (double)g_phases.host_ns.load() / 1000.0 / (double)n : 0.0;
  }
  if (reset) {
    g_phases.requests = 0;
    g_phases.stamped = 0;
    g_phases.host_ns = 0;
    for (auto &t : g_phases.ticks) t = 0;
  }
  return ADL_OK;
}

extern "C" int adl_bloom_probe_server_launches(uint64_t *launches) {
  if (!launches) return ADL_ERR_INVALID_ARG;
  *launches = adl_srv::launches();
  return ADL_OK;
}
