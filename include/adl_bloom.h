/*
 * include/adl_bloom.h -- C-ABI of the MI355X (gfx950) SSTable bloom-filter
 * build/probe layer (libadlbloom.so).
 *
 * This is the drop-in boundary for the reference's filter path
 * (adlternative/adlsm-tree):
 *   - src/murmur3_hash.hpp:9        uint32_t murmur3_hash(seed, data, len)
 *   - src/filter_block.hpp:22-34    class BloomFilter : FilterAlgorithm
 *       Keys2Block(const vector<string>&, string&)   (src/filter_block.cpp:9-33)
 *       IsKeyExists(string_view key, string_view bm) (src/filter_block.cpp:49-62)
 *   - src/filter_block.hpp:36-73    FilterBlockWriter / FilterBlockReader
 * The host C++ mirror of those classes (adlsm-tree_amd/csrc/filter_block.hpp)
 * and any FFI binding (ctypes) call only what is declared
 * here: plain pointers and sizes, no C++ or torch types, no exceptions.
 *
 * Key sets are packed: `keys` is a byte buffer; key i is
 *   keys[offsets[i] .. offsets[i+1])          when offsets != NULL (n+1 entries)
 *   keys[i*key_stride .. (i+1)*key_stride)    when offsets == NULL
 * Bitmaps are the reference's bytes exactly: n*bits_per_key + 7 bytes, bit b
 * of the filter is bit (b & 7) of byte (b >> 3).
 *
 * Every function returns an adl_status (0 = OK).  All entry points are
 * re-entrant and thread-safe: work is enqueued on the caller's HIP stream
 * (`stream`, a hipStream_t) and nothing global is mutated after the
 * once-guarded device query.  Functions named *_device take device pointers
 * and do not synchronise; there NULL = the null stream.  The others take host
 * pointers and return when the results are in host memory; there NULL = a
 * non-blocking stream of the calling thread (created on first use), so calls
 * from different threads run side by side on the device instead of queueing
 * on the legacy null stream.
 */
#ifndef ADL_BLOOM_H_
#define ADL_BLOOM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ADL_BLOOM_ABI_VERSION 1

/* Status codes.  ADL_OK and ADL_FILTER_BLOCK_ERROR keep the values of the
 * reference's enum RC (src/rc.hpp:8-39: OK = 0, FILTER_BLOCK_ERROR = 13); the
 * negative codes are device/argument failures the CPU reference cannot have. */
typedef enum adl_status {
  ADL_OK = 0,
  ADL_FILTER_BLOCK_ERROR = 13, /* malformed filter block (src/filter_block.cpp:113-170) */
  ADL_ERR_INVALID_ARG = -1,    /* NULL pointer, negative bits_per_key, bad offsets/alignment */
  ADL_ERR_TOO_LARGE = -2,      /* n*bits_per_key+7 exceeds the reference's int range */
  ADL_ERR_DEVICE = -3,         /* HIP runtime / launch failure, no GPU */
  ADL_ERR_OUT_OF_MEMORY = -4,  /* device allocation failed */
  ADL_ERR_WORKSPACE = -5       /* caller workspace smaller than required */
} adl_status;

/* Human-readable text for a status (static storage). */
const char *adl_bloom_strerror(int status);

/* ABI version of the loaded library (== ADL_BLOOM_ABI_VERSION). */
int adl_bloom_abi_version(void);

/* k = (int)(bits_per_key * 0.69) clamped to [1, 30]  (src/filter_block.cpp:44-46). */
int32_t adl_bloom_num_probes(int32_t bits_per_key);

/* Bitmap size in bytes, n*bits_per_key + 7 (src/filter_block.cpp:11-14); 0 when
 * the reference's `int` arithmetic would overflow or bits_per_key < 0. */
uint64_t adl_bloom_bitmap_bytes(uint64_t n, int32_t bits_per_key);

/* Device buffer size a *_device build writes for one filter: the bitmap rounded
 * up to 16 bytes (the pad bytes are written as zero). */
uint64_t adl_bloom_bitmap_alloc_bytes(uint64_t n, int32_t bits_per_key);

/* ---------------------------------------------------------------- build */

/* Workspace (device bytes) adl_bloom_build_device / _segmented_device need for
 * filters with the given key counts (num_filters entries).  key_counts is a
 * HOST array. */
uint64_t adl_bloom_build_workspace_bytes(const uint64_t *key_counts, uint32_t num_filters,
                                         int32_t bits_per_key);

/* Build one filter from device-resident keys into a device bitmap.
 * Replaces BloomFilter::Keys2Block (src/filter_block.cpp:9-33) for a batch.
 *   d_bitmap: adl_bloom_bitmap_alloc_bytes(n, bpk) bytes, 16-byte aligned;
 *             every byte is written (no pre-zeroing needed).
 *   d_workspace: adl_bloom_build_workspace_bytes(&n, 1, bpk) bytes, 256-B aligned.
 *   d_keys: no alignment or padding is required.  When it is 16-byte aligned
 *   the kernels may load whole aligned 16-byte blocks that hold key bytes, so
 *   up to 15 bytes past the last key's end are read (never a block that holds
 *   no key byte, so never a page the keys do not touch); when it is not, every
 *   access stays inside the key bytes. */
int adl_bloom_build_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n,
                           uint32_t key_stride, int32_t bits_per_key, uint8_t *d_bitmap,
                           void *d_workspace, uint64_t workspace_bytes, void *stream);

/* Build num_filters independent filters (one per SSTable) in one pass pair
 * (split only past 2^31 / k keys, where u32 position indices would overflow).
 * Filter f owns keys [key_begin[f], key_begin[f+1]) of the key set and writes
 * its bitmap at d_bitmaps + bitmap_off[f] (16-byte aligned, room for
 * adl_bloom_bitmap_alloc_bytes(n_f, bpk)).  key_begin (num_filters+1 entries)
 * and bitmap_off (num_filters entries) are HOST arrays. */
int adl_bloom_build_segmented_device(const uint8_t *d_keys, const uint64_t *d_offsets,
                                     uint32_t key_stride, const uint64_t *key_begin,
                                     uint32_t num_filters, int32_t bits_per_key,
                                     uint8_t *d_bitmaps, const uint64_t *bitmap_off,
                                     void *d_workspace, uint64_t workspace_bytes, void *stream);

/* Flags for adl_bloom_build_segmented_device_ex. */
#define ADL_BLOOM_SKIP_ADJACENT_DUPLICATES 1u /* a key equal to the previous key of its
  filter is not hashed: same bitmap (OR is idempotent, and m still counts every key
  as Keys2Block's keys.size() does), less work when versions of one user key arrive
  in a row (memtable order, src/keys.cpp:61-74; SSTableWriter::Add, src/sstable.cpp:28) */

/* adl_bloom_build_segmented_device with flags (0 = identical to it). */
int adl_bloom_build_segmented_device_ex(const uint8_t *d_keys, const uint64_t *d_offsets,
                                        uint32_t key_stride, const uint64_t *key_begin,
                                        uint32_t num_filters, int32_t bits_per_key,
                                        uint8_t *d_bitmaps, const uint64_t *bitmap_off, uint32_t flags,
                                        void *d_workspace, uint64_t workspace_bytes, void *stream);

/* Host-pointer convenience: upload keys, build, download exactly
 * adl_bloom_bitmap_bytes(n, bpk) bytes into h_bitmap (which may be unaligned,
 * e.g. the tail of a std::string as in Keys2Block).  Synchronous.  The same
 * path as adl_bloom_build_segmented with one filter: pinned (hipHostMalloc'd /
 * registered) key and bitmap buffers are DMAed directly, pageable ones staged
 * through per-thread pinned buffers.  Replaces BloomFilter::Keys2Block
 * (src/filter_block.cpp:9-33). */
int adl_bloom_build(const uint8_t *h_keys, const uint64_t *h_offsets, uint64_t n,
                    uint32_t key_stride, int32_t bits_per_key, uint8_t *h_bitmap,
                    void *stream);

/* Host-pointer segmented build for many filters (the compaction shape: one
 * filter per SSTable, keys and bitmaps in host memory), pipelined: filters go
 * in groups (~128 MB of keys, one launch pair each) whose key upload, build
 * (on `stream`) and bitmap download overlap on three streams.  Filter f's bitmap,
 * exactly adl_bloom_bitmap_bytes(n_f, bpk) bytes, is written at
 * h_bitmaps + h_bitmap_off[f] (any alignment, e.g. packed back to back as in
 * a filter block).  Pinned (hipHostMalloc'd / registered) buffers are DMAed
 * directly; pageable ones are staged through per-thread pinned buffers.
 * key_begin (num_filters+1) and h_bitmap_off (num_filters) are HOST arrays.
 * Synchronous.  Replaces num_filters calls of BloomFilter::Keys2Block
 * (src/filter_block.cpp:9-33) from SSTableWriter::Final (src/sstable.cpp:58). */
int adl_bloom_build_segmented(const uint8_t *h_keys, const uint64_t *h_offsets, uint32_t key_stride,
                              const uint64_t *key_begin, uint32_t num_filters, int32_t bits_per_key,
                              uint8_t *h_bitmaps, const uint64_t *h_bitmap_off, void *stream);

/* adl_bloom_build_segmented with flags (ADL_BLOOM_SKIP_ADJACENT_DUPLICATES; 0 =
 * identical to it): the host side of SSTableWriter::Final (src/sstable.cpp:58),
 * whose filters hold the user keys of a memtable run, versions of one user key
 * in a row (src/sstable.cpp:28, src/keys.cpp:61-74). */
int adl_bloom_build_segmented_ex(const uint8_t *h_keys, const uint64_t *h_offsets, uint32_t key_stride,
                                 const uint64_t *key_begin, uint32_t num_filters, int32_t bits_per_key,
                                 uint8_t *h_bitmaps, const uint64_t *h_bitmap_off, uint32_t flags, void *stream);

/* ------------------------------------------------- filter block on the device */

/* Size of the filter block FilterBlockWriter::Final (src/filter_block.cpp:77-102)
 * writes for num_filters filters, filter f holding keys [key_begin[f],
 * key_begin[f+1]) (HOST array, num_filters+1 entries): the bitmaps back to back
 * (n_f*bpk+7 bytes each), then i32 offsets[F], i32 offsets_start, i32 F,
 * "bf:" + i32 bpk, i32 7.  0 on invalid input or a block beyond the
 * reference's int offsets. */
uint64_t adl_bloom_filter_block_bytes(const uint64_t *key_begin, uint32_t num_filters,
                                      int32_t bits_per_key);

/* Workspace for adl_bloom_filter_block_build_device: the build workspace plus
 * the 16-byte-aligned bitmaps before they are packed. */
uint64_t adl_bloom_filter_block_workspace_bytes(const uint64_t *key_begin, uint32_t num_filters,
                                                int32_t bits_per_key);

/* Build num_filters filters from device-resident keys and frame them as one
 * filter block in d_block (16-byte aligned, >= adl_bloom_filter_block_bytes):
 * byte-identical to FilterBlockWriter::Keys2Block() per filter followed by
 * Final() (src/filter_block.cpp:77-109), so one D2H -- or one direct file
 * write -- emits the block.  num_filters == 0 gives the 19-byte empty block. */
int adl_bloom_filter_block_build_device(const uint8_t *d_keys, const uint64_t *d_offsets,
                                        uint32_t key_stride, const uint64_t *key_begin,
                                        uint32_t num_filters, int32_t bits_per_key,
                                        uint8_t *d_block, uint64_t block_bytes, void *d_workspace,
                                        uint64_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------- probe */

/* Probe n keys against one device bitmap of bitmap_bytes bytes (the exact
 * reference length; m = bitmap_bytes*8 as in src/filter_block.cpp:50).
 * d_out[i] = 1 if key i may be present, 0 if it is certainly absent.
 * Replaces BloomFilter::IsKeyExists (src/filter_block.cpp:49-62) for a batch. */
int adl_bloom_probe_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n,
                           uint32_t key_stride, int32_t bits_per_key, const uint8_t *d_bitmap,
                           uint64_t bitmap_bytes, uint8_t *d_out, void *stream);

/* Probe n keys, key i against filter d_filter_id[i] of num_filters resident
 * bitmaps; filter f is d_bitmaps[d_bitmap_off[f] .. d_bitmap_off[f+1]) (device
 * array, num_filters+1 entries).  A filter id >= num_filters answers 0, as
 * FilterBlockReader::IsKeyExists does (src/filter_block.cpp:174). */
int adl_bloom_probe_multi_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n,
                                 uint32_t key_stride, const uint32_t *d_filter_id,
                                 uint32_t num_filters, const uint8_t *d_bitmaps,
                                 const uint64_t *d_bitmap_off, int32_t bits_per_key,
                                 uint8_t *d_out, void *stream);

/* Like adl_bloom_probe_multi_device, with filter f = d_bitmaps[d_begin[f] ..
 * d_end[f]) (device arrays, num_filters entries each): the filters may sit
 * anywhere in one device arena, in any order (adl_bloom_filter_cache). */
int adl_bloom_probe_ranges_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n,
                                  uint32_t key_stride, const uint32_t *d_filter_id,
                                  uint32_t num_filters, const uint8_t *d_bitmaps,
                                  const uint64_t *d_begin, const uint64_t *d_end,
                                  int32_t bits_per_key, uint8_t *d_out, void *stream);

/* Large-batch probe with a workspace: the answers of adl_bloom_probe_multi_device
 * (d_bitmap_end == NULL) or adl_bloom_probe_ranges_device (filter f =
 * d_bitmaps[d_bitmap_off[f] .. d_bitmap_end[f])).  For big batches of 16-byte
 * keys over up to 4096 filters (n >= 2^20) it runs the tile-binned pipeline
 * (queries grouped by filter, positions sorted by 2^20-bit tile, bits tested
 * in LDS: streaming traffic instead of random bitmap reads);
 * otherwise the direct kernel.  A filter of 0 bytes or of 2^31 bits or more
 * answers 0.  Replaces BloomFilter::IsKeyExists (src/filter_block.cpp:49-62)
 * over a multi-get batch.  d_workspace: 256-byte aligned,
 * adl_bloom_probe_batch_workspace_bytes(n, num_filters, bpk, key_stride) bytes. */
uint64_t adl_bloom_probe_batch_workspace_bytes(uint64_t n, uint32_t num_filters, int32_t bits_per_key,
                                               uint32_t key_stride);
int adl_bloom_probe_batch_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n, uint32_t key_stride,
                                 const uint32_t *d_filter_id, uint32_t num_filters, const uint8_t *d_bitmaps,
                                 const uint64_t *d_bitmap_off, const uint64_t *d_bitmap_end, int32_t bits_per_key,
                                 uint8_t *d_out, void *d_workspace, uint64_t workspace_bytes, void *stream);

/* Host-pointer convenience for adl_bloom_probe_device.  Synchronous. */
int adl_bloom_probe(const uint8_t *h_keys, const uint64_t *h_offsets, uint64_t n,
                    uint32_t key_stride, int32_t bits_per_key, const uint8_t *h_bitmap,
                    uint64_t bitmap_bytes, uint8_t *h_out, void *stream);

/* ------------------------------------------------- device-resident filter sets */

/* A set of filters resident in device memory (the reader side: one set per
 * SSTable filter block, or many SSTables' filters for a multi-get).  Replaces
 * the mmapped, non-owning bitmaps FilterBlockReader probes
 * (src/filter_block.cpp:172-184, src/sstable.cpp:195-204). */
typedef struct adl_bloom_filter_set adl_bloom_filter_set;

/* Upload num_filters bitmaps: filter f = h_bitmaps[h_bitmap_off[f] ..
 * h_bitmap_off[f+1]) (HOST arrays, num_filters+1 offsets).  Synchronous. */
int adl_bloom_filter_set_create(const uint8_t *h_bitmaps, const uint64_t *h_bitmap_off,
                                uint32_t num_filters, int32_t bits_per_key,
                                adl_bloom_filter_set **out);

/* Probe n host keys; key i against filter h_filter_id[i], or against
 * `filter` for every key when h_filter_id is NULL.  h_out[i] = 0/1.
 * Synchronous on `stream`. */
int adl_bloom_filter_set_probe(const adl_bloom_filter_set *set, const uint8_t *h_keys,
                               const uint64_t *h_offsets, uint64_t n, uint32_t key_stride,
                               const uint32_t *h_filter_id, uint32_t filter, uint8_t *h_out,
                               void *stream);

/* Device views of a set, for callers that keep queries on the device and call
 * adl_bloom_probe_multi_device themselves. */
int adl_bloom_filter_set_device_view(const adl_bloom_filter_set *set, const uint8_t **d_bitmaps,
                                     const uint64_t **d_bitmap_off, uint32_t *num_filters);

int adl_bloom_filter_set_destroy(adl_bloom_filter_set *set);

/* ------------------------------------------- filter cache keyed by SSTable oid */

/* Device-resident filter blocks of many SSTables in one arena of
 * capacity_bytes, keyed by oid (any byte string, e.g. the SHA-256 file name),
 * least recently used evicted first, at most max_tables blocks: the filter
 * side of DB::table_cache_ (src/db.hpp:96-97, LRUCache src/cache.hpp:23-93).
 * Blocks of any bits_per_key share one cache: each is probed with the k of
 * its own "bf:" info, as FilterBlockReader::CreateFilterAlgorithm reads it per
 * block (src/filter_block.cpp:158-170), so a level of tables written under
 * different DBOptions::bits_per_key is served by one cache and one launch.
 * bits_per_key (>= 0) is kept for source compatibility and not otherwise
 * used.  Thread-safe (one mutex per cache). */
typedef struct adl_bloom_filter_cache adl_bloom_filter_cache;

int adl_bloom_filter_cache_create(uint64_t capacity_bytes, uint32_t max_tables, int32_t bits_per_key,
                                  adl_bloom_filter_cache **out);
int adl_bloom_filter_cache_destroy(adl_bloom_filter_cache *cache);

/* Insert (or replace) the filter block of table `oid`: validated as
 * FilterBlockReader::Init does (ADL_FILTER_BLOCK_ERROR); its bitmaps are
 * uploaded once, its k taken from its own bits_per_key, and it becomes the
 * most recently used.  Synchronous. */
int adl_bloom_filter_cache_put(adl_bloom_filter_cache *cache, const char *oid, uint64_t oid_len,
                               const uint8_t *h_block, uint64_t block_len);

/* 1 if cached (and now most recently used), else 0. */
int adl_bloom_filter_cache_contains(adl_bloom_filter_cache *cache, const char *oid, uint64_t oid_len);

/* 1 if removed, 0 if it was not cached. */
int adl_bloom_filter_cache_remove(adl_bloom_filter_cache *cache, const char *oid, uint64_t oid_len);

int adl_bloom_filter_cache_stats(adl_bloom_filter_cache *cache, uint32_t *tables, uint64_t *bytes_used);

/* Multi-get: query i (host keys) probes filter `filter` (0 for SSTables) of
 * table h_table[i], an index into the oid list oids[0..num_tables).  One
 * launch for the batch.  A query bound for a table that is not cached
 * answers 1 ("may be present": read the table); one bound for a filter the
 * block does not have answers 0 (src/filter_block.cpp:174).  *h_uncached
 * (optional) counts the queries whose table was not cached.  Synchronous.
 * Replaces SSTableReader::Get's filter check (src/sstable.cpp:238) across the
 * tables of a multi-get. */
int adl_bloom_filter_cache_probe(adl_bloom_filter_cache *cache, const char *const *oids,
                                 const uint64_t *oid_lens, uint32_t num_tables, uint32_t filter,
                                 const uint8_t *h_keys, const uint64_t *h_offsets, uint64_t n,
                                 uint32_t key_stride, const uint32_t *h_table, uint8_t *h_out,
                                 uint64_t *h_uncached, void *stream);

/* ---------------------------------------------------------------- hash */

/* The reference's murmur3 variant (src/murmur3_hash.cpp:11-65) on the GPU for a
 * batch: d_out[2i] = murmur3_hash(seed_a, key_i), d_out[2i+1] = (seed_b, key_i). */
int adl_bloom_murmur3_device(const uint8_t *d_keys, const uint64_t *d_offsets, uint64_t n,
                             uint32_t key_stride, uint32_t seed_a, uint32_t seed_b,
                             uint32_t *d_out, void *stream);

/* Single-key form of murmur3_hash(seed, data, len) (src/murmur3_hash.hpp:9),
 * computed on the GPU.  Synchronous; on failure *h_out is left untouched. */
int adl_bloom_murmur3(uint32_t seed, const void *data, uint64_t len, uint32_t *h_out);

/* The calling thread's current HIP device (every device pointer above belongs
 * to it), and setting it: for host code that hands a build to another thread
 * (SSTableWriter::BeginFinal's worker), whose current device starts at 0. */
int adl_bloom_get_device(int32_t *device);
int adl_bloom_set_device(int32_t device);

/* ---------------------------------------------------------------- instrumentation */

/* Per-kernel timing of the build for the calling thread: while enabled, each
 * build takes start/stop timestamps of pass A (bloom_bin_kernel) and pass B
 * (bloom_tile_kernel) from their dispatch packets (hipExtLaunchKernel events,
 * nothing extra enqueued between the launches); up to `capacity` builds are kept.  collect()
 * synchronises on the recorded events, writes the summed milliseconds of the
 * two kernels to ms[0] (pass A) and ms[1] (pass B), the number of timed builds
 * to *builds, and disables timing.  Used by bench.py for the live roofline. */
int adl_bloom_profile_enable(uint32_t capacity);
int adl_bloom_profile_collect(double *ms, uint32_t *builds);
/* The same timings one launch pair at a time, without stopping: ms_ab[2i] =
 * pass A and ms_ab[2i+1] = pass B of pair i, for up to `capacity` pairs (for
 * medians); call before adl_bloom_profile_collect. */
int adl_bloom_profile_each(double *ms_ab, uint32_t capacity, uint32_t *launch_pairs);

/* Bit-sets a build wrote as positions (pass A's output, after it skipped
 * repeated hash pairs), read back from the workspace of the last build made
 * with these key counts: *positions = the sum over its chunks.  For the
 * bench's traffic accounting (profiles/).  Synchronous on `stream`. */
int adl_bloom_build_positions(const uint64_t *key_counts, uint32_t num_filters, int32_t bits_per_key,
                              const void *d_workspace, uint64_t *positions, void *stream);

/* Test-only fault injection (the error-path tests; never set by the product).
 * ADL_TEST_FAULT_PIPELINE_GROUP, arg g >= 0: the next adl_bloom_build_segmented
 * call fails in its group g's build, with earlier groups' copies in flight.
 * ADL_TEST_FAULT_CACHE_COMPLETION, arg >= 0: the next filter-cache probe that
 * waits for its answers in the mapped buffer sees its kernel's completion
 * report a device error after all answers have arrived.  arg < 0 disarms. */
#define ADL_TEST_FAULT_PIPELINE_GROUP 1
#define ADL_TEST_FAULT_CACHE_COMPLETION 2
int adl_bloom_test_fault(int site, int64_t arg);

/* The tuning and test switches (ADL_BLOOM_* environment variables, DESIGN.md
 * §8) are read once per process, at the first call that needs them.  This
 * reads them again (tests that change them; no other call of the library may
 * be running). */
int adl_bloom_reload_knobs(void);

/* Resident probe server kernels launched by this process so far (first
 * launches and relaunches after an idle or life-limit exit), for the latency
 * tests (readpath_test --tails). */
int adl_bloom_probe_server_launches(uint64_t *launches);

/* (instrumentation) The resident probe server's request phases, averaged over
 * the requests since the last reset: *requests served, *stamped of them with
 * the kernel's stamps read back, and avg_us[7] = the kernel's gap since its
 * previous poll, then from the poll that found the request: its loads back,
 * the slot staged in LDS, the hashes done, the bit reads back, the answer
 * stored; avg_us[6] = the host's time per request (the request written to the
 * answer read).  reset != 0 clears the counters after reading them. */
int adl_bloom_probe_server_phases(uint64_t *requests, uint64_t *stamped, double *avg_us, int reset);

/* ---------------------------------------------------------------- synthetic data */

/* SURVEY.md §8d SplitMix64 16-byte keys, generated on the device: key i of the
 * stream seeded `seed`, skipping the first `skip` keys, = LE64(next) || LE64(next). */
int adl_synth_keys16_device(uint8_t *d_out, uint64_t seed, uint64_t skip, uint64_t n,
                            void *stream);

/* Variable-length synthetic keys (DESIGN.md "Synthetic inputs"): lengths
 * 8 + (r-1), r ~ Zipf(s) on [1, 249] by inverse CDF over a SplitMix64 counter
 * stream; d_lengths (n entries, uint32) must then be prefix-summed by the
 * caller into offsets, after which adl_synth_varlen_fill_device writes the
 * bytes (byte j of the packed buffer = byte j%8 of SplitMix64 output j/8). */
int adl_synth_varlen_lengths_device(uint32_t *d_lengths, uint64_t seed, uint64_t n, double zipf_s,
                                    void *stream);
int adl_synth_varlen_fill_device(uint8_t *d_out, uint64_t seed, uint64_t total_bytes, void *stream);

/* Probe queries of BASELINE.json configs[4] (DESIGN.md "Synthetic inputs"):
 * global query q = q0 + i draws four SplitMix64 outputs of the stream seeded
 * `seed` (calls 4q+1 .. 4q+4): r0 -> filter id r0 % num_tables; r1 odd -> an
 * inserted key, key j = (r1 >> 1) % keys_per_table of table t's key stream
 * (adl_synth_keys16_device(seed = table_seed0 + t)); r1 even -> a fresh key
 * LE64(r2) || LE64(r3).  d_member[i] = 1 for inserted keys (may be NULL). */
int adl_synth_probe_queries_device(uint8_t *d_keys, uint32_t *d_filter_id, uint8_t *d_member,
                                   uint64_t seed, uint64_t q0, uint64_t n, uint32_t num_tables,
                                   uint64_t table_seed0, uint64_t keys_per_table, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* ADL_BLOOM_H_ */
