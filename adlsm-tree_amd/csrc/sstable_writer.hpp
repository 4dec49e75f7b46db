// adlsm-tree_amd/csrc/sstable_writer.hpp -- the SSTable build path of the
// reference (src/sstable.{hpp,cpp} SSTableWriter, src/block.cpp BlockWriter,
// src/footer_block.cpp FooterBlockWriter) on top of the gfx950-backed filter
// mirror (filter_block.hpp).  SURVEY.md §8f rank 1: it proves the drop-in at
// file level -- the same SSTable bytes and oid (SHA-256 of the file) as the
// reference for the same memtable.
//
// What differs from the reference underneath:
//   * Add() feeds the user key into FilterBlockWriter's packed arena (no
//     per-key std::string); Final() builds the filter on the GPU in one
//     launch pair and checks its RC (the reference ignores it,
//     src/sstable.cpp:58).
//   * AddBatch() takes a whole sorted run (packed inner keys + values) at
//     once -- the memtable flush / MergeRuns output -- with the same result as
//     Add() per entry.
//   * File I/O goes through a small Sink (a string, or a POSIX file renamed
//     to <dir>/<oid>.sst on Final); the reference's WritAbleFile / FileManager
//     (src/file_util.cpp) is storage-engine code outside this tier.
#pragma once
#include <stdint.h>

#include <future>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

#include <openssl/evp.h>

#include "filter_block.hpp"
#include "rc.hpp"

namespace adl {

using namespace std;

/* RESTARTS_BLOCK_LEN, src/block.hpp:16 */
constexpr int kRestartsBlockLen = 12;

/* src/block.hpp:19-33 -- prefix-compressed entries with restart points. */
class BlockWriter {
 public:
  RC Add(string_view key, string_view value);
  RC Final(string &result);
  size_t EstimatedSize() const;
  void Reset();
  bool Empty() const { return entries_ == 0; }

 private:
  string buffer_;
  vector<int> restarts_;
  int entries_ = 0;
  string last_key_;
};

/* src/block.hpp:144-162 */
struct BlockHandle {
  int block_offset_ = 0;
  int block_size_ = 0;
  void EncodeMeta(string &ret) const;
  void SetMeta(int offset, int size) {
    block_offset_ = offset;
    block_size_ = size;
  }
};

/* src/footer_block.hpp:11-21 -- meta handle + index handle + magic 0x12 0x34. */
class FooterBlockWriter {
 public:
  static constexpr size_t footer_size = 18;
  RC Add(string_view meta_block_handle, string_view index_block_handle);
  RC Final(string &result);

 private:
  string meta_, index_;
};

/* Incremental SHA-256 of the file (its oid), OpenSSL EVP like the reference. */
class Sha256 {
 public:
  Sha256();
  ~Sha256();
  Sha256(const Sha256 &) = delete;
  Sha256 &operator=(const Sha256 &) = delete;
  void Update(const void *data, size_t len);
  void Final(unsigned char digest[32]);

 private:
  EVP_MD_CTX *ctx_;
};

string Sha256Hex(const unsigned char digest[32]);

/* Where the SSTable bytes go (stands in for WritAbleFile, src/file_util.hpp). */
class Sink {
 public:
  virtual ~Sink() = default;
  virtual RC Append(string_view data) = 0;
  /* called by Final with the oid; a file sink renames itself */
  virtual RC Finish(string_view /*oid_hex*/) { return OK; }
};

class StringSink : public Sink {
 public:
  RC Append(string_view data) override {
    out_.append(data.data(), data.size());
    return OK;
  }
  const string &data() const { return out_; }

 private:
  string out_;
};

/* Temp file in `dir`, renamed to <dir>/<oid>.sst by Finish (src/sstable.cpp:93-97). */
class PosixFileSink : public Sink {
 public:
  explicit PosixFileSink(string dir);
  ~PosixFileSink() override;
  RC Open();
  RC Append(string_view data) override;
  RC Finish(string_view oid_hex) override;
  const string &path() const { return path_; }

 private:
  string dir_, path_;
  int fd_ = -1;
};

/* what a filter build hands back to EndFinal */
struct FilterOutcome {
  RC rc;
  double seconds;
};

/* src/sstable.hpp:21-71 */
class SSTableWriter {
 public:
  SSTableWriter(Sink *sink, int bits_per_key = 10);
  /* any FilterAlgorithm (src/filter_block.hpp:13-20), e.g. one written
   * against the reference's interface */
  SSTableWriter(Sink *sink, unique_ptr<FilterAlgorithm> &&filter);
  /* waits for a filter build BeginFinal started and EndFinal did not collect */
  ~SSTableWriter();
  SSTableWriter(const SSTableWriter &) = delete;
  SSTableWriter &operator=(const SSTableWriter &) = delete;
  /* inner_key = user_key + LE64 seq + op byte (src/keys.cpp:76-84) */
  RC Add(string_view inner_key, string_view value);
  /* entries i = [key_off[i], key_off[i+1]) of keys, [val_off[i], val_off[i+1])
   * of values, in memtable order; same bytes as Add() per entry */
  RC AddBatch(const char *keys, const uint64_t *key_off, const char *values, const uint64_t *val_off,
              size_t n);
  RC Final(unsigned char sha256_digit[32]);
  /* Final() in two halves, so a caller that writes several tables -- a
   * compaction's outputs, src/db.cpp:428-509 -- can fill the next table while
   * this one's filter builds on the GPU.  BeginFinal flushes the data tail and
   * hands the filter build to the calling thread's filter worker (one
   * persistent thread per calling thread, running on the caller's current HIP
   * device); EndFinal waits for it and writes the filter, meta, index and
   * footer blocks.  No Add between the two (BAD_RECORD); the file and its oid
   * are the same as Final's.  Final itself builds on the calling thread. */
  RC BeginFinal();
  RC EndFinal(unsigned char sha256_digit[32]);
  int GetFileSize() const { return offset_; }
  /* filter keys added so far that equal their predecessor (user keys of
   * consecutive versions); Final skips them on the device when frequent */
  uint64_t filter_duplicates() const { return filter_block_.adjacent_duplicates(); }
  /* wall time of the filter block build of the last Final() / EndFinal();
   * not valid between BeginFinal and EndFinal */
  double filter_seconds() const { return filter_seconds_; }

 private:
  RC FlushDataBlock();
  RC Emit(const string &block);
  RC WriteTail(unsigned char sha256_digit[32]);

  Sink *sink_;
  int offset_ = 0;
  Sha256 sha256_;
  BlockWriter data_block_, index_block_, meta_data_block_;
  FooterBlockWriter foot_block_;
  FilterBlockWriter filter_block_;
  BlockHandle data_block_handle_, filter_block_handle_, meta_data_block_handle_, index_block_handle_;
  string last_key_;
  string buffer_;
  double filter_seconds_ = 0;
  /* BeginFinal's build and the block it writes.  The future comes from a
   * packaged_task on the filter worker, so its destructor does not wait:
   * ~SSTableWriter waits for a pending build, which uses filter_block_ and
   * filter_out_. */
  string filter_out_;
  future<FilterOutcome> filter_job_;
  static constexpr size_t need_flush_size_ = 1u << 12; /* 4KB, src/sstable.hpp:40 */
};

}  // namespace adl
