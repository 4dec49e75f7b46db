// adlsm-tree_amd/csrc/sstable_writer.cpp -- SSTable build path over the
// gfx950 filter mirror.  See sstable_writer.hpp for what differs from the
// reference's src/sstable.cpp underneath.
#include "sstable_writer.hpp"

#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>

#include "../../include/adl_bloom.h"

namespace adl {

namespace {
void Put32(string &dst, int v) { dst.append(reinterpret_cast<const char *>(&v), sizeof(int)); }
}  // namespace

// ------------------------------------------------------------ BlockWriter
/* src/block.cpp:18-43: a restart point (full key) every 12 entries, else the
 * key's prefix shared with the previous key is elided. */
RC BlockWriter::Add(string_view key, string_view value) {
  int shared = 0;
  if (entries_ % kRestartsBlockLen == 0) {
    restarts_.push_back((int)buffer_.size());
  } else {
    const size_t lim = std::min(key.size(), last_key_.size());
    while ((size_t)shared < lim && key[shared] == last_key_[shared]) ++shared;
  }
  Put32(buffer_, shared);
  Put32(buffer_, (int)key.size() - shared);
  Put32(buffer_, (int)value.size());
  buffer_.append(key.data() + shared, key.size() - shared);
  buffer_.append(value.data(), value.size());
  ++entries_;
  last_key_.assign(key.data(), key.size());
  return OK;
}

/* src/block.cpp:45-55: restart offsets, their count; the buffer moves out. */
RC BlockWriter::Final(string &result) {
  for (int r : restarts_) Put32(buffer_, r);
  Put32(buffer_, (int)restarts_.size());
  result = std::move(buffer_);
  buffer_.clear();
  return OK;
}

/* src/block.cpp:57-59 */
size_t BlockWriter::EstimatedSize() const { return buffer_.size() + (restarts_.size() + 1) * sizeof(int); }

void BlockWriter::Reset() {
  entries_ = 0;
  buffer_.clear();
  restarts_.clear();
  last_key_.clear();
}

void BlockHandle::EncodeMeta(string &ret) const {
  Put32(ret, block_offset_);
  Put32(ret, block_size_);
}

// ------------------------------------------------------------ footer
RC FooterBlockWriter::Add(string_view meta_block_handle, string_view index_block_handle) {
  meta_.assign(meta_block_handle.data(), meta_block_handle.size());
  index_.assign(index_block_handle.data(), index_block_handle.size());
  return OK;
}

/* src/footer_block.cpp:12-32 */
RC FooterBlockWriter::Final(string &result) {
  if (meta_.size() != 8 || index_.size() != 8) return UN_SUPPORTED_FORMAT;
  string f = meta_ + index_;
  f.push_back((char)0x12);
  f.push_back((char)0x34);
  result = std::move(f);
  return OK;
}

// ------------------------------------------------------------ SHA-256
// OpenSSL's SHA-256 (EVP), as the reference (src/sstable.cpp:2,22,40).
Sha256::Sha256() : ctx_(EVP_MD_CTX_new()) {
  if (!ctx_ || EVP_DigestInit_ex(ctx_, EVP_sha256(), nullptr) != 1) abort();
}

Sha256::~Sha256() { EVP_MD_CTX_free(ctx_); }

void Sha256::Update(const void *data, size_t len) {
  if (EVP_DigestUpdate(ctx_, data, len) != 1) abort();
}

void Sha256::Final(unsigned char digest[32]) {
  unsigned int n = 0;
  if (EVP_DigestFinal_ex(ctx_, digest, &n) != 1 || n != 32) abort();
}

string Sha256Hex(const unsigned char digest[32]) {
  static const char *hex = "0123456789abcdef";
  string s(64, '0');
  for (int i = 0; i < 32; ++i) s[2 * i] = hex[digest[i] >> 4], s[2 * i + 1] = hex[digest[i] & 15];
  return s;
}

// ------------------------------------------------------------ file sink
PosixFileSink::PosixFileSink(string dir) : dir_(std::move(dir)) {}

PosixFileSink::~PosixFileSink() {
  if (fd_ >= 0) close(fd_);
}

RC PosixFileSink::Open() {
  string tmpl = dir_ + "/tmp_sst_XXXXXX";
  fd_ = mkstemp(tmpl.data());
  if (fd_ < 0) return MAKESTEMP_ERROR;
  path_ = tmpl;
  return OK;
}

RC PosixFileSink::Append(string_view data) {
  if (fd_ < 0) return IO_ERROR;
  const char *p = data.data();
  size_t left = data.size();
  while (left) {
    const ssize_t w = write(fd_, p, left);
    if (w < 0) {
      if (errno == EINTR) continue;
      return IO_ERROR;
    }
    p += w, left -= (size_t)w;
  }
  return OK;
}

RC PosixFileSink::Finish(string_view oid_hex) {
  if (fd_ < 0) return IO_ERROR;
  const string dst = dir_ + "/" + string(oid_hex) + ".sst";
  if (rename(path_.c_str(), dst.c_str()) != 0) return RENAME_FILE_ERROR;
  path_ = dst;
  const int rc = close(fd_);
  fd_ = -1;
  return rc == 0 ? OK : CLOSE_FILE_ERROR;
}

// ------------------------------------------------------------ SSTableWriter
SSTableWriter::SSTableWriter(Sink *sink, int bits_per_key)
    : sink_(sink), filter_block_(make_unique<BloomFilter>(bits_per_key)) {}

SSTableWriter::SSTableWriter(Sink *sink, unique_ptr<FilterAlgorithm> &&filter)
    : sink_(sink), filter_block_(std::move(filter)) {}

/* a build BeginFinal posted writes filter_block_ and filter_out_: it must end
 * before they do (an error path that drops a writer between the halves) */
SSTableWriter::~SSTableWriter() {
  if (filter_job_.valid()) filter_job_.wait();
}

/* src/sstable.cpp:26-35: the user key (inner key minus seq and op,
 * src/keys.cpp:7-9) goes to the filter, the entry to the data block. */
RC SSTableWriter::Add(string_view inner_key, string_view value) {
  if (inner_key.size() < 9 || filter_job_.valid()) return BAD_RECORD;
  filter_block_.Update(inner_key.substr(0, inner_key.size() - 9));
  RC rc = data_block_.Add(inner_key, value);
  if (rc) return rc;
  last_key_.assign(inner_key.data(), inner_key.size());
  if (data_block_.EstimatedSize() > need_flush_size_) return FlushDataBlock();
  return OK;
}

/* A packed sorted run (memtable flush, src/mem_table.cpp:96-105; MergeRuns
 * output, src/db.cpp:428-509): the user keys go into the filter arena in one
 * bulk append (one reservation, no per-entry call), then the entries into the
 * data blocks.  Same bytes as Add() per entry.  Every record is checked before
 * anything is added, so a BAD_RECORD leaves the writer unchanged; an error
 * from the sink while a data block is flushed does not (the filter then holds
 * keys of entries that were not written), and the table must be abandoned, as
 * after any failed Add. */
RC SSTableWriter::AddBatch(const char *keys, const uint64_t *key_off, const char *values,
                           const uint64_t *val_off, size_t n) {
  if (filter_job_.valid()) return BAD_RECORD;
  for (size_t i = 0; i < n; ++i)
    if (key_off[i + 1] < key_off[i] || key_off[i + 1] - key_off[i] < 9) return BAD_RECORD;
  filter_block_.UpdateBatch(keys, key_off, n, 9);
  for (size_t i = 0; i < n; ++i) {
    const string_view k(keys + key_off[i], key_off[i + 1] - key_off[i]);
    RC rc = data_block_.Add(k, string_view(values + val_off[i], val_off[i + 1] - val_off[i]));
    if (rc) return rc;
    if (data_block_.EstimatedSize() > need_flush_size_) {
      last_key_.assign(k.data(), k.size());
      if ((rc = FlushDataBlock())) return rc;
    }
  }
  if (n) last_key_.assign(keys + key_off[n - 1], key_off[n] - key_off[n - 1]);
  return OK;
}

RC SSTableWriter::Emit(const string &block) {
  sha256_.Update(block.data(), block.size());
  return sink_->Append(block);
}

/* src/sstable.cpp:37-52 */
RC SSTableWriter::FlushDataBlock() {
  data_block_.Final(buffer_);
  RC rc = Emit(buffer_);
  if (rc) return rc;
  data_block_handle_.SetMeta(offset_, (int)buffer_.size());
  offset_ += (int)buffer_.size();
  data_block_.Reset();
  string handle;
  data_block_handle_.EncodeMeta(handle);
  return index_block_.Add(last_key_, handle);
}

// ------------------------------------------------------------ filter worker
/* One worker thread per calling thread, created by its first BeginFinal and
 * joined when that thread exits: the filter builds of consecutive tables run
 * on one thread, so the library's per-thread staging buffers, streams and
 * device workspace are allocated once, not per table.  Each job first makes
 * the caller's HIP device current (a thread starts on device 0). */
class FilterWorker {
 public:
  FilterWorker() : th_([this] { Run(); }) {}
  ~FilterWorker() {
    {
      lock_guard<mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_one();
    th_.join();
  }
  future<FilterOutcome> Post(function<FilterOutcome()> job) {
    packaged_task<FilterOutcome()> task(std::move(job));
    future<FilterOutcome> f = task.get_future();
    {
      lock_guard<mutex> g(mu_);
      q_.push_back(std::move(task));
    }
    cv_.notify_one();
    return f;
  }
  static FilterWorker &ForThisThread() {
    thread_local unique_ptr<FilterWorker> w;
    if (!w) w = make_unique<FilterWorker>();
    return *w;
  }

 private:
  void Run() {
    for (;;) {
      packaged_task<FilterOutcome()> task;
      {
        unique_lock<mutex> g(mu_);
        cv_.wait(g, [this] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;  // stop_, and every posted build has run
        task = std::move(q_.front());
        q_.pop_front();
      }
      task();
    }
  }
  mutex mu_;
  condition_variable cv_;
  deque<packaged_task<FilterOutcome()>> q_;
  bool stop_ = false;
  thread th_;
};

/* src/sstable.cpp:54-99: data tail, filter block (GPU build), meta block
 * ("filter" -> handle), index block, footer; the oid is the SHA-256 of it all.
 * Final builds the filter on the calling thread (its HIP device, its
 * adl_bloom_profile_enable timing). */
RC SSTableWriter::Final(unsigned char sha256_digit[32]) {
  if (filter_job_.valid()) return BAD_RECORD;
  RC rc;
  if (!data_block_.Empty() && (rc = FlushDataBlock())) return rc;
  const auto f0 = std::chrono::steady_clock::now();
  rc = filter_block_.Final(filter_out_);  // the reference drops this RC
  filter_seconds_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - f0).count();
  if (rc) return rc;
  return WriteTail(sha256_digit);
}

RC SSTableWriter::BeginFinal() {
  if (filter_job_.valid()) return BAD_RECORD;
  RC rc;
  if (!data_block_.Empty() && (rc = FlushDataBlock())) return rc;
  int32_t dev = 0;
  if (adl_bloom_get_device(&dev) != ADL_OK) return DEVICE_ERROR;
  // the worker owns filter_block_ and filter_out_ until EndFinal's get()
  filter_job_ = FilterWorker::ForThisThread().Post([this, dev]() -> FilterOutcome {
    if (adl_bloom_set_device(dev) != ADL_OK) return {DEVICE_ERROR, 0.0};
    const auto f0 = std::chrono::steady_clock::now();
    const RC r = filter_block_.Final(filter_out_);
    return {r, std::chrono::duration<double>(std::chrono::steady_clock::now() - f0).count()};
  });
  return OK;
}

RC SSTableWriter::EndFinal(unsigned char sha256_digit[32]) {
  if (!filter_job_.valid()) return BAD_RECORD;
  const FilterOutcome out = filter_job_.get();
  filter_seconds_ = out.seconds;
  if (out.rc) return out.rc;
  return WriteTail(sha256_digit);
}

RC SSTableWriter::WriteTail(unsigned char sha256_digit[32]) {
  RC rc;
  buffer_ = std::move(filter_out_);
  if ((rc = Emit(buffer_))) return rc;
  filter_block_handle_.SetMeta(offset_, (int)buffer_.size());
  offset_ += (int)buffer_.size();
  string fh;
  filter_block_handle_.EncodeMeta(fh);

  meta_data_block_.Add("filter", fh);
  meta_data_block_.Final(buffer_);
  if ((rc = Emit(buffer_))) return rc;
  meta_data_block_handle_.SetMeta(offset_, (int)buffer_.size());
  offset_ += (int)buffer_.size();

  index_block_.Final(buffer_);
  if ((rc = Emit(buffer_))) return rc;
  index_block_handle_.SetMeta(offset_, (int)buffer_.size());
  offset_ += (int)buffer_.size();

  string mh, ih;
  meta_data_block_handle_.EncodeMeta(mh);
  index_block_handle_.EncodeMeta(ih);
  foot_block_.Add(mh, ih);
  if ((rc = foot_block_.Final(buffer_))) return rc;
  if ((rc = Emit(buffer_))) return rc;
  offset_ += (int)buffer_.size();

  sha256_.Final(sha256_digit);
  return sink_->Finish(Sha256Hex(sha256_digit));
}

}  // namespace adl
