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
namespace {
constexpr uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
inline uint32_t ror(uint32_t x, int c) { return (x >> c) | (x << (32 - c)); }
}  // namespace

Sha256::Sha256()
    : h_{0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19} {}

void Sha256::Block(const unsigned char *p) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i)
    w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
    const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h_[0], b = h_[1], c = h_[2], d = h_[3], e = h_[4], f = h_[5], g = h_[6], h = h_[7];
  for (int i = 0; i < 64; ++i) {
    const uint32_t t1 = h + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + kK[i] + w[i];
    const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g, g = f, f = e, e = d + t1, d = c, c = b, b = a, a = t1 + t2;
  }
  h_[0] += a, h_[1] += b, h_[2] += c, h_[3] += d, h_[4] += e, h_[5] += f, h_[6] += g, h_[7] += h;
}

void Sha256::Update(const void *data, size_t len) {
  const unsigned char *p = static_cast<const unsigned char *>(data);
  total_ += len;
  if (used_) {
    const size_t take = std::min(len, 64 - used_);
    memcpy(buf_ + used_, p, take);
    used_ += take, p += take, len -= take;
    if (used_ < 64) return;
    Block(buf_);
    used_ = 0;
  }
  for (; len >= 64; p += 64, len -= 64) Block(p);
  memcpy(buf_, p, len);
  used_ = len;
}

void Sha256::Final(unsigned char digest[32]) {
  const uint64_t bits = total_ * 8;
  const unsigned char pad = 0x80, zero = 0;
  Update(&pad, 1);
  while (used_ != 56) Update(&zero, 1);
  unsigned char len_be[8];
  for (int i = 0; i < 8; ++i) len_be[i] = (unsigned char)(bits >> (56 - 8 * i));
  Update(len_be, 8);
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 4; ++j) digest[4 * i + j] = (unsigned char)(h_[i] >> (24 - 8 * j));
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

/* src/sstable.cpp:26-35: the user key (inner key minus seq and op,
 * src/keys.cpp:7-9) goes to the filter, the entry to the data block. */
RC SSTableWriter::Add(string_view inner_key, string_view value) {
  if (inner_key.size() < 9) return BAD_RECORD;
  filter_block_.Update(inner_key.substr(0, inner_key.size() - 9));
  RC rc = data_block_.Add(inner_key, value);
  if (rc) return rc;
  last_key_.assign(inner_key.data(), inner_key.size());
  if (data_block_.EstimatedSize() > need_flush_size_) return FlushDataBlock();
  return OK;
}

RC SSTableWriter::AddBatch(const char *keys, const uint64_t *key_off, const char *values,
                           const uint64_t *val_off, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    RC rc = Add(string_view(keys + key_off[i], key_off[i + 1] - key_off[i]),
                string_view(values + val_off[i], val_off[i + 1] - val_off[i]));
    if (rc) return rc;
  }
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

/* src/sstable.cpp:54-99: data tail, filter block (GPU build), meta block
 * ("filter" -> handle), index block, footer; the oid is the SHA-256 of it all. */
RC SSTableWriter::Final(unsigned char sha256_digit[32]) {
  RC rc;
  if (!data_block_.Empty() && (rc = FlushDataBlock())) return rc;

  if ((rc = filter_block_.Final(buffer_))) return rc;  // the reference drops this RC
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
