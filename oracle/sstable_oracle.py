"""oracle/sstable_oracle.py -- TEST INFRASTRUCTURE ONLY (the parity checker).

Pure-Python restatement of the reference's SSTable build path, the file-level
pin of the filter block:

* ``memtable_order``   -- MemKey::operator< (src/keys.cpp:61-74): user key
  ascending, then seq descending, then op descending; inner key =
  user_key + LE64(seq) + op byte (MemKey::ToKey, src/keys.cpp:76-84).
* ``BlockWriterOracle`` -- BlockWriter::Add / Final / EstimatedSize
  (src/block.cpp:18-60): entries [shared:i32][unshared:i32][vlen:i32][key
  suffix][value], a restart point every RESTARTS_BLOCK_LEN = 12 entries
  (src/block.hpp:16), then the restart offsets and their count.
* ``sstable_bytes``    -- SSTableWriter::Add / FlushDataBlock / Final
  (src/sstable.cpp:26-99): data blocks flushed when EstimatedSize() > 4096
  (src/sstable.hpp:40) after an Add; the index block maps each block's last
  inner key to its BlockHandle (i32 offset, i32 size; src/block.hpp:144-162);
  the filter block is FilterBlockWriter::Final over the user keys
  (InnerKeyToUserKey, src/keys.cpp:7-9) -- one filter, built by the C oracle;
  the meta block maps "filter" to its handle; the footer is meta handle +
  index handle + 0x12 0x34 (src/footer_block.cpp:12-32).  The SSTable oid is
  the SHA-256 of every byte appended, i.e. of the whole file (src/sstable.cpp
  :40,59,67,74,90).

Only tests/ may import this module.  The product (adlsm-tree_amd/) never does.
"""
from __future__ import annotations

import hashlib
import struct

import numpy as np

import oracle as O

RESTARTS_BLOCK_LEN = 12  # src/block.hpp:16
NEED_FLUSH_SIZE = 1 << 12  # src/sstable.hpp:40
OP_PUT, OP_DELETE = 0, 1  # src/keys.hpp:10-13


def inner_key(user_key: bytes, seq: int, op: int) -> bytes:
    """MemKey::ToKey, src/keys.cpp:76-84."""
    return bytes(user_key) + struct.pack("<q", seq) + bytes([op])


def memtable_order(entries):
    """entries: (user_key, seq, op, value) -> sorted by MemKey::operator<
    (src/keys.cpp:61-74).  Equal MemKeys keep the later Put (SkipList insert
    of an equal key is not exercised by the reference tests; we keep all)."""
    return sorted(entries, key=lambda e: (bytes(e[0]), -e[1], -e[2]))


class BlockWriterOracle:
    """src/block.cpp:18-60."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.buf = bytearray()
        self.restarts = []
        self.entries = 0
        self.last_key = b""

    def add(self, key: bytes, value: bytes):
        shared = 0
        if self.entries % RESTARTS_BLOCK_LEN == 0:
            self.restarts.append(len(self.buf))
        else:
            m = min(len(key), len(self.last_key))
            while shared < m and key[shared] == self.last_key[shared]:
                shared += 1
        self.buf += struct.pack("<iii", shared, len(key) - shared, len(value))
        self.buf += key[shared:]
        self.buf += value
        self.entries += 1
        self.last_key = bytes(key)

    def estimated_size(self) -> int:
        return len(self.buf) + (len(self.restarts) + 1) * 4

    def empty(self) -> bool:
        return self.entries == 0

    def final(self) -> bytes:
        out = bytes(self.buf) + b"".join(struct.pack("<i", r) for r in self.restarts)
        out += struct.pack("<i", len(self.restarts))
        self.buf = bytearray()  # moved out (std::move(buffer_))
        return out


def sstable_bytes(sorted_entries, bits_per_key: int = 10) -> bytes:
    """SSTableWriter over (inner_key, value) pairs in memtable order -> file bytes."""
    out = bytearray()
    data = BlockWriterOracle()
    index = BlockWriterOracle()
    user_keys = []
    last_key = b""

    def flush():
        blk = data.final()
        off = len(out)
        out.extend(blk)
        data.reset()
        index.add(last_key, struct.pack("<ii", off, len(blk)))

    for ik, value in sorted_entries:
        user_keys.append(ik[:-9])
        data.add(ik, value)
        last_key = ik
        if data.estimated_size() > NEED_FLUSH_SIZE:
            flush()
    if not data.empty():
        flush()
    # filter block: one filter over every user key (Final calls Keys2Block)
    if user_keys:
        bm = O.keys2block(user_keys, bits_per_key=bits_per_key).tobytes()
        fblock = O.filter_block_final([bm], bits_per_key)
    else:
        fblock = O.filter_block_final([], bits_per_key)
    foff = len(out)
    out += fblock
    meta = BlockWriterOracle()
    meta.add(b"filter", struct.pack("<ii", foff, len(fblock)))
    mblk = meta.final()
    moff = len(out)
    out += mblk
    iblk = index.final()
    ioff = len(out)
    out += iblk
    out += struct.pack("<ii", moff, len(mblk)) + struct.pack("<ii", ioff, len(iblk)) + b"\x12\x34"
    return bytes(out)


def oid(file_bytes: bytes) -> str:
    return hashlib.sha256(file_bytes).hexdigest()


def sstable_test_entries(which: int = 1):
    """The memtables of test/sstable_test.cpp: BuildSSTable (:9-27, which=1) and
    BuildSSTable2 (:29-43, which=2), as sorted (inner_key, value) pairs; which=3
    is a memtable of many versions per user key."""
    ents = []
    if which == 1:
        for i in range(10000):
            ents.append((b"key%d" % i, i, OP_PUT, b"value%d" % i))
    elif which == 2:
        for i in range(10000):
            ents.append((b"key%d" % (i // 2), i, OP_PUT if i % 2 == 0 else OP_DELETE, b"value%d" % (i // 2)))
    elif which == 3:
        # not a reference memtable: 1-5 versions of each of 4 000 user keys
        # (adlsm-tree_amd/csrc/sstable_test.cpp Memtable(3))
        seq = 0
        for j in range(4000):
            for _r in range((j * 7) % 5 + 1):
                ents.append((b"user%d" % j, seq, OP_DELETE if seq % 3 == 2 else OP_PUT, b"v%d" % seq))
                seq += 1
    else:
        raise ValueError(which)
    return [(inner_key(u, s, o), v) for (u, s, o, v) in memtable_order(ents)]


def filter_block_of(file_bytes: bytes) -> bytes:
    """Footer -> meta block -> "filter" handle -> the filter block bytes."""
    moff, mlen, _ioff, _ilen = struct.unpack_from("<iiii", file_bytes, len(file_bytes) - 18)
    meta = file_bytes[moff:moff + mlen]
    _sh, ksz, vsz = struct.unpack_from("<iii", meta, 0)
    assert meta[12:12 + ksz] == b"filter" and vsz == 8
    foff, flen = struct.unpack_from("<ii", meta, 12 + ksz)
    return file_bytes[foff:foff + flen]


__all__ = ["inner_key", "memtable_order", "BlockWriterOracle", "sstable_bytes", "oid",
           "sstable_test_entries", "filter_block_of", "np"]
