"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY (the parity checker).

ctypes front end to oracle/liboracle.so (the C restatement in
oracle/bloom_oracle.c) plus a pure-Python restatement of the filter-block
container framing of the reference:

* ``filter_block_final``  -- FilterBlockWriter::Final, src/filter_block.cpp:77-102
* ``FilterBlockReaderOracle`` -- FilterBlockReader::Init / IsKeyExists,
  src/filter_block.cpp:113-184

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product (adlsm-tree_amd/) never does.
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None

SEED1 = 0xE2C6928A  # src/filter_block.cpp:22
SEED2 = 0xBAEA8A8F  # src/filter_block.cpp:23
FILTER_BLOCK_ERROR = 13  # src/rc.hpp:22 (enum position)


def build() -> None:
    """Compile liboracle.so (and oracle/_ref when the reference is present)."""
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)
    if os.path.isdir("/root/reference/src"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        u8p = ctypes.c_void_p
        L.oracle_murmur3.restype = ctypes.c_uint32
        L.oracle_murmur3.argtypes = [ctypes.c_uint32, u8p, ctypes.c_uint64]
        L.oracle_num_probes.restype = ctypes.c_int
        L.oracle_num_probes.argtypes = [ctypes.c_int]
        L.oracle_bitmap_bytes.restype = ctypes.c_uint64
        L.oracle_bitmap_bytes.argtypes = [ctypes.c_uint64, ctypes.c_int]
        L.oracle_keys2block.restype = ctypes.c_int
        L.oracle_keys2block.argtypes = [u8p, u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, u8p]
        L.oracle_probe.restype = ctypes.c_int
        L.oracle_probe.argtypes = [u8p, u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                   u8p, ctypes.c_uint64, u8p]
        L.oracle_probe_multi.restype = ctypes.c_int
        L.oracle_probe_multi.argtypes = [u8p, u8p, ctypes.c_uint64, ctypes.c_uint64, u8p,
                                         ctypes.c_uint32, u8p, u8p, ctypes.c_int, u8p]
        L.oracle_murmur3_batch.restype = None
        L.oracle_murmur3_batch.argtypes = [u8p, u8p, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_uint32, ctypes.c_uint32, u8p]
        L.oracle_splitmix_keys16.restype = None
        L.oracle_splitmix_keys16.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u8p]
        L.oracle_synth_probe_queries.restype = None
        L.oracle_synth_probe_queries.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                 ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                                 u8p, u8p, u8p]
        L.oracle_synth_varlen_lengths.restype = None
        L.oracle_synth_varlen_lengths.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double, u8p]
        L.oracle_synth_varlen_fill.restype = None
        L.oracle_synth_varlen_fill.argtypes = [ctypes.c_uint64, ctypes.c_uint64, u8p]
        _LIB = L
    return _LIB


def ref_lib():
    """The reference's own src/murmur3_hash.cpp compiled into oracle/_ref/ (None if absent)."""
    global _REF
    if _REF is None:
        path = os.path.join(HERE, "_ref", "libref_murmur3.so")
        if not os.path.exists(path):
            return None
        L = ctypes.CDLL(path)
        L.ref_murmur3.restype = ctypes.c_uint32
        L.ref_murmur3.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
        L.ref_murmur3_batch.restype = None
        L.ref_murmur3_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                        ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_void_p]
        _REF = L
    return _REF


def _ptr(a):
    return None if a is None else a.ctypes.data


# ---------------------------------------------------------------- key sets
def splitmix_keys16(seed: int, n: int, skip: int = 0) -> np.ndarray:
    """SURVEY.md §8d SplitMix64 16-byte keys: (n,16) uint8."""
    out = np.empty((n, 16), dtype=np.uint8)
    lib().oracle_splitmix_keys16(seed, skip, n, _ptr(out))
    return out


def synth_probe_queries(n: int, seed: int = 0xFEED, q0: int = 0, num_tables: int = 256,
                        table_seed0: int = 0x5EED, keys_per_table: int = 1_000_000):
    """Probe queries of BASELINE.json configs[4]: (keys (n,16) u8, filter_id u32, member u8)."""
    keys = np.empty((n, 16), dtype=np.uint8)
    fid = np.empty(n, dtype=np.uint32)
    member = np.empty(n, dtype=np.uint8)
    lib().oracle_synth_probe_queries(seed, q0, n, num_tables, table_seed0, keys_per_table,
                                     _ptr(keys), _ptr(fid), _ptr(member))
    return keys, fid, member


def synth_varlen(n: int, seed: int = 0x5EED, zipf_s: float = 1.1):
    """configs[2] variable-length keys (restating adl_synth_varlen_*_device):
    (packed bytes uint8, offsets uint64[n+1])."""
    lengths = np.empty(max(n, 1), dtype=np.uint32)
    lib().oracle_synth_varlen_lengths(seed, n, zipf_s, _ptr(lengths))
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lengths[:n], dtype=np.uint64)
    total = int(offs[-1])
    data = np.empty(total + 16, dtype=np.uint8)
    lib().oracle_synth_varlen_fill(seed, total, _ptr(data))
    data[total:] = 0
    return data, offs


def pack(keys) -> tuple[np.ndarray, np.ndarray]:
    """list[bytes] -> (packed uint8 bytes, uint64 offsets[n+1])."""
    offs = np.zeros(len(keys) + 1, dtype=np.uint64)
    if keys:
        offs[1:] = np.cumsum([len(k) for k in keys], dtype=np.uint64)
    data = np.frombuffer(b"".join(keys) + b"\0", dtype=np.uint8).copy()
    return data, offs


def _keyargs(keys, offsets):
    """Normalise (keys, offsets) -> (data, offsets|None, n, stride)."""
    if isinstance(keys, (list, tuple)):
        data, offsets = pack(list(keys))
        return data, offsets, len(keys), 0
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    if offsets is None:
        assert keys.ndim == 2
        return keys, None, keys.shape[0], keys.shape[1]
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    return keys, offsets, len(offsets) - 1, 0


# ---------------------------------------------------------------- algorithm
def murmur3(seed: int, data: bytes) -> int:
    """src/murmur3_hash.cpp:11-65 (quirky Murmur3-x86-32)."""
    buf = np.frombuffer(bytes(data) + b"\0", dtype=np.uint8)
    return lib().oracle_murmur3(seed, buf.ctypes.data, len(data))


def murmur3_batch(keys, offsets=None, seed_a=SEED1, seed_b=SEED2) -> np.ndarray:
    data, offs, n, stride = _keyargs(keys, offsets)
    out = np.empty((n, 2), dtype=np.uint32)
    lib().oracle_murmur3_batch(_ptr(data), _ptr(offs), n, stride, seed_a, seed_b, _ptr(out))
    return out


def num_probes(bits_per_key: int) -> int:
    return lib().oracle_num_probes(bits_per_key)


def bitmap_bytes(n: int, bits_per_key: int) -> int:
    return lib().oracle_bitmap_bytes(n, bits_per_key)


def keys2block(keys, offsets=None, bits_per_key: int = 10) -> np.ndarray:
    """BloomFilter::Keys2Block (src/filter_block.cpp:9-33) -> bitmap bytes."""
    data, offs, n, stride = _keyargs(keys, offsets)
    nbytes = bitmap_bytes(n, bits_per_key)
    if nbytes == 0:
        raise ValueError("filter too large for the reference's int arithmetic")
    out = np.empty(nbytes, dtype=np.uint8)
    rc = lib().oracle_keys2block(_ptr(data), _ptr(offs), n, stride, bits_per_key, _ptr(out))
    assert rc == 0
    return out


def probe(keys, bitmap: np.ndarray, offsets=None, bits_per_key: int = 10) -> np.ndarray:
    """BloomFilter::IsKeyExists (src/filter_block.cpp:49-62), batched -> uint8[n]."""
    data, offs, n, stride = _keyargs(keys, offsets)
    bitmap = np.ascontiguousarray(bitmap, dtype=np.uint8)
    out = np.empty(n, dtype=np.uint8)
    rc = lib().oracle_probe(_ptr(data), _ptr(offs), n, stride, bits_per_key,
                            _ptr(bitmap), bitmap.size, _ptr(out))
    if rc != 0:
        raise ValueError("empty or oversized bitmap")
    return out


def probe_multi(keys, filter_id, bitmaps: np.ndarray, bitmap_off: np.ndarray, offsets=None,
                bits_per_key: int = 10) -> np.ndarray:
    data, offs, n, stride = _keyargs(keys, offsets)
    fid = np.ascontiguousarray(filter_id, dtype=np.uint32)
    bitmaps = np.ascontiguousarray(bitmaps, dtype=np.uint8)
    boff = np.ascontiguousarray(bitmap_off, dtype=np.uint64)
    out = np.empty(n, dtype=np.uint8)
    rc = lib().oracle_probe_multi(_ptr(data), _ptr(offs), n, stride, _ptr(fid), len(boff) - 1,
                                  _ptr(bitmaps), _ptr(boff), bits_per_key, _ptr(out))
    if rc != 0:
        raise ValueError("empty or oversized bitmap")
    return out


# ---------------------------------------------------------------- container
def filter_info(bits_per_key: int) -> bytes:
    """BloomFilter::FilterInfo, src/filter_block.cpp:64-67: "bf:" + raw int32."""
    return b"bf:" + struct.pack("<i", bits_per_key)


def filter_block_final(bitmaps: list[bytes], bits_per_key: int) -> bytes:
    """FilterBlockWriter::Final, src/filter_block.cpp:77-102.

    bitmaps: one Keys2Block result per filter, in order (each appended at the
    current buffer size, :104-109)."""
    buf = bytearray()
    offsets = []
    for bm in bitmaps:
        offsets.append(len(buf))
        buf += bytes(bm)
    offset_begin = len(buf)
    for o in offsets:
        buf += struct.pack("<i", o)
    buf += struct.pack("<i", offset_begin)
    buf += struct.pack("<i", len(offsets))
    info = filter_info(bits_per_key)
    buf += info
    buf += struct.pack("<i", len(info))
    return bytes(buf)


class FilterBlockReaderOracle:
    """FilterBlockReader, src/filter_block.cpp:111-184 (Python restatement)."""

    def __init__(self):
        self.filters_nums = 0

    def init(self, block: bytes) -> int:
        """Init, :113-155.  Returns 0 (OK) or FILTER_BLOCK_ERROR."""
        b = bytes(block)
        self.block = b
        L = len(b)
        if L < 4:
            return FILTER_BLOCK_ERROR
        info_len_off = L - 4
        (info_len,) = struct.unpack_from("<i", b, info_len_off)
        if info_len > info_len_off or info_len <= 0:
            return FILTER_BLOCK_ERROR
        info_off = info_len_off - info_len
        info = b[info_off:info_off + info_len]
        # CreateFilterAlgorithm, :158-170 -- type "bf", bpk read at info[3]
        if info[:2] != b"bf":
            return FILTER_BLOCK_ERROR
        if len(info) < 7:
            return FILTER_BLOCK_ERROR  # reference reads past the view here (UB)
        (self.bits_per_key,) = struct.unpack_from("<i", info, 3)
        if info_off < 4:
            return FILTER_BLOCK_ERROR
        nums_off = info_off - 4
        (self.filters_nums,) = struct.unpack_from("<i", b, nums_off)
        if nums_off < 4:
            return FILTER_BLOCK_ERROR
        (self.offsets_off,) = struct.unpack_from("<i", b, nums_off - 4)
        if self.offsets_off < 0:
            return FILTER_BLOCK_ERROR
        if self.offsets_off + 4 > L:
            return FILTER_BLOCK_ERROR  # reference reads out of bounds here (UB)
        (zero,) = struct.unpack_from("<i", b, self.offsets_off)
        if zero != 0:
            return FILTER_BLOCK_ERROR
        return 0

    def filter_range(self, i: int):
        (o1,) = struct.unpack_from("<i", self.block, self.offsets_off + 4 * i)
        if i + 1 == self.filters_nums:
            o2 = self.offsets_off
        else:
            (o2,) = struct.unpack_from("<i", self.block, self.offsets_off + 4 * (i + 1))
        return o1, o2

    def is_key_exists(self, i: int, key: bytes) -> bool:
        """IsKeyExists, :172-184."""
        if i >= self.filters_nums or i < 0:
            return False
        o1, o2 = self.filter_range(i)
        bm = np.frombuffer(self.block[o1:o2], dtype=np.uint8)
        return bool(probe([bytes(key)], bm, bits_per_key=self.bits_per_key)[0])


# ---------------------------------------------------------------- level lookup
def _decode_inner(k: bytes):
    """MemKey::FromKey (src/keys.cpp:86-91): user key, int64 seq, op byte."""
    if len(k) < 9:
        return k, 0, 0
    return k[:-9], struct.unpack("<q", k[-9:-1])[0], k[-1]


def _memkey_less(a, b) -> bool:
    """MemKey::operator< (src/keys.cpp:61-74)."""
    if a[0] != b[0]:
        return a[0] < b[0]
    if a[1] != b[1]:
        return a[1] > b[1]
    return a[2] > b[2]


def level_candidates(tables, user_key: bytes, seq: int):
    """Level::Get's visiting order and range test (src/revision.cpp:278-287):
    files_meta_ ordered by min_inner_key (src/file_util.hpp:163-165), walked in
    reverse; a table is skipped when (mk < min && mk.user != min.user) or
    max < mk, mk = MemKey(user_key, seq, OP_PUT).  tables: [(min_inner, max_inner)].
    Returns the indices of the tables Get reads, in order."""
    import functools

    mins = [_decode_inner(t[0]) for t in tables]
    order = sorted(range(len(tables)),
                   key=functools.cmp_to_key(lambda a, b: -1 if _memkey_less(mins[a], mins[b])
                                            else (1 if _memkey_less(mins[b], mins[a]) else 0)))
    mk = (user_key, seq, 0)
    out = []
    for t in reversed(order):
        mn, mx = mins[t], _decode_inner(tables[t][1])
        if (_memkey_less(mk, mn) and user_key != mn[0]) or _memkey_less(mx, mk):
            continue
        out.append(t)
    return out
