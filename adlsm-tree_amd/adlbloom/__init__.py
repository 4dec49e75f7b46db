"""adlbloom -- Python binding of libadlbloom.so (include/adl_bloom.h) over ctypes.

The product path: every build/probe here runs the gfx950 HIP kernels through
the C-ABI.  There is no CPU fallback -- if the shared library or a GPU is
missing, the calls raise.  torch is used only for device memory and streams.

Reference interfaces mirrored (adlternative/adlsm-tree):
  * build()  ~ BloomFilter::Keys2Block          src/filter_block.cpp:9-33
  * probe()  ~ BloomFilter::IsKeyExists         src/filter_block.cpp:49-62
  * murmur3  ~ murmur3_hash                     src/murmur3_hash.cpp:11-65
  * num_probes / bitmap_bytes                   src/filter_block.cpp:11-14, 44-46
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ADL_BLOOM_LIB: diagnostics only (tools/stamps.py points it at the
# s_memtime-instrumented build, lib_stamps/libadlbloom.so)
LIB_PATH = os.environ.get("ADL_BLOOM_LIB") or os.path.join(PKG_DIR, "lib", "libadlbloom.so")

SEED1 = 0xE2C6928A  # src/filter_block.cpp:22
SEED2 = 0xBAEA8A8F  # src/filter_block.cpp:23

ADL_OK = 0
ADL_FILTER_BLOCK_ERROR = 13

# every symbol include/adl_bloom.h declares (tests check the .so exports them all)
EXPORTS = (
    "adl_bloom_strerror", "adl_bloom_abi_version", "adl_bloom_num_probes",
    "adl_bloom_bitmap_bytes", "adl_bloom_bitmap_alloc_bytes", "adl_bloom_build_workspace_bytes",
    "adl_bloom_build_device", "adl_bloom_build_segmented_device", "adl_bloom_build",
    "adl_bloom_build_segmented", "adl_bloom_filter_block_bytes", "adl_bloom_filter_block_workspace_bytes",
    "adl_bloom_filter_block_build_device", "adl_bloom_probe_ranges_device", "adl_bloom_build_segmented_device_ex",
    "adl_bloom_filter_cache_create", "adl_bloom_filter_cache_destroy", "adl_bloom_filter_cache_put",
    "adl_bloom_filter_cache_contains", "adl_bloom_filter_cache_remove", "adl_bloom_filter_cache_stats",
    "adl_bloom_filter_cache_probe",
    "adl_bloom_probe_device", "adl_bloom_probe_multi_device", "adl_bloom_probe",
    "adl_bloom_filter_set_create", "adl_bloom_filter_set_probe",
    "adl_bloom_filter_set_device_view", "adl_bloom_filter_set_destroy",
    "adl_bloom_murmur3_device", "adl_bloom_murmur3", "adl_synth_keys16_device",
    "adl_synth_varlen_lengths_device", "adl_synth_varlen_fill_device",
    "adl_bloom_profile_enable", "adl_bloom_profile_collect", "adl_synth_probe_queries_device",
    "adl_bloom_profile_each", "adl_bloom_probe_batch_workspace_bytes", "adl_bloom_probe_batch_device",
    "adl_bloom_test_fault", "adl_bloom_build_positions", "adl_bloom_get_device", "adl_bloom_set_device",
    "adl_bloom_reload_knobs", "adl_bloom_build_segmented_ex", "adl_bloom_probe_server_launches",
    "adl_bloom_probe_server_phases",
)

_LIB = None


class AdlBloomError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        msg = lib().adl_bloom_strerror(status).decode()
        super().__init__(f"{what}: {msg} (status {status})" if what else f"{msg} (status {status})")


def lib() -> ctypes.CDLL:
    """Load libadlbloom.so (raises if it has not been built -- no fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C adlsm-tree_amd)")
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int32
    sig = {
        "adl_bloom_strerror": (ctypes.c_char_p, [ctypes.c_int]),
        "adl_bloom_abi_version": (ctypes.c_int, []),
        "adl_bloom_num_probes": (i32, [i32]),
        "adl_bloom_bitmap_bytes": (u64, [u64, i32]),
        "adl_bloom_bitmap_alloc_bytes": (u64, [u64, i32]),
        "adl_bloom_build_workspace_bytes": (u64, [vp, u32, i32]),
        "adl_bloom_build_device": (ctypes.c_int, [vp, vp, u64, u32, i32, vp, vp, u64, vp]),
        "adl_bloom_build_segmented_device": (ctypes.c_int, [vp, vp, u32, vp, u32, i32, vp, vp, vp, u64, vp]),
        "adl_bloom_build": (ctypes.c_int, [vp, vp, u64, u32, i32, vp, vp]),
        "adl_bloom_build_segmented": (ctypes.c_int, [vp, vp, u32, vp, u32, i32, vp, vp, vp]),
        "adl_bloom_build_segmented_ex": (ctypes.c_int, [vp, vp, u32, vp, u32, i32, vp, vp, u32, vp]),
        "adl_bloom_filter_block_bytes": (u64, [vp, u32, i32]),
        "adl_bloom_filter_block_workspace_bytes": (u64, [vp, u32, i32]),
        "adl_bloom_filter_block_build_device": (ctypes.c_int, [vp, vp, u32, vp, u32, i32, vp, u64, vp, u64, vp]),
        "adl_bloom_build_segmented_device_ex": (ctypes.c_int, [vp, vp, u32, vp, u32, i32, vp, vp, u32, vp, u64, vp]),
        "adl_bloom_probe_ranges_device": (ctypes.c_int, [vp, vp, u64, u32, vp, u32, vp, vp, vp, i32, vp, vp]),
        "adl_bloom_filter_cache_create": (ctypes.c_int, [u64, u32, i32, ctypes.POINTER(vp)]),
        "adl_bloom_filter_cache_destroy": (ctypes.c_int, [vp]),
        "adl_bloom_filter_cache_put": (ctypes.c_int, [vp, ctypes.c_char_p, u64, vp, u64]),
        "adl_bloom_filter_cache_contains": (ctypes.c_int, [vp, ctypes.c_char_p, u64]),
        "adl_bloom_filter_cache_remove": (ctypes.c_int, [vp, ctypes.c_char_p, u64]),
        "adl_bloom_filter_cache_stats": (ctypes.c_int, [vp, ctypes.POINTER(u32), ctypes.POINTER(u64)]),
        "adl_bloom_filter_cache_probe": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_char_p), vp, u32, u32, vp, vp,
                                                         u64, u32, vp, vp, ctypes.POINTER(u64), vp]),
        "adl_bloom_probe_device": (ctypes.c_int, [vp, vp, u64, u32, i32, vp, u64, vp, vp]),
        "adl_bloom_probe_batch_workspace_bytes": (u64, [u64, u32, i32, u32]),
        "adl_bloom_probe_batch_device": (ctypes.c_int, [vp, vp, u64, u32, vp, u32, vp, vp, vp, i32, vp, vp, u64, vp]),
        "adl_bloom_probe_multi_device": (ctypes.c_int, [vp, vp, u64, u32, vp, u32, vp, vp, i32, vp, vp]),
        "adl_bloom_probe": (ctypes.c_int, [vp, vp, u64, u32, i32, vp, u64, vp, vp]),
        "adl_bloom_filter_set_create": (ctypes.c_int, [vp, vp, u32, i32, ctypes.POINTER(vp)]),
        "adl_bloom_filter_set_probe": (ctypes.c_int, [vp, vp, vp, u64, u32, vp, u32, vp, vp]),
        "adl_bloom_filter_set_device_view": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                                            ctypes.POINTER(u32)]),
        "adl_bloom_filter_set_destroy": (ctypes.c_int, [vp]),
        "adl_bloom_murmur3_device": (ctypes.c_int, [vp, vp, u64, u32, u32, u32, vp, vp]),
        "adl_bloom_murmur3": (ctypes.c_int, [u32, vp, u64, ctypes.POINTER(u32)]),
        "adl_synth_keys16_device": (ctypes.c_int, [vp, u64, u64, u64, vp]),
        "adl_synth_varlen_lengths_device": (ctypes.c_int, [vp, u64, u64, ctypes.c_double, vp]),
        "adl_synth_varlen_fill_device": (ctypes.c_int, [vp, u64, u64, vp]),
        "adl_synth_probe_queries_device": (ctypes.c_int, [vp, vp, vp, u64, u64, u64, u32, u64, u64, vp]),
        "adl_bloom_profile_enable": (ctypes.c_int, [u32]),
        "adl_bloom_profile_collect": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u32)]),
        "adl_bloom_profile_each": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), u32, ctypes.POINTER(u32)]),
        "adl_bloom_test_fault": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64]),
        "adl_bloom_build_positions": (ctypes.c_int, [vp, u32, i32, vp, ctypes.POINTER(u64), vp]),
        "adl_bloom_get_device": (ctypes.c_int, [ctypes.POINTER(i32)]),
        "adl_bloom_set_device": (ctypes.c_int, [i32]),
        "adl_bloom_reload_knobs": (ctypes.c_int, []),
        "adl_bloom_probe_server_launches": (ctypes.c_int, [ctypes.POINTER(u64)]),
        "adl_bloom_probe_server_phases": (ctypes.c_int, [ctypes.POINTER(u64), ctypes.POINTER(u64),
                                                          ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = L
    return L


def reload_knobs() -> None:
    """Re-read the ADL_BLOOM_* switches (the library reads them once per
    process; tests that change them call this, with no call running)."""
    _check(lib().adl_bloom_reload_knobs(), "adl_bloom_reload_knobs")


def _check(status: int, what: str) -> None:
    if status != ADL_OK:
        raise AdlBloomError(status, what)


# ------------------------------------------------------------------ host math
def num_probes(bits_per_key: int) -> int:
    return lib().adl_bloom_num_probes(bits_per_key)


def bitmap_bytes(n: int, bits_per_key: int) -> int:
    return lib().adl_bloom_bitmap_bytes(n, bits_per_key)


def bitmap_alloc_bytes(n: int, bits_per_key: int) -> int:
    return lib().adl_bloom_bitmap_alloc_bytes(n, bits_per_key)


def workspace_bytes(counts, bits_per_key: int) -> int:
    arr = np.ascontiguousarray(counts, dtype=np.uint64)
    return lib().adl_bloom_build_workspace_bytes(arr.ctypes.data, len(arr), bits_per_key)


# ------------------------------------------------------------------ torch plumbing
def _torch():
    import torch
    return torch


def _stream(stream=None):
    torch = _torch()
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def _dptr(t) -> int | None:
    if t is None:
        return None
    assert t.is_cuda, "device tensor expected"
    return t.data_ptr()


def empty_device(nbytes: int, device="cuda"):
    """uint8 device buffer of nbytes (256-byte aligned by the caching allocator)."""
    return _torch().empty(max(int(nbytes), 1), dtype=_torch().uint8, device=device)


def _keyset(keys, offsets):
    """(keys, offsets) device tensors -> (ptr keys, ptr offs, n, stride)."""
    if offsets is None:
        assert keys.dim() == 2, "fixed-size keys: (n, stride) uint8 tensor"
        return _dptr(keys), None, keys.shape[0], keys.shape[1]
    return _dptr(keys), _dptr(offsets), offsets.numel() - 1, 0


class Builder:
    """Reusable device workspace + bitmap for repeated builds of one shape (bench)."""

    def __init__(self, n: int, bits_per_key: int = 10, device="cuda"):
        self.n, self.bpk = int(n), int(bits_per_key)
        self.nbytes = bitmap_bytes(self.n, self.bpk)
        if self.nbytes == 0:
            raise AdlBloomError(-2, "bitmap size")
        self.bitmap = empty_device(bitmap_alloc_bytes(self.n, self.bpk), device)
        self.ws_bytes = workspace_bytes([self.n], self.bpk)
        self.ws = empty_device(self.ws_bytes, device)

    def positions(self, stream=None) -> int:
        """Positions (bit-sets after repeated pairs were skipped) the last build wrote."""
        cnt = np.array([self.n], dtype=np.uint64)
        v = ctypes.c_uint64()
        _check(lib().adl_bloom_build_positions(cnt.ctypes.data, 1, self.bpk, _dptr(self.ws), ctypes.byref(v),
                                               _stream(stream)), "adl_bloom_build_positions")
        return v.value

    def build(self, keys, offsets=None, stream=None):
        pk, po, n, stride = _keyset(keys, offsets)
        assert n == self.n
        _check(lib().adl_bloom_build_device(pk, po, n, stride, self.bpk, _dptr(self.bitmap),
                                            _dptr(self.ws), self.ws_bytes, _stream(stream)),
               "adl_bloom_build_device")
        return self.bitmap[: self.nbytes]


class SegmentedBuilder:
    """Reusable buffers for repeated segmented builds (many SSTable filters per launch pair)."""

    def __init__(self, key_begin, bits_per_key: int = 10, device="cuda"):
        self.kb = np.ascontiguousarray(key_begin, dtype=np.uint64)
        self.bpk = int(bits_per_key)
        F = len(self.kb) - 1
        counts = self.kb[1:] - self.kb[:-1]
        self.sizes = np.array([bitmap_bytes(int(c), self.bpk) for c in counts], dtype=np.uint64)
        alloc = np.array([bitmap_alloc_bytes(int(c), self.bpk) for c in counts], dtype=np.uint64)
        self.boff = np.zeros(F, dtype=np.uint64)
        if F > 1:
            self.boff[1:] = np.cumsum(alloc[:-1])
        self.out = empty_device(int(alloc.sum()), device)
        self.ws_bytes = workspace_bytes(counts, self.bpk)
        self.ws = empty_device(self.ws_bytes, device)

    def build(self, keys, offsets=None, stream=None):
        stride = 0 if offsets is not None else keys.shape[1]
        _check(lib().adl_bloom_build_segmented_device(_dptr(keys), _dptr(offsets), stride, self.kb.ctypes.data,
                                                      len(self.kb) - 1, self.bpk, _dptr(self.out),
                                                      self.boff.ctypes.data, _dptr(self.ws), self.ws_bytes,
                                                      _stream(stream)), "adl_bloom_build_segmented_device")
        return self.out

    def positions(self, stream=None) -> int:
        """Positions (bit-sets after repeated pairs were skipped) the last build wrote."""
        counts = np.ascontiguousarray(self.kb[1:] - self.kb[:-1], dtype=np.uint64)
        v = ctypes.c_uint64()
        _check(lib().adl_bloom_build_positions(counts.ctypes.data, len(counts), self.bpk, _dptr(self.ws),
                                               ctypes.byref(v), _stream(stream)), "adl_bloom_build_positions")
        return v.value

    def bitmap(self, f: int):
        o = int(self.boff[f])
        return self.out[o:o + int(self.sizes[f])]


def build(keys, offsets=None, bits_per_key: int = 10, stream=None):
    """Keys2Block on the GPU: returns the (n*bpk+7)-byte bitmap as a uint8 device tensor."""
    pk, po, n, stride = _keyset(keys, offsets)
    return Builder(n, bits_per_key, keys.device).build(keys, offsets, stream)


SKIP_ADJACENT_DUPLICATES = 1


def build_segmented(keys, key_begin, offsets=None, bits_per_key: int = 10, stream=None, flags: int = 0):
    """Many independent filters in one pass pair.  key_begin: host ints (F+1).
    Returns (device bitmaps buffer, host bitmap byte offsets (F), exact sizes (F))."""
    torch = _torch()
    kb = np.ascontiguousarray(key_begin, dtype=np.uint64)
    F = len(kb) - 1
    counts = kb[1:] - kb[:-1]
    sizes = np.array([bitmap_bytes(int(c), bits_per_key) for c in counts], dtype=np.uint64)
    alloc = np.array([bitmap_alloc_bytes(int(c), bits_per_key) for c in counts], dtype=np.uint64)
    boff = np.zeros(F, dtype=np.uint64)
    if F > 1:
        boff[1:] = np.cumsum(alloc[:-1])
    out = empty_device(int(alloc.sum()), keys.device)
    ws_bytes = workspace_bytes(counts, bits_per_key)
    ws = empty_device(ws_bytes, keys.device)
    pk = _dptr(keys)
    po = _dptr(offsets)
    stride = 0 if offsets is not None else keys.shape[1]
    _check(lib().adl_bloom_build_segmented_device_ex(pk, po, stride, kb.ctypes.data, F, bits_per_key,
                                                     _dptr(out), boff.ctypes.data, flags, _dptr(ws), ws_bytes,
                                                     _stream(stream)), "adl_bloom_build_segmented_device_ex")
    torch.cuda.current_stream().synchronize()  # ws/out lifetimes end with this call's tensors
    return out, boff, sizes


def filter_block_bytes(key_begin, bits_per_key: int = 10) -> int:
    kb = np.ascontiguousarray(key_begin, dtype=np.uint64)
    return lib().adl_bloom_filter_block_bytes(kb.ctypes.data, len(kb) - 1, bits_per_key)


def build_filter_block(keys, key_begin, offsets=None, bits_per_key: int = 10, stream=None):
    """FilterBlockWriter: Keys2Block() per filter + Final(), framed on the device
    (adl_bloom_filter_block_build_device).  Returns the whole block as a uint8
    device tensor, byte-identical to the reference's."""
    kb = np.ascontiguousarray(key_begin, dtype=np.uint64)
    F = len(kb) - 1
    L = lib()
    nbytes = L.adl_bloom_filter_block_bytes(kb.ctypes.data, F, bits_per_key)
    if nbytes == 0:
        raise AdlBloomError(-2, "filter block size")
    ws_bytes = L.adl_bloom_filter_block_workspace_bytes(kb.ctypes.data, F, bits_per_key)
    dev = keys.device if keys is not None else "cuda"
    block = empty_device(nbytes, dev)
    ws = empty_device(ws_bytes, dev)
    stride = 0 if offsets is not None else (int(keys.shape[1]) if keys is not None else 16)
    _check(L.adl_bloom_filter_block_build_device(_dptr(keys), _dptr(offsets), stride, kb.ctypes.data, F,
                                                 bits_per_key, _dptr(block), nbytes, _dptr(ws), ws_bytes,
                                                 _stream(stream)), "adl_bloom_filter_block_build_device")
    _torch().cuda.current_stream().synchronize()  # ws lifetime ends with this call
    return block[:nbytes]


def _host_ptr(a):
    """Host address of a numpy array or a CPU (possibly pinned) torch tensor."""
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    assert not a.is_cuda, "host buffer expected"
    return a.data_ptr()


def build_segmented_host(keys, key_begin, out, bitmap_off, offsets=None, bits_per_key: int = 10, stream=None,
                         flags: int = 0):
    """Host-pointer pipelined segmented build (adl_bloom_build_segmented, or
    _ex with flags): keys (n, stride) uint8 or packed bytes + offsets (n+1) in
    host memory (numpy, or CPU torch tensors -- pinned ones are DMAed
    directly); filter f's exact-length bitmap lands at out[bitmap_off[f]:]
    (out: host uint8 buffer)."""
    kb = np.ascontiguousarray(key_begin, dtype=np.uint64)
    bo = np.ascontiguousarray(bitmap_off, dtype=np.uint64)
    stride = 0 if offsets is not None else int(keys.shape[1])
    args = (_host_ptr(keys), None if offsets is None else _host_ptr(offsets), stride, kb.ctypes.data, len(kb) - 1,
            bits_per_key, _host_ptr(out), bo.ctypes.data)
    if flags:
        _check(lib().adl_bloom_build_segmented_ex(*args, flags, _stream(stream)), "adl_bloom_build_segmented_ex")
    else:
        _check(lib().adl_bloom_build_segmented(*args, _stream(stream)), "adl_bloom_build_segmented")
    return out


def probe(keys, bitmap, nbytes: int | None = None, offsets=None, bits_per_key: int = 10, stream=None):
    """IsKeyExists on the GPU for a batch: uint8 device tensor of 0/1."""
    pk, po, n, stride = _keyset(keys, offsets)
    nbytes = bitmap.numel() if nbytes is None else nbytes
    out = _torch().empty(max(n, 1), dtype=_torch().uint8, device=keys.device)
    _check(lib().adl_bloom_probe_device(pk, po, n, stride, bits_per_key, _dptr(bitmap), nbytes,
                                        _dptr(out), _stream(stream)), "adl_bloom_probe_device")
    return out[:n]


def probe_multi(keys, filter_id, bitmaps, bitmap_off, offsets=None, bits_per_key: int = 10, stream=None):
    """Key i against filter filter_id[i]; bitmap_off: device uint64 tensor (F+1)."""
    pk, po, n, stride = _keyset(keys, offsets)
    out = _torch().empty(max(n, 1), dtype=_torch().uint8, device=keys.device)
    _check(lib().adl_bloom_probe_multi_device(pk, po, n, stride, _dptr(filter_id), bitmap_off.numel() - 1,
                                              _dptr(bitmaps), _dptr(bitmap_off), bits_per_key,
                                              _dptr(out), _stream(stream)), "adl_bloom_probe_multi_device")
    return out[:n]


def probe_batch(keys, filter_id, bitmaps, bitmap_off, offsets=None, bits_per_key: int = 10, stream=None,
                bitmap_end=None, out=None):
    """Large-batch multi-filter probe (adl_bloom_probe_batch_device): the answers of
    probe_multi, through the tile-binned pipeline when the batch is large.  The
    workspace comes from torch's caching allocator.  `out`: an optional uint8
    device tensor of at least n bytes (any alignment) to answer into."""
    pk, po, n, stride = _keyset(keys, offsets)
    F = bitmap_off.numel() - (0 if bitmap_end is not None else 1)
    L = lib()
    wsb = L.adl_bloom_probe_batch_workspace_bytes(n, F, bits_per_key, stride)
    ws = empty_device(wsb, keys.device)
    if out is None:
        out = _torch().empty(max(n, 1), dtype=_torch().uint8, device=keys.device)
    elif out.dtype != _torch().uint8 or out.numel() < n or not out.is_contiguous():
        raise ValueError("out must be a contiguous uint8 tensor of at least n elements")
    _check(L.adl_bloom_probe_batch_device(pk, po, n, stride, _dptr(filter_id), F, _dptr(bitmaps), _dptr(bitmap_off),
                                          _dptr(bitmap_end), bits_per_key, _dptr(out), _dptr(ws), wsb,
                                          _stream(stream)), "adl_bloom_probe_batch_device")
    return out[:n]


def murmur3_batch(keys, offsets=None, seed_a=SEED1, seed_b=SEED2, stream=None):
    pk, po, n, stride = _keyset(keys, offsets)
    out = _torch().empty((max(n, 1), 2), dtype=_torch().int32, device=keys.device)
    _check(lib().adl_bloom_murmur3_device(pk, po, n, stride, seed_a, seed_b, _dptr(out), _stream(stream)),
           "adl_bloom_murmur3_device")
    return out[:n]


def murmur3(seed: int, data: bytes) -> int:
    """murmur3_hash(seed, data, len) evaluated on the GPU."""
    buf = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    h = ctypes.c_uint32(0)
    _check(lib().adl_bloom_murmur3(seed, ctypes.cast(buf, ctypes.c_void_p), len(data), ctypes.byref(h)),
           "adl_bloom_murmur3")
    return h.value


# test-only fault injection (include/adl_bloom.h, adl_bloom_test_fault)
TEST_FAULT_PIPELINE_GROUP = 1
TEST_FAULT_CACHE_COMPLETION = 2


def test_fault(site: int, arg: int) -> None:
    """Arm (arg >= 0) or disarm (arg < 0) a one-shot injected failure."""
    _check(lib().adl_bloom_test_fault(site, arg), "adl_bloom_test_fault")


def probe_server_launches() -> int:
    """Probe-server kernels this process has launched (relaunches included)."""
    n = ctypes.c_uint64(0)
    _check(lib().adl_bloom_probe_server_launches(ctypes.byref(n)), "adl_bloom_probe_server_launches")
    return n.value


def profile_enable(capacity: int = 4096) -> None:
    """Start per-kernel HIP-event timing of builds issued by this thread."""
    _check(lib().adl_bloom_profile_enable(capacity), "adl_bloom_profile_enable")


def profile_each(capacity: int = 4096):
    """-> [(pass A ms, pass B ms)] per timed launch pair so far (timing keeps running)."""
    buf = (ctypes.c_double * (2 * capacity))()
    n = ctypes.c_uint32(0)
    _check(lib().adl_bloom_profile_each(buf, capacity, ctypes.byref(n)), "adl_bloom_profile_each")
    return [(buf[2 * i], buf[2 * i + 1]) for i in range(n.value)]


def profile_collect():
    """-> (pass A ms summed, pass B ms summed, builds timed); stops timing."""
    ms = (ctypes.c_double * 2)()
    nb = ctypes.c_uint32(0)
    _check(lib().adl_bloom_profile_collect(ms, ctypes.byref(nb)), "adl_bloom_profile_collect")
    return ms[0], ms[1], nb.value


# ------------------------------------------------------------------ host-pointer API
def build_host(keys: np.ndarray, offsets: np.ndarray | None = None, bits_per_key: int = 10,
               out: np.ndarray | None = None) -> np.ndarray:
    """adl_bloom_build: host keys in, host bitmap out (upload + build + download).
    `out`: an optional uint8 host array (any alignment; pinned or pageable) of
    at least the bitmap's size to write it into."""
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    if offsets is None:
        n, stride, po = keys.shape[0], keys.shape[1], None
    else:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n, stride, po = len(offsets) - 1, 0, offsets.ctypes.data
    nb = bitmap_bytes(n, bits_per_key)
    if nb == 0:
        raise AdlBloomError(-2, "bitmap size")
    if out is None:
        out = np.empty(nb, dtype=np.uint8)
    elif out.dtype != np.uint8 or out.size < nb or not out.flags["C_CONTIGUOUS"]:
        raise ValueError("out must be a contiguous uint8 array of at least the bitmap's size")
    kp = keys.ctypes.data if keys.size else np.zeros(1, np.uint8).ctypes.data
    _check(lib().adl_bloom_build(kp, po, n, stride, bits_per_key, out.ctypes.data, None), "adl_bloom_build")
    return out[:nb]


def probe_host(keys: np.ndarray, bitmap: np.ndarray, offsets: np.ndarray | None = None,
               bits_per_key: int = 10) -> np.ndarray:
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    bitmap = np.ascontiguousarray(bitmap, dtype=np.uint8)
    if offsets is None:
        n, stride, po = keys.shape[0], keys.shape[1], None
    else:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n, stride, po = len(offsets) - 1, 0, offsets.ctypes.data
    out = np.empty(max(n, 1), dtype=np.uint8)
    _check(lib().adl_bloom_probe(keys.ctypes.data, po, n, stride, bits_per_key, bitmap.ctypes.data,
                                 bitmap.size, out.ctypes.data, None), "adl_bloom_probe")
    return out[:n]


class FilterSet:
    """Device-resident bitmaps (adl_bloom_filter_set): the reader side."""

    def __init__(self, bitmaps: np.ndarray, bitmap_off: np.ndarray, bits_per_key: int = 10):
        bitmaps = np.ascontiguousarray(bitmaps, dtype=np.uint8)
        off = np.ascontiguousarray(bitmap_off, dtype=np.uint64)
        self._h = ctypes.c_void_p()
        _check(lib().adl_bloom_filter_set_create(bitmaps.ctypes.data, off.ctypes.data, len(off) - 1,
                                                 bits_per_key, ctypes.byref(self._h)),
               "adl_bloom_filter_set_create")

    def probe(self, keys: np.ndarray, filter_id=None, filter: int = 0, offsets=None) -> np.ndarray:
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        if offsets is None:
            n, stride, po = keys.shape[0], keys.shape[1], None
        else:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            n, stride, po = len(offsets) - 1, 0, offsets.ctypes.data
        fid = None if filter_id is None else np.ascontiguousarray(filter_id, dtype=np.uint32)
        out = np.empty(max(n, 1), dtype=np.uint8)
        _check(lib().adl_bloom_filter_set_probe(self._h, keys.ctypes.data, po, n, stride,
                                                None if fid is None else fid.ctypes.data, filter,
                                                out.ctypes.data, None), "adl_bloom_filter_set_probe")
        return out[:n]

    def close(self):
        if self._h:
            lib().adl_bloom_filter_set_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FilterCache:
    """Device-resident filter blocks keyed by SSTable oid, LRU (adl_bloom_filter_cache)."""

    def __init__(self, capacity_bytes: int, max_tables: int = 64, bits_per_key: int = 10):
        self._h = ctypes.c_void_p()
        _check(lib().adl_bloom_filter_cache_create(capacity_bytes, max_tables, bits_per_key, ctypes.byref(self._h)),
               "adl_bloom_filter_cache_create")

    def put(self, oid: bytes, block: bytes) -> None:
        b = np.frombuffer(block, dtype=np.uint8)
        _check(lib().adl_bloom_filter_cache_put(self._h, oid, len(oid), b.ctypes.data, b.size),
               "adl_bloom_filter_cache_put")

    def put_status(self, oid: bytes, block: bytes) -> int:
        b = np.frombuffer(block, dtype=np.uint8)
        return lib().adl_bloom_filter_cache_put(self._h, oid, len(oid), b.ctypes.data, b.size)

    def __contains__(self, oid: bytes) -> bool:
        return lib().adl_bloom_filter_cache_contains(self._h, oid, len(oid)) == 1

    def remove(self, oid: bytes) -> bool:
        return lib().adl_bloom_filter_cache_remove(self._h, oid, len(oid)) == 1

    def stats(self):
        t, b = ctypes.c_uint32(), ctypes.c_uint64()
        _check(lib().adl_bloom_filter_cache_stats(self._h, ctypes.byref(t), ctypes.byref(b)), "stats")
        return t.value, b.value

    def probe(self, oids, table, keys: np.ndarray, offsets=None, filter: int = 0):
        """Query i against filter `filter` of table oids[table[i]]; returns (0/1 array, uncached count)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        if offsets is None:
            n, stride, po = keys.shape[0], keys.shape[1], None
        else:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            n, stride, po = len(offsets) - 1, 0, offsets.ctypes.data
        arr = (ctypes.c_char_p * max(len(oids), 1))(*oids)
        lens = np.array([len(o) for o in oids] or [0], dtype=np.uint64)
        tab = np.ascontiguousarray(table, dtype=np.uint32)
        out = np.empty(max(n, 1), dtype=np.uint8)
        unc = ctypes.c_uint64()
        _check(lib().adl_bloom_filter_cache_probe(self._h, arr, lens.ctypes.data, len(oids), filter,
                                                  keys.ctypes.data, po, n, stride, tab.ctypes.data,
                                                  out.ctypes.data, ctypes.byref(unc), None),
               "adl_bloom_filter_cache_probe")
        return out[:n], unc.value

    def close(self):
        if self._h:
            lib().adl_bloom_filter_cache_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ synthetic inputs
def synth_keys16(n: int, seed: int = 0x5EED, skip: int = 0, device="cuda", stream=None):
    """SURVEY.md §8d SplitMix64 16-byte keys generated on the device: (n,16) uint8."""
    keys = _torch().empty((max(n, 1), 16), dtype=_torch().uint8, device=device)
    _check(lib().adl_synth_keys16_device(_dptr(keys), seed, skip, n, _stream(stream)), "adl_synth_keys16_device")
    return keys[:n]


def synth_varlen(n: int, seed: int = 0x5EED, zipf_s: float = 1.1, device="cuda", stream=None):
    """Variable-length keys (8..256 B, Zipf lengths) on the device: (bytes, offsets[n+1] uint64)."""
    torch = _torch()
    lengths = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    _check(lib().adl_synth_varlen_lengths_device(_dptr(lengths), seed, n, zipf_s, _stream(stream)),
           "adl_synth_varlen_lengths_device")
    offs = torch.zeros(n + 1, dtype=torch.int64, device=device)
    if n:
        offs[1:] = torch.cumsum(lengths[:n].to(torch.int64), 0)
    total = int(offs[-1].item())
    data = torch.empty(((total + 15) // 16) * 16 + 16, dtype=torch.uint8, device=device)
    _check(lib().adl_synth_varlen_fill_device(_dptr(data), seed, total, _stream(stream)),
           "adl_synth_varlen_fill_device")
    return data, offs  # int64 storage, read as uint64 offsets by the C-ABI


def synth_probe_queries(n: int, seed: int = 0xFEED, q0: int = 0, num_tables: int = 256,
                        table_seed0: int = 0x5EED, keys_per_table: int = 1_000_000, device="cuda", stream=None):
    """Probe queries of BASELINE.json configs[4] on the device: (keys (n,16) u8, filter_id int32
    (read as uint32), member u8) -- see adl_synth_probe_queries_device."""
    torch = _torch()
    keys = torch.empty((max(n, 1), 16), dtype=torch.uint8, device=device)
    fid = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    member = torch.empty(max(n, 1), dtype=torch.uint8, device=device)
    _check(lib().adl_synth_probe_queries_device(_dptr(keys), _dptr(fid), _dptr(member), seed, q0, n, num_tables,
                                                table_seed0, keys_per_table, _stream(stream)),
           "adl_synth_probe_queries_device")
    return keys[:n], fid[:n], member[:n]
