"""CPU: the C-ABI library builds, loads, and exports every symbol
include/adl_bloom.h declares; host-side arithmetic matches the oracle.
No compute call is made here (no GPU in this container)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "adl_bloom.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(adl_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import adlbloom

    L = adlbloom.lib()
    decl = declared_functions()
    assert len(decl) >= 20
    for name in decl:
        assert hasattr(L, name), name
    assert sorted(adlbloom.EXPORTS) == decl
    nm = subprocess.run(["nm", "-D", "--defined-only", adlbloom.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r" T (adl_\w+)", nm))
    assert set(decl) <= exported


def test_library_is_gfx950_code_object():
    import adlbloom

    blob = open(adlbloom.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # the offload bundle carries gfx950 code
    assert b"bloom_bin_kernel" in blob and b"bloom_tile_kernel" in blob


def test_abi_version_and_strerror():
    import adlbloom

    L = adlbloom.lib()
    assert L.adl_bloom_abi_version() == 1
    assert L.adl_bloom_strerror(0) == b"ok"
    assert L.adl_bloom_strerror(13) == b"filter block error"
    assert b"device" in L.adl_bloom_strerror(-3).lower()


@pytest.mark.parametrize("bpk", [-1, 0, 1, 2, 3, 5, 8, 9, 10, 11, 12, 16, 20, 30, 43, 44, 45, 100])
def test_num_probes_matches_oracle(oracle, bpk):
    import adlbloom

    if bpk < 0:
        return
    assert adlbloom.num_probes(bpk) == oracle.num_probes(bpk)


@pytest.mark.parametrize("n,bpk", [(0, 10), (1, 10), (10_000_000, 10), (26_843_544, 10), (26_843_545, 10),
                                   (268_435_448, 1), (268_435_449, 1), (5, 0), (3, -1), (2**40, 10)])
def test_bitmap_bytes_matches_oracle(oracle, n, bpk):
    import adlbloom

    assert adlbloom.bitmap_bytes(n, bpk) == oracle.bitmap_bytes(n, bpk)
    a = adlbloom.bitmap_alloc_bytes(n, bpk)
    b = adlbloom.bitmap_bytes(n, bpk)
    assert (a == 0) == (b == 0)
    assert a % 16 == 0 and a >= b and a - b < 16


def test_workspace_bytes():
    import adlbloom

    ws = adlbloom.workspace_bytes([10_000_000], 10)
    # 6 positions x 4 B per key + (tile, chunk) table + (h1, h2) 8 B per key
    # (variable-length keys are hashed into the workspace before pass A)
    assert 320_000_000 <= ws < 340_000_000
    assert adlbloom.workspace_bytes([0], 10) > 0
    assert adlbloom.workspace_bytes([1_000_000] * 32, 10) > 0
    assert adlbloom.workspace_bytes([2**31], 10) == 0  # too large -> 0


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    import adlbloom

    monkeypatch.setattr(adlbloom, "_LIB", None)
    monkeypatch.setattr(adlbloom, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(RuntimeError):
        adlbloom.lib()


def test_filter_block_bytes_matches_oracle_framing(oracle):
    """adl_bloom_filter_block_bytes (host arithmetic only) equals the length of
    the block FilterBlockWriter::Final writes (oracle framing, src/filter_block.cpp:77-102)."""
    import numpy as np

    import adlbloom

    rng = np.random.default_rng(3)
    for nf in (0, 1, 2, 7, 65, 200):
        for bpk in (1, 10, 23):
            sizes = rng.integers(0, 3000, size=nf)
            kb = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
            want = len(oracle.filter_block_final([bytes(oracle.bitmap_bytes(int(n), bpk)) for n in sizes], bpk))
            assert adlbloom.filter_block_bytes(kb, bpk) == want
    # beyond the reference's int offsets -> 0
    kb = (np.arange(10, dtype=np.uint64) * 26_000_000)  # 9 valid filters, 2.34 GB together
    assert adlbloom.filter_block_bytes(kb[:8], 10) > 0
    assert adlbloom.filter_block_bytes(kb, 10) == 0


def test_segmented_ex_rejects_unknown_flags():
    """Argument checks run before any device call (no GPU here)."""
    import ctypes

    import adlbloom

    L = adlbloom.lib()
    kb = (ctypes.c_uint64 * 2)(0, 16)
    off = (ctypes.c_uint64 * 1)(0)
    buf = ctypes.create_string_buffer(64)
    rc = L.adl_bloom_build_segmented_device_ex(ctypes.addressof(buf), None, 16, kb, 1, 10,
                                               ctypes.addressof(buf), off, 0x80, None, 0, None)
    assert rc == -1  # ADL_ERR_INVALID_ARG
