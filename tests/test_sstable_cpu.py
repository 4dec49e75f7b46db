"""SSTable build path, CPU side.

* the oracle's restatement of the reference's SSTable format
  (oracle/sstable_oracle.py) reproduces the reference's own SSTable oid for
  the test/sstable_test.cpp:9-27 memtable;
* the writer's SHA-256 (adlsm-tree_amd/csrc/sstable_writer.cpp), which names
  the file, agrees with hashlib at every padding boundary;
* the test binary fails loudly (non-zero, "device error") without a GPU
  rather than falling back to a CPU filter.
"""
import hashlib
import os
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "adlsm-tree_amd", "bin", "sstable_test")


@pytest.fixture(scope="module")
def S(oracle):
    import sstable_oracle

    return sstable_oracle


def test_oracle_sstable_oid_matches_reference(S, golden):
    g = golden["appendix_b"]["sstable_test"]
    b = S.sstable_bytes(S.sstable_test_entries(1))
    assert len(b) == g["bytes"]
    assert S.oid(b) == g["oid"]


def test_oracle_sstable_structure(S, oracle):
    """Footer -> meta -> filter handle; the filter block is the reference's
    one-filter block over the user keys; data blocks restart every 12 entries."""
    ents = S.sstable_test_entries(2)
    b = S.sstable_bytes(ents)
    assert b[-2:] == b"\x12\x34"
    moff, mlen, ioff, ilen = struct.unpack_from("<iiii", b, len(b) - 18)
    assert ioff == moff + mlen and ioff + ilen == len(b) - 18
    fb = S.filter_block_of(b)
    user = [k[:-9] for k, _ in ents]
    bm = oracle.keys2block(user, bits_per_key=10).tobytes()
    assert fb == oracle.filter_block_final([bm], 10)
    # first data block: restart count and offsets at its tail
    blk = S.BlockWriterOracle()
    for i in range(30):
        blk.add(ents[i][0], ents[i][1])
    raw = blk.final()
    (nr,) = struct.unpack_from("<i", raw, len(raw) - 4)
    assert nr == 3  # entries 0, 12, 24
    r = struct.unpack_from("<3i", raw, len(raw) - 16)
    assert r[0] == 0 and struct.unpack_from("<i", raw, r[1])[0] == 0  # restart: shared = 0


def test_oracle_memtable_order(S):
    e = S.memtable_order([(b"b", 1, 0, b""), (b"a", 1, 0, b""), (b"a", 5, 0, b""), (b"a", 5, 1, b"")])
    assert [(u, s, o) for u, s, o, _ in e] == [(b"a", 5, 1), (b"a", 5, 0), (b"a", 1, 0), (b"b", 1, 0)]


@pytest.mark.parametrize("size", [0, 1, 55, 56, 63, 64, 65, 119, 120, 128, 4097, 100000])
def test_writer_sha256(size, tmp_path):
    data = hashlib.sha256(str(size).encode()).digest() * (size // 32 + 1)
    data = data[:size]
    p = tmp_path / "f.bin"
    p.write_bytes(data)
    r = subprocess.run([EXE, "sha256", str(p)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == hashlib.sha256(data).hexdigest()


def test_sstable_binary_fails_loudly_without_gpu(tmp_path):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present: the GPU parity test covers this binary")
    r = subprocess.run([EXE, "1", str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "device error" in r.stderr
    assert not list(tmp_path.glob("*.sst"))
