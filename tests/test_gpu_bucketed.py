"""GPU: the bucketed build (adlsm-tree_amd/csrc/bloom_bucket.hip, ADL_BLOOM_BK=1)
against the oracle and the reference's SHA-256s.

Not the default (measured slower overall than the chunk/table build, DESIGN.md
§5 round 4), but a complete, selectable build: per-slice LDS buckets per
2^20-bit tile (pass A), per-(slice, tile) regions read as long runs (pass B),
overflow extents for skewed key sets, u32 or 24-bit entries (ADL_BLOOM_BK_P3),
16-byte keys and variable-length keys through the hashing pass.  Every bitmap
must equal BloomFilter::Keys2Block (reference src/filter_block.cpp:9-33).
"""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    torch.cuda.set_device(0)
    return torch


@pytest.fixture(scope="module")
def ab():
    import adlbloom

    adlbloom.lib()
    return adlbloom


@pytest.fixture(params=["0", "1"], ids=["u32", "p3"])
def bk(request, monkeypatch):
    monkeypatch.setenv("ADL_BLOOM_BK", "1")
    monkeypatch.setenv("ADL_BLOOM_BK_P3", request.param)
    return request.param


@pytest.mark.parametrize("n,bpk", [(1, 10), (5, 1), (20000, 10), (1_000_000, 10), (1_000_003, 3),
                                   (3_000_000, 20), (300_000, 44)])
def test_bucketed_build_vs_oracle(dev, ab, oracle, bk, n, bpk):
    keys = ab.synth_keys16(n, seed=n + bpk)
    bm = ab.build(keys, bits_per_key=bpk).cpu().numpy()
    assert np.array_equal(bm, oracle.keys2block(keys.cpu().numpy(), bits_per_key=bpk))


def test_bucketed_headline_reference_sha(dev, ab, golden, bk):
    """10M x 16 B keys, bpk 10: the reference's Appendix B SHA-256, three times
    into a dirty bitmap and workspace."""
    import hashlib

    want = {g["n"]: g["sha256"] for g in golden["appendix_b"]["bitmaps"]}[10_000_000]
    keys = ab.synth_keys16(10_000_000, seed=0x5EED)
    b = ab.Builder(10_000_000, 10)
    b.bitmap.fill_(0xFF)
    b.ws.fill_(0x5A)
    for _ in range(3):
        got = hashlib.sha256(b.build(keys).cpu().numpy().tobytes()).hexdigest()
        assert got == want


def test_bucketed_duplicate_keys(dev, ab, oracle, bk):
    base = ab.synth_keys16(7, seed=1).cpu().numpy()
    keys = np.repeat(base, 20000, axis=0)
    bm = ab.build(dev.from_numpy(keys).cuda()).cpu().numpy()
    assert np.array_equal(bm, oracle.keys2block(keys))


def test_bucketed_skewed_overflow_extents(dev, ab, oracle, bk):
    """Overflow extents: 9 distinct keys (h1 != h2, so the pair table does not
    skip them) repeated to 400 000 keys put every slice's ~9 400 positions on
    at most 54 bits in a few of the filter's 31 tiles, far past a region's
    capacity (its uniform share plus six sigma), so most entries go through
    chained overflow extents."""
    rng = np.random.default_rng(5)
    base = rng.integers(0, 256, (64, 16), dtype=np.uint8)
    h = oracle.murmur3_batch(base)
    base = base[h[:, 0] != h[:, 1]][:9]
    keys = np.repeat(base, 400_000 // len(base) + 1, axis=0)[:400_000]
    rng.shuffle(keys)
    bm = ab.build(dev.from_numpy(keys).cuda()).cpu().numpy()
    assert np.array_equal(bm, oracle.keys2block(keys))


def test_bucketed_segmented_16b(dev, ab, oracle, bk):
    """13 filters (the descriptor table), empty and 1-key filters."""
    sizes = [0, 1, 1000, 50_000, 7, 123_456, 6144, 6145, 3, 200_000, 10, 99_999, 2]
    kb = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    keys = ab.synth_keys16(int(kb[-1]), seed=42)
    out, boff, nbytes = ab.build_segmented(keys, kb)
    out, hk = out.cpu().numpy(), keys.cpu().numpy()
    for f in range(len(sizes)):
        assert np.array_equal(out[int(boff[f]):int(boff[f]) + int(nbytes[f])],
                              oracle.keys2block(hk[kb[f]:kb[f + 1]])), f


def test_bucketed_varlen(dev, ab, oracle, bk):
    data, offs = ab.synth_varlen(300_000, seed=0x5EED)
    bm = ab.build(data, offs).cpu().numpy()
    assert np.array_equal(bm, oracle.keys2block(data.cpu().numpy(), offs.cpu().numpy().view(np.uint64)))


def test_bucketed_segmented_varlen_many_filters(dev, ab, oracle, bk):
    rng = random.Random(77)
    sizes = [0, 1, 511, 512, 513, 40000, 7, 0, 1, 90000, 3, 1025, 20000]
    keys = [rng.randbytes(rng.randrange(0, 120)) for _ in range(sum(sizes))]
    data, offs = oracle.pack(keys)
    pad = np.zeros(((data.size + 15) // 16) * 16 + 16, dtype=np.uint8)
    pad[: data.size] = data
    kb = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    out, boff, nbytes = ab.build_segmented(dev.from_numpy(pad).cuda(), kb,
                                           offsets=dev.from_numpy(offs.view(np.int64)).cuda())
    out = out.cpu().numpy()
    for f in range(len(sizes)):
        want = oracle.keys2block(keys[int(kb[f]):int(kb[f + 1])])
        assert np.array_equal(out[int(boff[f]):int(boff[f]) + int(nbytes[f])], want), f
