"""GPU: pass A's claim layout (ADL_BLOOM_CLAIM; bloom_bin16_kernel<..., CL> in
adlsm-tree_amd/csrc/bloom_build.hip) against the oracle and the reference's
SHA-256s.

Each tile of a chunk region gets a fixed share of slots and a position claims
one with a single LDS atomic (no count pass, no scan).  A chunk in which a tile
outgrows its share is counting-sorted exactly instead.  The "tight" settings
force that fallback: ADL_BLOOM_CLAIM=2 skips the plan's share test and
ADL_BLOOM_CLAIM_CAP=101 leaves about 1 % slack, so most chunks overflow; "mid"
(107 %) mixes overflowing and claimed chunks in one launch.  Every bitmap must
equal BloomFilter::Keys2Block (reference src/filter_block.cpp:9-33).
"""
import hashlib
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SETTINGS = {
    "default": {},
    "auto": {"ADL_BLOOM_CLAIM": "1"},
    "mid": {"ADL_BLOOM_CLAIM": "2", "ADL_BLOOM_CLAIM_CAP": "107"},
    "tight": {"ADL_BLOOM_CLAIM": "2", "ADL_BLOOM_CLAIM_CAP": "101"},
}


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


@pytest.fixture(params=list(SETTINGS), ids=list(SETTINGS))
def claim(request, knobs):
    for k, v in SETTINGS[request.param].items():
        knobs.set(k, v)
    return request.param


def test_claim_plan_selected(dev, ab, knobs, capfd):
    """ADL_BLOOM_CLAIM=1 takes the claim layout for 32 filters of 100 K keys
    (31 tiles of 2^18 bits each, about 800 positions per tile and chunk) and
    refuses it for the headline's single 10 M-key filter (763 tiles of 2^20
    bits, about 44 per tile and chunk: too few for a fixed share)."""
    knobs.set("ADL_BLOOM_CLAIM", "1")
    knobs.set("ADL_BLOOM_DEBUG", "1")
    assert ab.workspace_bytes([100_000] * 32, 10) > 0
    assert "(claim)" in capfd.readouterr().err
    assert ab.workspace_bytes([10_000_000], 10) > 0
    assert "(claim)" not in capfd.readouterr().err
    # default: only filters of at most 10 tiles (256 x 10 K: 4 tiles each)
    knobs.unset("ADL_BLOOM_CLAIM")
    assert ab.workspace_bytes([10_000] * 256, 10) > 0
    assert "(claim)" in capfd.readouterr().err
    assert ab.workspace_bytes([100_000] * 32, 10) > 0
    assert "(claim)" not in capfd.readouterr().err


def test_claim_headline_reference_sha(dev, ab, golden, claim):
    """10M x 16 B keys, bpk 10: the reference's Appendix B SHA-256, three times
    into a dirty bitmap and workspace."""
    want = {g["n"]: g["sha256"] for g in golden["appendix_b"]["bitmaps"]}[10_000_000]
    keys = ab.synth_keys16(10_000_000, seed=0x5EED)
    b = ab.Builder(10_000_000, 10)
    b.bitmap.fill_(0xFF)
    b.ws.fill_(0x5A)
    for _ in range(3):
        got = hashlib.sha256(b.build(keys).cpu().numpy().tobytes()).hexdigest()
        assert got == want


@pytest.mark.parametrize("n,bpk", [(20000, 10), (1_000_003, 3), (3_000_000, 20), (2_000_000, 44)])
def test_claim_build_vs_oracle(dev, ab, oracle, claim, n, bpk):
    keys = ab.synth_keys16(n, seed=n + bpk)
    bm = ab.build(keys, bits_per_key=bpk).cpu().numpy()
    assert np.array_equal(bm, oracle.keys2block(keys.cpu().numpy(), bits_per_key=bpk))


def test_claim_duplicate_keys(dev, ab, oracle, claim):
    """7 distinct keys repeated 20 000 times: every position of a chunk lands
    in at most 42 bits, far past any tile's share."""
    base = ab.synth_keys16(7, seed=1).cpu().numpy()
    keys = np.repeat(base, 20000, axis=0)
    bm = ab.build(dev.from_numpy(keys).cuda()).cpu().numpy()
    assert np.array_equal(bm, oracle.keys2block(keys))


def test_claim_skewed_keys(dev, ab, oracle, claim):
    """9 distinct keys with h1 != h2 (not skipped by the pair table) shuffled
    into 400 000: a few tiles take every position."""
    rng = np.random.default_rng(5)
    base = rng.integers(0, 256, (64, 16), dtype=np.uint8)
    h = oracle.murmur3_batch(base)
    base = base[h[:, 0] != h[:, 1]][:9]
    keys = np.repeat(base, 400_000 // len(base) + 1, axis=0)[:400_000]
    rng.shuffle(keys)
    bm = ab.build(dev.from_numpy(keys).cuda()).cpu().numpy()
    assert np.array_equal(bm, oracle.keys2block(keys))


@pytest.mark.parametrize("sizes", [
    [10_000] * 256,
    [1_000_000] * 8,
    [0, 1, 1000, 2_000_000, 7, 123_456, 6144, 6145, 3, 1_500_000, 10, 99_999, 2],
    [40_000] * 256,
], ids=["256x10K", "8x1M", "13-mixed", "256x40K"])
def test_claim_segmented_16b(dev, ab, oracle, claim, sizes):
    kb = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    keys = ab.synth_keys16(int(kb[-1]), seed=42 + len(sizes))
    out, boff, nbytes = ab.build_segmented(keys, kb)
    out, hk = out.cpu().numpy(), keys.cpu().numpy()
    for f in range(len(sizes)):
        assert np.array_equal(out[int(boff[f]):int(boff[f]) + int(nbytes[f])],
                              oracle.keys2block(hk[kb[f]:kb[f + 1]])), f


def test_claim_varlen(dev, ab, oracle, claim):
    """Variable-length keys: the hashing pass, then the claim pass A over the
    (h1, h2) pairs."""
    data, offs = ab.synth_varlen(3_000_000, seed=0x5EED)
    bm = ab.build(data, offs).cpu().numpy()
    assert np.array_equal(bm, oracle.keys2block(data.cpu().numpy(), offs.cpu().numpy().view(np.uint64)))


def test_claim_segmented_varlen_many_filters(dev, ab, oracle, claim):
    rng = random.Random(77)
    sizes = [0, 1, 511, 512, 513, 400_000, 7, 0, 1, 900_000, 3, 1025, 20000]
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


def test_claim_positions_count(dev, ab, oracle, claim, knobs):
    """adl_bloom_build_positions reads the claim layout's (start, length)
    entries: with the pair table off every key writes k = 6 positions, and
    the bitmaps still equal the oracle's (256 filters of 10 K keys, the
    default's claim shape)."""
    knobs.set("ADL_BLOOM_HASH_DEDUP", "0")
    sizes = [10_000] * 255 + [9_999]
    kb = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    keys = ab.synth_keys16(int(kb[-1]), seed=99)
    sb = ab.SegmentedBuilder(kb)
    out = sb.build(keys).cpu().numpy()
    assert sb.positions() == 6 * int(kb[-1])
    hk = keys.cpu().numpy()
    for f in (0, 1, 128, 255):
        o = int(sb.boff[f])
        assert np.array_equal(out[o:o + int(sb.sizes[f])], oracle.keys2block(hk[kb[f]:kb[f + 1]])), f


def test_builds_with_a_resident_server(dev, ab, oracle, golden):
    """While a resident probe server exists (a reader), pass A and pass B take
    their chunks and tiles from the work queues (GroupQueue, bloom_build.hip)
    instead of the static stripes.  The same bitmaps: the 10 M reference SHA
    (chunk/table layout), 256 x 10 K (claim layout), 32 x 100 K (two pass-B
    workgroups per CU), var-len keys, built while single-key Gets keep the
    server running."""
    blk_keys = oracle.splitmix_keys16(0x5151, 20_000)
    bm0 = oracle.keys2block(blk_keys)
    cache = ab.FilterCache(8 << 20, max_tables=8)
    # a one-filter block in the reference's framing
    cache.put(b"t0", oracle.filter_block_final([bm0.tobytes()], bits_per_key=10))
    t = np.zeros(1, np.uint32)

    def get(i):
        got, _ = cache.probe([b"t0"], t, blk_keys[i:i + 1])
        assert got[0] == 1  # an inserted key

    try:
        get(0)  # the server now exists
        g = golden["appendix_b"]["bitmaps"][5]
        keys = ab.synth_keys16(g["n"], seed=0x5EED)
        b = ab.Builder(g["n"], 10)
        for r in range(3):
            get(r + 1)
            bm = b.build(keys).cpu().numpy()
            assert hashlib.sha256(bm.tobytes()).hexdigest() == g["sha256"], r
        del keys, b
        for sizes in ([10_000] * 256, [100_000] * 32, [1, 0, 70_000, 5]):
            get(7)
            kb = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
            hk = oracle.splitmix_keys16(0xAB + len(sizes), int(kb[-1]))
            out, boff, nbytes = ab.build_segmented(dev.from_numpy(hk).cuda(), kb)
            out = out.cpu().numpy()
            for f in range(len(sizes)):
                if sizes[f]:
                    assert np.array_equal(out[int(boff[f]):int(boff[f]) + int(nbytes[f])],
                                          oracle.keys2block(hk[int(kb[f]):int(kb[f + 1])])), (len(sizes), f)
        data, offs = ab.synth_varlen(300_000, seed=5)
        get(9)
        got = ab.build(data, offs).cpu().numpy()
        assert np.array_equal(got, oracle.keys2block(data.cpu().numpy(), offs.cpu().numpy().view(np.uint64)))
    finally:
        cache.close()
