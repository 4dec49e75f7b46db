"""GPU: the read side of the filter path and the
host-pointer pipeline's corner cases.

* The level multi-get (LevelMultiGetFilter: Level::Get's candidate tables,
  src/revision.cpp:265-310, each checked as SSTableReader::Get does,
  src/sstable.cpp:238) over 24 cached SSTables, run single-threaded and from 8
  threads with tables coming and going (and, in a cache too small for the
  level, evicted under running probes): bin/readpath_test.  Its answers are
  checked here pair by pair against the oracle (the Python restatement of
  Level::Get's range test and FilterBlockReader over the same blocks).
* The filter cache's C-ABI probed from Python threads while other threads put
  and remove tables.
* adl_bloom_build_segmented (pipelined groups) with fixed strides whose group
  starts are not 16-byte aligned, and a build failing mid-pipeline.
"""
import os
import subprocess
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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


@pytest.mark.parametrize("server", ["1", "0"])
def test_level_multiget_threaded_vs_oracle(dev, oracle, tmp_path, server):
    """The level's tables are written with bits_per_key 10, 3 and 16 in turn
    and share one cache: every answer is checked against the oracle with each
    block's own bits_per_key.  server=0 sends the single-key IsKeyExists calls
    through a launched probe instead of the resident server."""
    exe = os.path.join(ROOT, "adlsm-tree_amd", "bin", "readpath_test")
    r = subprocess.run([exe, str(tmp_path), "8", "10" if server == "1" else "4"], capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, ADL_BLOOM_PROBE_SERVER=server))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "phase 1 (level cached) 0 mismatches" in r.stdout and "phase 2 (evicting) 0 mismatches" in r.stdout

    tables = []
    for line in (tmp_path / "tables.txt").read_text().split("\n"):
        if line:
            oid, mn, mx = line.split()
            tables.append((bytes.fromhex(mn), bytes.fromhex(mx)))
    assert len(tables) >= 16
    blocks = [(tmp_path / f"table_{t}.blk").read_bytes() for t in range(len(tables))]
    readers = []
    for b in blocks:
        rd = oracle.FilterBlockReaderOracle()
        assert rd.init(b) == 0
        readers.append(rd)
    queries = [bytes.fromhex(x) for x in (tmp_path / "queries.txt").read_text().split("\n") if x]
    got = {}
    for line in (tmp_path / "multiget.txt").read_text().split("\n"):
        if line:
            f = line.split()
            got[int(f[0])] = [(int(p.split(":")[0]), int(p.split(":")[1])) for p in f[1:]]
    assert len(got) == len(queries)
    # every table's filter 0 over every query, by the oracle
    want_bits = []
    assert sorted({rd.bits_per_key for rd in readers}) == [3, 10, 16]
    for rd in readers:
        o1, o2 = rd.filter_range(0)
        bm = np.frombuffer(rd.block[o1:o2], dtype=np.uint8)
        want_bits.append(oracle.probe(queries, bm, bits_per_key=rd.bits_per_key))
    pairs = hits = 0
    for i, q in enumerate(queries):
        cand = oracle.level_candidates(tables, q, 2**63 - 1)
        assert [t for t, _ in got[i]] == cand, i
        for t, m in got[i]:
            assert m == want_bits[t][i], (i, t)
            pairs += 1
            hits += m
    assert pairs > len(queries)  # overlapping ranges: several candidates per key
    assert 0 < hits < pairs


def _block(oracle, seed, n, bpk=10):
    keys = oracle.splitmix_keys16(seed, n)
    return keys, oracle.filter_block_final([oracle.keys2block(keys, bits_per_key=bpk).tobytes()], bpk)


def test_filter_cache_concurrent_put_probe(dev, ab, oracle):
    """Probes from 4 threads while 2 threads put/remove other tables and
    re-put the probed ones (no lock is held across a probe's kernel)."""
    T = 16
    tabs = [_block(oracle, 1000 + t, 20_000) for t in range(T)]
    cache = ab.FilterCache(64 << 20, max_tables=64)
    oids = [b"sst-%02d" % t for t in range(T)]
    for o, (_, blk) in zip(oids, tabs):
        cache.put(o, blk)
    rng = np.random.default_rng(5)
    n = 20_000
    table = rng.integers(0, T, n).astype(np.uint32)
    fresh = oracle.splitmix_keys16(0xF00D, n)
    q = np.where((rng.integers(0, 2, n) == 1)[:, None],
                 np.stack([tabs[t][0][i % 20_000] for i, t in enumerate(table)]), fresh)
    want = np.empty(n, np.uint8)
    for t in range(T):
        sel = table == t
        want[sel] = oracle.probe(q[sel], oracle.keys2block(tabs[t][0]))
    errors = []
    stop = threading.Event()

    def prober(k):
        for r in range(15):
            got, unc = cache.probe(oids, table, q)
            if unc or not np.array_equal(got, want):
                errors.append((k, r, int(unc), int((got != want).sum())))

    def churn(k):
        i = 0
        while not stop.is_set():
            cache.put(b"other-%d-%d" % (k, i % 4), tabs[i % T][1])
            cache.remove(b"other-%d-%d" % (k, (i + 2) % 4))
            cache.put(oids[(i * 3 + k) % T], tabs[(i * 3 + k) % T][1])  # replace a probed table
            i += 1

    th = [threading.Thread(target=prober, args=(k,)) for k in range(4)]
    ch = [threading.Thread(target=churn, args=(k,)) for k in range(2)]
    for t in th + ch:
        t.start()
    for t in th:
        t.join()
    stop.set()
    for t in ch:
        t.join()
    cache.close()
    assert not errors, errors[:5]


def test_filter_cache_small_batch_under_eviction(dev, ab, oracle):
    """Small batches (<= 4096 keys: the mapped buffer, answers watched instead
    of a stream synchronize) from 4 threads while a churn thread puts tables
    into a cache that holds about 6 of them, so probed tables are evicted while
    probes pin them.  An uncached table answers 1 ("may be present"); a
    range released too early would answer 0 for an inserted key."""
    T = 8
    tabs = [_block(oracle, 2000 + t, 20_000) for t in range(T)]
    blk_bytes = len(tabs[0][1])
    cache = ab.FilterCache(6 * blk_bytes + (64 << 10), max_tables=64)
    oids = [b"ev-%02d" % t for t in range(T)]
    rng = np.random.default_rng(11)
    n = 3000
    table = rng.integers(0, T, n).astype(np.uint32)
    fresh = oracle.splitmix_keys16(0xBEEF, n)
    q = np.where((rng.integers(0, 2, n) == 1)[:, None],
                 np.stack([tabs[t][0][(7 * i) % 20_000] for i, t in enumerate(table)]), fresh)
    want = np.empty(n, np.uint8)
    for t in range(T):
        sel = table == t
        want[sel] = oracle.probe(q[sel], oracle.keys2block(tabs[t][0]))
    errors, exact = [], [0]
    stop = threading.Event()

    def prober(k):
        for r in range(40):
            got, unc = cache.probe(oids, table, q)
            if np.any(got < want) or (unc == 0 and not np.array_equal(got, want)):
                errors.append((k, r, int(unc), int((got < want).sum())))
            exact[0] += unc == 0

    def churn():
        i = 0
        while not stop.is_set():
            cache.put(oids[i % T], tabs[i % T][1])
            cache.put(b"filler-%d" % (i % 3), tabs[(i + 3) % T][1])
            i += 1

    for o, (_, blk) in zip(oids[:6], tabs[:6]):
        cache.put(o, blk)
    th = [threading.Thread(target=prober, args=(k,)) for k in range(4)]
    ch = threading.Thread(target=churn)
    for t in th + [ch]:
        t.start()
    for t in th:
        t.join()
    stop.set()
    ch.join()
    cache.close()
    assert not errors, errors[:5]


def test_filter_cache_completion_fault(dev, ab, oracle):
    """A small batch whose launch reports an error after every answer has
    arrived in the mapped buffer fails (it does not return those answers), and
    the next call on the same thread is exact again."""
    keys, blk = _block(oracle, 3000, 20_000)
    cache = ab.FilterCache(8 << 20, max_tables=8)
    cache.put(b"t0", blk)
    q = np.concatenate([keys[:500], oracle.splitmix_keys16(0xCAFE, 500)])
    table = np.zeros(len(q), np.uint32)
    want = oracle.probe(q, oracle.keys2block(keys))
    got, unc = cache.probe([b"t0"], table, q)
    assert unc == 0 and np.array_equal(got, want)
    ab.test_fault(ab.TEST_FAULT_CACHE_COMPLETION, 0)
    try:
        with pytest.raises(ab.AdlBloomError):
            cache.probe([b"t0"], table, q)
    finally:
        ab.test_fault(ab.TEST_FAULT_CACHE_COMPLETION, -1)
    got, unc = cache.probe([b"t0"], table, q)
    assert unc == 0 and np.array_equal(got, want)
    cache.close()


@pytest.mark.parametrize("stride", [8, 24])
def test_pipeline_fixed_stride_unaligned_groups(dev, ab, oracle, stride):
    """adl_bloom_build_segmented with fixed-stride keys: more than 8 filters (so
    several pipeline groups), an odd first key, group starts at byte offsets that
    are not multiples of 16 -- every bitmap equal to the oracle's."""
    rng = np.random.default_rng(stride)
    sizes = [3, 1001, 0, 17, 5000, 1, 777, 4096, 33, 12345, 9, 2, 70_000, 11]
    first = 5  # keys before the first filter: key_begin[0] is odd
    kb = (first + np.concatenate([[0], np.cumsum(sizes)])).astype(np.uint64)
    hk = rng.integers(0, 256, (int(kb[-1]) + 3, stride), dtype=np.uint8)
    nbytes = [ab.bitmap_bytes(s, 10) for s in sizes]
    boff = np.concatenate([[0], np.cumsum(nbytes)[:-1]]).astype(np.uint64)
    out = np.zeros(int(sum(nbytes)), dtype=np.uint8)
    ab.build_segmented_host(hk, kb, out, boff)
    for f, s in enumerate(sizes):
        want = oracle.keys2block(hk[int(kb[f]):int(kb[f + 1])])
        assert np.array_equal(out[int(boff[f]):int(boff[f]) + nbytes[f]], want), f


@pytest.mark.parametrize("pinned", [False, True])
def test_pipeline_fault_mid_pipeline(dev, ab, oracle, knobs, pinned):
    """A build failing in group 2 (adl_bloom_test_fault) returns the error only
    after every copy into the caller's buffer has finished: the buffer does not
    change after the call returns.  The next call succeeds."""
    sizes = [400_000] * 24  # 5 groups (32 MB of keys each)
    kb = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    hk = oracle.splitmix_keys16(99, int(kb[-1]))
    nbytes = [ab.bitmap_bytes(s, 10) for s in sizes]
    boff = np.concatenate([[0], np.cumsum(nbytes)[:-1]]).astype(np.uint64)
    total = int(sum(nbytes))
    if pinned:
        keys = dev.from_numpy(hk).pin_memory()
        out = dev.zeros(total, dtype=dev.uint8).pin_memory()
        view = lambda: out.numpy().copy()  # noqa: E731
    else:
        keys, out = hk, np.zeros(total, dtype=np.uint8)
        view = lambda: out.copy()  # noqa: E731
    knobs.set("ADL_BLOOM_PIPE_MB", "32")  # groups of 5 filters: group 2 exists
    ab.test_fault(ab.TEST_FAULT_PIPELINE_GROUP, 2)
    try:
        with pytest.raises(ab.AdlBloomError):
            ab.build_segmented_host(keys, kb, out, boff)
    finally:
        ab.test_fault(ab.TEST_FAULT_PIPELINE_GROUP, -1)
    a = view()
    time.sleep(0.2)
    assert np.array_equal(a, view()), "the caller's buffer changed after the error returned"
    ab.build_segmented_host(keys, kb, out, boff)
    full = view()
    for f in (0, 9, 23):
        want = oracle.keys2block(hk[int(kb[f]):int(kb[f + 1])])
        assert np.array_equal(full[int(boff[f]):int(boff[f]) + nbytes[f]], want), f


# ------------------------------------------------ resident probe server (single-key Get)
def _varlen_block(oracle, seed, n, bpk):
    """A one-filter block over n keys of 0..64 bytes; (key list, block, bitmap)."""
    rng = np.random.default_rng(seed)
    keys = [rng.integers(0, 256, int(rng.integers(0, 65)), dtype=np.uint8).tobytes() for _ in range(n)]
    offs = np.concatenate([[0], np.cumsum([len(k) for k in keys])]).astype(np.uint64)
    data = np.frombuffer(b"".join(keys) + b"\0", np.uint8)
    bm = oracle.keys2block(data, offs, bits_per_key=bpk)
    return keys, oracle.filter_block_final([bm.tobytes()], bpk), bm


def _pack(keys):
    offs = np.concatenate([[0], np.cumsum([len(k) for k in keys])]).astype(np.uint64)
    return np.frombuffer(b"".join(keys) + b"\0", np.uint8), offs


@pytest.mark.parametrize("bpk", [3, 10, 44])
def test_probe_server_single_keys_vs_oracle(dev, ab, oracle, knobs, bpk):
    """Batches of 1..8 queries (keys of 0..288 bytes, several tables, an
    uncached table, a filter index the block does not have) through the
    resident server equal the oracle and the launched probe."""
    T = 3
    tabs = [_varlen_block(oracle, 40 + t + bpk, 3000, bpk) for t in range(T)]
    cache = ab.FilterCache(16 << 20, max_tables=8, bits_per_key=bpk)
    oids = [b"srv-%d" % t for t in range(T)] + [b"not-cached"]
    for o, (_, blk, _) in zip(oids, tabs):
        cache.put(o, blk)
    rng = np.random.default_rng(bpk)
    checked = 0
    for it in range(400):
        n = 1 + it % 8
        table = rng.integers(0, T + 1, n).astype(np.uint32)
        qs = []
        for i in range(n):
            t = int(table[i])
            if t < T and rng.integers(0, 2):
                qs.append(tabs[t][0][int(rng.integers(0, 3000))])  # a member
            else:
                qs.append(rng.integers(0, 256, int(rng.integers(0, 289 // n)), dtype=np.uint8).tobytes())
        data, offs = _pack(qs)
        want = np.array([1 if t == T else
                         int(oracle.probe(data, tabs[t][2], offsets=offs[i:i + 2].copy(), bits_per_key=bpk)[0])
                         for i, t in enumerate(table)], np.uint8)
        got, unc = cache.probe(oids, table, data, offs)
        assert np.array_equal(got, want), (it, got, want)
        assert unc == int((table == T).sum())
        knobs.set("ADL_BLOOM_PROBE_SERVER", "0")
        got2, _ = cache.probe(oids, table, data, offs)
        knobs.unset("ADL_BLOOM_PROBE_SERVER")
        assert np.array_equal(got2, want)
        # filter 1 does not exist in these one-filter blocks: absent
        got3, _ = cache.probe(oids, table, data, offs, filter=1)
        assert np.array_equal(got3, (table == T).astype(np.uint8))
        checked += n
    assert checked > 1500
    cache.close()


def test_filter_cache_mixed_bpk(dev, ab, oracle, knobs):
    """Tables written with bits_per_key 3, 10 and 16 in ONE cache: multi-get
    batches (one launch: a k per table), single-key and small batches through
    the resident server (a k per query) and through a launched probe, all equal
    to the oracle with each block's own bits_per_key (the reference builds the
    BloomFilter of each block from its "bf:" info, src/filter_block.cpp:158-170;
    Level::Get reads every table of a level, src/revision.cpp:265-310)."""
    bpks = [3, 10, 16, 3, 16, 10, 0, 44]  # (0: a 7-byte bitmap, k = 1; 44: k = 30)
    tabs = [_varlen_block(oracle, 70 + t, 2500, b) for t, b in enumerate(bpks)]
    cache = ab.FilterCache(16 << 20, max_tables=len(bpks))
    oids = [b"mix-%d" % t for t in range(len(bpks))]
    for o, (_, blk, _) in zip(oids, tabs):
        cache.put(o, blk)
    T = len(bpks)

    def want_of(qs, table):
        data, offs = _pack(qs)
        return np.array([int(oracle.probe(data, tabs[t][2], offsets=offs[i:i + 2].copy(), bits_per_key=bpks[t])[0])
                         for i, t in enumerate(table)], np.uint8)

    rng = np.random.default_rng(77)
    # a large batch: one launch
    n = 6000
    table = rng.integers(0, T, n).astype(np.uint32)
    qs = [tabs[t][0][int(rng.integers(0, 2500))] if i % 2 else
          rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes() for i, t in enumerate(table)]
    want = want_of(qs, table)
    data, offs = _pack(qs)
    got, unc = cache.probe(oids, table, data, offs)
    assert unc == 0 and np.array_equal(got, want)
    assert 0 < int(want.sum()) < n
    # small batches: the server (per-query k), then launched
    for server in ("1", "0"):
        knobs.set("ADL_BLOOM_PROBE_SERVER", server)
        for it in range(240):
            m = 1 + it % 8
            sel = rng.integers(0, n, m)
            sub = [qs[int(i)] for i in sel]
            d, o = _pack(sub)
            got, _ = cache.probe(oids, table[sel], d, o)
            assert np.array_equal(got, want[sel]), (server, it)
    knobs.unset("ADL_BLOOM_PROBE_SERVER")
    cache.close()


def test_probe_server_relaunch_and_teardown(dev, ab, oracle, knobs):
    """A server that exits when idle (100 us) or at its life limit (2 ms) is
    relaunched by the next request; closing the cache while the server is
    running stops it; an armed completion fault fails one call only."""
    knobs.set("ADL_BLOOM_SERVER_IDLE_US", "100")
    knobs.set("ADL_BLOOM_SERVER_LIFE_US", "2000")
    keys, blk = _block(oracle, 3100, 20_000)
    bm = oracle.keys2block(keys)
    q = np.concatenate([keys[:300], oracle.splitmix_keys16(0xD00D, 300)])
    want = oracle.probe(q, bm)
    for round_ in range(3):
        cache = ab.FilterCache(8 << 20, max_tables=8)
        cache.put(b"t0", blk)
        t = np.zeros(1, np.uint32)
        for i in range(len(q)):
            got, _ = cache.probe([b"t0"], t, q[i:i + 1])
            assert got[0] == want[i], (round_, i)
            if i % 97 == 0:
                time.sleep(0.002)  # idle: the server exits, the next call relaunches it
        ab.test_fault(ab.TEST_FAULT_CACHE_COMPLETION, 0)
        try:
            with pytest.raises(ab.AdlBloomError):
                cache.probe([b"t0"], t, q[:1])
        finally:
            ab.test_fault(ab.TEST_FAULT_CACHE_COMPLETION, -1)
        got, _ = cache.probe([b"t0"], t, q[:1])
        assert got[0] == want[0]
        cache.close()  # the server is (most likely) still running here


def test_probe_server_threads(dev, ab, oracle):
    """8 threads issuing single-key probes at once (one server slot each),
    while a ninth runs large batches on its own stream: every answer exact,
    and the large batches are not held up behind the resident kernel."""
    T = 4
    tabs = [_block(oracle, 3200 + t, 20_000) for t in range(T)]
    cache = ab.FilterCache(32 << 20, max_tables=8)
    oids = [b"th-%d" % t for t in range(T)]
    for o, (_, blk) in zip(oids, tabs):
        cache.put(o, blk)
    rng = np.random.default_rng(9)
    n = 2000
    table = rng.integers(0, T, n).astype(np.uint32)
    fresh = oracle.splitmix_keys16(0xABCD, n)
    q = np.where((rng.integers(0, 2, n) == 1)[:, None],
                 np.stack([tabs[t][0][(3 * i) % 20_000] for i, t in enumerate(table)]), fresh)
    want = np.empty(n, np.uint8)
    for t in range(T):
        sel = table == t
        want[sel] = oracle.probe(q[sel], oracle.keys2block(tabs[t][0]))
    errors, big_ms = [], []

    def single(k):
        for i in range(k, n, 8):
            got, _ = cache.probe(oids, table[i:i + 1], q[i:i + 1])
            if got[0] != want[i]:
                errors.append((k, i))

    def big():
        for _ in range(10):
            t0 = time.perf_counter()
            got, _ = cache.probe(oids, table, q)
            big_ms.append((time.perf_counter() - t0) * 1e3)
            if not np.array_equal(got, want):
                errors.append(("big", int((got != want).sum())))

    th = [threading.Thread(target=single, args=(k,)) for k in range(8)] + [threading.Thread(target=big)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    cache.close()
    assert not errors, errors[:5]
    assert sorted(big_ms)[len(big_ms) // 2] < 15.0, big_ms


def _readpath_json(args, timeout=300, **env):
    import json

    exe = os.path.join(ROOT, "adlsm-tree_amd", "bin", "readpath_test")
    r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=timeout, env=dict(os.environ, **env))
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_gets_beside_builds(dev, golden):
    """Single-key Gets through the resident probe server while the headline
    build and a configs[3]-shaped build (256 tables x 1 M keys) run on another
    thread (the reference's DB::Get during DoCompaction, src/db.cpp:164-172,
    263): every answer equals the one given with the GPU idle, the headline
    bitmap equals the reference's SHA-256 and the 256 tables equal the oracle
    pins, idle and concurrent alike.  The server's wave fits beside pass A
    (2 KiB of LDS and 32 VGPRs left free on every CU), so the Gets do not
    wait for a build; the times are printed (profiles/ holds the measured
    runs)."""
    import hashlib
    import json

    d = _readpath_json(["--coexist", "2"])
    print(d)
    assert d["get_mismatches"] == 0
    sha10m = golden["appendix_b"]["bitmaps"][5]
    assert sha10m["n"] == 10_000_000
    assert d["headline_sha256"] == [sha10m["sha256"]] * 2
    with open(os.path.join(ROOT, "tests", "golden", "full_size.json")) as f:
        pins = json.load(f)["compaction"]
    want = hashlib.sha256("".join(pins["bitmap_sha256"]).encode()).hexdigest()
    assert d["compaction_sha_of_shas"] == [want, want]
    assert d["get_us_during_builds"]["calls"] > 100


def test_probe_server_tails(dev):
    """20 000 single-key Gets in a row with a 2 ms server life: the requests
    that meet an exiting server are answered by its last poll or by a
    relaunch (no timeout path), every answer exact."""
    d = _readpath_json(["--tails", "20000"], ADL_BLOOM_SERVER_LIFE_US="2000")
    print(d)
    assert d["mismatches"] == 0
    assert d["single_key_us"]["calls"] == 20000
    assert d["server_launches"] >= 10


def test_probe_server_exit_with_queued_successor(dev):
    """A process that returns from main while the server has a successor
    kernel queued behind the running one exits promptly: the atexit stop path
    waits on the mapped control words until the queued successor has started,
    seen stop and left, before the runtime's teardown."""
    exe = os.path.join(ROOT, "adlsm-tree_amd", "bin", "readpath_test")
    t0 = time.perf_counter()
    r = subprocess.run([exe, "--exit-queued"], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, ADL_BLOOM_DEBUG="1"))
    print(r.stdout, r.stderr[-2000:])
    assert r.returncode == 0, r.stdout + r.stderr
    assert time.perf_counter() - t0 < 30
    line = [x for x in r.stderr.splitlines() if "adl_bloom server at exit" in x]
    assert line and "drained" in line[-1] and "NOT drained" not in line[-1], r.stderr[-2000:]
