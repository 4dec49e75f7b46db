"""GPU parity at BASELINE.json's full sizes, against pins the oracle computed
(tests/golden/full_size.json, written by tests/golden/make_full_pins.py):

  configs[2]  10M variable-length keys (8-256 B, Zipf 1.1): the generated
              lengths and the bitmap, by SHA-256;
  configs[3]  256 SSTables x 1M x 16 B keys, one filter each, in one
              segmented build: all 256 bitmaps by SHA-256;
  configs[4]  100M probe queries against those 256 device-resident filters:
              the SHA-256 of all 100M answers, every inserted key found, and
              the false-positive count on fresh keys.
(configs[1], the 10M x 16 B headline, is pinned to the reference's own
SHA-256 in test_gpu_parity.py.)
"""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def pins():
    with open(os.path.join(ROOT, "tests", "golden", "full_size.json")) as f:
        return json.load(f)


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


def test_config2_varlen_10m(dev, ab, pins):
    p = pins["varlen"]
    data, offs = ab.synth_varlen(p["n"], seed=p["seed"], zipf_s=p["zipf_s"])
    o = offs.cpu().numpy().view(np.uint64)
    lengths = (o[1:] - o[:-1]).astype(np.uint32)
    assert int(o[-1]) == p["total_key_bytes"]
    assert hashlib.sha256(lengths.tobytes()).hexdigest() == p["lengths_sha256"]
    bm = ab.Builder(p["n"], 10).build(data, offs)
    assert hashlib.sha256(bm.cpu().numpy().tobytes()).hexdigest() == p["bitmap_sha256"]


@pytest.fixture(scope="module")
def arena(dev, ab, pins):
    """configs[3]: all 256 tables built in one segmented build; returns the
    exact-length bitmaps packed back to back (device) and their offsets."""
    p = pins["compaction"]
    T, per = p["tables"], p["keys_per_table"]
    keys = dev.cat([ab.synth_keys16(per, seed=p["seed0"] + t) for t in range(T)])
    kb = np.arange(T + 1, dtype=np.uint64) * per
    sb = ab.SegmentedBuilder(kb, 10)
    out = sb.build(keys)
    dev.cuda.synchronize()
    del keys
    pieces = [sb.bitmap(t) for t in range(T)]
    packed = dev.cat(pieces)
    off = np.concatenate([[0], np.cumsum([x.numel() for x in pieces])]).astype(np.uint64)
    del out, sb, pieces
    return packed, off


def test_config3_compaction_256_tables(arena, pins):
    packed, off = arena
    host = packed.cpu().numpy()
    got = [hashlib.sha256(host[int(off[t]):int(off[t + 1])].tobytes()).hexdigest() for t in range(len(off) - 1)]
    want = pins["compaction"]["bitmap_sha256"]
    bad = [t for t in range(len(want)) if got[t] != want[t]]
    assert not bad, f"tables {bad[:10]} differ from the oracle"


@pytest.mark.parametrize("path", ["direct", "batch"])
def test_config4_probe_100m(dev, ab, arena, pins, path):
    """direct: bloom_probe_multi_kernel; batch: adl_bloom_probe_batch_device, the
    tile-binned pipeline at this size (bench.py's probe step)."""
    p = pins["probe"]
    packed, off = arena
    d_off = dev.from_numpy(off.view(np.int64)).cuda()
    h = hashlib.sha256()
    n_ins = hits = fps = 0
    step = 25_000_000 if path == "direct" else p["queries"]
    for q0 in range(0, p["queries"], step):
        k, f, m = ab.synth_probe_queries(min(step, p["queries"] - q0), seed=p["seed"], q0=q0,
                                         num_tables=p["tables"], keys_per_table=p["keys_per_table"])
        r = (ab.probe_multi if path == "direct" else ab.probe_batch)(k, f, packed, d_off)
        rh, mh = r.cpu().numpy(), m.cpu().numpy()
        h.update(rh.tobytes())
        n_ins += int(mh.sum())
        hits += int((rh & mh).sum())
        fps += int((rh & (1 - mh)).sum())
    assert n_ins == p["queries_inserted"] and hits == p["hits_inserted"] == n_ins
    assert fps == p["false_positives_fresh"]
    assert h.hexdigest() == p["results_sha256"]
