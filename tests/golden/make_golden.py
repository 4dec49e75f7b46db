"""tests/golden/make_golden.py -- regenerate the committed golden fixtures.

Sources (never the restatement under test):
  * murmur3_ref.json: the reference's own src/murmur3_hash.cpp, compiled
    unmodified into oracle/_ref/libref_murmur3.so by oracle/Makefile (needs
    /root/reference, i.e. this container -- not the GPU box).
  * appendix_b.json: SURVEY.md Appendix B, produced during the survey by the
    compiled reference src/filter_block.cpp + src/murmur3_hash.cpp (bitmap
    SHA-256s / popcounts for SplitMix64 keys, probe false-positive counts and
    masks, the test/filter_block_test.cpp block, the test/sstable_test.cpp
    SSTable oid and size).  Transcribed here verbatim.

Run: python tests/golden/make_golden.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402

SEEDS = (0xE2C6928A, 0xBAEA8A8F)


def murmur_vectors():
    R = O.ref_lib()
    if R is None:
        raise SystemExit("oracle/_ref/libref_murmur3.so missing: make -C oracle ref (needs /root/reference)")
    rng = random.Random(20261015)
    keys = [b"", b"a", b"ab", b"abc", b"abcd", b"hello", b"hello-ddl0", bytes([0x80, 0xFF, 0x7F, 0x01])]
    # every length 0..64 with bytes >= 0x80 forced in, all len%4 tails
    for L in range(0, 65):
        keys.append(bytes(rng.randrange(256) for _ in range(L)))
        keys.append(bytes(rng.randrange(128, 256) for _ in range(L)))
        keys.append(bytes(rng.randrange(32, 127) for _ in range(L)))
    for _ in range(200):
        L = rng.randrange(65, 300)
        keys.append(bytes(rng.randrange(256) for _ in range(L)))
    out = []
    for k in keys:
        out.append({"key": k.hex(), "h1": R.ref_murmur3(SEEDS[0], k, len(k)),
                    "h2": R.ref_murmur3(SEEDS[1], k, len(k)),
                    "s0": R.ref_murmur3(0, k, len(k))})
    return out


APPENDIX_B = {
    "source": "SURVEY.md Appendix B (compiled reference src/filter_block.cpp + src/murmur3_hash.cpp)",
    "keys": "SplitMix64 seed 0x5EED, key i = LE64(next) || LE64(next)",
    "bits_per_key": 10,
    "bitmaps": [
        {"n": 1, "bytes": 17, "popcount": 6,
         "sha256": "cd5cc0045fb5e83e52f7e2bad3c4df2a1e7f94457cd91931ee991ad01df8110a"},
        {"n": 2, "bytes": 27, "popcount": 12,
         "sha256": "6f4e8856cb39275ae9396f1a0deedd15f8d86bf0377610cd25193634e324c1e3",
         "hex": "020840008020000002100000000000004530000000000000000000"},
        {"n": 1000, "bytes": 10007, "popcount": 5374,
         "sha256": "26ce06e6ae4bdd85ef41e9e5842f846ead889c3a9a3b266c8b6d562bf37d5da1"},
        {"n": 100000, "bytes": 1000007, "popcount": 431546,
         "sha256": "adb59bc2c083dd89a36a6a7a33d38e384d025e4d0bb1e7b6bab12ad6fc08bed4"},
        {"n": 1000000, "bytes": 10000007, "popcount": 3998627,
         "sha256": "641829d3f5a5dbeb469bceb021d526f66d8037461f13d1ecf4ad86b0d6d150de"},
        {"n": 10000000, "bytes": 100000007, "popcount": 37449647,
         "sha256": "b80f0b985b23cab91cd49be48692f09c3eeeafee1b269eb21c021c7d98eedb4c"},
    ],
    "probes": [
        {"n": 1000, "queries": "next 1000 keys of the same stream", "false_positives": 65,
         "first64_mask_lsb_first": "0240004000000020"},
        {"n": 100000, "queries": "next 100000 keys of the same stream", "false_positives": 25776,
         "first64_mask_lsb_first": "90012c80080610a4"},
    ],
    "filter_block_test": {
        "scenario": "test/filter_block_test.cpp:7-31 (filter 0: hello, world, hello-yly, hello-ddl, "
                    "hello-ddl0..9999; filter 1: adl, dont, like-apple)",
        "bytes": 100111,
        "sha256": "68cb3322ec5d66d7dbd58781011cb955a62f31a89e7a41d3d3aca4e458ace57e",
        "last30_hex": "00010000000000cf860100f48601000200000062663a0a00000007000000",
    },
    "sstable_test": {
        "scenario": "test/sstable_test.cpp:9-27 BuildSSTable (10,000 x key{i}/value{i}, seq=i, OP_PUT), "
                    "MemTable::BuildSSTable -> SSTableWriter, bits_per_key=10",
        "oid": "15c52c5634ae0b6eb9529a93c797a4acd1cfbde1a7a85a33565d99c4f5a2d8a6",
        "bytes": 420270,
    },
    "murmur3_kat": [
        {"key": "", "h1": "389d2042", "h2": "1f2c6e1c"},
        {"key": "61", "h1": "4ec17aca", "h2": "c1b2ac76"},
        {"key": "6162", "h1": "0856e6d0", "h2": "e8796178"},
        {"key": "616263", "h1": "a79c2abf", "h2": "affb1f13"},
        {"key": "61626364", "h1": "37a2ddba", "h2": "c5802bfa"},
        {"key": "68656c6c6f", "h1": "6d84082c", "h2": "c6ba3a6b"},
        {"key": "68656c6c6f2d64646c30", "h1": "d6619413", "h2": "94025c34"},
        {"key": "80ff7f01", "h1": "fcae0523", "h2": "ea9e7223"},
    ],
}


def main():
    with open(os.path.join(HERE, "murmur3_ref.json"), "w") as f:
        json.dump({"source": "reference src/murmur3_hash.cpp via oracle/_ref (unmodified)",
                   "seeds": [hex(s) for s in SEEDS], "vectors": murmur_vectors()}, f, indent=0)
    with open(os.path.join(HERE, "appendix_b.json"), "w") as f:
        json.dump(APPENDIX_B, f, indent=1)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
