#!/usr/bin/env python3
"""tools/sstable_bench.py -- SSTable flush through the GPU filter, end to end
(SURVEY.md §8f rank 1).  Needs a GPU for the flush; the oracle is only the
checker and the CPU filter timing.

For each memtable size n ("key%012d" user keys, 100-byte values, seq = i):
  * bin/sstable_test bench n: best-of-3 time of the SSTableWriter Add loop
    (data + index blocks, keys into the filter arena), of Final (meta, index,
    footer, SHA-256) and of the filter build inside it (filter_s: H2D keys,
    two kernels, D2H bitmap, block framing);
  * the file is compared byte for byte with oracle/sstable_oracle.py (n <= 1M);
  * the reference's filter build (BloomFilter::Keys2Block over the same user
    keys, oracle C restatement, 1 core) is timed for comparison: the same flush
    with the CPU filter would take add_s + final_s - filter_s + cpu_filter_s.
usage: python tools/sstable_bench.py [n ...]  -> one JSON line per n
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402
import sstable_oracle as S  # noqa: E402

EXE = os.path.join(ROOT, "adlsm-tree_amd", "bin", "sstable_test")


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [100_000, 1_000_000, 4_000_000]
    for n in sizes:
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([EXE, "bench", str(n), d], capture_output=True, text=True, timeout=600)
            if r.returncode:
                raise SystemExit(r.stderr)
            res = json.loads(r.stdout)
            user = [b"key%012d" % i for i in range(n)]
            if n <= 1_000_000:
                ents = [(S.inner_key(u, i, 0), bytes([97 + i % 26]) * 100) for i, u in enumerate(user)]
                want = S.sstable_bytes(ents)
                got = open(os.path.join(d, res["oid"] + ".sst"), "rb").read()
                res["parity"] = "byte-identical to oracle" if got == want else "MISMATCH"
            else:
                res["parity"] = None
        data, offs = O.pack(user)
        best = 1e30
        for _ in range(2):
            t0 = time.perf_counter()
            O.keys2block(data, offsets=offs, bits_per_key=10)
            best = min(best, time.perf_counter() - t0)
        res["cpu_filter_s"] = round(best, 6)
        res["gpu_flush_s"] = round(res["add_s"] + res["final_s"], 6)
        # the same flush with the reference's CPU filter in place of the GPU one
        res["cpu_flush_s_est"] = round(res["add_s"] + res["final_s"] - res["filter_s"] + best, 6)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
