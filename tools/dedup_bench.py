#!/usr/bin/env python3
"""tools/dedup_bench.py -- cost and gain of ADL_BLOOM_SKIP_ADJACENT_DUPLICATES.

10 M 16-byte keys per build, with every key repeated r times in a row
(r = 1: no duplicates; r = 2 / 4: half / three quarters of the keys repeat
their predecessor), built with flags 0 and 1.  Prints ms per build (HIP
events around 10 builds after 3 warm-ups) and checks the two bitmaps agree.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adlsm-tree_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import adlbloom as ab  # noqa: E402


def time_build(keys, kb, flags, reps=10):
    for _ in range(3):
        out, _, _ = ab.build_segmented(keys, kb, flags=flags)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        out, _, _ = ab.build_segmented(keys, kb, flags=flags)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps, out


def main():
    n = 10_000_000
    print(f"{'repeat':>6} {'flags=0 ms':>11} {'flags=1 ms':>11}")
    for r in (1, 2, 4):
        base = ab.synth_keys16((n + r - 1) // r)
        keys = base.repeat_interleave(r, dim=0)[:n].contiguous()
        kb = np.array([0, n], dtype=np.uint64)
        t0, b0 = time_build(keys, kb, 0)
        t1, b1 = time_build(keys, kb, ab.SKIP_ADJACENT_DUPLICATES)
        assert torch.equal(b0, b1), "dedup changed the bitmap"
        print(f"{r:>6} {t0:>11.3f} {t1:>11.3f}")


if __name__ == "__main__":
    main()
