#!/usr/bin/env python3
"""tools/tl_shapes.py -- the build's automatic tile size / pass-B occupancy
choice against the round-3 choice on several filter shapes: pass A + pass B
per build from HIP events on the kernels (adlbloom.profile_*), the two
settings interleaved, bitmaps compared byte for byte between them.

round 3: ADL_BLOOM_TILE_LOG2 = the largest tile giving >= 512 tiles in all,
ADL_BLOOM_B_OCC=1, ADL_BLOOM_DEPTH=8."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "adlsm-tree_amd"))
import torch  # noqa: E402

import adlbloom as ab  # noqa: E402


def old_tl(counts):
    for tl in range(20, 9, -1):
        tiles = sum(((c * 10 + 7) * 8 + (1 << tl) - 1) >> tl for c in counts)
        if tiles >= 512:
            return tl
    return 10


def run(keys, kb, reps):
    ab.profile_enable(4 * reps + 8)
    outs = None
    for _ in range(reps):
        outs = ab.build_segmented(keys, kb)
    a, b, n = ab.profile_collect()
    return a / reps * 1e3, b / reps * 1e3, outs[0].cpu().numpy()


SHAPES = [("256 x 1M", [1_000_000] * 256), ("8 x 1M", [1_000_000] * 8), ("32 x 100K", [100_000] * 32),
          ("256 x 10K", [10_000] * 256), ("64 x 300K", [300_000] * 64)]
for name, counts in SHAPES:
    keys = torch.cat([ab.synth_keys16(c, seed=0x5EED + i) for i, c in enumerate(counts)])
    kb = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    reps = 5 if sum(counts) > 50_000_000 else 20
    res = {}
    for rnd in range(2):
        for label, env in (("auto", {}), ("round3", {"ADL_BLOOM_TILE_LOG2": str(old_tl(counts)),
                                                       "ADL_BLOOM_B_OCC": "1", "ADL_BLOOM_DEPTH": "8"})):
            for k in ("ADL_BLOOM_TILE_LOG2", "ADL_BLOOM_B_OCC", "ADL_BLOOM_DEPTH"):
                os.environ.pop(k, None)
            os.environ.update(env)
            a, b, bm = run(keys, kb, reps)
            res.setdefault(label, []).append((a, b))
            res[label + "_bm"] = bm
    same = np.array_equal(res["auto_bm"], res["round3_bm"])
    print(f"{name}: auto " + " ".join(f"{a:.1f}+{b:.1f}" for a, b in res["auto"]) +
          " us | round3 " + " ".join(f"{a:.1f}+{b:.1f}" for a, b in res["round3"]) + f" us | bitmaps equal: {same}",
          flush=True)
    del keys
    torch.cuda.empty_cache()
