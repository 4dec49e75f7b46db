#!/usr/bin/env python3
"""tools/claim_shapes.py -- pass A's claim layout (ADL_BLOOM_CLAIM) against the
chunk/table build on the filter shapes the plan gives it (and, forced with
ADL_BLOOM_CLAIM=2, on two it refuses): pass A + pass B per build from HIP
events on the kernels (adlbloom.profile_*), the settings interleaved, bitmaps
compared byte for byte between them."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "adlsm-tree_amd"))
import torch  # noqa: E402

import adlbloom as ab  # noqa: E402


def run(keys, kb, reps):
    ab.profile_enable(4 * reps + 8)
    outs = None
    for _ in range(reps):
        outs = ab.build_segmented(keys, kb)
    a, b, n = ab.profile_collect()
    return a / reps * 1e3, b / reps * 1e3, outs[0].cpu().numpy()


SHAPES = [("256 x 10K", [10_000] * 256, "1"), ("32 x 100K", [100_000] * 32, "1"),
          ("256 x 40K", [40_000] * 256, "1"), ("64 x 300K", [300_000] * 64, "1"),
          ("8 x 1M (forced)", [1_000_000] * 8, "2"), ("1 x 10M (forced)", [10_000_000], "2")]
if len(sys.argv) > 1 and sys.argv[1] == "threshold":  # around the default's 8-tile limit
    SHAPES = [("512 x 5K", [5_000] * 512, "1"), ("256 x 20K", [20_000] * 256, "1"),
              ("128 x 30K", [30_000] * 128, "1"), ("128 x 60K", [60_000] * 128, "1")]
for name, counts, mode in SHAPES:
    keys = torch.cat([ab.synth_keys16(c, seed=0x5EED + i) for i, c in enumerate(counts)])
    kb = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    reps = 20
    res = {}
    for rnd in range(2):
        for label, val in (("base", "0"), ("claim", mode)):
            os.environ["ADL_BLOOM_CLAIM"] = val
            a, b, bm = run(keys, kb, reps)
            res.setdefault(label, []).append((a, b))
            res[label + "_bm"] = bm
    same = np.array_equal(res["base_bm"], res["claim_bm"])
    print(f"{name}: base " + " ".join(f"{a:.1f}+{b:.1f}" for a, b in res["base"]) +
          " us | claim " + " ".join(f"{a:.1f}+{b:.1f}" for a, b in res["claim"]) + f" us | bitmaps equal: {same}",
          flush=True)
    del keys
    torch.cuda.empty_cache()
