#!/usr/bin/env python3
"""tools/e2e_parts.py -- where a single host-to-host build's time goes
(bench.py's e2e "single" against the sum of its parts): the 160 MB key upload,
the build, the 100 MB bitmap download, alone and chained on one stream, and
the same chain through the C-ABI host API (adl_bloom_build: one pipeline
group).  Prints one JSON line of median milliseconds over REPS runs."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adlsm-tree_amd"))
import adlbloom as ab  # noqa: E402

n = 10_000_000
REPS = int(os.environ.get("REPS", "7"))
keys_d = ab.synth_keys16(n, seed=0x5EED)
keys_h = torch.empty((n, 16), dtype=torch.uint8, pin_memory=True)
keys_h.copy_(keys_d)
b = ab.Builder(n, 10)
out_h = torch.empty(b.nbytes, dtype=torch.uint8, pin_memory=True)
out_h2 = torch.empty(b.nbytes + 64, dtype=torch.uint8, pin_memory=True)
dst = torch.empty_like(keys_d)
bm = b.build(dst.copy_(keys_d))
st = torch.cuda.current_stream()


def med(fn):
    ts = []
    for i in range(REPS + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        st.synchronize()
        if i:
            ts.append((time.perf_counter() - t0) * 1e3)
    return round(float(np.median(ts)), 3)


res = {
    "h2d": med(lambda: dst.copy_(keys_h, non_blocking=True)),
    "build": med(lambda: b.build(dst)),
    "d2h": med(lambda: out_h.copy_(b.bitmap[:b.nbytes], non_blocking=True)),
    "d2h_aligned_len": med(lambda: out_h2[:b.nbytes + 9].copy_(b.bitmap[:b.nbytes + 9], non_blocking=True)),
    "h2d_build": med(lambda: (dst.copy_(keys_h, non_blocking=True), b.build(dst))),
    "build_d2h": med(lambda: (b.build(dst), out_h.copy_(b.bitmap[:b.nbytes], non_blocking=True))),
    "h2d_build_d2h": med(lambda: (dst.copy_(keys_h, non_blocking=True), b.build(dst),
                                  out_h.copy_(b.bitmap[:b.nbytes], non_blocking=True))),
}
hk = keys_h.numpy()
ho = out_h.numpy()
res["c_abi_adl_bloom_build"] = med(lambda: ab.lib().adl_bloom_build(hk.ctypes.data, None, n, 16, 10, ho.ctypes.data,
                                                                    None))
print(json.dumps(res))
