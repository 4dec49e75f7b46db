#!/usr/bin/env python3
"""tools/probe_shapes.py -- the large-batch probe (adl_bloom_probe_batch_device)
on several batch shapes, each answer array checked against the oracle on a
sample, timed with HIP events around the call (median of reps).  ADL_BLOOM_LIB
selects the library (tools/ab_lib.sh style A/B).  One JSON line per shape.

usage: python tools/probe_shapes.py [reps]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adlsm-tree_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import adlbloom as ab  # noqa: E402
import oracle as O  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
torch.cuda.set_device(0)
# (filters, keys per filter, queries, share of queries to filter 0 or None for uniform)
SHAPES = [(1, 1_000_000, 20_000_000, None), (16, 1_000_000, 20_000_000, None), (256, 100_000, 20_000_000, None),
          (4096, 5_000, 20_000_000, None), (64, 300_000, 20_000_000, 0.9)]
only = os.environ.get("PROBE_SHAPES")  # e.g. "3" or "0,3": indices into SHAPES
for si, (F, per, n, skew) in enumerate(SHAPES):
    if only and str(si) not in only.split(","):
        continue
    keys_t = ab.synth_keys16(F * per, seed=0x5EED, device="cuda")
    kb = np.arange(F + 1, dtype=np.uint64) * per
    bms, boff, nbytes = ab.build_segmented(keys_t, kb)
    rng = np.random.default_rng(F)
    if skew is None:
        fid = rng.integers(0, F, n).astype(np.uint32)
    else:
        fid = np.where(rng.random(n) < skew, 0, rng.integers(0, F, n)).astype(np.uint32)
    q = ab.synth_keys16(n, seed=0xFEED, device="cuda")
    d_fid = torch.from_numpy(fid.view(np.int32)).cuda()
    d_off = torch.from_numpy(np.asarray(boff, dtype=np.uint64).view(np.int64)).cuda()
    d_end = torch.from_numpy((np.asarray(boff, dtype=np.uint64) + np.asarray(nbytes, dtype=np.uint64)).view(np.int64)).cuda()
    out = ab.probe_batch(q, d_fid, bms, d_off, bitmap_end=d_end)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = ab.probe_batch(q, d_fid, bms, d_off, bitmap_end=d_end, out=out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    # sampled check against the oracle (the filter bytes and 200K queries)
    idx = rng.choice(n, 200_000, replace=False)
    h_bm = bms.cpu().numpy()
    h_off = np.asarray(boff, dtype=np.uint64)
    arena = np.concatenate([h_bm[int(h_off[f]):int(h_off[f]) + int(nbytes[f])] for f in range(F)] + [np.zeros(16, np.uint8)])
    aoff = np.concatenate([[0], np.cumsum(np.asarray(nbytes, dtype=np.uint64))]).astype(np.uint64)
    want = O.probe_multi(q.cpu().numpy()[idx], fid[idx], arena, aoff)
    ok = bool(np.array_equal(out.cpu().numpy()[idx], want))
    print(json.dumps({"filters": F, "keys_per_filter": per, "queries": n, "skew_to_filter0": skew,
                      "ms_median": round(float(np.median(ts)), 4), "ms_all": [round(t, 4) for t in ts],
                      "sampled_answers_equal_oracle": ok}), flush=True)
    del keys_t, bms, q, d_fid, out
    torch.cuda.empty_cache()
