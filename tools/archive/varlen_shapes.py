#!/usr/bin/env python3
"""tools/varlen_shapes.py -- variable-length build time (pass A = hashing pass +
pass A over pairs, or the fused pass A) by key-length shape, for
ADL_BLOOM_VAR_HASH=0/1: configs[2]'s Zipf keys and uniform-length keys of
32, 128 and 512 bytes on average (2M keys each).  Bitmaps are compared
between the two paths."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "adlsm-tree_amd"))
import adlbloom as ab  # noqa: E402


def shape(n, lo, hi, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    lens = torch.randint(lo, hi + 1, (n,), device="cuda", generator=g, dtype=torch.int64)
    offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    offs[1:] = torch.cumsum(lens, 0)
    data = torch.randint(0, 256, (int(offs[-1].item()) + 16,), device="cuda", generator=g, dtype=torch.uint8)
    return data, offs


def timed(data, offs, n, vh):
    os.environ["ADL_BLOOM_VAR_HASH"] = vh
    b = ab.Builder(n, 10)
    for _ in range(2):
        b.build(data, offs)
    torch.cuda.synchronize()
    ab.profile_enable(64)
    for _ in range(10):
        b.build(data, offs)
    torch.cuda.synchronize()
    pairs = ab.profile_each(64)
    ab.profile_collect()
    pa = sorted(p[0] for p in pairs)[len(pairs) // 2] * 1e3
    pb = sorted(p[1] for p in pairs)[len(pairs) // 2] * 1e3
    return pa, pb, b.bitmap[: b.nbytes].clone()


cases = {"zipf 8-256 (configs[2], 10M)": ab.synth_varlen(10_000_000, seed=0x5EED)}
for name, (lo, hi) in {"uniform 16-48": (16, 48), "uniform 64-192": (64, 192), "uniform 256-768": (256, 768)}.items():
    cases[name + " (2M)"] = shape(2_000_000, lo, hi, lo)
for name, (data, offs) in cases.items():
    n = offs.numel() - 1
    r = {vh: timed(data, offs, n, vh) for vh in ("0", "1")}
    same = torch.equal(r["0"][2], r["1"][2])
    print(f"{name:30s} fused pass A {r['0'][0]:8.1f} us | hashing pass + pass A {r['1'][0]:8.1f} us | "
          f"pass B {r['1'][1]:6.1f} us | bitmaps equal: {same}")
