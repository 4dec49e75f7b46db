#!/usr/bin/env python3
"""tools/pass_b_data.py -- pass A / pass B kernel times of a 10M-key build as a
function of the key bytes: the SplitMix keys of the headline, the same keys
with every byte < 0x80 (no sign-extension collapse in the reference's murmur
variant) and with every byte >= 0x80 (maximal collapse).  Also reports the
bitmap popcount, i.e. how many distinct bit positions the keys set."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "adlsm-tree_amd"))
import adlbloom as ab  # noqa: E402

n = 10_000_000
base = ab.synth_keys16(n, seed=0x5EED)
variants = {"splitmix": base, "bytes<0x80": base & 0x7F, "bytes>=0x80": base | 0x80}
b = ab.Builder(n, 10)
for name, keys in variants.items():
    for _ in range(3):
        b.build(keys)
    torch.cuda.synchronize()
    ab.profile_enable(64)
    for _ in range(20):
        b.build(keys)
    torch.cuda.synchronize()
    pairs = ab.profile_each(64)
    ab.profile_collect()
    pa = sorted(p[0] for p in pairs)[len(pairs) // 2] * 1e3
    pb = sorted(p[1] for p in pairs)[len(pairs) // 2] * 1e3
    pop = int(torch.bitwise_count(b.bitmap[: b.nbytes]).sum().item()) if hasattr(torch, "bitwise_count") else -1
    if pop < 0:
        bm = b.bitmap[: b.nbytes].cpu().numpy()
        import numpy as np
        pop = int(np.unpackbits(bm).sum())
    print(f"{name:12s} pass A {pa:7.1f} us  pass B {pb:7.1f} us  popcount {pop}")
