"""tools/pipe_probe.py -- the pipelined host build (adl_bloom_build_segmented)
on configs[3]'s shape (256 tables x 1M x 16 B keys, pinned host memory) at
several group sizes (ADL_BLOOM_PIPE_MB), next to the unpipelined sequence
(all keys up, one segmented build, all bitmaps down).  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "adlsm-tree_amd"))
import adlbloom as ab  # noqa: E402


def main():
    T, per = int(os.environ.get("TABLES", 256)), int(os.environ.get("PER", 1_000_000))
    kb = np.arange(T + 1, dtype=np.uint64) * per
    n = int(kb[-1])
    keys_d = ab.synth_keys16(n, seed=0x5EED)
    keys_h = torch.empty((n, 16), dtype=torch.uint8, pin_memory=True)
    keys_h.copy_(keys_d)
    sizes = [ab.bitmap_bytes(per, 10)] * T
    boff = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    out_h = torch.zeros(int(sum(sizes)), dtype=torch.uint8, pin_memory=True)
    res = {}
    for mb in [int(x) for x in os.environ.get("MBS", "32,128,256,512").split(",")]:
        os.environ["ADL_BLOOM_PIPE_MB"] = str(mb)
        ab.build_segmented_host(keys_h, kb, out_h, boff)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            ab.build_segmented_host(keys_h, kb, out_h, boff)
        res[f"pipe_{mb}MB_ms"] = round((time.perf_counter() - t0) / 3 * 1e3, 2)
    b = ab.SegmentedBuilder(kb, 10)
    dst = torch.empty_like(keys_d)
    seq_h = torch.empty(b.out.numel(), dtype=torch.uint8, pin_memory=True)

    def seq():
        dst.copy_(keys_h, non_blocking=True)
        o = b.build(dst)
        seq_h.copy_(o, non_blocking=True)
        torch.cuda.current_stream().synchronize()
    seq()
    t0 = time.perf_counter()
    for _ in range(3):
        seq()
    res["serial_ms"] = round((time.perf_counter() - t0) / 3 * 1e3, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
