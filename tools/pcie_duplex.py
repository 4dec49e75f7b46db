"""tools/pcie_duplex.py -- host<->device copy rates on this box: H2D alone,
D2H alone, and both at once on two streams (pinned host memory), to see
whether the link (and the copy engines HIP uses) overlap the two directions.
Diagnostics for the pipelined host build (bloom_pipeline.hip)."""
import json
import time

import torch


def rate(fn, nbytes, iters=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return nbytes * iters / (time.perf_counter() - t0) / 1e9


def main():
    up_n, down_n = 2 << 30, 1 << 30
    h_up = torch.empty(up_n, dtype=torch.uint8, pin_memory=True)
    h_down = torch.empty(down_n, dtype=torch.uint8, pin_memory=True)
    d_up = torch.empty(up_n, dtype=torch.uint8, device="cuda")
    d_down = torch.ones(down_n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = {}
    out["h2d_GBs"] = rate(lambda: d_up.copy_(h_up, non_blocking=True), up_n)
    out["d2h_GBs"] = rate(lambda: h_down.copy_(d_down, non_blocking=True), down_n)

    def both():
        with torch.cuda.stream(s1):
            d_up.copy_(h_up, non_blocking=True)
        with torch.cuda.stream(s2):
            h_down.copy_(d_down, non_blocking=True)
    t = rate(both, up_n + down_n)
    out["both_GBs_total"] = t
    # chunked both (many 32 MB copies interleaved), as the pipeline issues them
    ch = 32 << 20

    def both_chunked():
        for i in range(up_n // ch):
            with torch.cuda.stream(s1):
                d_up[i * ch:(i + 1) * ch].copy_(h_up[i * ch:(i + 1) * ch], non_blocking=True)
            if i < down_n // ch:
                with torch.cuda.stream(s2):
                    h_down[i * ch:(i + 1) * ch].copy_(d_down[i * ch:(i + 1) * ch], non_blocking=True)
    out["both_chunked_GBs_total"] = rate(both_chunked, up_n + down_n)
    print(json.dumps({k: round(v, 1) for k, v in out.items()}))


if __name__ == "__main__":
    main()
