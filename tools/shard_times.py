#!/usr/bin/env python3
"""tools/shard_times.py -- every rank's share of the sharded workloads at
N = 1, 2, 4, 8, timed on ONE GPU: the compaction build (configs[3]: rank r's
256/N tables, one segmented build) and the owner-bucketed probe (configs[4]:
rank r's own tables' share of the 100M-query batch).  bench.py --gpus N runs
exactly these per-rank steps with no collective on the data path, so the
slowest rank's time here bounds the N-GPU step from below (the node's own
effects -- clocks, the host, the final 16-byte all-reduce -- are the driver's
SCALE run to show).  One JSON line per (workload, N, rank).

usage: [SHARD_KINDS=compaction,probe] [SHARD_NS=1,2,4,8] python tools/shard_times.py [steps]
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "adlsm-tree_amd"))
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
torch.cuda.set_device(0)
kinds = os.environ.get("SHARD_KINDS", "compaction,probe").split(",")
ns = [int(x) for x in os.environ.get("SHARD_NS", "1,2,4,8").split(",")]
for kind in kinds:
    for N in ns:
        for rank in sorted({0, N - 1}):
            w = bench.Workload(kind, rank, 0, N, 100_000_000 if kind == "probe" else 0)
            if kind == "probe":
                w.kernel_events = None
            for _ in range(2):
                w.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                w.step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            units = w.n
            print(json.dumps({"workload": kind, "N": N, "rank": rank, "units_this_rank": units,
                              "tables_this_rank": len(w.tables), "ms_per_step": round(ms, 4),
                              "rank_rate_M_per_s": round(units / ms / 1e3, 1)}), flush=True)
            del w
            torch.cuda.empty_cache()
