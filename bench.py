#!/usr/bin/env python3
"""bench.py -- MI355X bloom-filter build benchmark (BASELINE.json metric:
"Mkeys/s bloom-filter build (device-resident), 16B keys, bits/key=10").

A step is one bloom-filter build over one batch of device-resident synthetic
keys (SURVEY.md §8d SplitMix64), through the C-ABI (adl_bloom_build_device):
pass A (hash + bin) and pass B (LDS tile OR + bitmap write).  Workloads:

  single      (default) one 10M x 16 B-key filter per GPU, bpk=10 (BASELINE.json
              configs[1]); weak scaling: rank r builds its own SSTable filter.
  compaction  32 SSTables x 1M x 16 B keys per GPU in one segmented build
              (configs[3]: 256 tables over 8 GPUs).
  varlen      10M variable-length keys (8-256 B, Zipf(1.1) lengths) per GPU (configs[2]).

Multi-GPU: one process per GPU (torch.distributed.run); no collective on the
data path -- each rank owns whole filters.  RCCL reduces only the key counter
(sum) and the elapsed time (max).  Rank 0 prints one JSON line.
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "adlsm-tree_amd"))

BPK = 10
ALGO_BYTES_PER_KEY16 = 26  # 16 B key read + (n*bpk+7)/n ~ 10 B bitmap write
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="single", choices=["single", "compaction", "varlen"])
    ap.add_argument("--keys", type=int, default=10_000_000, help="keys per filter (single/varlen)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget")
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


class Workload:
    """Device-resident inputs + a step() that performs one build."""

    def __init__(self, kind, rank, n, world=1):
        import numpy as np
        import torch

        import adlbloom as ab

        self.kind = kind
        if kind == "single":
            self.n = n
            self.keys = ab.synth_keys16(n, seed=0x5EED + rank)
            self.builder = ab.Builder(n, BPK)
            self.bytes_per_launch = ALGO_BYTES_PER_KEY16 * n
            self.config = {"workload": f"{n // 1_000_000}M x 16B keys, bits_per_key={BPK}, one filter per GPU",
                           "keys_per_gpu": n, "key_bytes": 16, "bits_per_key": BPK, "filters_per_gpu": 1}
            self.dtype = "u32"
        elif kind == "varlen":
            self.n = n
            self.keys, self.offs = ab.synth_varlen(n, seed=0x5EED + rank)
            total = int(self.offs[-1].item())
            self.builder = ab.Builder(n, BPK)
            # sum(len) + 8 B offset + ~10 B bitmap per key
            self.bytes_per_launch = total + 8 * (n + 1) + ab.bitmap_bytes(n, BPK)
            self.config = {"workload": f"{n // 1_000_000}M var-len keys (8-256 B, Zipf 1.1), bits_per_key={BPK}",
                           "keys_per_gpu": n, "mean_key_bytes": round(total / n, 2), "bits_per_key": BPK,
                           "filters_per_gpu": 1}
            self.dtype = "u32"
        else:  # compaction: 32 tables x 1M keys per GPU; table t lives on GPU t // 32
            from adlbloom import dist as D

            per = 1_000_000
            tables = D.table_shard(32 * world, world, rank)
            T = len(tables)
            self.n = T * per
            self.keys = torch.cat([ab.synth_keys16(per, seed=0x5EED + t) for t in tables])
            kb = np.arange(T + 1, dtype=np.uint64) * per
            self.builder = ab.SegmentedBuilder(kb, BPK)
            self.bytes_per_launch = ALGO_BYTES_PER_KEY16 * self.n
            self.config = {"workload": "compaction: 32 SSTables x 1M x 16B keys per GPU (256 over 8 GPUs)",
                           "keys_per_gpu": self.n, "key_bytes": 16, "bits_per_key": BPK, "filters_per_gpu": T}
            self.dtype = "u32"

    def step(self):
        if self.kind == "varlen":
            return self.builder.build(self.keys, self.offs)
        return self.builder.build(self.keys)


def cpu_baseline(budget_s):
    """The oracle's C restatement of BloomFilter::Keys2Block (single thread,
    gcc -O2) on the same 10M x 16 B SplitMix64 workload, repeated within budget."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    n = 10_000_000
    keys = O.splitmix_keys16(0x5EED, n)
    reps, t_total = 0, 0.0
    while reps < 20 and t_total < budget_s:
        t0 = time.perf_counter()
        O.keys2block(keys, bits_per_key=BPK)
        t_total += time.perf_counter() - t0
        reps += 1
    return {"value": round(n * reps / t_total / 1e6, 3), "unit": "Mkeys/s", "cores": 1, "kind": "port",
            "sample": f"{reps} x full 10M x 16B-key build (seed 0x5EED, bpk=10), oracle_keys2block "
                      f"(C restatement of src/filter_block.cpp:9-33, gcc -O2), {t_total:.1f} s"}


def e2e(n, iters=5):
    """Host keys (pinned) -> H2D -> build -> D2H bitmap; reported separately."""
    import torch

    import adlbloom as ab

    keys_d = ab.synth_keys16(n, seed=0x5EED)
    keys_h = torch.empty((n, 16), dtype=torch.uint8, pin_memory=True)
    keys_h.copy_(keys_d)
    b = ab.Builder(n, BPK)
    out_h = torch.empty(b.nbytes, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty_like(keys_d)
    st = torch.cuda.current_stream()

    def once():
        dst.copy_(keys_h, non_blocking=True)
        bm = b.build(dst)
        out_h.copy_(bm, non_blocking=True)

    once()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        once()
    st.synchronize()
    dt = (time.perf_counter() - t0) / iters
    return {"value": round(n / dt / 1e6, 1), "unit": "Mkeys/s", "ms_per_build": round(dt * 1e3, 3),
            "h2d_bytes": n * 16, "d2h_bytes": b.nbytes, "host_memory": "pinned"}


def parity_check(bm_dev, n):
    """Rank-0 bitmap vs the reference's SHA-256 for the seed-0x5EED key set."""
    path = os.path.join(ROOT, "tests", "golden", "appendix_b.json")
    try:
        gold = {g["n"]: g["sha256"] for g in json.load(open(path))["bitmaps"]}
    except OSError:
        return None
    if n not in gold:
        return None
    sha = hashlib.sha256(bm_dev.cpu().numpy().tobytes()).hexdigest()
    return "bit-identical to reference (sha256)" if sha == gold[n] else f"MISMATCH sha256 {sha}"


def load_traffic(workload, bytes_per_launch):
    """HBM bytes per build from the committed rocprofv3 PMC summary (profiles/), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    e = d.get(workload)
    return None if e is None else e.get("hbm_bytes_per_build")


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import adlbloom as ab

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    w = Workload(args.workload, rank, args.keys, world)
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        w.step()
    barrier()
    ab.profile_enable(max(args.steps, 1) * 64)  # launch pairs: a segmented build runs one per 8 filters
    t0 = time.perf_counter()
    for _ in range(args.steps):
        bm = w.step()
    barrier()
    elapsed = time.perf_counter() - t0
    ms_a, ms_b, nb = ab.profile_collect()

    # RCCL: the only collective -- sum of keys built, max of elapsed time
    from adlbloom import dist as D

    total_keys, elapsed_max = D.reduce_throughput(float(w.n) * args.steps, elapsed, device="cuda")

    parity = parity_check(bm, w.n) if (rank == 0 and args.workload == "single") else None

    if rank == 0:
        # kernel time per step (a segmented build is one launch pair per group of 8 filters)
        kern_ms = (ms_a + ms_b) / max(args.steps, 1)
        achieved = w.bytes_per_launch / (kern_ms * 1e-3) / 1e9 if nb else None
        traffic = load_traffic(args.workload, w.bytes_per_launch)
        out = {
            "metric": "Mkeys/s bloom-filter build (device-resident), 16B keys, bits/key=10"
            if args.workload != "varlen" else "Mkeys/s bloom-filter build (device-resident), var-len keys, bits/key=10",
            "value": round(total_keys / elapsed_max / 1e6, 1),
            "unit": "Mkeys/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / max(args.steps, 1) * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": w.dtype,
            "data": "synthetic (SplitMix64 keys generated on device, SURVEY.md §8d)",
            "config": dict(w.config, parallelism=f"whole filters per GPU x{world}, no data-path collective"),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1) if achieved else None,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic,
                "kernel": "bloom_bin_kernel + bloom_tile_kernel (one build = the pair)",
                "algorithmic_bytes_per_build": w.bytes_per_launch,
                "us_per_build": {"bloom_bin_kernel": round(ms_a / max(args.steps, 1) * 1e3, 2),
                                 "bloom_tile_kernel": round(ms_b / max(args.steps, 1) * 1e3, 2)},
                "launch_pairs_per_build": round(nb / max(args.steps, 1), 2),
                "read_only_frac": round(16 * w.n / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                if (nb and args.workload != "varlen") else None,
            },
            "parity": parity,
        }
        if world == 1 and args.workload == "single" and not args.no_e2e:
            out["e2e"] = e2e(w.n)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
