#!/usr/bin/env python3
"""bench.py -- MI355X bloom-filter build benchmark (BASELINE.json metric:
"Mkeys/s bloom-filter build (device-resident), 16B keys, bits/key=10").

A step is one bloom-filter build over one batch of device-resident synthetic
keys (SURVEY.md §8d SplitMix64), through the C-ABI (adl_bloom_build_device):
pass A (hash + bin) and pass B (LDS tile OR + bitmap write).  Workloads:

  single      (default) one 10M x 16 B-key filter per GPU, bpk=10 (BASELINE.json
              configs[1]); weak scaling: rank r builds its own SSTable filter.
  compaction  256 SSTables x 1M x 16 B keys, one filter each (configs[3]), tables
              t -> GPU t // (256/N), each GPU one segmented build of its tables
              (strong scaling: the 256 tables are fixed).
  varlen      10M variable-length keys (8-256 B, Zipf(1.1) lengths) per GPU (configs[2]).
  probe       100M 16 B queries against 256 device-resident 1M-key filters (configs[4]);
              filters t -> GPU t // (256/N).  At N > 1 the batch is bucketed by owner
              before upload, so each GPU is handed exactly its own
              tables' queries: no collective on the data path; strong scaling, the
              100M total is fixed.  The routed form (every rank asks a slice of the
              batch; two RCCL all-to-alls per step, adlbloom.dist.route_probe) is
              timed after it and reported as roofline.routing_variant.

Multi-GPU: one process per GPU (torch.distributed.run).  No workload has a
collective on its data path -- each rank owns whole filters.  RCCL reduces the
key counter (sum) and the elapsed time (max).  The default workload also
reports configs[3] as a `compaction_strong` sub-record (256 tables split over
the N GPUs, strong scaling), the north star's multi-GPU target, the same
build in a process serving Gets (`headline_with_reader`), and configs[4] and
configs[2] as `probe` and `varlen` sub-records, each with its own parity,
roofline and CPU baseline.  Rank 0 prints one JSON line.
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "adlsm-tree_amd"))

BPK = 10
ALGO_BYTES_PER_KEY16 = 26  # 16 B key read + (n*bpk+7)/n ~ 10 B bitmap write
ALGO_BYTES_PER_QUERY = 21  # 16 B query + 4 B filter id + 1 B result
PROBE_TABLES, PROBE_KEYS_PER_TABLE = 256, 1_000_000
COMPACTION_TABLES = 256   # BASELINE.json configs[3]
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="single", choices=["single", "compaction", "varlen", "probe"])
    ap.add_argument("--keys", type=int, default=10_000_000, help="keys per filter (single/varlen)")
    ap.add_argument("--queries", type=int, default=100_000_000, help="total probe queries (probe)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget")
    ap.add_argument("--no-compaction-strong", action="store_true",
                    help="single: skip the configs[3] compaction_strong sub-record")
    ap.add_argument("--no-sub-records", action="store_true",
                    help="single: skip the configs[4] probe and configs[2] varlen sub-records")
    ap.add_argument("--no-reader", action="store_true",
                    help="single: skip the headline_with_reader record")
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


class Workload:
    """Device-resident inputs + a step() that performs one build."""

    def __init__(self, kind, rank, n, world=1, queries=0):
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
        elif kind == "probe":
            self._init_probe(rank, world, queries)
        else:  # compaction: 256 tables x 1M keys; table t lives on GPU t // (256/N)
            from adlbloom import dist as D

            per = 1_000_000
            tables = D.table_shard(COMPACTION_TABLES, world, rank)
            self.tables = tables
            T = len(tables)
            self.n = T * per
            self.keys = torch.cat([ab.synth_keys16(per, seed=0x5EED + t) for t in tables])
            kb = np.arange(T + 1, dtype=np.uint64) * per
            self.builder = ab.SegmentedBuilder(kb, BPK)
            self.bytes_per_launch = ALGO_BYTES_PER_KEY16 * self.n
            self.config = {"workload": f"compaction: {COMPACTION_TABLES} SSTables x 1M x 16B keys, one filter each, "
                                       f"{T} per GPU",
                           "tables_total": COMPACTION_TABLES, "keys_per_gpu": self.n, "key_bytes": 16,
                           "bits_per_key": BPK, "filters_per_gpu": T}
            self.dtype = "u32"

    def _init_probe(self, rank, world, queries):
        """configs[4]: 256 tables x 1M keys (this rank's share built on the device in
        segmented builds of 32 tables), compacted to exact-length bitmaps.  Rank r
        asks the slice [r*Q/N, (r+1)*Q/N) of the global query stream (generated on
        the device); at N > 1 each step routes the queries to their filters' ranks
        and the answers back (adlbloom.dist.route_probe)."""
        import numpy as np
        import torch

        import adlbloom as ab
        from adlbloom import dist as D

        per = PROBE_KEYS_PER_TABLE
        tables = D.table_shard(PROBE_TABLES, world, rank)
        self.tables = tables
        self.world = world
        pieces, sizes = [], []
        for g0 in range(tables.start, tables.stop, 32):
            grp = range(g0, min(g0 + 32, tables.stop))
            keys = torch.cat([ab.synth_keys16(per, seed=0x5EED + t) for t in grp])
            bms, boff, sz = ab.build_segmented(keys, np.arange(len(grp) + 1, dtype=np.uint64) * per)
            pieces += [bms[int(o):int(o) + int(z)] for o, z in zip(boff, sz)]
            sizes += [int(z) for z in sz]
            del keys
        self.bitmaps = torch.cat(pieces)
        del pieces
        off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
        self.bitmap_off_host = off
        self.bitmap_off = torch.from_numpy(off.view(np.int64)).cuda()
        own, lid = D.owner_table(PROBE_TABLES, world)
        self.owner = torch.from_numpy(own).cuda()
        self.local_id = torch.from_numpy(lid).cuda()
        if queries % world:
            raise SystemExit(f"--queries {queries} must divide over {world} ranks")
        self.gidx = None  # batch positions of this rank's queries (owner-bucketed, N > 1)
        self.bucketing_ms = None
        if world == 1:
            self.n = queries
            self.keys, self.fid, self.member = ab.synth_probe_queries(queries, num_tables=PROBE_TABLES,
                                                                      keys_per_table=per)
        else:
            # owner-bucketed: the whole batch, bucketed by owner before
            # upload -- this rank keeps exactly its own tables' queries, batch order kept;
            # self.fid holds filter ids local to this rank.  Its cost (outside the timed
            # loop: a lookup is issued where its level's tables live) is reported as
            # probe_bucketing_ms.
            torch.cuda.synchronize()
            tb0 = time.perf_counter()
            ks, fs, ms, ix = [], [], [], []
            chunk = 8_000_000
            for q0 in range(0, queries, chunk):
                k, f, m = ab.synth_probe_queries(min(chunk, queries - q0), q0=q0, num_tables=PROBE_TABLES,
                                                 keys_per_table=per)
                idx, lf = D.owner_select(f, self.owner, self.local_id, rank)
                ks.append(k[idx])
                fs.append(lf)
                ms.append(m[idx])
                ix.append(idx + q0)
                del k, f, m
            self.keys, self.fid, self.member, self.gidx = (torch.cat(ks), torch.cat(fs), torch.cat(ms),
                                                           torch.cat(ix))
            torch.cuda.synchronize()
            self.bucketing_ms = (time.perf_counter() - tb0) * 1e3
            self.n = int(self.keys.shape[0])
            # the routed variant's input: this rank's contiguous slice of the batch
            rq0, rn = rank * (queries // world), queries // world
            self.route_n = rn
            self.route_keys, self.route_fid, _ = ab.synth_probe_queries(rn, q0=rq0, num_tables=PROBE_TABLES,
                                                                        keys_per_table=per)
        self.total_queries = queries
        self.bytes_per_launch = ALGO_BYTES_PER_QUERY * self.n
        self.kernel_events = []  # (start, stop) of every probe launch
        self.served = self.n
        self.routing = None
        self.config = {"workload": f"probe: {queries // 1_000_000}M x 16B queries vs {PROBE_TABLES} device-resident "
                                   f"filters of {per // 1_000_000}M keys (50% inserted keys)",
                       "queries_total": queries, "queries_this_gpu": self.n, "filters_total": PROBE_TABLES,
                       "filters_per_gpu": len(tables), "keys_per_filter": per, "bits_per_key": BPK,
                       "routing": "none (one GPU)" if world == 1 else
                       "owner-bucketed: each GPU is handed its own tables' queries (bucketed by owner before "
                       "upload); no collective on the data path"}
        self.dtype = "u32"

    def _probe_local(self, keys, lfid):
        import torch

        import adlbloom as ab

        if self.kernel_events is None:  # the throughput pass: no events
            return ab.probe_batch(keys, lfid, self.bitmaps, self.bitmap_off)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = ab.probe_batch(keys, lfid, self.bitmaps, self.bitmap_off)
        e1.record()
        self.kernel_events.append((e0, e1))
        return out

    def step(self):
        if self.kind == "probe":
            return self._probe_local(self.keys, self.fid)
        if self.kind == "varlen":
            return self.builder.build(self.keys, self.offs)
        return self.builder.build(self.keys)

    def step_routed(self):
        """The routed probe (N > 1): this rank's slice of the batch goes to the
        tables' owners and the answers come back, two RCCL all-to-alls."""
        import adlbloom as ab
        from adlbloom import dist as D

        st = {}
        out, _ = D.route_probe(self.route_keys, self.route_fid, self.owner, self.local_id,
                               lambda k, f: ab.probe_batch(k, f, self.bitmaps, self.bitmap_off), stats=st)
        # DESIGN.md §6's cost model: (N-1)/N of the queries cross xGMI, 20 B out and 1 B back
        self.routing = dict(st, bytes_per_query_out=D.ROUTE_BYTES_OUT, bytes_per_query_back=D.ROUTE_BYTES_BACK,
                            offrank_fraction=round(st["queries_sent_offrank"] / max(self.route_n, 1), 4),
                            model_offrank_fraction=round((self.world - 1) / self.world, 4))
        return out



def _cpu_cores():
    """Host threads for the multi-filter CPU baselines: this process's CPU share,
    capped at 16 (the GPU box's share per GPU)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def _timed_reps(fn, budget_s, max_reps=20):
    reps, t_total = 0, 0.0
    while reps < max_reps and t_total < budget_s:
        t0 = time.perf_counter()
        fn()
        t_total += time.perf_counter() - t0
        reps += 1
    return reps, t_total


def cpu_baseline(budget_s, workload="single", w=None):
    """The oracle's C restatement of the reference path (gcc -O2) on the same
    synthetic inputs, timed on this host: BloomFilter::Keys2Block
    (src/filter_block.cpp:9-33) single-threaded for one filter, one filter per
    thread for the 32-table compaction shard, and IsKeyExists
    (src/filter_block.cpp:49-62) over query slices per thread for the probe."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np

    import oracle as O

    if workload == "varlen":
        data = w.keys.cpu().numpy()
        offs = w.offs.cpu().numpy().view(np.uint64)
        n = len(offs) - 1
        reps, t = _timed_reps(lambda: O.keys2block(data, offsets=offs, bits_per_key=BPK), budget_s)
        return {"value": round(n * reps / t / 1e6, 3), "unit": "Mkeys/s", "cores": 1, "kind": "port",
                "sample": f"{reps} x full {n // 1_000_000}M var-len-key build (same keys as the GPU run), "
                          f"oracle_keys2block (C restatement of src/filter_block.cpp:9-33, gcc -O2), {t:.1f} s"}
    if workload == "compaction":
        per, T = 1_000_000, 32
        cores = _cpu_cores()
        tables = [O.splitmix_keys16(0x5EED + t, per) for t in range(T)]
        with ThreadPoolExecutor(cores) as ex:
            def run():
                list(ex.map(lambda k: O.keys2block(k, bits_per_key=BPK), tables))
            reps, t = _timed_reps(run, budget_s)
        return {"value": round(T * per * reps / t / 1e6, 3), "unit": "Mkeys/s", "cores": cores, "kind": "port",
                "sample": f"{reps} x 32 of the 256 tables x 1M x 16B keys, one filter per thread on "
                          f"{cores} threads, oracle_keys2block (gcc -O2), {t:.1f} s"}
    if workload == "probe":
        cores = _cpu_cores()
        ns = min(w.n, 2_000_000)
        q = w.keys[:ns].cpu().numpy()
        fid = w.fid[:ns].cpu().numpy().view(np.uint32)
        bms = w.bitmaps.cpu().numpy()
        off = w.bitmap_off_host
        sl = [slice(i, min(ns, i + (ns + cores - 1) // cores)) for i in range(0, ns, (ns + cores - 1) // cores)]
        with ThreadPoolExecutor(cores) as ex:
            def run():
                list(ex.map(lambda s_: O.probe_multi(q[s_], fid[s_], bms, off, bits_per_key=BPK), sl))
            reps, t = _timed_reps(run, budget_s)
        return {"value": round(ns * reps / t / 1e6, 3), "unit": "Mqueries/s", "cores": cores, "kind": "port",
                "sample": f"{reps} x the first {ns // 1000}k queries of this GPU's batch, query slices on "
                          f"{cores} threads, oracle_probe_multi (C restatement of src/filter_block.cpp:49-62), "
                          f"{t:.1f} s"}
    n = 10_000_000
    keys = O.splitmix_keys16(0x5EED, n)
    reps, t_total = _timed_reps(lambda: O.keys2block(keys, bits_per_key=BPK), budget_s)
    return {"value": round(n * reps / t_total / 1e6, 3), "unit": "Mkeys/s", "cores": 1, "kind": "port",
            "sample": f"{reps} x full 10M x 16B-key build (seed 0x5EED, bpk=10), oracle_keys2block "
                      f"(C restatement of src/filter_block.cpp:9-33, gcc -O2), {t_total:.1f} s"}


def load_pins():
    """Full-size oracle pins of configs[2]-[4] (tests/golden/full_size.json), or None."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "full_size.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def gather_all(t, world):
    """Every rank's equal-length slice, concatenated in rank order (all ranks call)."""
    if world == 1:
        return t
    import torch
    import torch.distributed as dist

    if dist.get_backend() == "gloo":  # host tensors (the 2-rank test on one GPU)
        parts = [torch.empty_like(t.cpu()) for _ in range(world)]
        dist.all_gather(parts, t.contiguous().cpu())
        return torch.cat(parts).to(t.device)
    out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.contiguous())
    return out


def probe_check(w, out, rank, world):
    """Probe results (all ranks call; rank 0 returns the record): all 100M answers,
    gathered in global query order, against the oracle's SHA-256
    (tests/golden/full_size.json); every inserted key found; the false-positive
    rate on fresh keys; and the bitmap reads per query with the reference's early
    exit, counted on a sample of rank 0's queries to its own filters."""
    import numpy as np

    if world > 1:  # owner-bucketed: every rank's answers back in batch order
        from adlbloom import dist as D

        allout = D.scatter_answers(out, w.gidx, w.total_queries)
        allmem = D.scatter_answers(w.member, w.gidx, w.total_queries)
    else:
        allout, allmem = out, w.member
    if rank != 0:
        return None
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    mem = allmem.bool()
    hits_ins = int(allout[mem].sum().item())
    n_ins = int(mem.sum().item())
    fp = int(allout[~mem].sum().item())
    n_fresh = int(allout.numel()) - n_ins
    rec = {"hit_rate_inserted": round(hits_ins / max(n_ins, 1), 6), "false_negatives": n_ins - hits_ins,
           "fpr_fresh": round(fp / max(n_fresh, 1), 6), "queries_inserted": n_ins, "queries_fresh": n_fresh}
    pins = load_pins()
    if pins and pins["probe"]["queries"] == w.total_queries:
        sha = hashlib.sha256(allout.cpu().numpy().tobytes()).hexdigest()
        rec["oracle"] = ("all %dM answers bit-identical to the oracle (sha256)" % (w.total_queries // 1_000_000)
                         if sha == pins["probe"]["results_sha256"] else f"MISMATCH sha256 {sha}")
    else:  # no pin for this batch: rank 0's first 200K queries (all to its own filters) against the oracle
        sel0 = np.arange(min(w.n, 200_000))
        want = O.probe_multi(w.keys[:sel0.size].cpu().numpy(), w.fid[:sel0.size].cpu().numpy().astype(np.uint32),
                             w.bitmaps.cpu().numpy(), np.asarray(w.bitmap_off_host, dtype=np.uint64),
                             bits_per_key=BPK)
        got = out[:sel0.size].cpu().numpy()
        rec["oracle"] = ("parity unpinned (no pin for this batch); %d sampled answers identical to the oracle"
                         % sel0.size if np.array_equal(got, want) else "MISMATCH on sampled answers")
    # reads per query on rank 0's own filters (w.fid: filter ids local to this rank)
    fid_all = w.fid.cpu().numpy().astype(np.int64)
    sel = np.arange(min(w.n, 200_000))
    bms = w.bitmaps.cpu().numpy()
    off = np.asarray(w.bitmap_off_host, dtype=np.int64)
    h = O.murmur3_batch(w.keys[:sel.size].cpu().numpy())
    lf = fid_all[sel]
    base = off[lf]
    m = (off[lf + 1] - base) * 8
    alive = np.ones(sel.size, dtype=bool)
    reads = np.zeros(sel.size, dtype=np.int64)
    for j in range(O.num_probes(BPK)):
        pos = ((h[:, 0].astype(np.uint64) + np.uint64(j) * h[:, 1].astype(np.uint64)) % np.uint64(1 << 32)
               ).astype(np.int64) % m
        bit = (bms[base + (pos >> 3)] >> (pos & 7)) & 1
        reads += alive
        alive &= bit.astype(bool)
    rec["bitmap_reads_per_query"] = round(float(reads.mean()), 4)
    return rec


def build_parity(w, rank):
    """Rank 0's bitmaps against the oracle pins (varlen, compaction)."""
    pins = load_pins() or {"varlen": {"n": -1}, "compaction": {"bitmap_sha256": {}}}
    if rank != 0:
        return None
    if w.kind == "varlen":
        p = pins["varlen"]
        if w.n != p["n"]:
            return oracle_build_check(w.builder.bitmap[:w.builder.nbytes], w.keys, w.offs, w.n)
        sha = hashlib.sha256(w.builder.bitmap[:w.builder.nbytes].cpu().numpy().tobytes()).hexdigest()
        return "bit-identical to the oracle (sha256)" if sha == p["bitmap_sha256"] else f"MISMATCH sha256 {sha}"
    if w.kind == "compaction":
        want = pins["compaction"]["bitmap_sha256"]
        if isinstance(want, dict) or len(want) != COMPACTION_TABLES:  # no pins: two tables against the oracle
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O

            bad = [t for i, t in list(enumerate(w.tables))[:2]
                   if not np.array_equal(w.builder.bitmap(i).cpu().numpy(),
                                         O.keys2block(O.splitmix_keys16(0x5EED + t, 1_000_000), bits_per_key=BPK))]
            return ("parity unpinned (no pins): 2 tables bit-identical to the oracle" if not bad
                    else f"MISMATCH tables {bad}")
        bad = [t for i, t in enumerate(w.tables)
               if hashlib.sha256(w.builder.bitmap(i).cpu().numpy().tobytes()).hexdigest() != want[t]]
        return (f"all {len(w.tables)} bitmaps of this GPU bit-identical to the oracle (sha256)" if not bad
                else f"MISMATCH tables {bad[:8]}")
    return None


def hbm_stream_read_gbs(nbytes=4 << 30, reps=5):
    """Measured streaming-read bandwidth of this GPU (lib/libadlhbm.so, nontemporal
    16 B loads, persistent grid), best of `reps` over a buffer 16x the Infinity Cache."""
    import ctypes

    import torch

    path = os.path.join(ROOT, "adlsm-tree_amd", "lib", "libadlhbm.so")
    L = ctypes.CDLL(path)
    L.adl_hbm_stream_read.restype = ctypes.c_int
    L.adl_hbm_stream_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                      ctypes.c_void_p]
    buf = torch.ones(nbytes // 8, dtype=torch.int64, device="cuda")
    sink = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    best = 0.0
    for _ in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        rc = L.adl_hbm_stream_read(buf.data_ptr(), nbytes, sink.data_ptr(), sink.numel(),
                                   ctypes.c_void_p(st.cuda_stream))
        e1.record(st)
        e1.synchronize()
        if rc:
            return None
        best = max(best, nbytes / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    del buf
    return round(best, 1)


def hbm_random_read_gps(buf, iters=64, reps=3):
    """Measured random single-byte read rate (G reads/s) over `buf` (the probe's own
    filter arena, so the same working set), lib/libadlhbm.so's hbm_random_read_kernel."""
    import ctypes

    import torch

    L = ctypes.CDLL(os.path.join(ROOT, "adlsm-tree_amd", "lib", "libadlhbm.so"))
    L.adl_hbm_random_read.restype = ctypes.c_uint64
    L.adl_hbm_random_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                      ctypes.c_uint32, ctypes.c_void_p]
    sink = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    best = 0.0
    for _ in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        nreads = L.adl_hbm_random_read(buf.data_ptr(), buf.numel(), iters, sink.data_ptr(), sink.numel(),
                                       ctypes.c_void_p(st.cuda_stream))
        e1.record(st)
        e1.synchronize()
        if not nreads:
            return None
        best = max(best, nreads / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    return round(best, 2)


def e2e(n, iters=5, flushes=5):
    """End to end through host memory (pinned), reported beside the
    device-resident headline:
      * single: one build's latency -- H2D 16n B of keys, the build, D2H the
        bitmap, serial on one stream; its floor is the two copies at the link's
        measured one-way rates (every bit of the bitmap can depend on the last
        key, so the download cannot start before the upload ends);
      * flush_stream: `flushes` memtable-sized filters back to back through
        adl_bloom_build_segmented (the pipelined host API: filter i's bitmap
        downloads while filter i+1's keys upload), the SSTable-flush / compaction
        producer's steady state (src/sstable.cpp:54-62, src/db.cpp:428-509)."""
    import numpy as np
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

    def timed_ms(fn, reps):
        """median over reps of one call, the stream drained before and after it"""
        ts = []
        for i in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            st.synchronize()
            if i:
                ts.append((time.perf_counter() - t0) * 1e3)
        return float(np.median(ts))

    dt = timed_ms(once, iters)
    bm_dev = b.bitmap[:b.nbytes]
    h2d_ms = timed_ms(lambda: dst.copy_(keys_h, non_blocking=True), iters)
    d2h_ms = timed_ms(lambda: out_h.copy_(bm_dev, non_blocking=True), iters)
    parity = parity_check(out_h, n, None) if n == 10_000_000 else None
    rec = {"value": round(n / (dt * 1e-3) / 1e6, 1), "unit": "Mkeys/s", "ms_per_build": round(dt, 3),
           "h2d_bytes": n * 16, "d2h_bytes": b.nbytes, "host_memory": "pinned",
           "single": {"ms_per_build": round(dt, 3), "h2d_ms": round(h2d_ms, 3), "d2h_ms": round(d2h_ms, 3),
                      "h2d_gbs": round(n * 16 / (h2d_ms * 1e-3) / 1e9, 1),
                      "d2h_gbs": round(b.nbytes / (d2h_ms * 1e-3) / 1e9, 1),
                      "floor_ms": round(h2d_ms + d2h_ms, 3), "parity": parity}}
    del dst
    # back-to-back flushes through the pipelined host API
    F = flushes
    kh = torch.empty((F * n, 16), dtype=torch.uint8, pin_memory=True)
    for f in range(F):
        kh[f * n:(f + 1) * n].copy_(keys_d)
    kb = np.arange(F + 1, dtype=np.uint64) * n
    nb = ab.bitmap_bytes(n, BPK)
    boff = np.arange(F, dtype=np.uint64) * nb
    outs = torch.zeros(F * nb, dtype=torch.uint8, pin_memory=True)
    ab.build_segmented_host(kh, kb, outs, boff)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 2
    for _ in range(reps):
        ab.build_segmented_host(kh, kb, outs, boff)
    ds = (time.perf_counter() - t0) / reps / F * 1e3
    same = all(torch.equal(outs[f * nb:(f + 1) * nb], out_h) for f in range(F))
    rec["flush_stream"] = {"ms_per_build": round(ds, 3), "value": round(n / (ds * 1e-3) / 1e6, 1),
                           "filters": F, "api": "adl_bloom_build_segmented (pipelined groups, one filter each)",
                           "parity": "every filter's bitmap equal to the single build's" if same else "MISMATCH"}
    rec["ms_per_build_stream"] = round(ds, 3)
    del kh, outs
    return rec


def e2e_compaction(w, iters=3):
    """Compaction shape end to end: 32 tables' keys in pinned host memory ->
    adl_bloom_build_segmented (groups of filters: key upload, build and bitmap
    download overlapped on three streams) -> exact-length bitmaps packed back
    to back in pinned host memory (the filter-block layout).  Also times the
    unpipelined sequence (all keys up, one segmented build, all bitmaps down)."""
    import numpy as np
    import torch

    import adlbloom as ab

    kb = w.builder.kb
    n = int(kb[-1])
    keys_h = torch.empty((n, 16), dtype=torch.uint8, pin_memory=True)
    keys_h.copy_(w.keys)
    sizes = [ab.bitmap_bytes(int(kb[f + 1] - kb[f]), BPK) for f in range(len(kb) - 1)]
    boff = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    out_h = torch.zeros(int(sum(sizes)), dtype=torch.uint8, pin_memory=True)
    ab.build_segmented_host(keys_h, kb, out_h, boff)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        ab.build_segmented_host(keys_h, kb, out_h, boff)
    dt = (time.perf_counter() - t0) / iters
    # unpipelined: H2D all keys, one segmented build, D2H the device bitmaps
    dst = torch.empty_like(w.keys)
    seq_h = torch.empty(w.builder.out.numel(), dtype=torch.uint8, pin_memory=True)

    def seq():
        dst.copy_(keys_h, non_blocking=True)
        out = w.builder.build(dst)
        seq_h.copy_(out, non_blocking=True)
        torch.cuda.current_stream().synchronize()

    seq()
    t0 = time.perf_counter()
    for _ in range(iters):
        seq()
    ds = (time.perf_counter() - t0) / iters
    return {"value": round(n / dt / 1e6, 1), "unit": "Mkeys/s", "ms_per_build": round(dt * 1e3, 3),
            "h2d_bytes": n * 16, "d2h_bytes": int(sum(sizes)), "host_memory": "pinned",
            "api": "adl_bloom_build_segmented (pipelined groups)",
            "unpipelined": {"value": round(n / ds / 1e6, 1), "ms_per_build": round(ds * 1e3, 3)}}


def parity_check(bm_dev, n, keys=None):
    """Rank-0 bitmap vs the reference's SHA-256 for the seed-0x5EED key set; for
    a size the pins do not cover, against the oracle's build of the same keys
    (up to 20M keys), else a sampled statement."""
    path = os.path.join(ROOT, "tests", "golden", "appendix_b.json")
    try:
        gold = {g["n"]: g["sha256"] for g in json.load(open(path))["bitmaps"]}
    except (OSError, ValueError):
        gold = {}
    if n in gold:
        sha = hashlib.sha256(bm_dev.cpu().numpy().tobytes()).hexdigest()
        return "bit-identical to reference (sha256)" if sha == gold[n] else f"MISMATCH sha256 {sha}"
    return oracle_build_check(bm_dev, keys, None, n)


def oracle_build_check(bm_dev, keys, offs, n):
    """Parity of a build the pins do not cover: the oracle's bitmap of the same
    keys (n <= 20M: a few seconds of CPU), or -- larger -- 'parity unpinned'
    with a sampled check that every bit of 100K of the keys is set."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    got = bm_dev.cpu().numpy()
    hk = keys.cpu().numpy()
    ho = offs.cpu().numpy().view(np.uint64) if offs is not None else None
    if n <= 20_000_000:
        want = O.keys2block(hk, offsets=ho, bits_per_key=BPK)
        return ("bit-identical to the oracle (full build of the same keys)" if np.array_equal(got, want)
                else f"MISMATCH vs the oracle ({int((got != want).sum())} bytes differ)")
    idx = np.random.default_rng(1).choice(n, 100_000, replace=False)
    if ho is None:
        ok = O.probe(hk[idx], got, bits_per_key=BPK).all()
    else:
        ks = [hk[int(ho[i]):int(ho[i + 1])].tobytes() for i in idx]
        ok = O.probe(ks, got, bits_per_key=BPK).all()
    return ("parity unpinned (no pin for this size); sampled: every bit of 100K keys set" if ok
            else "MISMATCH: a sampled key has a clear bit")


def load_pmc(workload):
    """This workload's entry of the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, tools/pmc_traffic.py), or {}."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        return json.load(open(path)).get(workload) or {}
    except (OSError, ValueError):
        return {}


def load_traffic(workload, bytes_per_launch):
    """HBM bytes per build from the committed rocprofv3 PMC summary (profiles/), or None."""
    return load_pmc(workload).get("hbm_bytes_per_build")


# Integer issue ceiling (MI355X_MICROARCH.md): 256 CUs x 4 SIMDs, one wave64
# VALU instruction per SIMD every 2 cycles, at the clock the PMC pass measured
# (GRBM_GUI_ACTIVE / 8 XCDs / kernel time).
def alu_roofline(workload, n_keys, kernels_us):
    """roofline.alu (SURVEY.md §8(d)'s secondary bound) from the committed PMC
    pass: VALU wave-instructions per key of each pass, and the fraction of the
    integer issue ceiling they take at this run's kernel times."""
    e = load_pmc(workload).get("alu")
    if not e:
        return None
    out = {"source": "profiles/pmc_traffic.json (SQ_INSTS_VALU, GRBM_GUI_ACTIVE per kernel)",
           "issue_model": "256 CUs x 4 SIMDs x 1 wave64 VALU instruction / 2 cycles"}
    for k, v in e.items():
        us = kernels_us.get(k)
        clk = v.get("clock_ghz") or 2.4
        ceiling = 256 * 4 / 2 * clk * 1e9  # wave-instructions / s
        out[k] = {"valu_wave_insts": v["valu_wave_insts"],
                  "valu_lane_ops_per_key": round(v["valu_wave_insts"] * 64 / n_keys, 1),
                  "clock_ghz": clk,
                  "issue_frac": round(v["valu_wave_insts"] / (us * 1e-6) / ceiling, 4) if us else None}
    return out


def lds_roofline(workload, kernels_us):
    """roofline.lds from the committed PMC pass (tools/pmc_lds.py): per build
    pass, the LDS array's cycles and the share of them spent in bank
    conflicts, as a busy fraction of this run's kernel time, and the array
    time with and without the conflict cycles (the floor an LDS-bound pass
    could reach, MI355X_MICROARCH.md §LDS)."""
    e = load_pmc(workload).get("lds")
    if not e:
        return None
    out = {"source": "profiles/pmc_traffic.json (SQ_LDS_IDX_ACTIVE, SQ_LDS_BANK_CONFLICT, GRBM_GUI_ACTIVE)",
           "model": "array cycles summed over 256 CUs; busy = cycles / (256 x kernel cycles)"}
    if workload == "single":
        # the bound measured directly: the same pass A
        # with a conflict-free counting sort (diagnostics build, wrong tiles)
        out["conflict_free_pass_a_us"] = {"real_sort": 101.0, "conflict_free": 97.7, "gain_frac": 0.034,
                                          "source": "profiles/r05/r05b_lds_conflict_free_ab.log"}
    for k, v in e.items():
        us = kernels_us.get(k)
        clk = v.get("clock_ghz") or 2.4
        arr_us = v["array_cycles"] / 256 / (clk * 1e3)
        out[k] = {"conflict_frac": v.get("conflict_frac"), "clock_ghz": clk,
                  "array_us": round(arr_us, 2),
                  "array_us_without_conflicts": round((v["array_cycles"] - v["conflict_cycles"]) / 256 / (clk * 1e3), 2),
                  "array_busy_frac": round(arr_us / us, 4) if us else None}
    return out


_STREAM_GBS = []


def stream_gbs_once():
    """hbm_stream_read_gbs, measured once per process (every record reuses it)."""
    if not _STREAM_GBS:
        _STREAM_GBS.append(hbm_stream_read_gbs())
    return _STREAM_GBS[0]


def measure(kind, args, rank, world, backend, barrier, timed, sub=False):
    """One workload's record: warmup, the timed K steps (the throughput), the
    same K steps again with per-kernel HIP events (the roofline), parity
    against the reference / oracle pins, and (rank 0, one GPU) its CPU
    baseline.  All ranks call; rank 0 gets the dict, the others None.
    sub: a sub-record of the default line (smaller CPU-baseline budget, no
    e2e)."""
    import torch

    import adlbloom as ab
    from adlbloom import dist as D

    w = Workload(kind, rank, args.keys, world, args.queries)
    probe = kind == "probe"
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        w.step()
    barrier()
    # Pass 1, the throughput: K steps with nothing but the work in flight.
    # Timing events on the kernels' dispatch packets add ~9.5 us at every
    # launch boundary (tools/gap_check.sh: 0 us between the passes without
    # them, 9.4-9.5 with them), so they stay out of this pass.
    w.kernel_events = None
    t0 = time.perf_counter()
    for i in range(args.steps):
        out = w.step()
    barrier()
    elapsed = time.perf_counter() - t0
    # Pass 2, the kernel durations: the same K steps again, each kernel timed by
    # HIP events on its own dispatch packets (build) or on torch's current
    # stream around the probe pipeline (Workload._probe_local).
    ab.profile_enable(max(args.steps, 1) * 64)  # launch pairs: a segmented build runs one per 8 filters
    if probe:
        w.kernel_events = []
    t1 = time.perf_counter()
    for i in range(args.steps):
        out = w.step()
    barrier()
    elapsed_instrumented = time.perf_counter() - t1
    pairs = ab.profile_each(max(args.steps, 1) * 64)
    ms_a, ms_b, nb = ab.profile_collect()
    probe_ms = sum(a.elapsed_time(b) for a, b in w.kernel_events) / max(args.steps, 1) if probe else 0.0
    if probe:  # the kernel's own work: the queries this rank probed (its filters' share of all ranks')
        w.bytes_per_launch = ALGO_BYTES_PER_QUERY * w.served

    # RCCL: the only collective -- sum of keys built, max of elapsed time
    total_keys, elapsed_max = D.reduce_throughput(float(w.n) * args.steps, elapsed, device="cuda")

    # the routed probe (N > 1), reported beside the owner-bucketed measurement
    routing_variant = None
    if probe and world > 1:
        el = timed(w.step_routed, args.steps)
        routing_variant = {
            "form": "routed: every GPU asks a contiguous slice of the batch; each step sends every query to its "
                    "table's GPU and the answer back (2 RCCL all-to-alls, adlbloom.dist.route_probe)",
            "value": round(w.total_queries * args.steps / el / 1e6, 1), "unit": "Mqueries/s",
            "ms_per_step": round(el / max(args.steps, 1) * 1e3, 4), "rank0_traffic": w.routing}

    if rank == 0 and kind == "single":
        parity = parity_check(out, w.n, w.keys)
    elif probe:
        parity = probe_check(w, out, rank, world)
    else:
        parity = build_parity(w, rank)

    rec = None
    if rank == 0:
        if probe:
            kern_ms = probe_ms
            kernels = {"probe (adl_bloom_probe_batch_device)": round(probe_ms * 1e3, 2)}
            kname = ("adl_bloom_probe_batch_device: tile-binned pipeline pb_* (9 launches) for large 16-byte "
                     "batches, bloom_probe_multi_kernel otherwise")
            med = None
        else:
            # kernel time per step (every filter of a segmented build in one launch pair)
            kern_ms = (ms_a + ms_b) / max(args.steps, 1)
            kernels = {"bloom_bin_kernel": round(ms_a / max(args.steps, 1) * 1e3, 2),
                       "bloom_tile_kernel": round(ms_b / max(args.steps, 1) * 1e3, 2)}
            kname = "bloom_bin_kernel + bloom_tile_kernel (one build = the pair)"
            if kind == "varlen":
                kname = ("hash_var_kernel + bloom_bin16_kernel<SrcH> (the pass-A interval) + bloom_tile_kernel "
                         "(one build)")
            # median over the steps: each step's launch pairs summed
            per = len(pairs) // max(args.steps, 1)
            if per and len(pairs) == per * args.steps:
                steps_ms = [[sum(p[j] for p in pairs[i * per:(i + 1) * per]) for j in (0, 1)]
                            for i in range(args.steps)]
                med = {"bloom_bin_kernel": round(float(np.median([x[0] for x in steps_ms])) * 1e3, 2),
                       "bloom_tile_kernel": round(float(np.median([x[1] for x in steps_ms])) * 1e3, 2),
                       "build": round(float(np.median([x[0] + x[1] for x in steps_ms])) * 1e3, 2)}
            else:
                med = None
        is_timed = kern_ms > 0 and (probe or nb)
        achieved = w.bytes_per_launch / (kern_ms * 1e-3) / 1e9 if is_timed else None
        traffic = load_traffic(kind, w.bytes_per_launch)
        stream_gbs = stream_gbs_once()
        if probe:
            metric = "Mqueries/s bloom-filter probe (device-resident), 16B keys, 256 filters, bits/key=10"
            if world > 1:
                metric += ", owner-bucketed"
        elif kind == "varlen":
            metric = "Mkeys/s bloom-filter build (device-resident), var-len keys, bits/key=10"
        elif kind == "compaction":
            metric = ("Mkeys/s bloom-filter build (device-resident), 16B keys, bits/key=10, "
                      "configs[3]: 256 SSTables x 1M keys")
        else:
            metric = "Mkeys/s bloom-filter build (device-resident), 16B keys, bits/key=10"
        rec = {
            "metric": metric,
            "value": round(total_keys / elapsed_max / 1e6, 1),
            "unit": "Mqueries/s" if probe else "Mkeys/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / max(args.steps, 1) * 1e3, 4),
            "ms_per_step_kernel_timed": round(elapsed_instrumented / max(args.steps, 1) * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if kind in ("probe", "compaction") else "weak",
            "vs_baseline": None,
            "dtype": w.dtype,
            "data": "synthetic (SplitMix64 keys generated on device, SURVEY.md §8d)",
            "config": dict(w.config, parallelism=f"whole filters per GPU x{world}, no data-path collective"),
            "world": {"size": world, "backend": backend or "none (one process)"},
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1) if achieved else None,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic,
                "kernel": kname,
                "kernel_timing": "HIP events on each kernel's dispatch packets (probe: on the stream around the "
                                 "pipeline), over a second pass of the same K steps right after the timed one",
                "algorithmic_bytes_per_step": w.bytes_per_launch,
                "us_per_step": kernels,
                "median_us_per_step": med,
                "zero_fill_us": None if probe else 0.0,  # none: pass B writes every bitmap byte
                "launch_pairs_per_build": None if probe else round(nb / max(args.steps, 1), 2),
                "read_only_frac": round(16 * w.n / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                if (is_timed and kind in ("single", "compaction")) else None,
                "measured_stream_read_gbs": stream_gbs,
                "frac_of_measured_stream_read": round(achieved / stream_gbs, 4) if (achieved and stream_gbs) else None,
            },
            "parity": parity,
        }
        if traffic and is_timed:
            rec["roofline"]["traffic_gbs"] = round(traffic / (kern_ms * 1e-3) / 1e9, 1)
            rec["roofline"]["traffic_over_algorithmic"] = round(traffic / w.bytes_per_launch, 3)
        if probe and parity and is_timed:
            # what the direct kernel (one query per lane, random bitmap reads) would be
            # bound by: the measured random-read rate over the same 2.56 GB arena, at the
            # reference's early-exit read count; the binned pipeline replaces those reads
            rr = hbm_random_read_gps(w.bitmaps)
            rec["roofline"]["random_reads"] = {
                "reads_per_query_direct_kernel": parity["bitmap_reads_per_query"],
                "measured_random_read_greads_per_s": rr,
                "direct_kernel_ceiling_mqueries_per_s": round(rr * 1e3 / parity["bitmap_reads_per_query"], 1)
                if rr else None,
                "working_set_bytes": int(w.bitmaps.numel()),
            }
        if probe and w.bucketing_ms is not None:
            rec["probe_bucketing_ms"] = round(w.bucketing_ms, 2)
        if not probe:
            rec["roofline"]["alu"] = alu_roofline(kind, w.n, kernels)
            rec["roofline"]["lds"] = lds_roofline(kind, kernels)
            pos = w.builder.positions()
            rec["roofline"]["positions_per_build"] = {
                "positions": pos, "per_key": round(pos / w.n, 3),
                "round_trip_bytes": 8 * pos,  # 4 B written by pass A, read by pass B
                "note": "k bit-sets per key, less the keys whose hash pair their workgroup had already counted"}
        if routing_variant:
            rec["roofline"]["routing_variant"] = routing_variant
        if world == 1 and kind == "single" and not args.no_e2e and not sub:
            rec["e2e"] = e2e(w.n)
        if world == 1 and kind == "compaction" and not args.no_e2e and not sub:
            rec["e2e"] = e2e_compaction(w)
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(min(args.cpu_seconds, 5.0) if sub else args.cpu_seconds, kind, w)
        else:
            rec["cpu_baseline"] = None
    del w
    torch.cuda.empty_cache()
    return rec


def with_reader(args, rank, world, timed):
    """The headline build in a process that serves Gets.

    reader_idle: a FilterCache with one table has served a single-key Get
    (the resident probe server launched), and after the server's 2 ms idle
    limit the same K builds are timed as the headline: no kernel resident, the
    static work order.

    gets_beside_builds (one GPU): bin/readpath_test --coexist, the C++
    harness (no interpreter lock between the threads): one thread issues
    single-key Gets through the server back to back while another builds the
    headline filter and configs[3] on its own stream; build times idle and
    with Gets, Get latencies idle and during builds, every answer and both
    SHA-256s compared (the reference's DB::Get beside DoCompaction,
    src/db.cpp:164-172, 263).  (A Python thread issuing the Gets measured the
    interpreter: the building thread's launches starved.)"""
    import subprocess

    import torch

    import adlbloom as ab

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    keys = O.splitmix_keys16(0x7AB1E, 20_000)
    blk = O.filter_block_final([O.keys2block(keys, bits_per_key=BPK).tobytes()], BPK)
    cache = ab.FilterCache(8 << 20, max_tables=4)
    cache.put(b"reader-table", blk)
    w = Workload("single", rank, args.keys, world)
    for _ in range(args.warmup):
        w.step()
    torch.cuda.synchronize()
    launches0 = ab.probe_server_launches()
    got, _ = cache.probe([b"reader-table"], np.zeros(1, np.uint32), keys[:1])
    assert got[0] == 1
    time.sleep(0.02)  # past the server's idle limit: its kernel leaves
    el_idle = timed(w.step, args.steps)
    launches = ab.probe_server_launches() - launches0
    cache.close()
    parity = parity_check(w.builder.bitmap[:w.builder.nbytes], w.n, w.keys) if rank == 0 else None
    del w
    torch.cuda.empty_cache()
    rec = {"reader_idle": {"ms_per_step": round(el_idle / max(args.steps, 1) * 1e3, 4),
                           "note": "the same builds in a process whose FilterCache has served a Get, after the "
                                   "server's idle exit"},
           "server_launches": int(launches), "parity": parity}
    exe = os.path.join(ROOT, "adlsm-tree_amd", "bin", "readpath_test")
    if world == 1 and os.path.exists(exe):
        r = subprocess.run([exe, "--coexist", "10"], capture_output=True, text=True, timeout=300)
        if r.returncode == 0:
            c = json.loads(r.stdout.strip().splitlines()[-1])
            b = c["build_ms"]
            rec["gets_beside_builds"] = {
                "harness": "bin/readpath_test --coexist 10 (C++: one thread Gets, one builds)",
                "headline_ms": {"idle": b["headline_idle"], "with_gets": b["headline_with_gets"],
                                "vs_idle": round(b["headline_with_gets"] / b["headline_idle"] - 1.0, 4)},
                "compaction_ms": {"idle": b["compaction_idle"], "with_gets": b["compaction_with_gets"],
                                  "vs_idle": round(b["compaction_with_gets"] / b["compaction_idle"] - 1.0, 4)},
                "get_us_idle": {k: c["get_us_idle"][k] for k in ("calls", "p50", "p99", "max")},
                "get_us_during_builds": {k: c["get_us_during_builds"][k] for k in ("calls", "p50", "p99", "max")},
                "get_mismatches": c["get_mismatches"],
                "shas_equal_idle_and_concurrent": c["headline_sha256"][0] == c["headline_sha256"][1]
                and c["compaction_sha_of_shas"][0] == c["compaction_sha_of_shas"][1]}
        else:
            rec["gets_beside_builds"] = {"error": f"readpath_test rc {r.returncode}: {r.stderr[-300:]}"}
    return rec


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    # (several ranks share a GPU only in the one-GPU test of the N > 1 line)
    torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
    backend = None
    if world > 1:
        # RCCL (backend "nccl") on a node; ADL_BENCH_BACKEND=gloo lets a test run
        # the N > 1 line as several ranks on one GPU (RCCL refuses that)
        be = os.environ.get("ADL_BENCH_BACKEND", "nccl")
        if be == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(be)
        world = dist.get_world_size()
        backend = dist.get_backend()

    from adlbloom import dist as D

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def timed(fn, steps, warmup=2):
        """max over ranks of the wall time of `steps` calls, barriers on both sides"""
        for _ in range(warmup):
            fn()
        barrier()
        t = time.perf_counter()
        for _ in range(steps):
            fn()
        barrier()
        return D.reduce_throughput(0.0, time.perf_counter() - t, device="cuda")[1]

    out_json = measure(args.workload, args, rank, world, backend, barrier, timed)

    if args.workload == "single":
        # configs[3] beside the headline: the north star's multi-GPU target (256
        # tables split over the N GPUs, strong scaling), its own clock
        if not args.no_compaction_strong:
            wc = Workload("compaction", rank, 0, world)
            el = timed(wc.step, args.steps)
            tot = D.reduce_throughput(float(wc.n) * args.steps, 0.0, device="cuda")[0]
            comp_strong = {"metric": "Mkeys/s bloom-filter build (device-resident), 16B keys, bits/key=10, "
                                     "configs[3]: 256 SSTables x 1M keys split over the GPUs",
                           "value": round(tot / el / 1e6, 1), "unit": "Mkeys/s",
                           "ms_per_step": round(el / max(args.steps, 1) * 1e3, 4), "steps": args.steps,
                           "scaling": "strong", "tables_total": COMPACTION_TABLES, "tables_per_gpu": len(wc.tables),
                           "parity": build_parity(wc, rank)}
            if rank == 0 and not args.no_cpu_baseline:
                # every N: the reference's filter builds on this host's cores for the same tables
                comp_strong["cpu_baseline"] = cpu_baseline(min(args.cpu_seconds, 5.0), "compaction", wc)
            del wc
            torch.cuda.empty_cache()
            if rank == 0:
                out_json["compaction_strong"] = comp_strong
        if not args.no_reader:
            wr = with_reader(args, rank, world, timed)
            if rank == 0:
                head = out_json["ms_per_step"]
                k = "reader_idle"
                wr[k]["value"] = round(args.keys * world / (wr[k]["ms_per_step"] * 1e-3) / 1e6, 1)
                wr[k]["vs_headline"] = round(wr[k]["ms_per_step"] / head - 1.0, 4)
                out_json["headline_with_reader"] = wr
        # configs[4] and configs[2] on the driver's default run
        for kind in ([] if args.no_sub_records else ["probe", "varlen"]):
            rec = measure(kind, args, rank, world, backend, barrier, timed, sub=True)
            if rank == 0:
                out_json[kind] = rec

    if rank == 0:
        print(json.dumps(out_json), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
