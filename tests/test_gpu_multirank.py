"""GPU, world size 2: bench.py's real sharded workloads with GPU builds, two
processes on cuda:0 over gloo (RCCL refuses two ranks on one GPU; the 8-GPU
RCCL run is the driver's).  SURVEY.md §8e:

* compaction -- the 256 tables of configs[3] split 128 / 128 by
  adlbloom.dist.table_shard, each rank one segmented build of its share;
  every table of both ranks against the oracle's SHA-256
  (tests/golden/full_size.json);
* probe -- configs[4]'s 100M queries, both forms of bench.py's N > 1 probe:
  owner-bucketed (the measured path: the batch bucketed by owner before
  upload, each rank probing only its own tables' queries, the answers put back
  in batch order by adlbloom.dist.scatter_answers) and routed (rank r asking
  [r*50M, (r+1)*50M), sent to the rank owning each query's filter and back by
  adlbloom.dist.route_probe, two all-to-alls); the 100M answers of each, in
  query order, against the oracle's SHA-256.
"""
import json
import os
import socket

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import hashlib
    import sys

    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import bench

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        res = {}
        w = bench.Workload("compaction", rank, 0, world, 0)
        w.step()
        torch.cuda.synchronize()
        res["tables"] = list(w.tables)
        res["sha"] = [hashlib.sha256(w.builder.bitmap(i).cpu().numpy().tobytes()).hexdigest()
                      for i in range(len(w.tables))]
        del w
        torch.cuda.empty_cache()
        from adlbloom import dist as D

        p = bench.Workload("probe", rank, 0, world, 100_000_000)
        out = p.step()
        out = p.step()  # twice: nothing leaks between steps
        torch.cuda.synchronize()
        res["served"] = p.served
        allout = D.scatter_answers(out, p.gidx, 100_000_000)
        if rank == 0:
            res["probe_sha"] = hashlib.sha256(allout.cpu().numpy().tobytes()).hexdigest()
        del allout
        out = p.step_routed()
        out = p.step_routed()  # routing state does not leak between steps
        torch.cuda.synchronize()
        allout = bench.gather_all(out, world)
        if rank == 0:
            res["routed_sha"] = hashlib.sha256(allout.cpu().numpy().tobytes()).hexdigest()
        q.put((rank, res))
    except Exception as e:  # report, do not hang the other rank's test
        q.put((rank, {"error": repr(e)}))
        raise
    finally:
        dist.destroy_process_group()


def test_two_ranks_one_gpu_compaction_and_probe_routing():
    import torch.multiprocessing as mp

    with open(os.path.join(ROOT, "tests", "golden", "full_size.json")) as f:
        pins = json.load(f)
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=280) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in out[r], out[r]
    assert [p.exitcode for p in procs] == [0, 0]
    want = pins["compaction"]["bitmap_sha256"]
    assert out[0]["tables"] + out[1]["tables"] == list(range(256))
    for r in range(world):
        for t, sha in zip(out[r]["tables"], out[r]["sha"]):
            assert sha == want[t], (r, t)
    assert out[0]["served"] + out[1]["served"] == 100_000_000
    assert out[0]["probe_sha"] == pins["probe"]["results_sha256"]
    assert out[0]["routed_sha"] == pins["probe"]["results_sha256"]


def _rccl_worker(port, q):
    """One rank on cuda:0 over backend "nccl" (RCCL on ROCm): the device-tensor
    collectives bench.py and adlbloom.dist use at N > 1 -- the throughput
    counters' SUM / MAX all-reduce, route_probe's three all-to-alls and
    scatter_answers' SUM all-reduce of a uint8 vector -- run for real through
    RCCL (world size 1: a single GPU box; the N > 1 run is the driver's)."""
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "adlsm-tree_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import torch
    import torch.distributed as dist

    import adlbloom as ab
    import oracle as O
    from adlbloom import dist as D

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    try:
        res = {"backend": dist.get_backend()}
        k = torch.tensor([3.0], dtype=torch.float64, device="cuda")
        e = torch.tensor([0.25], dtype=torch.float64, device="cuda")
        dist.all_reduce(k, op=dist.ReduceOp.SUM)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        res["reduce"] = [k.item(), e.item()]
        T, per, n = 8, 20_000, 300_000
        bms = [O.keys2block(O.splitmix_keys16(0x5EED + t, per)) for t in range(T)]
        off = np.concatenate([[0], np.cumsum([b.size for b in bms])]).astype(np.uint64)
        arena = np.concatenate(bms + [np.zeros(16, np.uint8)])
        keys, fid, _ = O.synth_probe_queries(n, num_tables=T, keys_per_table=per)
        want = O.probe_multi(keys, fid, arena, off)
        d_arena = torch.from_numpy(arena).cuda()
        d_off = torch.from_numpy(off.view(np.int64)).cuda()
        own, lid = D.owner_table(T, 1)
        own_t, lid_t = torch.from_numpy(own).cuda(), torch.from_numpy(lid).cuda()
        probe_fn = lambda kk, ff: ab.probe_multi(kk, ff, d_arena, d_off)
        stats = {}
        got, served = D.route_probe(torch.from_numpy(keys).cuda(), torch.from_numpy(fid.view(np.int32)).cuda(),
                                    own_t, lid_t, probe_fn, stats=stats)
        res["routed_equal"] = bool(np.array_equal(got.cpu().numpy(), want))
        res["served"] = served
        idx = torch.arange(n, device="cuda")
        full = D.scatter_answers(got, idx, n)
        res["scatter_equal"] = bool(np.array_equal(full.cpu().numpy(), want))
        q.put(res)
    except Exception as ex:
        q.put({"error": repr(ex)})
        raise
    finally:
        dist.destroy_process_group()


def test_rccl_world1_collectives():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=200)
    p.join(timeout=60)
    assert "error" not in res, res
    assert p.exitcode == 0
    assert res["backend"] == "nccl"
    assert res["reduce"] == [3.0, 0.25]
    assert res["routed_equal"] and res["scatter_equal"]
    assert res["served"] == 300_000


def test_bench_line_two_ranks_one_gpu(tmp_path):
    """bench.py's whole N > 1 default line -- the headline, compaction_strong,
    headline_with_reader and the probe / varlen sub-records -- as two ranks on
    cuda:0 over gloo (torch.distributed.run, 127.0.0.1): it runs to the end
    and rank 0's JSON line carries every record with its parity, so the
    driver's 8-GPU run of the same code has been exercised end to end."""
    import subprocess
    import sys

    port = _free_port()
    env = dict(os.environ, ADL_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--no-cpu-baseline", "--no-e2e"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["world"]["size"] == 2
    assert d["parity"] == "bit-identical to reference (sha256)"
    assert "MISMATCH" not in json.dumps(d)
    assert d["compaction_strong"]["tables_per_gpu"] == 128
    assert d["probe"]["parity"]["oracle"].startswith("all 100M answers bit-identical")
    assert d["varlen"]["parity"] == "bit-identical to the oracle (sha256)"
    assert d["headline_with_reader"]["parity"] == "bit-identical to reference (sha256)"
