"""CPU, world_size 2 over gloo: the multi-GPU plumbing of bench.py / adlbloom.dist
(whole filters per rank, no data-path collective, one counter all-reduce), and
that sharded builds reassemble to the single-process result."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "adlsm-tree_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch.distributed as dist

    from adlbloom import dist as D
    import oracle as O

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        # each rank builds the filters of its own tables (CPU oracle stands in for the GPU here)
        tables = D.table_shard(8, world, rank)
        n = 2000
        built = {t: O.keys2block(O.splitmix_keys16(0x5EED + t, n)) for t in tables}
        keys_local = n * len(tables)
        total, tmax = D.reduce_throughput(keys_local, 0.5 + rank, device="cpu")
        q.put((rank, list(tables), {t: bm.tobytes() for t, bm in built.items()}, total, tmax))
    finally:
        dist.destroy_process_group()


def test_table_shard_covers_all():
    from adlbloom import dist as D

    for T, W in [(256, 8), (256, 1), (10, 3), (7, 2), (3, 8)]:
        seen = []
        for r in range(W):
            seen.extend(D.table_shard(T, W, r))
        assert seen == list(range(T))
        own = D.owner_of(np.arange(T), T, W)
        for r in range(W):
            assert all(own[t] == r for t in D.table_shard(T, W, r))
    assert list(D.table_shard(256, 8, 3)) == list(range(96, 128))  # t -> GPU t // 32


def test_partition_queries_is_stable_and_invertible():
    from adlbloom import dist as D

    rng = np.random.default_rng(0)
    fid = rng.integers(0, 256, size=5000)
    order, counts = D.partition_queries(fid, 256, 8)
    assert counts.sum() == 5000
    own = D.owner_of(fid[order], 256, 8)
    assert np.all(np.diff(own) >= 0)
    # stability: inside a rank's slice, original indices increase
    start = 0
    for c in counts:
        assert np.all(np.diff(order[start:start + c]) > 0)
        start += c
    # results scatter back
    res = fid[order] * 3
    back = np.empty_like(res)
    back[order] = res
    assert np.array_equal(back, fid * 3)


def test_two_ranks_gloo_sharded_build_and_counter_reduce():
    import torch.multiprocessing as mp

    import oracle as O

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    all_tables = [t for _, tables, _, _, _ in out for t in tables]
    assert all_tables == list(range(8))
    for _, _, built, total, tmax in out:
        assert total == 8 * 2000          # sum over ranks
        assert tmax == pytest.approx(1.5)  # max over ranks
    # sharded results equal the single-process build of every table
    for _, tables, built, _, _ in out:
        for t in tables:
            assert built[t] == O.keys2block(O.splitmix_keys16(0x5EED + t, 2000)).tobytes()


def _probe_worker(rank, world, port, q):
    """route_probe over gloo: rank r originates queries [r*Q/world, (r+1)*Q/world)
    of the configs[4] stream (scaled down) and gets every answer back in order."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "adlsm-tree_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch
    import torch.distributed as dist

    from adlbloom import dist as D
    import oracle as O

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        T, per, Q = 16, 3000, 20000
        tables = D.table_shard(T, world, rank)
        bms = [O.keys2block(O.splitmix_keys16(0x5EED + t, per)) for t in tables]
        arena = np.concatenate(bms)
        off = np.concatenate([[0], np.cumsum([b.size for b in bms])]).astype(np.uint64)
        own, lid = D.owner_table(T, world)
        q0, n = rank * Q // world, Q // world
        k, f, m = O.synth_probe_queries(n, q0=q0, num_tables=T, keys_per_table=per)
        probed = []

        def probe_fn(keys, lfid):
            probed.append(int(keys.shape[0]))
            return torch.from_numpy(O.probe_multi(keys.numpy(), lfid.numpy().astype(np.uint32), arena, off))

        out, served = D.route_probe(torch.from_numpy(k), torch.from_numpy(f.astype(np.int64)),
                                    torch.from_numpy(own), torch.from_numpy(lid), probe_fn)
        q.put((rank, out.numpy().tobytes(), served, q0, n))
    finally:
        dist.destroy_process_group()


def test_two_ranks_gloo_probe_routing_matches_single_process():
    import torch.multiprocessing as mp

    import oracle as O

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_probe_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    T, per, Q = 16, 3000, 20000
    bms = [O.keys2block(O.splitmix_keys16(0x5EED + t, per)) for t in range(T)]
    off = np.concatenate([[0], np.cumsum([b.size for b in bms])]).astype(np.uint64)
    k, f, m = O.synth_probe_queries(Q, num_tables=T, keys_per_table=per)
    want = O.probe_multi(k, f, np.concatenate(bms), off)
    got = np.concatenate([np.frombuffer(o[1], dtype=np.uint8) for o in out])
    assert np.array_equal(got, want)
    assert sum(o[2] for o in out) == Q  # every query probed exactly once, by its table's owner
    assert got[m.astype(bool)].all()


def _owner_worker(rank, world, port, q):
    """Owner-bucketed probe over gloo (bench.py's measured path at N > 1): the
    whole configs[4] batch (scaled down) is bucketed by owner before upload,
    each rank probes only its own tables' queries -- no collective on the data
    path -- and scatter_answers puts every answer back in batch order."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "adlsm-tree_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch
    import torch.distributed as dist

    from adlbloom import dist as D
    import oracle as O

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        T, per, Q = 16, 3000, 20000
        tables = D.table_shard(T, world, rank)
        bms = [O.keys2block(O.splitmix_keys16(0x5EED + t, per)) for t in tables]
        arena = np.concatenate(bms)
        off = np.concatenate([[0], np.cumsum([b.size for b in bms])]).astype(np.uint64)
        own, lid = D.owner_table(T, world)
        k, f, m = O.synth_probe_queries(Q, num_tables=T, keys_per_table=per)
        idx, lf = D.owner_select(torch.from_numpy(f.astype(np.int64)), torch.from_numpy(own),
                                 torch.from_numpy(lid), rank)
        assert np.all(np.diff(idx.numpy()) > 0)  # batch order kept
        assert np.all(own[f[idx.numpy()]] == rank)
        ans = torch.from_numpy(O.probe_multi(k[idx.numpy()], lf.numpy().astype(np.uint32), arena, off))
        full = D.scatter_answers(ans, idx, Q)
        q.put((rank, full.numpy().tobytes(), int(idx.numel())))
    finally:
        dist.destroy_process_group()


def test_two_ranks_gloo_owner_bucketed_probe_matches_single_process():
    import torch.multiprocessing as mp

    import oracle as O

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_owner_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    T, per, Q = 16, 3000, 20000
    bms = [O.keys2block(O.splitmix_keys16(0x5EED + t, per)) for t in range(T)]
    off = np.concatenate([[0], np.cumsum([b.size for b in bms])]).astype(np.uint64)
    k, f, m = O.synth_probe_queries(Q, num_tables=T, keys_per_table=per)
    want = O.probe_multi(k, f, np.concatenate(bms), off)
    for _, full, _ in out:  # every rank holds all answers in batch order
        assert np.array_equal(np.frombuffer(full, dtype=np.uint8), want)
    assert sum(o[2] for o in out) == Q  # each query probed once, by its table's owner
