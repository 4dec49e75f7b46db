"""adlbloom.dist -- multi-GPU plumbing for the sharded filter workloads.

The path shards by whole filters (one SSTable's filter never spans GPUs,
reference src/sstable.cpp:21 builds one filter per table), so the build has
no collective on its data path: one process per GPU, and torch.distributed
(backend "nccl" = RCCL on ROCm, "gloo" in the CPU tests) only combines the
throughput counters.  The probe does have a real exchange step: a query must
reach the GPU that holds its table's filter, and its answer must come back to
the rank that asked (bucket queries by owner, stable, and
scatter the results back).

Two forms of that step:
  * owner-bucketed (bench.py's measured path at N > 1): the host buckets the
    batch by owner once, before upload (owner_select), so each rank is handed
    exactly its own tables' queries and probes them with no collective at all;
    the answers are put back in the batch's order afterwards (scatter_answers,
    outside the timed loop).  This is the LSM's natural case: a lookup is
    issued where its level's tables live.
  * routed (route_probe): every rank holds an arbitrary slice of the batch and
    two all-to-alls per step move queries to their owners and answers back;
    bench.py reports it as roofline.routing_variant.
"""
from __future__ import annotations

import numpy as np


def table_shard(num_tables: int, world: int, rank: int) -> range:
    """Contiguous block of table ids owned by `rank` (256 tables over 8 GPUs ->
    32 each: table t lives on GPU t // 32).  Remainders go to the low ranks."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(num_tables, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def owner_of(table_id: np.ndarray, num_tables: int, world: int) -> np.ndarray:
    """Owning rank of each table id (inverse of table_shard)."""
    table_id = np.asarray(table_id, dtype=np.int64)
    base, extra = divmod(num_tables, world)
    cut = extra * (base + 1)
    return np.where(table_id < cut, table_id // max(base + 1, 1),
                    extra + (table_id - cut) // max(base, 1))


def partition_queries(filter_id: np.ndarray, num_tables: int, world: int):
    """Stable partition of a probe batch by owning rank.

    Returns (order, counts): queries order[sum(counts[:r]) : sum(counts[:r+1])]
    go to rank r, in their original relative order, so results scatter back
    with out[order] = concatenated per-rank results."""
    own = owner_of(filter_id, num_tables, world)
    order = np.argsort(own, kind="stable")
    counts = np.bincount(own, minlength=world)
    return order, counts


def reduce_throughput(keys_local: float, elapsed_local: float, device=None):
    """All-reduce (sum of keys processed, max of elapsed seconds) over the
    default process group -- the only collective (16 bytes)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(keys_local), float(elapsed_local)
    k = torch.tensor([float(keys_local)], dtype=torch.float64, device=device)
    e = torch.tensor([float(elapsed_local)], dtype=torch.float64, device=device)
    dist.all_reduce(k, op=dist.ReduceOp.SUM)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    return k.item(), e.item()


def owner_table(num_tables: int, world: int):
    """(owner rank, index within the owner's shard) of every table id, as numpy arrays."""
    t = np.arange(num_tables)
    own = owner_of(t, num_tables, world)
    first = np.array([table_shard(num_tables, world, r).start for r in range(world)])
    return own, t - first[own]


# bytes a routed query moves each way (route_probe): key + local filter id out,
# the answer back
ROUTE_BYTES_OUT, ROUTE_BYTES_BACK = 16 + 4, 1


def route_probe(keys, fid, owner, local_id, probe_fn, group=None, comm_cpu=None, stats=None):
    """Multi-get across ranks: this rank's queries (keys (n, 16) uint8, fid (n,)
    global table ids) are bucketed by the rank owning each table (stable, as
    partition_queries), sent there (all_to_all), probed against the owner's
    local filters by probe_fn(keys, local_fid) -> uint8 answers, and the
    answers sent back (all_to_all) and scattered into the original order.
    owner / local_id: per-table tensors on keys' device (owner_table).
    comm_cpu: stage the exchanges through host memory (default: when the
    backend is gloo, which moves host tensors; RCCL moves device memory).
    stats: an optional dict that receives this rank's off-rank traffic of the
    call (queries sent to other ranks, bytes out and back).
    Returns (answers uint8 (n,), queries this rank probed for others)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    dev = keys.device
    if comm_cpu is None:
        comm_cpu = dist.get_backend(group) == "gloo" and dev.type != "cpu"
    fid = fid.long()
    own = owner[fid]
    order = torch.sort(own, stable=True).indices
    counts = torch.bincount(own, minlength=world)
    xfer = (lambda t: t.cpu()) if comm_cpu else (lambda t: t)
    back = (lambda t: t.to(dev)) if comm_cpu else (lambda t: t)
    rcounts = xfer(torch.empty_like(counts))
    dist.all_to_all_single(rcounts, xfer(counts), group=group)
    send = counts.tolist()
    recv = rcounts.tolist()
    if stats is not None:
        me = dist.get_rank(group)
        off = sum(c for r, c in enumerate(send) if r != me)
        stats.update(queries_sent_offrank=off, bytes_out=off * ROUTE_BYTES_OUT,
                     bytes_back_in=off * ROUTE_BYTES_BACK,
                     queries_received=sum(c for r, c in enumerate(recv) if r != me))
    # keys as 2 x int64 per query (16 B), local filter ids as int32
    k_send = keys[order].contiguous().view(torch.int64).view(-1, 2)
    f_send = local_id[fid[order]].to(torch.int32)
    k_recv = torch.empty((sum(recv), 2), dtype=torch.int64, device=xfer(k_send).device)
    f_recv = torch.empty(sum(recv), dtype=torch.int32, device=k_recv.device)
    dist.all_to_all_single(k_recv, xfer(k_send), recv, send, group=group)
    dist.all_to_all_single(f_recv, xfer(f_send), recv, send, group=group)
    ans = probe_fn(back(k_recv).view(torch.uint8).view(-1, 16), back(f_recv))
    a_back = torch.empty(sum(send), dtype=torch.uint8, device=k_recv.device)
    dist.all_to_all_single(a_back, xfer(ans.to(torch.uint8).contiguous()), send, recv, group=group)
    out = torch.empty(keys.shape[0], dtype=torch.uint8, device=dev)
    out[order] = back(a_back)
    return out, int(sum(recv))


def owner_select(fid, owner, local_id, rank: int):
    """Owner-bucketed batch: the positions (ascending, so the batch order is
    kept) of the queries whose table `rank` owns, and their filter ids local
    to that rank.  fid: global table ids (torch tensor); owner / local_id:
    per-table tensors (owner_table) on fid's device."""
    import torch

    f = fid.long()
    idx = torch.nonzero(owner[f] == rank).squeeze(1)
    return idx, local_id[f[idx]].to(torch.int32)


def scatter_answers(ans, idx, total: int, group=None):
    """Inverse of owner_select over all ranks: every rank's answers `ans` (uint8)
    at batch positions `idx` into one (total,) uint8 tensor in batch order, on
    every rank.  Each position is answered by exactly one rank, so a SUM
    all-reduce of the zero-filled per-rank vectors assembles it (host tensors
    for gloo)."""
    import torch
    import torch.distributed as dist

    dev = ans.device
    full = torch.zeros(total, dtype=torch.uint8, device=dev)
    full[idx] = ans.to(torch.uint8)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return full
    if dist.get_backend(group) == "gloo":
        host = full.to("cpu", torch.int32)
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        return host.to(torch.uint8).to(dev)
    dist.all_reduce(full, op=dist.ReduceOp.SUM, group=group)
    return full
