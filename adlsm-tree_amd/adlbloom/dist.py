"""adlbloom.dist -- multi-GPU plumbing for the sharded filter workloads.

The path shards by whole filters (one SSTable's filter never spans GPUs,
reference src/sstable.cpp:21 builds one filter per table), so there is no
collective on the data path.  One process per GPU; torch.distributed
(backend "nccl" = RCCL on ROCm, "gloo" in the CPU tests) is used only to
combine the throughput counters.  SURVEY.md §8e.
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
