"""Multi-GPU plumbing: one process per GPU, groups sharded by id.

Raft groups are independent (no inter-group messages) and the trace RNG is
keyed by the GLOBAL group id, so a shard is just (group_base, groups) and
results are invariant under the number of shards. The only collective on
the data path is the tick-statistics sum, done by the engine's own RCCL
communicator; torch.distributed is used for the id exchange, barriers and
the max-over-ranks timing.
"""


def shard(groups_total, world, rank):
    """Contiguous balanced range of global group ids owned by `rank`."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    if groups_total < world:   # raft_engine_create rejects an empty shard
        raise ValueError(f"{groups_total} groups cannot be sharded over {world} ranks (need groups_total >= world)")
    lo = groups_total * rank // world
    hi = groups_total * (rank + 1) // world
    return lo, hi - lo


def exchange_comm_id(dist, rank, make_id):
    """Rank 0 creates the RCCL unique id; every rank receives it, with rank
    0's world size: a rank whose process group disagrees fails here, with a
    message, before it reaches raft_comm_init (whose own wait is bounded by
    RAFTSTEP_COMM_TIMEOUT_S)."""
    world = dist.get_world_size()
    box = [(make_id(), world) if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    uid, world0 = box[0]
    if world0 != world or not 0 <= rank < world:
        raise RuntimeError(f"rank {rank}: world size {world}, rank 0 has {world0}")
    return uid


def max_over_ranks(dist, value, device=None):
    """Wall time of the slowest rank (the job's time)."""
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, values, device=None):
    import torch
    t = torch.tensor([int(v) for v in values], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(x) for x in t.tolist()]
