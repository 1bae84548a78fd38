"""Multi-GPU partitioning of the match path: replicas only.

A frame's decision depends on the frame, the rule table and its own source's
carried 1-entry cache (/root/reference/src/endpoint.rs:186-191).  Distinct rx
queues are distinct sources, so the GPUs of a node share nothing but a
replica of the rule table: rank r owns a disjoint set of rx queues and
classifies only their rings.  There is no collective on the data path; the
process group carries the bench's barrier and max-over-ranks timing only.
"""
from __future__ import annotations


def rank_queues(total_queues: int, world: int, rank: int) -> list[int]:
    """Rx queue ids owned by `rank` (contiguous block; every queue has exactly one owner)."""
    if not (0 <= rank < world) or total_queues < world:
        raise ValueError("need at least one queue per rank")
    per, extra = divmod(total_queues, world)
    start = rank * per + min(rank, extra)
    return list(range(start, start + per + (1 if rank < extra else 0)))


def step_queues(frames_per_queue: int, world: int, rank: int, strong: bool = False,
                queues_per_rank: int = 1, strong_frames: int = 1 << 26) -> tuple[list[int], int]:
    """The rx queues `rank` drains in every poll round, and the job's queue count.

    Weak scaling: every rank owns `queues_per_rank` queues (the job grows with
    the world).  Strong scaling: the job is `strong_frames` frames per round in
    queues of `frames_per_queue`, split over the ranks (at least one each)."""
    if strong:
        total = max(world, strong_frames // frames_per_queue)
    else:
        total = queues_per_rank * world
    return rank_queues(total, world, rank), total


def rank_device(local_rank: int, ndev: int) -> int:
    """HIP device of a rank: its local rank on a node with one GPU per rank;
    round-robin when there are more ranks than visible GPUs (a rehearsal on
    one GPU); the local rank itself when no GPU count is known (ndev 0)."""
    if local_rank < 0:
        raise ValueError("local rank must be >= 0")
    return local_rank % ndev if ndev > 0 else local_rank


def queue_seed(queue: int, rnd: int) -> int:
    """Seed of the synthetic traffic of global rx queue `queue` in rotation
    round `rnd` (distinct across queues, hence across ranks; the rule table of
    a config does not depend on it)."""
    return 7919 * queue + 17 * rnd + 2


def batch_seed(rank: int, k: int) -> int:
    """Seed of the k-th synthetic batch generated on `rank` (distinct across ranks)."""
    return 1000 * rank + 17 * k + 2


def max_over_ranks(value: float, dist=None) -> float:
    """The bench's wall time is the slowest rank's (torch.distributed, any backend)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_objects(obj, dist=None):
    """All ranks' `obj` on every rank, in rank order (result collection, tests)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out
