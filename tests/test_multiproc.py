"""world_size-2 gloo tests of the multi-GPU path (CPU only, no GPU needed).

Replicas only: each rank owns disjoint rx queues (sources) and a replica of
the rule table.  The per-rank classifier here is the C oracle standing in for
the device (the same ranks on the GPU, through the product: tests/
test_gpu_multiproc.py); what is tested is the partition bench.py uses
(shard.rank_queues, shard.queue_seed): every queue is classified exactly
once, the union of the ranks' per-queue decision streams equals a single
process classifying every queue, and the timing reduction is a max over
ranks."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from usnetd_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _classify_queues(queues, n):
    import coracle
    from usnetd_amd import traffic
    out = {}
    o = coracle.Oracle()
    base = traffic.config("c2", n=n, seed=shard.batch_seed(0, 0))
    coracle.install_oracle(o, base)
    first = max(e[0] for e in base.endpoints) + 1
    for q in range(8):
        if q:
            o.add_endpoint(first + q - 1, 0, -1)
    for q in queues:
        src = 0 if q == 0 else first + q - 1
        cfg = traffic.config("c2", n=n, seed=shard.queue_seed(q, 0))   # as bench.py's Run
        d = o.forward_batch(src, cfg.frames, cfg.lens, stride=cfg.stride)
        out[q] = d.tolist()
    return out


def _worker(rank, world, port, n, ret):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = shard.rank_queues(8, world, rank)
    res = _classify_queues(mine, n)
    elapsed = shard.max_over_ranks(1.0 + rank, dist)
    allres = shard.gather_objects(res, dist)
    if rank == 0:
        merged = {}
        for r in allres:
            assert not set(r) & set(merged), "a queue was classified twice"
            merged.update(r)
        ret["merged"] = merged
        ret["elapsed"] = elapsed
    dist.barrier()
    dist.destroy_process_group()


def test_rank_queues_partition():
    for world in (1, 2, 3, 4, 8):
        got = [q for r in range(world) for q in shard.rank_queues(8, world, r)]
        assert got == list(range(8))
    with pytest.raises(ValueError):
        shard.rank_queues(2, 4, 0)
    assert shard.batch_seed(0, 3) != shard.batch_seed(1, 3)


def test_two_rank_replicas_match_single_process():
    import coracle
    coracle.build()
    n = 3000
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), n, ret), nprocs=2, join=True)
    single = _classify_queues(list(range(8)), n)
    merged = dict(ret["merged"])
    assert sorted(merged) == list(range(8))
    for q in range(8):
        assert np.array_equal(np.array(merged[q]) & 0xFFFFFF, np.array(single[q]) & 0xFFFFFF), q
    assert ret["elapsed"] == 2.0      # max over ranks (rank 1 reported 2.0)


def test_rank_device_mapping():
    """bench.py's rank -> HIP device map (shard.rank_device): one GPU per rank
    on an 8-GPU node, round-robin when ranks outnumber the visible GPUs."""
    assert [shard.rank_device(r, 8) for r in range(8)] == list(range(8))
    assert [shard.rank_device(r, 1) for r in range(8)] == [0] * 8
    assert [shard.rank_device(r, 4) for r in range(8)] == [0, 1, 2, 3, 0, 1, 2, 3]
    assert [shard.rank_device(r, 0) for r in range(3)] == [0, 1, 2]
    with pytest.raises(ValueError):
        shard.rank_device(-1, 8)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_strong_partition_covers_every_frame(world):
    """--strong: the 64M-frame job of c5 (8M-frame queues) split into disjoint
    per-rank queue sets that together cover every queue, hence every frame
    exactly once; weak scaling gives every rank its own queues_per_rank."""
    import bench
    n = bench.DEFAULT_FRAMES["c5"]
    owned, totals = [], set()
    for r in range(world):
        mine, total = shard.step_queues(n, world, r, True, 2, bench.STRONG_FRAMES)
        assert mine, "every rank drains at least one queue"
        owned += mine
        totals.add(total)
    assert totals == {max(world, bench.STRONG_FRAMES // n)}
    assert sorted(owned) == list(range(totals.pop()))
    assert max(world, 8) * n >= bench.STRONG_FRAMES and len(owned) * n == max(world, 8) * n
    weak = [shard.step_queues(n, world, r, False, 2)[0] for r in range(world)]
    assert sorted(q for m in weak for q in m) == list(range(2 * world))
    assert all(len(m) == 2 for m in weak)
