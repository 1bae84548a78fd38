"""The multi-GPU replicas path on the GPU: two ranks (processes, gloo for the
coordination only), each classifying the rx queues shard.rank_queues gives it
-- the partition bench.py uses -- with its own usn_ctx (a replica of the rule
table) through the C ABI, every decision checked against the oracle.  On the
one-GPU box both ranks share device 0 (bench.py's round-robin rehearsal
placement); on a node each rank takes LOCAL_RANK's GPU."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import json, os, sys
root = sys.argv[1]
sys.path[:0] = [root, os.path.join(root, "oracle"), os.path.join(root, "tests")]
import numpy as np
import torch.distributed as dist
import coracle, katrun
from usnetd_amd import lib, shard, traffic
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo")
nq, n = int(sys.argv[2]), int(sys.argv[3])
mine = shard.rank_queues(nq, world, rank)
ctx = lib.Ctx(0)
base = traffic.config("c5", n=1024)
traffic.install_ctx(ctx, base)
nics = [base.src] + traffic.extra_nics(base, len(mine) - 1, ctx)
o = coracle.Oracle()
coracle.install_oracle(o, base)
for nid in nics[1:]:
    o.add_endpoint(nid, 0, -1)
s = ctx.stream()
res = {}
for j, q in enumerate(mine):
    cfg = traffic.config("c5", n=n, seed=shard.queue_seed(q, 0))
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, nics[j], stride=cfg.stride)
    r = lib.DeviceResult(ctx, n)
    ctx.classify(b, r, s)
    ctx.finalize(b, r, s)
    got = r.decisions()
    want = o.forward_batch(nics[j], cfg.frames, cfg.lens, stride=cfg.stride)
    bad = int(((got ^ want) & katrun.PARITY_MASK).astype(bool).sum())
    res[q] = {"bad": bad, "hits": int((((got >> 16) & 0xF) == 1).sum())}
    b.free(); r.free()
allres = shard.gather_objects(res, dist)
t = shard.max_over_ranks(1.0 + rank, dist)
if rank == 0:
    with open(sys.argv[4], "w") as fh:
        json.dump({"per_rank": allres, "max_t": t}, fh)
ctx.close()
dist.destroy_process_group()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_classify_their_queues(tmp_path):
    from usnetd_amd import shard
    world, nq, n = 2, 6, 40000
    out = tmp_path / "res.json"
    port = _free_port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER, ROOT, str(nq), str(n), str(out)],
                                      env=env))
    rcs = [p.wait(timeout=240) for p in procs]
    assert rcs == [0] * world
    d = json.loads(out.read_text())
    merged = {}
    for r, part in enumerate(d["per_rank"]):
        assert sorted(int(q) for q in part) == shard.rank_queues(nq, world, r)
        for q, v in part.items():
            assert q not in merged, "a queue was classified twice"
            merged[q] = v
    assert sorted(int(q) for q in merged) == list(range(nq))
    assert all(v["bad"] == 0 for v in merged.values()), merged
    assert all(v["hits"] > 0.85 * n for v in merged.values())
    assert d["max_t"] == float(world)


def test_bench_self_launch_two_ranks():
    """`bench.py --gpus 2` with no launcher starts two ranks itself (both on
    the box's one GPU: the round-robin rehearsal placement) and reports
    n_gpus 2 from the ranks that joined, with each rank's device."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--config", "c2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                          "--no-extra", "--launch-probe", "4", "--ramp", "2"],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    line = lines[0]
    assert line["n_gpus"] == 2 and len(line["config"]["rank_devices"]) == 2
    assert line["value"] > 0
