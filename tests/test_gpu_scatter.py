"""The device-wide per-endpoint scatter's two ranking paths (SURVEY §2
scatter_by_endpoint; the reference writes each frame straight into its
target's ring, /root/reference/src/endpoint.rs:61-74, and floods at
:340-363).

The scatter kernel ranks a chunk's frames with one LDS atomic add per frame
(optimistic: the LDS serves same-word lanes of one instruction in lane
order) and verifies that every bin's run of the chunk is in frame order;
an unsorted chunk is ranked again by bit-sliced ballots.  These tests check
that the optimistic path is the one taken (no chunk fell back) and that the
ballot path, forced on every chunk (USN_SCATTER_SLOW_RANK=1, read once per
process: a subprocess), gives the same lists -- both against the sequential
oracle's decisions sorted stably by bin.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np
sys.path[:0] = [%(root)r, %(root)r + '/oracle', %(root)r + '/tests']
import coracle, katrun
from usnetd_amd import lib, traffic
coracle.build()
for name, n in (("c5", 1 << 20), ("c2", 1 << 20), ("c4", 300000)):
    cfg = traffic.config(name, n=n, seed=4242)
    o = coracle.Oracle()
    coracle.install_oracle(o, cfg)
    want = o.forward_batch(cfg.src, cfg.frames, cfg.lens, stride=cfg.stride)
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    s = ctx.stream()
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, cfg.src, stride=cfg.stride)
    r = lib.DeviceResult(ctx, n)
    before = ctx.scatter_fallbacks()
    ctx.classify(b, r, s)
    ctx.finalize(b, r, s)
    got = r.decisions()
    assert np.array_equal(got & katrun.PARITY_MASK, want & katrun.PARITY_MASK), name
    n_ep = max(e[0] for e in cfg.endpoints) + 1
    bins = lib.dec_bin(want, n_ep)
    assert np.array_equal(r.index(n), np.argsort(bins, kind="stable").astype(np.uint32)), name
    print(name, "fallback chunks", ctx.scatter_fallbacks() - before, flush=True)
    b.free(); r.free(); ctx.close()
print("ok")
"""


def _run(env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    p = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT}], env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    return p.stdout


def test_scatter_optimistic_ranks_not_redone():
    """Default path: lists equal the oracle's, and no chunk was ranked again."""
    out = _run({})
    assert out.strip().endswith("ok")
    for line in out.splitlines()[:-1]:
        assert line.endswith("fallback chunks 0"), line


def test_scatter_ballot_ranks_forced():
    """Every chunk also takes the ballot path and rewrites its stage: the
    lists are the same stable sort."""
    out = _run({"USN_SCATTER_SLOW_RANK": "1"})
    assert out.strip().endswith("ok")
    assert all(not l.endswith(" 0") for l in out.splitlines()[:-1]), out
