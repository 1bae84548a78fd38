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
process, in the test build: a subprocess), gives the same lists -- both against the sequential
oracle's decisions sorted stably by bin.  Small launches sum their count rows
in the scatter itself (self-scan, no scan launch); both ways are checked.
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
    ctx = lib.Ctx(0, libpath=lib.TEST_LIB_PATH)   # reads USN_SCATTER_SLOW_RANK
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


@pytest.mark.parametrize("kb", ["0", "1048576"])
def test_scatter_scan_or_self_scan(kb):
    """The chunk offsets from the scan launch everywhere (USN_SELFSCAN_KB=0),
    or summed by every launch whose chunks are all resident (self-scan even
    at c5's 2 KiB rows and c4's 300K frames): the same lists."""
    out = _run({"USN_SELFSCAN_KB": kb})
    assert out.strip().endswith("ok")


def _tile_plan(bins_of, rng, n_tiles):
    """Frame indices of a batch whose tiles hold bins with 254, 255, 256,
    511, 1020 and 1024 frames, the rest random, each tile shuffled."""
    from collections import defaultdict
    by = defaultdict(list)
    for i, b in enumerate(bins_of):
        by[int(b)].append(i)
    big = sorted(by, key=lambda b: -len(by[b]))[:6]
    allidx = np.arange(bins_of.size)
    plans = [
        {big[0]: 1024},
        {big[0]: 255, big[1]: 256, big[2]: 254},
        {big[0]: 255, big[1]: 255, big[2]: 255, big[3]: 255},
        {big[4]: 1020},
        {big[5]: 511, big[1]: 257},
    ]
    tiles = []
    for t in range(n_tiles):
        want = plans[t % (len(plans) + 2)] if t % (len(plans) + 2) < len(plans) else {}
        sel = []
        for b, k in want.items():
            sel.append(rng.choice(by[b], size=k, replace=True))
        rest = 1024 - sum(want.values())
        if rest:
            sel.append(rng.choice(allidx, size=rest, replace=True))
        tile = np.concatenate(sel)
        rng.shuffle(tile)
        tiles.append(tile)
    return np.concatenate(tiles)


@pytest.mark.parametrize("name", ["c5", "c2"])
def test_count_rows_heavy_bins(name):
    """Tiles whose frames crowd into few bins (a whole tile in one bin; bins
    at 254-256 frames, the edge of a one-byte count row, measured and
    rejected in DESIGN.md 6.1): decisions and the per-endpoint lists equal
    the oracle's.  c5 (1005 bins, a scan over 48 chunks) and c2 (19 bins)."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import coracle
    import katrun
    from usnetd_amd import lib, traffic
    coracle.build()
    base = traffic.config(name, n=1 << 18, seed=77)
    o = coracle.Oracle()
    coracle.install_oracle(o, base)
    d0 = o.forward_batch(base.src, base.frames, base.lens, stride=base.stride)
    n_ep = max(e[0] for e in base.endpoints) + 1
    rng = np.random.default_rng(5)
    idx = _tile_plan(lib.dec_bin(d0, n_ep), rng, 384)
    st = base.stride
    rows = np.asarray(base.frames, np.uint8)[: base.n * st].reshape(base.n, st)
    frames = np.concatenate([rows[idx].reshape(-1), np.zeros(64, np.uint8)])
    lens = np.asarray(base.lens)[idx]
    n = idx.size
    o2 = coracle.Oracle()
    coracle.install_oracle(o2, base)
    want = o2.forward_batch(base.src, frames, lens, stride=st)
    bins = lib.dec_bin(want, n_ep)
    counts = np.bincount((np.arange(n) // 1024) * (n_ep + 3) + bins)
    assert (counts == 255).any() and (counts == 1024).any() and (counts == 256).any()
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, base)
    s = ctx.stream()
    b = lib.DeviceBatch(ctx, frames, lens, base.src, stride=st)
    r = lib.DeviceResult(ctx, n)
    ctx.classify(b, r, s)
    ctx.finalize(b, r, s)
    got = r.decisions()
    assert np.array_equal(got & katrun.PARITY_MASK, want & katrun.PARITY_MASK)
    off = r.bin_off()
    assert np.array_equal(np.diff(off.astype(np.int64)), np.bincount(bins, minlength=n_ep + 3))
    assert np.array_equal(r.index(n), np.argsort(bins, kind="stable").astype(np.uint32))
    b.free(); r.free(); ctx.close()


CORRUPT_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [%(root)r]
from usnetd_amd import lib, traffic
for name, n in (("c5", 1 << 20), ("c2", 1 << 16), ("c4tx", 1 << 16)):
    cfg = traffic.c4tx(n=n, seed=6) if name == "c4tx" else traffic.config(name, n=n, seed=4242)
    ctx = lib.Ctx(0, libpath=lib.TEST_LIB_PATH)   # the test build: USN_DEBUG_CORRUPT
    traffic.install_ctx(ctx, cfg)
    s = ctx.stream()
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, cfg.src, stride=cfg.stride)
    r = lib.DeviceResult(ctx, n)
    ctx.classify(b, r, s)
    try:
        ctx.finalize(b, r, s)
        print(name, "no error", flush=True)
    except lib.UsnError as e:
        print(name, "error", str(e), flush=True)
    b.free(); r.free(); ctx.close()
print("ok")
"""


@pytest.mark.parametrize("mode", ["1", "2"])
def test_scatter_reports_inconsistent_counts(mode):
    """a count row that disagrees with the decisions (test
    hook USN_DEBUG_CORRUPT=1: +257 frames in one bin of the first tile) or a
    decision naming an endpoint past the batch's bins (=2) is reported by
    usn_finalize as USN_ELIST, on the rx path (c5 with the scan, c2) and on
    the tx path (c4tx, the finalize state gathered on the device)."""
    env = dict(os.environ, USN_DEBUG_CORRUPT=mode)
    p = subprocess.run([sys.executable, "-c", CORRUPT_CHILD % {"root": ROOT}], env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    lines = p.stdout.strip().splitlines()
    assert lines[-1] == "ok", p.stdout
    for line in lines[:-1]:
        assert " error " in line and "ELIST" in line, line
    assert len(lines) == 4, lines

