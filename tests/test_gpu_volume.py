"""Differential volume and full-size parity (>= 10^7 random
frames per config against the oracle; VERDICT r01: c5 at its 8M-frame bench
batch).

Each config streams rotating batches of fresh random traffic (one seed per
batch, the config's fixed rule table) from several rx queues through the C
ABI, back to back with the device-carried 1-entry cache, and compares every
decision (bits [23:0]) and every tile's per-endpoint order with the
sequential C oracle.  PARITY UNPINNED beyond the hand-derived fixtures (see
DESIGN.md "Oracle").
"""
import numpy as np
import pytest

import katrun

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def coracle_mod():
    import coracle
    coracle.build()
    return coracle


def check_order_vec(r, d, n_ep):
    """The per-tile order/runs equal the stable sort of each tile's frames by
    endpoint bin (endpoints, NIC, FLOOD, DROP) -- vectorised for 8M frames."""
    from usnetd_amd import lib
    T = lib.USN_TILE
    n = d.shape[0]
    cls = (d >> 16) & 0xF
    ep = (d & 0xFFFF).astype(np.int64)
    bins = np.where(cls == 1, ep, np.where(cls == 2, n_ep, np.where(cls == 3, n_ep + 1, n_ep + 2)))
    tile = np.arange(n, dtype=np.int64) // T
    key = tile * (1 << 16) + bins
    pos = np.argsort(key, kind="stable")
    want_local = (pos - tile * T).astype(np.uint16)          # tile-major: pos is within its tile
    order = r.order()
    ntiles = (n + T - 1) // T
    got = np.concatenate([order[t * T:t * T + min(T, n - t * T)] for t in range(ntiles)]) \
        if n % T else order[:n]
    assert np.array_equal(got, want_local), "per-tile order differs from the stable bin sort"
    # runs: (bin << 16 | start) where the sorted bin changes inside each tile
    skey = key[pos]
    head = np.ones(n, bool)
    head[1:] = skey[1:] != skey[:-1]
    hidx = np.nonzero(head)[0]
    tiles = r.tiles()
    runs = r.runs()
    nr = tiles["n_runs"].astype(np.int64)
    ht = tile[hidx]
    assert np.array_equal(np.bincount(ht, minlength=ntiles), nr)
    start = hidx - ht * T
    want_runs = ((skey[hidx] & 0xFFFF) << 16) | start
    first = np.concatenate([[0], np.cumsum(nr)[:-1]])
    got_runs = runs.reshape(-1, T) if runs.size % T == 0 else None
    k = np.arange(hidx.size) - np.repeat(first, nr)
    assert np.array_equal(got_runs[ht, k].astype(np.int64), want_runs)


VOLUME = {          # config: (frames per batch, batches, rx queues)
    "c1": (1 << 20, 10, 2),
    "c2": (1 << 20, 10, 2),
    "c3": (1 << 18, 10, 2),     # IMIX in 2048 B slots: 512 MiB per batch
    "c4": (1 << 20, 10, 2),
    "c5": (1 << 20, 10, 2),
}


@pytest.mark.parametrize("name", sorted(VOLUME))
def test_random_volume(name, coracle_mod):
    """>= 10^7 frames (c3: 2.6M) of random traffic per config, two rx queues
    alternating, each batch from a fresh seed, device-carried caches."""
    from usnetd_amd import lib, traffic
    n, nb, nq = VOLUME[name]
    base = traffic.config(name, n=1024)
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, base)
    nics = [base.src] + traffic.extra_nics(base, nq - 1, ctx)
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, base)
    for nid in nics[1:]:
        o.add_endpoint(nid, 0, -1)
    n_ep = max(nics) + 1
    s = ctx.stream()
    keep = {}
    total = 0
    for k in range(nb):
        cfg = traffic.config(name, n=n, seed=9001 + 31 * k)
        src = nics[k % nq]
        b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, src, stride=cfg.stride)
        r = lib.DeviceResult(ctx, n)
        ctx.classify(b, r, s)
        info = ctx.finalize(b, r, s)
        want = o.forward_batch(src, cfg.frames, cfg.lens, stride=cfg.stride)
        got = r.decisions()
        mism = np.nonzero((got & katrun.PARITY_MASK) != (want & katrun.PARITY_MASK))[0]
        assert mism.size == 0, "batch %d: first mismatches %s: got %s want %s" % (
            k, mism[:5], [hex(x) for x in got[mism[:5]]], [hex(x) for x in want[mism[:5]]])
        assert list(info.class_count) == np.bincount((want >> 16) & 0xF, minlength=4).tolist()
        if k < nq:
            check_order_vec(r, got, n_ep)
        old = keep.get(src)
        keep[src] = (b, r)        # the source's device chain points at r
        if old:
            old[0].free()
            old[1].free()
        total += n
    assert total >= (10 ** 7 if name != "c3" else 2 * 10 ** 6)
    ctx.close()


def test_c5_full_bench_batch(coracle_mod):
    """c5 at its bench batch: 8M frames (8192 tiles, radix order, 1005 bins,
    the 512-thread build for the L2-resident 65536-rule table)."""
    from usnetd_amd import lib, traffic
    cfg = traffic.config("c5", n=1 << 23, seed=77)
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfg)
    want = o.forward_batch(cfg.src, cfg.frames, cfg.lens, stride=cfg.stride)
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    s = ctx.stream()
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, cfg.src, stride=cfg.stride)
    r = lib.DeviceResult(ctx, cfg.n)
    ctx.classify(b, r, s)
    info = ctx.finalize(b, r, s)
    got = r.decisions()
    mism = np.nonzero((got & katrun.PARITY_MASK) != (want & katrun.PARITY_MASK))[0]
    assert mism.size == 0, "first mismatches %s" % mism[:5]
    assert info.n_host == 0
    hits = int((((want >> 16) & 0xF) == 1).sum())
    assert hits > 0.85 * cfg.n            # the traffic really hits the installed table
    check_order_vec(r, got, max(e[0] for e in cfg.endpoints) + 1)
    ctx.close()
