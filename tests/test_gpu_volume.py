"""Differential volume and full-size parity (>= 10^7 random
frames per config against the oracle; VERDICT r01: c5 at its 8M-frame bench
batch).

Each config streams rotating batches of fresh random traffic (one seed per
batch, the config's fixed rule table) from several rx queues through the C
ABI, back to back with the device-carried 1-entry cache, and compares every
decision (bits [23:0]) and the per-endpoint lists with the
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
    """The device-wide per-endpoint lists (usn_result.index / bin_off) equal
    the stable sort of the batch's frames by endpoint bin (endpoints, NIC,
    FLOOD, DROP) -- vectorised for 8M frames."""
    from usnetd_amd import lib
    n = d.shape[0]
    bins = lib.dec_bin(d, n_ep)
    want = np.argsort(bins, kind="stable").astype(np.uint32)
    off = r.bin_off()
    assert off.size == n_ep + 4 and off[0] == 0 and off[-1] == n
    assert np.array_equal(np.diff(off.astype(np.int64)), np.bincount(bins, minlength=n_ep + 3))
    assert np.array_equal(r.index(n), want), "index differs from the stable bin sort"


VOLUME = {          # config: (frames per batch, batches, rx queues)
    "c1": (1 << 20, 10, 2),
    "c2": (1 << 20, 10, 2),
    "c3": (1 << 18, 40, 2),     # IMIX in 2048 B slots: 512 MiB per batch, 10.5M frames
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
        check_order_vec(r, want, n_ep)      # the lists equal the oracle's ordered lists
        old = keep.get(src)
        keep[src] = (b, r)        # the source's device chain points at r
        if old:
            old[0].free()
            old[1].free()
        total += n
    assert total >= 10 ** 7
    ctx.close()


def test_c5_full_bench_batch(coracle_mod):
    """c5 at its bench batch: 8M frames (8192 tiles, 1005 bins, the 512-thread
    build for the L2-resident 65536-rule table): decisions and the
    device-wide per-endpoint lists against the oracle."""
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
    # every endpoint's list, the NIC, FLOOD and DROP lists: the oracle's, in frame order
    check_order_vec(r, want, max(e[0] for e in cfg.endpoints) + 1)
    assert ctx.scatter_fallbacks() == 0      # every chunk's optimistic ranks were stable
    ctx.close()
