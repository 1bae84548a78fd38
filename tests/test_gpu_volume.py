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


def test_c5_headline_launch(coracle_mod):
    """The bench's headline call itself: c5's two 8M-frame rx
    rings of two distinct NIC sources, generated as bench.py generates them
    (shard.queue_seed of queues 0 and 1), classified in ONE
    usn_classify_multi call -- 16384 tiles, the scan at 512 workgroups (32
    ranges of 64 chunks x 16 blocks of 64 bins), 2048 scatter chunks of 8
    tiles that span the boundary between the two batches.  Two poll rounds
    (the second from the device-carried caches of the first).  Every decision
    and every per-endpoint list of each ring against the sequential oracle."""
    import ctypes as C
    from usnetd_amd import lib, shard, traffic
    n = 1 << 23
    cfg0 = traffic.config("c5", n=n, seed=shard.queue_seed(0, 0))
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg0)
    nics = [cfg0.src] + traffic.extra_nics(cfg0, 1, ctx)
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfg0)
    o.add_endpoint(nics[1], 0, -1)
    n_ep = max(nics) + 1
    # the launch shape rocprof shows for the bench (profiles/r04/r04as): the
    # list plan of two 8192-tile batches at c5's bins
    L = C.CDLL(lib.LIB_PATH)
    f = L.usn_debug_scatter_plan
    f.argtypes = [C.POINTER(C.c_uint32), C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]
    nt = (C.c_uint32 * 2)(n >> 10, n >> 10)
    out = (C.c_uint32 * 4)()
    assert f(nt, 2, n_ep + 3, 256, out) == 0
    tc, cpt = out[0], out[1]
    assert (tc, cpt, out[2], out[3]) == (8, 4, 0, 0)
    chunks = 2 * (n >> 10) // tc
    assert chunks == 2048
    assert (chunks // (16 * cpt)) * (((n_ep + 3 + 7) // 8 * 8 + 63) // 64) == 512
    s = ctx.stream()
    for rnd in range(2):
        cfgs = [traffic.config("c5", n=n, seed=shard.queue_seed(q, rnd)) for q in range(2)]
        bs = [lib.DeviceBatch(ctx, c.frames, c.lens, nics[q], stride=c.stride) for q, c in enumerate(cfgs)]
        rs = [lib.DeviceResult(ctx, n) for _ in cfgs]
        ba = (lib.Batch * 2)(*[b.desc for b in bs])
        ra = (lib.Result * 2)(*[r.desc for r in rs])
        lib.check(ctx.L.usn_classify_multi(ctx.h, C.cast(ba, C.c_void_p), C.cast(ra, C.c_void_p), 2, s))
        for q, c in enumerate(cfgs):
            info = ctx.finalize(bs[q], rs[q], s)
            want = o.forward_batch(nics[q], c.frames, c.lens, stride=c.stride)
            got = rs[q].decisions()
            mism = np.nonzero((got & katrun.PARITY_MASK) != (want & katrun.PARITY_MASK))[0]
            assert mism.size == 0, "round %d ring %d: first mismatches %s" % (rnd, q, mism[:5])
            assert info.n_host == 0
            check_order_vec(rs[q], want, n_ep)
        if rnd == 0:
            keep = (bs, rs)          # the sources' device chains point at these results
        else:
            for x in keep[0] + keep[1]:
                x.free()
        del cfgs
    assert ctx.scatter_fallbacks() == 0
    ctx.close()
