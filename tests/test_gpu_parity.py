"""GPU parity: the HIP path (through the C ABI) against the C oracle.

Bit-exact on decision bits [23:0] (class, endpoint, drop reason); the
per-tile order must be the stable sort of the decisions by endpoint bin and
its expansion must equal the oracle's per-endpoint ordered frame lists.
PARITY UNPINNED beyond the hand-derived fixtures (see DESIGN.md "Oracle").
"""
import ctypes

import numpy as np
import pytest

import katrun
import randtraffic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def coracle_mod():
    import coracle
    coracle.build()
    return coracle


def _gpu():
    from gpu_backend import GpuBackend
    return GpuBackend()


def test_library_is_native_and_gfx950():
    from usnetd_amd import lib
    ctx = lib.Ctx(0)
    assert lib.load().usn_abi_version() == 5
    ctx.close()


@pytest.mark.parametrize("kat", katrun.load_kats(), ids=lambda k: k["name"])
def test_kat_gpu(kat, coracle_mod):
    bad = katrun.run_kat(kat, _gpu())
    assert not bad, "\n".join("step %d: got %#x want %#x (%s)" % b for b in bad)


@pytest.mark.parametrize("tx_frac", [0.0, 0.5])
@pytest.mark.parametrize("seed", range(8))
def test_random_streams_gpu(seed, tx_frac, coracle_mod):
    stream = randtraffic.make_stream(100 + seed, n_events=700, tx_frac=tx_frac)
    want = randtraffic.run_stream(stream, katrun.COracleBackend())
    got = randtraffic.run_stream(stream, _gpu())
    assert len(want) == len(got)
    for i, (x, y) in enumerate(zip(want, got)):
        if isinstance(x, tuple):
            assert x == y, (i, x, y)
        else:
            assert (x & katrun.PARITY_MASK) == (y & katrun.PARITY_MASK), (i, hex(x), hex(y))


@pytest.mark.parametrize("switch_p,ops_p,n_events", [(0.15, 0.02, 700), (0.0008, 0.0003, 6000)])
@pytest.mark.parametrize("seed", range(6))
def test_random_streams_two_rings_gpu(seed, switch_p, ops_p, n_events, coracle_mod):
    """Every sending endpoint's run goes to the device as 2-8 consecutive
    rings of one usn_classify_multi launch (one tx grid), split at seeded
    random frames: learning, fragments, DHCP and the decision cache cross the
    ring boundaries inside the grid.  Long runs (about 1000 frames) span tiles."""
    from gpu_backend import GpuBackend
    stream = randtraffic.make_stream(500 + seed, n_events=n_events, tx_frac=0.7, switch_p=switch_p, ops_p=ops_p)
    want = randtraffic.run_stream(stream, katrun.COracleBackend())
    got = randtraffic.run_stream(stream, GpuBackend(split_tx_seed=seed))
    assert len(want) == len(got)
    for i, (x, y) in enumerate(zip(want, got)):
        if isinstance(x, tuple):
            assert x == y, (i, x, y)
        else:
            assert (x & katrun.PARITY_MASK) == (y & katrun.PARITY_MASK), (i, hex(x), hex(y))


def _filler(n):
    """n rules no frame of randtraffic hits (dst 10.77.0.0/16): they push the
    image past LDS, so the rx kernel takes the projection table U."""
    out = []
    for i in range(n):
        conn = i % 2 == 0
        out.append({"op": "add_match", "owner": 1, "sticky": False,   # endpoint 1 is never removed
                    "want": {"dst": "10.77.%d.%d" % (i >> 8, i & 255), "proto": 17, "dport": 1000 + i % 7,
                             "src": "10.1.1.1" if conn else None, "sport": 5000 + i % 13 if conn else None}})
    return out


@pytest.mark.parametrize("tx_frac", [0.0, 0.5])
@pytest.mark.parametrize("seed", range(6))
def test_random_streams_projection_gpu(seed, tx_frac, coracle_mod):
    """Random streams over a table too large for LDS: 3000 filler rules plus
    40 random ones of every Want shape from small pools (several K1 rules per
    projection: the overflow table X).  The rx kernel reads U (+ X) with
    displacements in LDS; bit-exact against the oracle.  (NIC-owned rules:
    tests/test_table_image.py, through usn_table_build.)"""
    stream = randtraffic.make_stream(300 + seed, n_events=900, tx_frac=tx_frac, n_rules=40)
    stream["steps"] = _filler(3000) + stream["steps"]
    want = randtraffic.run_stream(stream, katrun.COracleBackend())
    gb = _gpu()
    got = randtraffic.run_stream(stream, gb)
    info = (ctypes.c_uint32 * 10)()
    gb.ctx.L.usn_debug_image_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    assert gb.ctx.L.usn_debug_image_info(gb.ctx.h, info) == 0
    assert info[5] & 4 and info[4] * 16 > 40000   # U built; the image is past LDS
    assert len(want) == len(got)
    for i, (x, y) in enumerate(zip(want, got)):
        if isinstance(x, tuple):
            assert x == y, (i, x, y)
        else:
            assert (x & katrun.PARITY_MASK) == (y & katrun.PARITY_MASK), (i, hex(x), hex(y))


def _oracle_lists(d, n_ep):
    cls = (d >> 16) & 0xF
    ep = d & 0xFFFF
    bins = np.where(cls == 1, ep, np.where(cls == 2, n_ep, np.where(cls == 3, n_ep + 1, n_ep + 2)))
    out = {}
    for b in np.unique(bins):
        out[int(b)] = np.nonzero(bins == b)[0]
    return out


@pytest.mark.parametrize("name,n,t512", [
    ("c1", 50000, None), ("c2", 1 << 20, None), ("c3", 1 << 17, None), ("c4", 1 << 18, None),
    ("c5", 1 << 20, None),
    # ragged last tiles; both classify builds for c5
    ("c3", 5003, None), ("c4", 70001, None), ("c5", 100003, "0"), ("c5", 100003, "1"),
    # 4093 pipes + NIC + host ring: the whole 12-bit endpoint id space (4098 bins)
    ("c5-4093", 300007, None),
    # connected rules on listening ports: most frames also probe the overflow table X
    ("c5x", 1 << 20, None)])
def test_config_parity(name, n, t512, coracle_mod, monkeypatch):
    from usnetd_amd import lib, traffic
    if t512 is not None:   # USN_T512 (test build, read at context creation): force one build
        monkeypatch.setenv("USN_T512", t512)
    kw = {}
    if name == "c5-4093":
        name, kw = "c5", {"n_ep": 4093}
    cfg = traffic.config(name, n=n, **kw)
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfg)
    want = o.forward_batch(cfg.src, cfg.frames, cfg.lens, stride=cfg.stride)
    # the forced build is a test knob: the test library reads it
    ctx = lib.Ctx(0, libpath=lib.TEST_LIB_PATH) if t512 is not None else lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    s = ctx.stream()
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, cfg.src, stride=cfg.stride)
    r = lib.DeviceResult(ctx, cfg.n)
    ctx.classify(b, r, s)
    info = ctx.finalize(b, r, s)
    got = r.decisions()
    mism = np.nonzero((got & katrun.PARITY_MASK) != (want & katrun.PARITY_MASK))[0]
    assert mism.size == 0, "first mismatches %s: got %s want %s" % (
        mism[:5], [hex(x) for x in got[mism[:5]]], [hex(x) for x in want[mism[:5]]])
    n_ep = max(e[0] for e in cfg.endpoints) + 1
    assert int(r.summary()["n_ep"]) == n_ep
    lists = r.lists(cfg.n)
    ref = _oracle_lists(want, n_ep)
    assert sorted(lists) == sorted(ref)
    for k in ref:
        assert np.array_equal(lists[k], ref[k]), k
    cc = np.bincount((want >> 16) & 0xF, minlength=4)
    assert list(info.class_count) == cc.tolist()
    ctx.close()


def test_pipelined_batches_carry_cache(coracle_mod):
    """Back-to-back batches of one source with no finalize in between: the
    1-entry cache is carried on the device (fixed 5-tuple flood, c1)."""
    from usnetd_amd import lib, traffic
    cfg = traffic.config("c1", n=3000, variant="fixed")
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfg)
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    s = ctx.stream()
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, 0, stride=cfg.stride)
    rs = [lib.DeviceResult(ctx, cfg.n) for _ in range(3)]
    for r in rs:
        ctx.classify(b, r, s)
    for r in rs:
        want = o.forward_batch(0, cfg.frames, cfg.lens, stride=cfg.stride)
        info = ctx.finalize(b, r, s)
        assert info.n_host == 0
        got = r.decisions()
        assert ((got & katrun.PARITY_MASK) == (want & katrun.PARITY_MASK)).all()
    ctx.close()


@pytest.mark.parametrize("n", [700, 5000])
def test_stale_cache_prefix(n, coracle_mod):
    """RemoveMatch leaves the NIC's cached decision in place: a fixed-5-tuple
    flood keeps going to the old endpoint (endpoint.rs:186-191, main.rs:608-625),
    inside tile 0 (device) and past it (ordered host stage)."""
    from usnetd_amd import lib, traffic
    cfg = traffic.config("c1", n=n, variant="fixed")
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfg)
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    s = ctx.stream()
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, 0, stride=cfg.stride)
    r1, r2, r3 = (lib.DeviceResult(ctx, n) for _ in range(3))
    ctx.classify(b, r1, s)
    ctx.finalize(b, r1, s)
    o.forward_batch(0, cfg.frames, cfg.lens, stride=cfg.stride)
    w = lib.make_want(traffic.LOCAL, 17, 3333)
    assert ctx.remove_match(w, 2) == 1
    assert o.remove_match(coracle_mod.make_want(traffic.LOCAL, 17, 3333), 2) == 1
    # second batch: a different flow in the middle ends the stale prefix
    frames = cfg.frames.copy()
    k = n // 2
    frames[k * 64 + 34:k * 64 + 36] = [0x12, 0x34]
    b2 = lib.DeviceBatch(ctx, frames, cfg.lens, 0, stride=cfg.stride)
    ctx.classify(b2, r2, s)
    info = ctx.finalize(b2, r2, s)
    want = o.forward_batch(0, frames, cfg.lens, stride=cfg.stride)
    got = r2.decisions()
    assert info.flags & lib.S_STALE
    assert ((got & katrun.PARITY_MASK) == (want & katrun.PARITY_MASK)).all()
    from gpu_backend import check_order
    check_order(r2, got)
    # third batch: the cache now holds the live (NOMATCH) decision
    ctx.classify(b2, r3, s)
    ctx.finalize(b2, r3, s)
    want = o.forward_batch(0, frames, cfg.lens, stride=cfg.stride)
    got = r3.decisions()
    assert ((got & katrun.PARITY_MASK) == (want & katrun.PARITY_MASK)).all()
    ctx.close()


def test_offsets_layout(coracle_mod):
    """Packed frames addressed through an offsets array (IMIX in one buffer)."""
    from usnetd_amd import lib, traffic
    cfg = traffic.config("c3", n=20000)
    n = cfg.n
    lens = cfg.lens.astype(np.int64)
    slot = ((lens + 15) // 16) * 16
    offs = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.uint64)
    buf = np.zeros(int(slot.sum()) + 64, np.uint8)
    for i in range(n):
        o_, l_ = int(offs[i]), int(lens[i])
        buf[o_:o_ + l_] = cfg.frames[i * cfg.stride:i * cfg.stride + l_]
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfg)
    want = o.forward_batch(0, buf, cfg.lens, offsets=offs)
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    s = ctx.stream()
    b = lib.DeviceBatch(ctx, buf, cfg.lens, 0, offsets=offs)
    r = lib.DeviceResult(ctx, n)
    ctx.classify(b, r, s)
    ctx.finalize(b, r, s)
    got = r.decisions()
    assert ((got & katrun.PARITY_MASK) == (want & katrun.PARITY_MASK)).all()
    ctx.close()


@pytest.mark.parametrize("name", ["c2", "c5"])
def test_classify_multi_matches_separate(name, coracle_mod):
    """One launch over the drained rings of several NICs (usn_classify_multi)
    gives each source exactly its sequential decisions and carried cache
    (c2: the image in LDS; c5: the projection table, whose tile-0 check of
    each carried cache runs through U too)."""
    import ctypes as C
    from usnetd_amd import lib, traffic
    cfgs = [traffic.config(name, n=n, seed=40 + k) for k, n in enumerate([5000, 1024, 20000])]
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfgs[0])
    nics = [0] + traffic.extra_nics(cfgs[0], 2, ctx)
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfgs[0])
    for nid in nics[1:]:
        o.add_endpoint(nid, 0, -1)
    s = ctx.stream()
    bs = [lib.DeviceBatch(ctx, c.frames, c.lens, nics[k], stride=c.stride) for k, c in enumerate(cfgs)]
    for rep in range(2):                      # the second launch uses the device-carried caches
        rs = [lib.DeviceResult(ctx, c.n) for c in cfgs]
        ba = (lib.Batch * 3)(*[b.desc for b in bs])
        ra = (lib.Result * 3)(*[r.desc for r in rs])
        lib.check(ctx.L.usn_classify_multi(ctx.h, C.cast(ba, C.c_void_p), C.cast(ra, C.c_void_p), 3, s))
        for k, c in enumerate(cfgs):
            ctx.finalize(bs[k], rs[k], s)
            want = o.forward_batch(nics[k], c.frames, c.lens, stride=c.stride)
            got = rs[k].decisions()
            assert ((got & katrun.PARITY_MASK) == (want & katrun.PARITY_MASK)).all(), (rep, k)
    # the same source twice in one launch is refused
    ba = (lib.Batch * 2)(bs[0].desc, bs[0].desc)
    ra = (lib.Result * 2)(rs[0].desc, rs[1].desc)
    assert ctx.L.usn_classify_multi(ctx.h, C.cast(ba, C.c_void_p), C.cast(ra, C.c_void_p), 2, s) == -22
    ctx.close()


@pytest.mark.parametrize("name", ["c2", "c5"])
def test_lists_async(name, coracle_mod):
    """usn_set_lists_async: the lists of each batch are built on the library's
    side stream while the caller's stream classifies the next batches; after
    usn_lists_wait (or usn_finalize) every batch's lists equal the oracle's
    ordered per-endpoint lists, and reusing a result waits for its lists."""
    from usnetd_amd import lib, traffic
    n = 200003
    cfgs = [traffic.config(name, n=n, seed=50 + k) for k in range(3)]
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfgs[0])
    ctx.set_lists_async(True)
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfgs[0])
    s = ctx.stream()
    bs = [lib.DeviceBatch(ctx, c.frames, c.lens, c.src, stride=c.stride) for c in cfgs]
    rs = [lib.DeviceResult(ctx, n) for _ in range(2)]
    wants = [o.forward_batch(c.src, c.frames, c.lens, stride=c.stride) for c in cfgs]
    for k, (b, want) in enumerate(zip(bs, wants)):
        r = rs[k % 2]                       # batch 2 reuses batch 0's result
        ctx.classify(b, r, s)
        if k == 1:                          # batch 0's lists, joined on the stream
            ctx.lists_wait(rs[0], s)
            ctx.sync(s)
            _check_lists(rs[0], wants[0])
    ctx.finalize(bs[2], rs[0], s)
    ctx.finalize(bs[1], rs[1], s)
    for r, want in ((rs[0], wants[2]), (rs[1], wants[1])):
        assert np.array_equal(r.decisions() & katrun.PARITY_MASK, want & katrun.PARITY_MASK)
        _check_lists(r, want)
    ctx.close()


def _check_lists(r, want):
    from usnetd_amd import lib
    n_ep = int(r.summary()["n_ep"])
    got = r.lists(want.shape[0])
    ref = lib.expected_lists(want, n_ep)
    assert sorted(got) == sorted(ref)
    for k in ref:
        assert np.array_equal(got[k], ref[k]), k


def test_endpoint_added_before_finalize(coracle_mod):
    """An rx batch whose later fragments need the host stage, then an endpoint
    added (the endpoint count grows) before its usn_finalize: the batch keeps
    the bins it was classified with (scratch, count rows, lists), and its
    decisions and lists equal the oracle's.  (Before round 3's fix, finalize
    carved the scratch with the grown endpoint count.)"""
    from gpu_backend import check_order
    from usnetd_amd import lib, traffic
    n = 1 << 16
    cfg = traffic.config("c2", n=n, seed=91)
    fr = np.asarray(cfg.frames, np.uint8)
    H = fr[: n * cfg.stride].reshape(n, cfg.stride)
    # frame 100: a first fragment (MF, offset 0); frames 2000 and 40000: later
    # fragments of the same datagram (offset 24 B), decided by the host stage
    H[100, 20:22] = [0x20, 0x00]
    for j in (2000, 40000):
        H[j, :] = H[100, :]
        H[j, 20:22] = [0x00, 0x03]
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfg)
    want = o.forward_batch(cfg.src, fr, cfg.lens, stride=cfg.stride)
    n_ep = max(e[0] for e in cfg.endpoints) + 1
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    s = ctx.stream()
    b = lib.DeviceBatch(ctx, fr, cfg.lens, cfg.src, stride=cfg.stride)
    r = lib.DeviceResult(ctx, n)
    ctx.classify(b, r, s)
    ctx.endpoint_add(n_ep + 40, lib.EP_PIPE, 0)      # 43 more bins from now on
    info = ctx.finalize(b, r, s)
    assert info.n_host >= 2
    got = r.decisions()
    assert np.array_equal(got & katrun.PARITY_MASK, want & katrun.PARITY_MASK)
    assert int(r.summary()["n_bins"]) == n_ep + 3
    check_order(r, got)
    b.free(); r.free(); ctx.close()


def test_stale_walk_names_endpoint_added_after_classify(coracle_mod):
    """the stale-prefix walk of usn_finalize resolves frames with
    today's registry.  A NIC's cached decision goes stale (RemoveMatch,
    main.rs:608-625); the next batch repeats the cached flow past tile 0 and
    then sends ONE frame of another flow; between that batch's classify and
    its finalize an endpoint and a rule for that flow are added.  The walk
    resolves the frame to the new endpoint (an id past the batch's bins), so
    the lists are rebuilt with today's bins: decisions and lists equal the
    oracle's, run with the same registry change before that frame."""
    from gpu_backend import check_order
    from usnetd_amd import lib, traffic
    n = 1 << 14
    k = 5000                                  # past tile 0: the walk, not the device, reaches it
    cfg = traffic.config("c1", n=n, variant="fixed")
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfg)
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    s = ctx.stream()
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, 0, stride=cfg.stride)
    r1, r2 = lib.DeviceResult(ctx, n), lib.DeviceResult(ctx, n)
    ctx.classify(b, r1, s)
    ctx.finalize(b, r1, s)
    o.forward_batch(0, cfg.frames, cfg.lens, stride=cfg.stride)
    assert ctx.remove_match(lib.make_want(traffic.LOCAL, 17, 3333), 2) == 1
    assert o.remove_match(coracle_mod.make_want(traffic.LOCAL, 17, 3333), 2) == 1
    frames = np.asarray(cfg.frames, np.uint8).copy()
    frames[k * 64 + 36:k * 64 + 38] = [0x12, 0x34]          # dport 4660 (UDP checksum untouched)
    n_ep = max(e[0] for e in cfg.endpoints) + 1
    new_id = n_ep + 40
    b2 = lib.DeviceBatch(ctx, frames, cfg.lens, 0, stride=cfg.stride)
    ctx.classify(b2, r2, s)
    ctx.endpoint_add(new_id, lib.EP_PIPE, 0)
    assert ctx.add_match(lib.make_want(traffic.LOCAL, 17, 0x1234), new_id) == 1
    info = ctx.finalize(b2, r2, s)
    got = r2.decisions()
    want0 = o.forward_batch(0, frames[: k * 64], cfg.lens[:k], stride=cfg.stride)
    o.add_endpoint(new_id, lib.EP_PIPE, 0)
    assert o.add_match(coracle_mod.make_want(traffic.LOCAL, 17, 0x1234), new_id) == 1
    want1 = o.forward_batch(0, frames[k * 64:], cfg.lens[k:], stride=cfg.stride)
    want = np.concatenate([want0, want1])
    assert info.flags & lib.S_STALE
    assert (got[k] & 0xFFFF) == new_id and ((got[k] >> 16) & 0xF) == lib.CLS_EP
    assert np.array_equal(got & katrun.PARITY_MASK, want & katrun.PARITY_MASK)
    assert int(r2.summary()["n_bins"]) == new_id + 1 + 3
    check_order(r2, got)
    b.free(); b2.free(); r1.free(); r2.free(); ctx.close()
