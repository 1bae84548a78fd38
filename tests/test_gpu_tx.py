"""GPU parity of the tx direction (a non-NIC endpoint sends; endpoint.rs:194-256).

c4tx (BASELINE.json configs[3], the ADD_MACS learned-MAC path) through the C
ABI against the sequential C oracle: decisions bit-exact on [23:0], and the
registry the batch leaves behind -- learned answer rules with their owner,
learned bridge MACs -- equal to the oracle's.  PARITY UNPINNED beyond the
hand-derived fixtures (see DESIGN.md "Oracle").
"""
import numpy as np
import pytest

import katrun
from gpu_backend import check_order

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def coracle_mod():
    import coracle
    coracle.build()
    return coracle


def _registry_gpu(ctx):
    return sorted((w.dst_addr, w.src_addr, w.dst_port, w.src_port, w.protocol, w.present, o)
                  for w, o, _ in ctx.rules())


def _run(cfg, coracle_mod, batches=2):
    from usnetd_amd import lib, traffic
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfg)
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, cfg.src, stride=cfg.stride)
    infos, keep = [], []
    for k in range(batches):   # the same ring again: learned state + carried cache
        want = o.forward_batch(cfg.src, cfg.frames, cfg.lens, stride=cfg.stride)
        r = lib.DeviceResult(ctx, cfg.n)
        ctx.classify(b, r)
        info = ctx.finalize(b, r)
        got = r.decisions()
        bad = np.nonzero((got & katrun.PARITY_MASK) != (want & katrun.PARITY_MASK))[0]
        assert bad.size == 0, "batch %d: %d mismatches, first %d: got %#x want %#x" % (
            k, bad.size, bad[0], got[bad[0]], want[bad[0]])
        check_order(r, got)
        assert sorted(o.rules()) == _registry_gpu(ctx), "batch %d: registry differs" % k
        assert o.bridge_count() == ctx.bridge_count()
        cls = np.bincount((want >> 16) & 0xF, minlength=4)
        assert list(info.class_count) == [int(x) for x in cls]
        infos.append(info)
        keep.append(r)
    return infos


@pytest.mark.parametrize("n", [1500, 1 << 16, 1 << 18, 1 << 20])
def test_c4tx_parity(n, coracle_mod):
    """Every batch is decided on the device (n_host == 0: no tile wait of the
    one-launch tx kernel gave up, no set overflowed)."""
    from usnetd_amd import traffic
    infos = _run(traffic.config("c4tx", n=n), coracle_mod, batches=3)
    assert infos[0].n_learned > 0
    assert [i.n_host for i in infos] == [0, 0, 0]


@pytest.mark.parametrize("n,at,src", [(5000, [2500], 0), (1 << 16, [0], 0),
                                      (1 << 16, [40000, 40001, 60000], 0),
                                      (5000, [2500], 0x00010203), (1 << 16, [777], 0x00FFFFFF)])
def test_c4tx_host_tail(n, at, src, coracle_mod):
    """A DHCP request (NIC.next_dhcp := S, endpoint.rs:214-226) sends the rest
    of the batch through the ordered host stage from that frame on; its
    source is unspecified anywhere in 0.0.0.0/8 (smoltcp 0.7.0, recalled:
    tests/golden kat_dhcp)."""
    from usnetd_amd import traffic
    infos = _run(traffic.c4tx(n=n, host_at=at, host_src=src), coracle_mod)
    assert infos[0].n_host == n - at[0]


@pytest.mark.parametrize("src", [0x01000000, 0x7F000001, 0x0A000001])
def test_c4tx_dhcp_shaped_not_unspecified(src, coracle_mod):
    """UDP 68 -> 67 to 255.255.255.255 from a source outside 0.0.0.0/8 is no
    DHCP request: it is decided on the device (it learns its answer rule,
    or is a loopback frame) and nothing goes to the host stage."""
    from usnetd_amd import traffic
    infos = _run(traffic.c4tx(n=5000, host_at=[100, 2500], host_src=src), coracle_mod)
    assert [i.n_host for i in infos] == [0, 0]


def test_tx_busy_until_finalize(coracle_mod):
    from usnetd_amd import lib, traffic
    cfg = traffic.config("c4tx", n=4096)
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, cfg.src, stride=cfg.stride)
    r = lib.DeviceResult(ctx, cfg.n)
    ctx.classify(b, r)
    L = lib.load()
    assert L.usn_rule_count(ctx.h) == lib.USN_EBUSY
    assert L.usn_classify(ctx.h, b.desc, r.desc, None) == lib.USN_EBUSY
    ctx.finalize(b, r)
    assert ctx.rule_count() > len(cfg.rules)
    info = ctx.finalize(b, r)   # again: already final
    assert info.n_host == 0


def test_bulk_table_build_and_bridge_set(coracle_mod):
    """usn_table_build / usn_bridge_set give the same decisions as rule-by-rule
    AddMatch + ADD_MACS (the listening triples aside, which only AddMatch records)."""
    from usnetd_amd import lib, traffic
    cfg = traffic.config("c4", n=1 << 14)
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfg)
    want = o.forward_batch(cfg.src, cfg.frames, cfg.lens, stride=cfg.stride)
    ctx = lib.Ctx(0)
    for eid, kind, for_nic in cfg.endpoints:
        ctx.endpoint_add(eid, kind, for_nic)
    rules = [(lib.make_want(w["dst"], w["proto"], w["dport"], w["src"], w["sport"]), owner, sticky)
             for w, owner, sticky in cfg.rules]
    assert ctx.table_build(rules + rules[:5]) == len(cfg.rules)
    ctx.bridge_set([bytes.fromhex("02000000b001"), bytes.fromhex("02000000b002")])
    assert ctx.bridge_count() == 2
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, cfg.src, stride=cfg.stride)
    r = lib.DeviceResult(ctx, cfg.n)
    ctx.classify(b, r)
    ctx.finalize(b, r)
    got = r.decisions()
    assert ((got & katrun.PARITY_MASK) == (want & katrun.PARITY_MASK)).all()
    assert _registry_gpu(ctx) == sorted(o.rules())


def _check(cfg, coracle_mod, offsets=None, frames=None, lens=None, src=None):
    from usnetd_amd import lib, traffic
    frames = cfg.frames if frames is None else frames
    lens = cfg.lens if lens is None else lens
    src = cfg.src if src is None else src
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfg)
    if offsets is None:
        want = o.forward_batch(src, frames, lens, stride=cfg.stride)
    else:
        want = o.forward_batch(src, frames, lens, offsets=offsets)
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    if offsets is None:
        b = lib.DeviceBatch(ctx, frames, lens, src, stride=cfg.stride)
    else:
        b = lib.DeviceBatch(ctx, frames, lens, src, offsets=offsets)
    r = lib.DeviceResult(ctx, len(lens))
    ctx.classify(b, r)
    info = ctx.finalize(b, r)
    got = r.decisions()
    bad = np.nonzero((got & katrun.PARITY_MASK) != (want & katrun.PARITY_MASK))[0]
    assert bad.size == 0, "%d mismatches, first %d: got %#x want %#x" % (
        bad.size, bad[0], got[bad[0]], want[bad[0]])
    check_order(r, got)
    assert sorted(o.rules()) == _registry_gpu(ctx)
    assert o.bridge_count() == ctx.bridge_count()
    return info


def test_tx_ragged_offsets(coracle_mod):
    """Ragged frame lengths packed through an offsets array, sent by an endpoint."""
    from usnetd_amd import traffic
    cfg = traffic.c4tx(n=20000, seed=11)
    rng = np.random.default_rng(3)
    n = cfg.n
    lens = rng.integers(0, 129, n).astype(np.uint16)
    lens[rng.random(n) < 0.7] = 64
    slot = ((lens.astype(np.int64) + 15) // 16) * 16
    offs = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.uint64)
    buf = np.zeros(int(slot.sum()) + 128, np.uint8)
    for i in range(n):
        o_, l_ = int(offs[i]), int(lens[i])
        c_ = min(l_, 64)
        buf[o_:o_ + c_] = cfg.frames[i * cfg.stride:i * cfg.stride + c_]
    _check(cfg, coracle_mod, offsets=offs, frames=buf, lens=lens)


def test_tx_fragments(coracle_mod):
    """First fragments sent by an endpoint are remembered in order; the first
    later fragment starts the ordered host tail."""
    from usnetd_amd import traffic
    cfg = traffic.c4tx(n=8192, seed=12)
    V = cfg.frames[:cfg.n * cfg.stride].reshape(cfg.n, cfg.stride)
    ip = np.nonzero((V[:, 12] == 8) & (V[:, 13] == 0))[0]
    first, later = ip[100:160], ip[3000:3010]
    V[first, 20], V[first, 21] = 0x20, 0x00            # MF, offset 0
    V[later, 20], V[later, 21] = 0x00, 0xB9            # offset 185
    V[later, 18:20] = V[first[:10], 18:20]             # same ident ...
    V[later, 26:34] = V[first[:10], 26:34]             # ... addresses
    V[later, 0:12] = V[first[:10], 0:12]               # ... and MACs: map hits
    V[later, 23] = V[first[:10], 23]
    info = _check(cfg, coracle_mod)
    assert info.n_host == cfg.n - int(later[0])


def test_tx_imix_stride_2048_from_pipe(coracle_mod):
    from usnetd_amd import traffic
    cfg = traffic.config("c3", n=1 << 15)
    info = _check(cfg, coracle_mod, src=2)          # endpoint 2 (a pipe) sends c3's frames
    assert info.n_learned > 0


@pytest.mark.parametrize("n", [1, 2, 1023, 1025])
def test_tx_tiny_and_tile_edges(n, coracle_mod):
    from usnetd_amd import traffic
    cfg = traffic.c4tx(n=n, seed=13)
    _check(cfg, coracle_mod)


def test_tx_runs_across_tiles(coracle_mod):
    """Runs of one repeated frame that cross tile boundaries (the run head's
    decision reaches the next tiles: an IPv4 flow, an ARP flood), and whole
    tiles without a cache-touching frame (the tile after looks further back)."""
    from usnetd_amd import traffic
    cfg = traffic.c4tx(n=9000, seed=14)
    st = cfg.stride
    V = cfg.frames[:cfg.n * st].reshape(cfg.n, st)
    ip = np.nonzero((V[:, 12] == 8) & (V[:, 13] == 0))[0]
    arp = np.nonzero((V[:, 12] == 8) & (V[:, 13] == 6))[0]
    V[1000:1100] = V[ip[5]]                    # crosses 1024
    V[2000:2200] = V[arp[3]]                   # crosses 2048
    V[3000:3100] = V[ip[7]]                    # a run up to the garbage tiles
    V[3100:5200, 12:14] = 0x12                 # no parse: tiles 4 (3072.. ) fully non-touching
    V[5200:5300] = V[ip[7]]                    # the same flow again after them: a cache hit
    V[8190:8200] = V[arp[4]]                   # crosses 8192
    _check(cfg, coracle_mod)


def test_tx_fixed_flow_all_hits(coracle_mod):
    """One 5-tuple sent 200000 times by the host endpoint: every frame after
    the first is a cache hit whose run head lies in tile 0."""
    from usnetd_amd import traffic
    cfg = traffic.config("c1", n=200000, variant="fixed")
    info = _check(cfg, coracle_mod, src=1)
    assert info.n_host == 0


def test_tx_runs_host_free(coracle_mod):
    """test_tx_runs_across_tiles' batch needs no host stage either."""
    from usnetd_amd import traffic
    cfg = traffic.c4tx(n=70000, seed=15)
    st = cfg.stride
    V = cfg.frames[:cfg.n * st].reshape(cfg.n, st)
    V[3100:69000, 12:14] = 0x12                # 64+ tiles in a row without a touching frame
    info = _check(cfg, coracle_mod)
    assert info.n_host == 0


def test_c4tx_more_tiles_than_resident(coracle_mod):
    """4M frames (4096 tiles): more tiles than the GPU keeps resident at once,
    so later tiles wait on tiles that were dispatched, not yet finished."""
    from usnetd_amd import traffic
    infos = _run(traffic.config("c4tx", n=1 << 22), coracle_mod, batches=2)
    assert [i.n_host for i in infos] == [0, 0]



def _pipelined(cfgs, coracle_mod, n_rings):
    """Rings of one sending endpoint, ring k + 1 classified before ring k's
    usn_finalize; decisions, lists and the registry against the sequential
    oracle, ring by ring."""
    from usnetd_amd import lib, traffic
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfgs[0])
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfgs[0])
    s = ctx.stream()
    bs = [lib.DeviceBatch(ctx, c.frames, c.lens, c.src, stride=c.stride) for c in cfgs]
    rs = [lib.DeviceResult(ctx, cfgs[0].n) for _ in range(2)]
    infos = []
    ctx.classify(bs[0], rs[0], s)
    for k in range(n_rings):
        if k + 1 < n_rings:
            ctx.classify(bs[(k + 1) % len(bs)], rs[(k + 1) % 2], s)
        info = ctx.finalize(bs[k % len(bs)], rs[k % 2], s)
        c = cfgs[k % len(cfgs)]
        want = o.forward_batch(c.src, c.frames, c.lens, stride=c.stride)
        got = rs[k % 2].decisions()
        bad = np.nonzero((got & katrun.PARITY_MASK) != (want & katrun.PARITY_MASK))[0]
        assert bad.size == 0, "ring %d: %d mismatches, first %d: got %#x want %#x" % (
            k, bad.size, bad[0], got[bad[0]], want[bad[0]])
        check_order(rs[k % 2], got)
        infos.append(info)
    assert sorted(o.rules()) == _registry_gpu(ctx)
    assert o.bridge_count() == ctx.bridge_count()
    ctx.close()
    return infos


@pytest.mark.parametrize("n", [3000, 1 << 20])
def test_tx_pipelined_rings(n, coracle_mod):
    """ring k + 1 enqueued before ring k's usn_finalize.  Ring
    0 learns, so ring 1 (which ran against the state ring 0 started from) is
    decided again on the host; rings 2.. run against the learned state and
    are final on the device."""
    from usnetd_amd import traffic
    infos = _pipelined([traffic.config("c4tx", n=n)], coracle_mod, 5)
    assert infos[0].n_learned > 0
    assert infos[1].n_host == n                  # redone on the host
    assert [i.n_host for i in infos[2:]] == [0, 0, 0]


def test_tx_pipelined_rings_all_learn(coracle_mod):
    """Back-to-back rings that all learn (new flows in every ring): each ring
    after the first is redone on the host, and every decision, the registry
    and the bridge equal the sequential oracle's."""
    from usnetd_amd import traffic
    cfgs = [traffic.c4tx(n=1 << 16, seed=6 + k) for k in range(4)]
    infos = _pipelined(cfgs, coracle_mod, 4)
    assert all(i.n_learned > 0 for i in infos)
    assert [i.n_host for i in infos[1:]] == [1 << 16] * 3


def test_tx_pipeline_order_and_busy(coracle_mod):
    """At most two tx rings in flight, of one source on one stream, finalized
    in order; nothing else while they are (USN_EBUSY)."""
    import ctypes as C
    from usnetd_amd import lib, traffic
    cfg = traffic.config("c4tx", n=4096)
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    s, s2 = ctx.stream(), ctx.stream()
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, cfg.src, stride=cfg.stride)
    r0, r1, r2 = (lib.DeviceResult(ctx, cfg.n) for _ in range(3))
    L = ctx.L
    ctx.classify(b, r0, s)
    assert L.usn_classify(ctx.h, C.byref(b.desc), C.byref(r1.desc), s2) == lib.USN_EBUSY   # other stream
    ctx.classify(b, r1, s)
    assert L.usn_classify(ctx.h, C.byref(b.desc), C.byref(r2.desc), s) == lib.USN_EBUSY    # a third
    info = lib.FinalizeInfo()
    assert L.usn_finalize(ctx.h, C.byref(b.desc), C.byref(r1.desc), s, C.byref(info)) == lib.USN_EBUSY
    w = lib.make_want(traffic.LOCAL, 17, 4444)
    assert ctx.L.usn_add_match(ctx.h, C.byref(w), 2, 0) == lib.USN_EBUSY
    ctx.finalize(b, r0, s)
    ctx.finalize(b, r1, s)
    ctx.classify(b, r2, s)
    ctx.finalize(b, r2, s)
    ctx.close()


def _ring_launches(rings, coracle_mod, pipelined=False, src=None, per=2):
    """Rings of one sending endpoint, `per` consecutive rings per
    usn_classify_multi launch (one tx grid: ring k's tiles order after ring
    k - 1's); with `pipelined`, launch j + 1 is enqueued before
    launch j's rings are finalized.  Every ring's decisions and lists, and
    the registry and bridge at the end, against the sequential oracle."""
    from usnetd_amd import lib, traffic
    src = rings[0].src if src is None else src
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, rings[0])
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, rings[0])
    s = ctx.stream()
    bs = [lib.DeviceBatch(ctx, c.frames, c.lens, src, stride=c.stride) for c in rings]
    rs = [lib.DeviceResult(ctx, c.n) for c in rings]
    pairs = [list(range(k, min(k + per, len(rings)))) for k in range(0, len(rings), per)]
    infos = [None] * len(rings)

    def launch(p):
        ctx.classify_multi([bs[k] for k in p], [rs[k] for k in p], s)

    def fin(k):
        infos[k] = ctx.finalize(bs[k], rs[k], s)
        c = rings[k]
        want = o.forward_batch(src, c.frames, c.lens, stride=c.stride)
        got = rs[k].decisions()
        bad = np.nonzero((got & katrun.PARITY_MASK) != (want & katrun.PARITY_MASK))[0]
        assert bad.size == 0, "ring %d: %d mismatches, first %d: got %#x want %#x" % (
            k, bad.size, bad[0], got[bad[0]], want[bad[0]])
        check_order(rs[k], got)
        cls = np.bincount((want >> 16) & 0xF, minlength=4)
        assert list(infos[k].class_count) == [int(x) for x in cls], k

    if pipelined:
        launch(pairs[0])
        for j, p in enumerate(pairs):
            if j + 1 < len(pairs):
                launch(pairs[j + 1])
            for k in p:
                fin(k)
    else:
        for p in pairs:
            launch(p)
            for k in p:
                fin(k)
    assert sorted(o.rules()) == _registry_gpu(ctx)
    assert o.bridge_count() == ctx.bridge_count()
    ctx.close()
    return infos


@pytest.mark.parametrize("n", [3000, 1 << 20])
def test_tx_two_rings_one_launch(n, coracle_mod):
    """Ring 1 learns; ring 2 (the same frames) saw that learning inside the
    grid, so it is final on the device: no host stage, nothing left to learn."""
    from usnetd_amd import traffic
    cfg = traffic.config("c4tx", n=n)
    infos = _ring_launches([cfg] * 4, coracle_mod)
    assert infos[0].n_learned > 0
    assert infos[1].n_learned == 0
    assert [i.n_host for i in infos] == [0, 0, 0, 0]


@pytest.mark.parametrize("n", [3000, 1 << 20])
def test_tx_two_ring_launches_pipelined(n, coracle_mod):
    """Launch 1 enqueued before launch 0's rings are finalized: launch 0
    learned, so both of launch 1's rings are decided again on the host;
    launch 2 was enqueued after launch 0's finalizes and is final on the
    device."""
    from usnetd_amd import traffic
    cfg = traffic.config("c4tx", n=n)
    infos = _ring_launches([cfg] * 8, coracle_mod, pipelined=True)
    assert infos[0].n_learned > 0
    assert infos[1].n_host == 0
    assert [i.n_host for i in infos[2:4]] == [n, n]
    assert [i.n_host for i in infos[4:]] == [0, 0, 0, 0]


def test_tx_two_rings_all_learn(coracle_mod):
    """Every ring brings new flows: ring 2 learns its own on the device, with
    ring 1's already visible to it (first learners across the ring boundary)."""
    from usnetd_amd import traffic
    rings = [traffic.c4tx(n=1 << 16, seed=30 + k) for k in range(4)]
    infos = _ring_launches(rings, coracle_mod)
    assert all(i.n_learned > 0 for i in infos)
    assert [i.n_host for i in infos] == [0, 0, 0, 0]


@pytest.mark.parametrize("first", [True, False])
def test_tx_two_rings_host_tail(first, coracle_mod):
    """A DHCP request sends the rest of its ring through the ordered host
    stage.  In ring 1, ring 2 is then decided again on the host (it ran
    behind ring 1's device results); in ring 2, ring 1 stays final."""
    from usnetd_amd import traffic
    a = traffic.c4tx(n=5000, host_at=[2500], seed=40)
    b = traffic.c4tx(n=5000, seed=41)
    rings = [a, b] if first else [b, a]
    infos = _ring_launches(rings, coracle_mod)
    if first:
        assert [i.n_host for i in infos] == [2500, 5000]
    else:
        assert [i.n_host for i in infos] == [0, 2500]


def test_tx_two_rings_cache_across(coracle_mod):
    """The carried cache across the ring boundary inside a grid: ragged
    rings, ring 2 opening with ring 1's last flow (cache hits on ring 1's
    frames), a ring without any cache-touching frame as ring 1 (ring 2 then
    compares with the cache carried into the launch) and as ring 2 (the next
    launch takes ring 1's cache through ring 2's summary)."""
    from usnetd_amd import traffic
    r1 = traffic.c4tx(n=3000, seed=50)
    r2 = traffic.c4tx(n=1025, seed=51)
    g = traffic.c4tx(n=2100, seed=52)
    st = r1.stride
    V1 = r1.frames[:r1.n * st].reshape(r1.n, st)
    V2 = r2.frames[:r2.n * st].reshape(r2.n, st)
    G = g.frames[:g.n * st].reshape(g.n, st)
    ip = np.nonzero((V1[:, 12] == 8) & (V1[:, 13] == 0))[0]
    V1[2990:3000] = V1[ip[5]]
    V2[0:50] = V1[ip[5]]
    G[:, 12:14] = 0x12                          # no parse: no frame touches the cache
    infos = _ring_launches([r1, r2, g, r1, r1, g, r2], coracle_mod)
    assert [i.n_host for i in infos] == [0] * 7


def test_tx_two_ring_launch_rules(coracle_mod):
    """Up to eight rings per tx launch: of one source, distinct results; at
    most two launches in flight; rings finalized in order."""
    import ctypes as C
    from usnetd_amd import lib, traffic
    cfg = traffic.config("c4tx", n=4096)
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    s = ctx.stream()
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, cfg.src, stride=cfg.stride)
    b2 = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, 2, stride=cfg.stride)
    rs = [lib.DeviceResult(ctx, cfg.n) for _ in range(9)]

    def multi(bb, rr):
        ba = (lib.Batch * len(bb))(*[x.desc for x in bb])
        ra = (lib.Result * len(rr))(*[x.desc for x in rr])
        return ctx.L.usn_classify_multi(ctx.h, C.cast(ba, C.c_void_p), C.cast(ra, C.c_void_p), len(bb), s)

    assert multi([b, b2], rs[:2]) == lib.USN_EINVAL          # two sources
    assert multi([b] * 9, rs[:9]) == lib.USN_EINVAL          # nine rings
    assert multi([b, b], [rs[0], rs[0]]) == lib.USN_EINVAL   # one result twice
    assert multi([b, b, b], [rs[0], rs[1], rs[0]]) == lib.USN_EINVAL
    assert multi([b, b, b2], rs[:3]) == lib.USN_EINVAL       # a third ring of another source
    assert multi([b, b], rs[:2]) == 0
    assert multi([b], [rs[1]]) == lib.USN_EBUSY              # a result in flight
    assert multi([b, b], rs[2:4]) == 0                       # the second launch
    assert multi([b], [rs[4]]) == lib.USN_EBUSY              # a third
    info = lib.FinalizeInfo()
    assert ctx.L.usn_finalize(ctx.h, C.byref(b.desc), C.byref(rs[1].desc), s, C.byref(info)) == lib.USN_EBUSY
    ctx.finalize(b, rs[0], s)
    assert multi([b], [rs[4]]) == lib.USN_EBUSY              # launch 0's ring 2 still in flight
    ctx.finalize(b, rs[1], s)
    assert multi([b], [rs[4]]) == 0
    for r in rs[2:5]:
        ctx.finalize(b, r, s)
    assert multi([b] * 8, rs[:8]) == 0                       # eight rings in one grid
    for r in rs[:8]:
        ctx.finalize(b, r, s)
    ctx.close()


def test_tx_finalize_on_another_stream_is_refused(coracle_mod):
    """a tx batch's state is copied on the stream its
    launches are on; usn_finalize on another stream returns USN_EINVAL and
    leaves the batch pending."""
    import ctypes as C
    from usnetd_amd import lib, traffic
    cfg = traffic.config("c4tx", n=4096)
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    s, s2 = ctx.stream(), ctx.stream()
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, cfg.src, stride=cfg.stride)
    r = lib.DeviceResult(ctx, cfg.n)
    ctx.classify(b, r, s)
    info = lib.FinalizeInfo()
    assert ctx.L.usn_finalize(ctx.h, C.byref(b.desc), C.byref(r.desc), s2, C.byref(info)) == lib.USN_EINVAL
    assert ctx.L.usn_rule_count(ctx.h) == lib.USN_EBUSY
    ctx.finalize(b, r, s)
    assert ctx.rule_count() > len(cfg.rules)
    ctx.close()


@pytest.mark.parametrize("n1,n2", [(1, 1), (1, 5000), (1023, 1), (1024, 1025), (2047, 2049)])
def test_tx_two_rings_tile_edges(n1, n2, coracle_mod):
    """Two rings in one grid at tile edges: single-frame rings, a ring 1
    that ends inside its last tile (ring 2 starts on a fresh tile of the
    grid), full tiles, and a ring 2 of one frame; every ring twice."""
    from usnetd_amd import traffic
    r1 = traffic.c4tx(n=n1, seed=70)
    r2 = traffic.c4tx(n=n2, seed=71)
    infos = _ring_launches([r1, r2, r1, r2], coracle_mod)
    assert [i.n_host for i in infos] == [0, 0, 0, 0]


@pytest.mark.parametrize("n", [3000, 1 << 20])
def test_tx_four_rings_one_launch(n, coracle_mod):
    """Four rings per grid: ring 0 learns, rings 1-3 (the same frames) saw
    it inside the grid; then the same with launch 1 enqueued before launch
    0's rings are finalized (all four decided again on the host)."""
    from usnetd_amd import traffic
    cfg = traffic.config("c4tx", n=n)
    infos = _ring_launches([cfg] * 8, coracle_mod, per=4)
    assert infos[0].n_learned > 0
    assert [i.n_learned for i in infos[1:]] == [0] * 7
    assert [i.n_host for i in infos] == [0] * 8
    infos = _ring_launches([cfg] * 12, coracle_mod, pipelined=True, per=4)
    assert [i.n_host for i in infos] == [0] * 4 + [n] * 4 + [0] * 4


@pytest.mark.parametrize("per", [3, 4, 8])
def test_tx_multi_rings_all_learn(per, coracle_mod):
    """Every ring brings new flows: each learns its own on the device, with
    the earlier rings' items already visible to it."""
    from usnetd_amd import traffic
    rings = [traffic.c4tx(n=1 << 15, seed=80 + k) for k in range(2 * per)]
    infos = _ring_launches(rings, coracle_mod, per=per)
    assert all(i.n_learned > 0 for i in infos)
    assert [i.n_host for i in infos] == [0] * (2 * per)


@pytest.mark.parametrize("at", [0, 1, 3])
def test_tx_four_rings_host_tail(at, coracle_mod):
    """A DHCP request in ring `at` of four: the rest of that ring goes to the
    host stage, and every later ring of the grid is decided again on the
    host; the rings before stay final."""
    from usnetd_amd import traffic
    rings = [traffic.c4tx(n=5000, seed=90 + k) for k in range(4)]
    rings[at] = traffic.c4tx(n=5000, host_at=[2500], seed=90 + at)
    infos = _ring_launches(rings, coracle_mod, per=4)
    assert [i.n_host for i in infos] == [0] * at + [2500] + [5000] * (3 - at)


@pytest.mark.parametrize("ns", [(1, 1, 1, 1), (1023, 1, 1025, 3), (1024, 2049, 1, 5000), (3000, 1025)])
def test_tx_multi_rings_tile_edges(ns, coracle_mod):
    """Three and four rings in one grid at tile edges (rings of one frame,
    rings ending inside a tile, full tiles); every launch twice."""
    from usnetd_amd import traffic
    rings = [traffic.c4tx(n=x, seed=100 + k) for k, x in enumerate(ns)]
    per = len(ns) if len(ns) > 2 else 3
    infos = _ring_launches(rings + rings, coracle_mod, per=per)
    assert [i.n_host for i in infos] == [0] * len(infos)


@pytest.mark.parametrize("n", [3000, 1 << 20])
def test_tx_eight_rings_one_launch(n, coracle_mod):
    """Eight rings per grid (the bench's c4tx launch): ring 0 learns, the
    rest saw it inside the grid; pipelined, launch 1's rings are all decided
    again on the host and launch 2's are final."""
    from usnetd_amd import traffic
    cfg = traffic.config("c4tx", n=n)
    infos = _ring_launches([cfg] * 24, coracle_mod, pipelined=True, per=8)
    assert infos[0].n_learned > 0
    assert [i.n_host for i in infos] == [0] * 8 + [n] * 8 + [0] * 8


@pytest.mark.parametrize("at,src", [(0, 0), (5, 0), (7, 0), (3, 0x00070707)])
def test_tx_eight_rings_host_tail(at, src, coracle_mod):
    """A DHCP request in ring `at` of eight: that ring's rest and every later
    ring go to the host stage (from 0.0.0.0, or another 0/8 source)."""
    from usnetd_amd import traffic
    rings = [traffic.c4tx(n=3000, seed=110 + k) for k in range(8)]
    rings[at] = traffic.c4tx(n=3000, host_at=[1500], seed=110 + at, host_src=src)
    infos = _ring_launches(rings, coracle_mod, per=8)
    assert [i.n_host for i in infos] == [0] * at + [1500] + [3000] * (7 - at)


def test_tx_eight_rings_all_learn_1m(coracle_mod):
    """The bench's launch shape with learning in every ring: eight 1M rings
    of distinct flows in one grid (8192 tiles, eight generations), each
    learning ~300K answer rules with the earlier rings' items visible."""
    from usnetd_amd import traffic
    rings = [traffic.c4tx(n=1 << 20, seed=200 + k) for k in range(8)]
    infos = _ring_launches(rings, coracle_mod, per=8)
    assert all(i.n_learned > 0 for i in infos)
    assert [i.n_host for i in infos] == [0] * 8
