"""One registry, several device replicas (usn_ctx_create_group): the
multi-GPU product path for a single daemon (include/usn_classify.h).

The reference keeps ONE match_register / innerl2bridge
(/root/reference/src/main.rs:447-449); a tx frame learns into it
(/root/reference/src/endpoint.rs:194-253) and AddMatch / RemoveMatch change it
(main.rs:546-625) between drains.  With the table replicated per GPU, every
such change must reach every replica before that replica's next batch.
These tests use two replicas on the one GPU of the box ([0, 0]: two device
copies of the image and bridge, two sets of tx scratch) and check every
decision against the sequential oracle running the same event order.
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


def _answers(cfg):
    """The NIC-side replies to cfg's frames: IPv4 addresses and ports swapped,
    addressed to the NIC's MAC."""
    from usnetd_amd import traffic
    n, st = cfg.n, cfg.stride
    V = cfg.frames[:n * st].reshape(n, st).copy()
    ip = (V[:, 12] == 0x08) & (V[:, 13] == 0x00)
    a, b = V[ip, 26:30].copy(), V[ip, 30:34].copy()
    V[ip, 26:30], V[ip, 30:34] = b, a
    a, b = V[ip, 34:36].copy(), V[ip, 36:38].copy()
    V[ip, 34:36], V[ip, 36:38] = b, a
    V[:, 0:6] = np.frombuffer(traffic.NICMAC, np.uint8)
    out = np.zeros(cfg.frames.shape[0], np.uint8)
    out[:n * st] = V.reshape(-1)
    return out


def _same(got, want, what):
    mism = np.nonzero((got & katrun.PARITY_MASK) != (want & katrun.PARITY_MASK))[0]
    assert mism.size == 0, "%s: first mismatches %s: got %s want %s" % (
        what, mism[:5], [hex(x) for x in got[mism[:5]]], [hex(x) for x in want[mism[:5]]])


def test_learned_rules_reach_the_other_replica(coracle_mod):
    """tx on replica 0 learns answer rules (and bridge MACs); the NIC's rx on
    replica 1 hits them in its very next batch; while the tx batch awaits
    usn_finalize, replica 1 cannot classify (USN_EBUSY)."""
    from usnetd_amd import lib, traffic
    cfg = traffic.config("c4tx", n=20000, seed=31)
    ctx = lib.Ctx(devices=[0, 0])
    assert ctx.replicas() == 2
    traffic.install_ctx(ctx, cfg)
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfg)
    rules0 = ctx.rule_count()
    ans = _answers(cfg)
    # replica 0: the host endpoint sends
    ctx.select(0)
    s0 = ctx.stream()
    bt = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, cfg.src, stride=cfg.stride)
    rt = lib.DeviceResult(ctx, cfg.n)
    ctx.classify(bt, rt, s0)
    # replica 1 must wait for the learned state
    ctx.select(1)
    s1 = ctx.stream()
    br = lib.DeviceBatch(ctx, ans, cfg.lens, 0, stride=cfg.stride)
    rr = lib.DeviceResult(ctx, cfg.n)
    with pytest.raises(lib.UsnError, match="EBUSY"):
        ctx.classify(br, rr, s1)
    ctx.finalize(bt, rt, s0)
    want_t = o.forward_batch(cfg.src, cfg.frames, cfg.lens, stride=cfg.stride)
    _same(rt.decisions(), want_t, "tx on replica 0")
    learned = ctx.rule_count() - rules0
    assert learned > 1000 and ctx.rule_count() == o.rule_count()
    # replica 1: the NIC receives the replies
    ctx.classify(br, rr, s1)
    ctx.finalize(br, rr, s1)
    want_r = o.forward_batch(0, ans, cfg.lens, stride=cfg.stride)
    got_r = rr.decisions()
    _same(got_r, want_r, "rx on replica 1")
    to_host = int(((((got_r >> 16) & 0xF) == 1) & ((got_r & 0xFFFF) == cfg.src)).sum())
    assert to_host > 1000            # the learned answer rules route replies to the sender
    ctx.close()


def test_control_plane_changes_and_moving_sources(coracle_mod):
    """AddMatch / RemoveMatch made between batches are seen by whichever
    replica classifies next; a NIC whose rings alternate between replicas
    carries its 1-entry decision cache across (a fixed 5-tuple flood, so the
    cache decides almost every frame, stale after RemoveMatch)."""
    from usnetd_amd import lib, traffic
    cfg = traffic.config("c1", n=3000, variant="fixed")
    ctx = lib.Ctx(devices=[0, 0])
    traffic.install_ctx(ctx, cfg)
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfg)
    streams = []
    for rep in (0, 1):
        ctx.select(rep)
        streams.append(ctx.stream())
    frames = cfg.frames.copy()
    k = cfg.n // 2
    frames[k * 64 + 34:k * 64 + 36] = [0x12, 0x34]          # one other flow mid-batch
    keep = []
    for step in range(6):
        rep = step % 2
        ctx.select(rep)
        if step == 2:      # RemoveMatch: the NIC's cached decision goes stale
            w = lib.make_want(traffic.LOCAL, 17, 3333)
            assert ctx.remove_match(w, 2) == 1
            assert o.remove_match(coracle_mod.make_want(traffic.LOCAL, 17, 3333), 2) == 1
        if step == 4:      # AddMatch: a new rule owned by pipe 3 (clears the NIC's cache)
            w = lib.make_want(traffic.LOCAL, 17, 3333)
            assert ctx.add_match(w, 3) == 1
            assert o.add_match(coracle_mod.make_want(traffic.LOCAL, 17, 3333), 3) == 1
        fr = frames if step % 3 == 1 else cfg.frames
        b = lib.DeviceBatch(ctx, fr, cfg.lens, 0, stride=cfg.stride)
        r = lib.DeviceResult(ctx, cfg.n)
        ctx.classify(b, r, streams[rep])
        ctx.finalize(b, r, streams[rep])
        want = o.forward_batch(0, fr, cfg.lens, stride=cfg.stride)
        _same(r.decisions(), want, "step %d on replica %d" % (step, rep))
        keep.append((b, r))
    ctx.close()


def test_two_ring_tx_launch_hands_its_cache_to_another_replica(coracle_mod):
    """Two tx rings in one grid on replica 1, the second without any
    cache-touching frame: the source's next ring, on replica 0, takes its
    carried cache from the launch's ring-2 summary (written inside the grid:
    the state ring 1 hands on) through the host.  Ring B's first frame repeats
    its last frame's PacketInfo with the gateway's dmac, so only the carried
    cache (a hit: the last frame's lookup) gives the oracle's decision."""
    from usnetd_amd import lib, traffic
    a = traffic.c4tx(n=5000, seed=81)
    b = traffic.c4tx(n=3000, seed=82)
    g = traffic.c4tx(n=2100, seed=83)
    st = b.stride
    B = b.frames[:b.n * st].reshape(b.n, st)
    ip = np.nonzero((B[:, 12] == 8) & (B[:, 13] == 0) & (B[:, 23] == 17))[0]
    B[b.n - 1] = B[ip[3]]
    B[b.n - 1, 0:6] = [0x02, 0, 0, 0, 0xB0, 0x07]            # a bridged MAC: get_endpoint
    B[0] = B[b.n - 1]
    B[0, 0:6] = np.frombuffer(traffic.NICMAC, np.uint8)       # not bridged: NIC unless cached
    G = g.frames[:g.n * st].reshape(g.n, st)
    G[:, 12:14] = 0x12                                        # no parse: nothing touches the cache
    ctx = lib.Ctx(devices=[0, 0])
    traffic.install_ctx(ctx, a)
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, a)
    streams = []
    for rep in (0, 1):
        ctx.select(rep)
        streams.append(ctx.stream())
    bufs = {}
    for name, cfg in (("a", a), ("b", b), ("g", g)):
        for rep in (0, 1):
            ctx.select(rep)
            bufs[name, rep] = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, a.src, stride=st)
    keep = []

    def check(cfg, r, what):
        want = o.forward_batch(a.src, cfg.frames, cfg.lens, stride=st)
        _same(r.decisions(), want, what)
        return want

    ctx.select(0)
    ra = lib.DeviceResult(ctx, a.n)
    ctx.classify(bufs["a", 0], ra, streams[0])
    ctx.finalize(bufs["a", 0], ra, streams[0])
    check(a, ra, "ring a, replica 0")
    ctx.select(1)
    rb, rg = lib.DeviceResult(ctx, b.n), lib.DeviceResult(ctx, g.n)
    ctx.classify_multi([bufs["b", 1], bufs["g", 1]], [rb, rg], streams[1])
    ctx.finalize(bufs["b", 1], rb, streams[1])
    check(b, rb, "ring b (ring 1 of the grid), replica 1")
    ctx.finalize(bufs["g", 1], rg, streams[1])
    check(g, rg, "ring g (ring 2 of the grid), replica 1")
    ctx.select(0)
    rb2 = lib.DeviceResult(ctx, b.n)
    ctx.classify(bufs["b", 0], rb2, streams[0])
    ctx.finalize(bufs["b", 0], rb2, streams[0])
    want = check(b, rb2, "ring b again, replica 0")
    assert (want[0] >> 16) & 0xF != lib.CLS_NIC                # decided by the carried cache
    assert ctx.rule_count() == o.rule_count()
    keep += [ra, rb, rg, rb2]
    ctx.close()
