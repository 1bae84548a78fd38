"""The usn_batch window contract (include/usn_classify.h): the device never
reads a frame past `window` bytes.  Frames whose L4 ports lie beyond it
(IPv4 with IHL >= 12 at a 64-byte window: extract_pkt_info reads the ports at
14+hl .. 17+hl, /root/reference/src/pkt.rs:177-186) are flagged
USN_R_WINDOW | USN_F_HOST and usn_finalize resolves them from the host frame
reader -- bit-exact against the oracle, which sees the whole frames.  Without
a reader, usn_finalize refuses the batch (USN_EINVAL) before any side effect.

This is INTEGRATION.md's copy path: the host copies each netmap slot's first
64 bytes to the device at stride 64, with the real slot lengths.
"""
import numpy as np
import pytest

import katrun

pytestmark = pytest.mark.gpu

FULL = 1536   # host slot size (frames up to 1500 B)


def _frames(n, seed, dmac=None):
    """IPv4 TCP/UDP/ICMP frames of 100-1500 B with IHL 5, 11 and 12-15."""
    from usnetd_amd import traffic
    rng = np.random.default_rng(seed)
    buf = np.zeros((n, FULL), np.uint8)
    buf[:, 64:] = rng.integers(0, 256, (n, FULL - 64), dtype=np.uint8)   # payload noise
    lens = rng.integers(100, 1501, n).astype(np.uint16)
    ihl = rng.choice(np.array([5, 11, 12, 13, 14, 15]), n, p=[0.2, 0.1, 0.175, 0.175, 0.175, 0.175])
    proto = rng.choice(np.array([6, 17, 1]), n, p=[0.45, 0.45, 0.1])
    dport = np.where(rng.random(n) < 0.8, 7000 + rng.integers(0, 16, n), rng.integers(20000, 30000, n))
    sport = rng.integers(1024, 65536, n)
    src = (10 << 24) | rng.integers(0, 1 << 16, n)
    for i in range(n):
        f = buf[i]
        f[0:6] = np.frombuffer(dmac or traffic.NICMAC, np.uint8)
        f[6:12] = np.frombuffer(traffic.REMMAC, np.uint8)
        f[12], f[13] = 0x08, 0x00
        hl = int(ihl[i]) * 4
        f[14] = 0x40 | int(ihl[i])
        f[15:14 + hl] = 0
        tl = int(lens[i]) - 14
        f[16], f[17] = tl >> 8, tl & 0xFF
        f[18], f[19] = (i >> 8) & 0xFF, i & 0xFF
        f[20], f[21] = 0x40, 0x00            # DF
        f[22], f[23] = 64, int(proto[i])
        f[26:30] = np.frombuffer(int(src[i]).to_bytes(4, "big"), np.uint8)
        f[30:34] = np.frombuffer(traffic.LOCAL.to_bytes(4, "big"), np.uint8)
        p = 14 + hl
        f[p:p + 2] = np.frombuffer(int(sport[i]).to_bytes(2, "big"), np.uint8)
        f[p + 2:p + 4] = np.frombuffer(int(dport[i]).to_bytes(2, "big"), np.uint8)
    return buf, lens, ihl


def _setup(n_pipes=16):
    """NIC 0, host ring 1 (for NIC 0), pipes 2.. with listening rules on 7000+k."""
    from usnetd_amd import lib, traffic
    eps = [(0, 0, None), (1, 1, 0)] + [(2 + k, 2, 0) for k in range(n_pipes)]
    rules = []
    for k in range(n_pipes):
        proto = 6 if k % 2 else 17
        rules.append((lib.make_want(traffic.LOCAL, proto, 7000 + k), 2 + k))
    rules.append((lib.make_want(traffic.LOCAL, 1), 3))   # ICMP to the local address
    return eps, rules


def _install(ctx, o, eps, rules):
    for eid, kind, for_nic in eps:
        ctx.endpoint_add(eid, kind, for_nic)
        o.add_endpoint(eid, kind, -1 if for_nic is None else for_nic)
    import coracle
    for w, owner in rules:
        assert ctx.add_match(w, owner) == 1
        ow = coracle.make_want(w.dst_addr, w.protocol,
                               w.dst_port if w.present & 1 else None,
                               w.src_addr if w.present & 2 else None,
                               w.src_port if w.present & 4 else None)
        assert o.add_match(ow, owner) == 1


@pytest.fixture(scope="module")
def coracle_mod():
    import coracle
    coracle.build()
    return coracle


@pytest.mark.parametrize("src", [0, 1], ids=["rx", "tx"])
def test_window64_ports_past_window(src, coracle_mod):
    """64-B windows at stride 64 (INTEGRATION.md copy path): IHL 12-15 frames
    of 100-1500 B resolved through the host frame reader, bit-exact."""
    from usnetd_amd import lib
    n = 3000
    full, lens, ihl = _frames(n, 11 + src)
    eps, rules = _setup()
    ctx = lib.Ctx(0)
    o = coracle_mod.Oracle()
    _install(ctx, o, eps, rules)
    want = o.forward_batch(src, full.reshape(-1), lens, stride=FULL)
    win = np.ascontiguousarray(full[:, :64]).reshape(-1)
    b = lib.DeviceBatch(ctx, win, lens, src, stride=64)
    assert b.desc.window == 64
    r = lib.DeviceResult(ctx, n)
    s = ctx.stream()
    ctx.classify(b, r, s)
    ctx.sync(s)
    pre = r.decisions()
    flagged = ((pre >> 20) & 0xF) == lib.R_WINDOW
    assert flagged.sum() > 0
    # exactly the frames with ports past byte 64 (IHL >= 12, TCP/UDP) are left to the host
    if src == 0:
        assert np.array_equal(np.nonzero(flagged)[0], np.nonzero(ihl >= 12)[0][
            np.isin(np.nonzero(ihl >= 12)[0], np.nonzero(full[:, 23] != 1)[0])])
    reads = []

    def reader(s_, i):
        reads.append(i)
        assert s_ == src
        return full[i, :int(lens[i])].tobytes()
    ctx.set_frame_reader(reader)
    ctx.finalize(b, r, s)
    got = r.decisions()
    mism = np.nonzero((got & katrun.PARITY_MASK) != (want & katrun.PARITY_MASK))[0]
    assert mism.size == 0, "first mismatches %s: got %s want %s" % (
        mism[:5], [hex(x) for x in got[mism[:5]]], [hex(x) for x in want[mism[:5]]])
    assert len(reads) > 0
    if src == 1:
        assert ctx.rule_count() == o.rule_count()
    ctx.close()


@pytest.mark.parametrize("window", [66, 67, 70, 78])
@pytest.mark.parametrize("src", [0, 1], ids=["rx", "tx"])
def test_window_not_multiple_of_4(window, src, coracle_mod):
    """Windows of 66/67/70/78 bytes at stride 80 (usn_batch.window is any
    value >= 64): every byte of a frame past its window is poisoned in HBM, so
    a read past the window changes a decision.  IHL 12 frames have their
    ports at 62..65 (inside a 66-byte window: decided on the device from the
    reloaded bytes 60..65), IHL >= 13 past it (resolved from the frame
    reader); bit-exact against the oracle on the whole frames."""
    from usnetd_amd import lib
    n = 3000
    full, lens, ihl = _frames(n, 31 + window + src)
    eps, rules = _setup()
    ctx = lib.Ctx(0)
    o = coracle_mod.Oracle()
    _install(ctx, o, eps, rules)
    want = o.forward_batch(src, full.reshape(-1), lens, stride=FULL)
    dev = np.ascontiguousarray(full[:, :80]).copy()
    dev[:, window:] = 0xA5                      # poison: never readable
    b = lib.DeviceBatch(ctx, dev.reshape(-1), lens, src, stride=80, window=window)
    assert b.desc.window == window
    r = lib.DeviceResult(ctx, n)
    s = ctx.stream()
    ctx.classify(b, r, s)
    ctx.sync(s)
    pre = r.decisions()
    flagged = ((pre >> 20) & 0xF) == lib.R_WINDOW
    if src == 0:
        # exactly the TCP/UDP frames whose ports end past the window (18 + hl > window)
        past = (18 + 4 * ihl > window) & (full[:, 23] != 1)
        assert np.array_equal(flagged, past)
        assert not (flagged & (ihl == 12)).any()        # ports at 62..65 lie inside
    ctx.set_frame_reader(lambda s_, i: full[i, :int(lens[i])].tobytes())
    ctx.finalize(b, r, s)
    got = r.decisions()
    mism = np.nonzero((got & katrun.PARITY_MASK) != (want & katrun.PARITY_MASK))[0]
    assert mism.size == 0, "first mismatches %s: got %s want %s" % (
        mism[:5], [hex(x) for x in got[mism[:5]]], [hex(x) for x in want[mism[:5]]])
    if src == 1:
        assert ctx.rule_count() == o.rule_count()
    ctx.close()


def test_window64_without_reader_is_refused(coracle_mod):
    """No frame reader: usn_finalize returns USN_EINVAL and changes nothing."""
    from usnetd_amd import lib
    n = 1200
    full, lens, _ = _frames(n, 21)
    eps, rules = _setup()
    ctx = lib.Ctx(0)
    o = coracle_mod.Oracle()
    _install(ctx, o, eps, rules)
    win = np.ascontiguousarray(full[:, :64]).reshape(-1)
    for src in (0, 1):
        b = lib.DeviceBatch(ctx, win, lens, src, stride=64)
        r = lib.DeviceResult(ctx, n)
        s = ctx.stream()
        nrules = ctx.rule_count()
        ctx.classify(b, r, s)
        with pytest.raises(lib.UsnError, match="EINVAL"):
            ctx.finalize(b, r, s)
        if src == 1:
            # nothing learned was applied, and the batch is still pending:
            # registry calls are busy until a finalize with a reader succeeds
            with pytest.raises(lib.UsnError, match="EBUSY"):
                ctx.rule_count()
            want = o.forward_batch(1, full.reshape(-1), lens, stride=FULL)
            ctx.set_frame_reader(lambda s_, i: full[i, :int(lens[i])].tobytes())
            ctx.finalize(b, r, s)
            got = r.decisions()
            assert np.array_equal(got & katrun.PARITY_MASK, want & katrun.PARITY_MASK)
            assert ctx.rule_count() == o.rule_count()
            ctx.set_frame_reader(None)
    ctx.close()


def test_window_validation():
    """window < 64, or a window larger than the stride, is an invalid batch."""
    from usnetd_amd import lib
    ctx = lib.Ctx(0)
    ctx.endpoint_add(0, 0, None)
    full, lens, _ = _frames(64, 3)
    win = np.ascontiguousarray(full[:, :64]).reshape(-1)
    r = lib.DeviceResult(ctx, 64)
    for stride, window in ((64, 80), (64, 32), (128, 129)):
        b = lib.DeviceBatch(ctx, np.zeros(64 * stride, np.uint8), lens, 0, stride=stride, window=window)
        with pytest.raises(lib.UsnError, match="EINVAL"):
            ctx.classify(b, r, None)
    b = lib.DeviceBatch(ctx, win, lens, 0, stride=64, window=64)
    ctx.classify(b, r, None)
    ctx.close()


def test_tx_redo_after_refused_finalize_keeps_host_tail_cache(coracle_mod):
    """ring k's finalize runs a host tail that leaves a
    carried cache the device chain does not (its last frame's ports lie past
    the window: UNKNOWN on the device, retained on the host); ring k + 1,
    enqueued before it, is redone from that cache.  A finalize of ring k + 1
    refused for want of a frame reader must not lose it: ring k + 1's first
    frame repeats ring k's last PacketInfo with a dmac outside the bridge, so
    only the host tail's cache (a hit: ring k's last decision) gives the
    oracle's decision; the device chain's would send it to the NIC."""
    from usnetd_amd import lib, traffic
    n = 2048
    fa, la, ihl = _frames(n, 61)
    fb, lb, _ = _frames(n, 62)
    # an IHL 15 UDP frame to an even pipe port (7000 + k, k even: a UDP rule of pipe 2 + k)
    dp = fa[:, 76].astype(np.int64) * 256 + fa[:, 77]
    j = int(np.nonzero((ihl == 15) & (fa[:, 23] == 17) & (dp >= 7000) & (dp < 7016) & (dp % 2 == 0))[0][0])
    fa[n - 1], la[n - 1] = fa[j], la[j]
    fa[n - 1, 0:6] = np.frombuffer(traffic.REMMAC, np.uint8)     # in the bridge: get_endpoint
    fb[0], lb[0] = fa[n - 1], la[n - 1]
    fb[0, 0:6] = np.frombuffer(traffic.NICMAC, np.uint8)         # not in the bridge
    eps, rules = _setup()
    ctx = lib.Ctx(0)
    o = coracle_mod.Oracle()
    _install(ctx, o, eps, rules)
    want_a = o.forward_batch(1, fa.reshape(-1), la, stride=FULL)
    want_b = o.forward_batch(1, fb.reshape(-1), lb, stride=FULL)
    assert (want_b[0] >> 16) & 0xF == lib.CLS_EP          # the cache hit on ring k's last frame
    s = ctx.stream()
    ba = lib.DeviceBatch(ctx, np.ascontiguousarray(fa[:, :64]).reshape(-1), la, 1, stride=64)
    bb = lib.DeviceBatch(ctx, np.ascontiguousarray(fb[:, :64]).reshape(-1), lb, 1, stride=64)
    ra, rb = lib.DeviceResult(ctx, n), lib.DeviceResult(ctx, n)
    ctx.classify(ba, ra, s)
    ctx.classify(bb, rb, s)                              # before ring k's finalize
    cur = {"f": fa, "l": la}
    ctx.set_frame_reader(lambda s_, i: cur["f"][i, :int(cur["l"][i])].tobytes())
    ctx.finalize(ba, ra, s)
    assert np.array_equal(ra.decisions() & katrun.PARITY_MASK, want_a & katrun.PARITY_MASK)
    ctx.set_frame_reader(None)
    with pytest.raises(lib.UsnError, match="EINVAL"):
        ctx.finalize(bb, rb, s)                          # refused: ring k + 1 stays pending
    cur.update(f=fb, l=lb)
    ctx.set_frame_reader(lambda s_, i: cur["f"][i, :int(cur["l"][i])].tobytes())
    info = ctx.finalize(bb, rb, s)
    assert info.n_host == n                              # redone from its first frame
    got = rb.decisions()
    mism = np.nonzero((got & katrun.PARITY_MASK) != (want_b & katrun.PARITY_MASK))[0]
    assert mism.size == 0, "first mismatches %s: got %s want %s" % (
        mism[:5], [hex(x) for x in got[mism[:5]]], [hex(x) for x in want_b[mism[:5]]])
    assert ctx.rule_count() == o.rule_count()
    ctx.close()
