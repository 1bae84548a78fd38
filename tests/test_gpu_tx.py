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


@pytest.mark.parametrize("n", [1500, 1 << 16, 1 << 18])
def test_c4tx_parity(n, coracle_mod):
    from usnetd_amd import traffic
    infos = _run(traffic.config("c4tx", n=n), coracle_mod)
    assert infos[0].n_host == 0 and infos[0].n_learned > 0


@pytest.mark.parametrize("n,at", [(5000, [2500]), (1 << 16, [0]), (1 << 16, [40000, 40001, 60000])])
def test_c4tx_host_tail(n, at, coracle_mod):
    """A DHCP request (NIC.next_dhcp := S, endpoint.rs:214-226) sends the rest
    of the batch through the ordered host stage from that frame on."""
    from usnetd_amd import traffic
    infos = _run(traffic.c4tx(n=n, host_at=at), coracle_mod)
    assert infos[0].n_host == n - at[0]


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
