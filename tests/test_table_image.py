"""CPU tests of the device rule image (perfect hash, usn_internal.h), built
from the registry by the product library on a registry-only context
(USN_HOST_ONLY) and probed on the host with the device's own hash functions
(test hook usn_debug_image_probe, which computes exactly what ph_probe in
usn_device.hip computes).

The image must answer get_endpoint's two exact-match lookups
(/root/reference/src/endpoint.rs:307-338): every rule key1 or key2 can hit is
found with its owner; nothing else is (other Want shapes never match a frame,
SURVEY.md A.3.6); and a probe reads one displacement and one slot."""
import ctypes as C

import numpy as np
import pytest

from usnetd_amd import lib, traffic

VALID = 1 << 11
META_MASK = 0x0FFF


def _ctx(test_build=False):
    L = lib.load(lib.TEST_LIB_PATH) if test_build else lib.load()
    h = C.c_void_p()
    assert L.usn_ctx_create(-1, C.byref(h)) == 0
    L.usn_debug_image_probe.restype = C.c_int64
    L.usn_debug_image_probe.argtypes = [C.c_void_p, C.c_int] + [C.c_uint32] * 4
    L.usn_debug_image_info.argtypes = [C.c_void_p, C.c_void_p]
    return L, h.value


def _packed(w):
    """(table, x, y, z, meta) of a Want as the device packs it."""
    p = w.present & 7
    z = (w.dst_port if p & 1 else 0) | ((w.src_port if p & 4 else 0) << 16)
    y = w.src_addr if p & 2 else 0
    meta = (w.protocol & 0xFF) | (p << 8) | VALID
    table = 0 if p in (2, 7) else 1 if p in (0, 1) else -1
    return table, w.dst_addr, y, z, meta


def _info(L, h):
    out = (C.c_uint32 * 10)()
    assert L.usn_debug_image_info(h, out) == 0
    return list(out)[:6]


def _uinfo(L, h):
    out = (C.c_uint32 * 10)()
    assert L.usn_debug_image_info(h, out) == 0
    return list(out)[6:8]


def test_image_finds_every_rule_c5():
    L, h = _ctx()
    cfg = traffic.config("c5", n=16)
    for eid, kind, for_nic in cfg.endpoints:
        assert L.usn_endpoint_add(h, eid, kind, -1 if for_nic is None else for_nic) == 0
    ws = []
    for w, owner, sticky in cfg.rules:
        want = lib.make_want(w["dst"], w["proto"], w["dport"], w["src"], w["sport"])
        assert L.usn_add_match(h, C.byref(want), owner, int(sticky)) == 1
        ws.append((want, owner))
    m0, g0, m1, g1, units, pmask = _info(L, h)
    assert pmask == 7                             # K1, K2, and U built
    assert m0 >= 32768 and m1 >= 32768 and m0 < 32768 / 0.49 and m1 < 32768 / 0.49
    mu, mx = _uinfo(L, h)
    assert (mu + mx) * 16 < 2.2 * 2 ** 20        # what rx reads is L2-resident (4 MiB per XCD)
    assert mu >= 32768 + 30000 and mx < 4000     # c5: ~5 % of connected rules share a projection
    for want, owner in ws:
        t, x, y, z, meta = _packed(want)
        got = L.usn_debug_image_probe(h, t, x, y, z, meta)
        assert got and (got >> 16) == owner and (got & META_MASK) == meta
        # never in the other table
        assert L.usn_debug_image_probe(h, 1 - t, x, y, z, meta) == 0
    rng = np.random.default_rng(3)
    for _ in range(20000):   # random keys of both shapes miss
        x = int(rng.integers(0, 2 ** 32))
        z = int(rng.integers(0, 2 ** 32))
        assert L.usn_debug_image_probe(h, 0, x, 7, z, 6 | (7 << 8) | VALID) == 0
        assert L.usn_debug_image_probe(h, 1, x, 0, z & 0xFFFF, 17 | (1 << 8) | VALID) == 0
    L.usn_ctx_destroy(h)


def test_image_shapes_owner_flags_and_updates():
    """Other Want shapes stay out of the image; NIC-owned rules carry the NIC
    bit (the exclusion of endpoint.rs:328-336); the image follows AddMatch /
    RemoveMatch / endpoint removal."""
    L, h = _ctx()
    assert L.usn_endpoint_add(h, 0, 0, -1) == 0      # NIC
    assert L.usn_endpoint_add(h, 1, 1, 0) == 0       # host ring
    assert L.usn_endpoint_add(h, 2, 2, 0) == 0       # pipe
    w_listen = lib.make_want("10.0.0.1", 6, 80)
    w_icmp = lib.make_want("10.0.0.1", 1)
    w_conn = lib.make_want("10.0.0.1", 6, 80, "10.9.9.9", 4444)
    w_src_only = lib.make_want("10.0.0.1", 1, None, "10.9.9.9")
    w_odd = lib.make_want("10.0.0.1", 6, 80, "10.9.9.9")           # dport+src, no sport
    for w, o in ((w_listen, 1), (w_icmp, 2), (w_conn, 2), (w_src_only, 1), (w_odd, 2)):
        assert L.usn_add_match(h, C.byref(w), o, 0) == 1
    for w, o in ((w_listen, 1), (w_icmp, 2), (w_conn, 2), (w_src_only, 1)):
        t, x, y, z, meta = _packed(w)
        got = L.usn_debug_image_probe(h, t, x, y, z, meta)
        assert (got >> 16) == o and not got & (1 << 12)
    t, x, y, z, meta = _packed(w_odd)
    assert t == -1
    assert L.usn_debug_image_probe(h, 0, x, y, z, meta) == 0
    assert L.usn_debug_image_probe(h, 1, x, y, z, meta) == 0
    # RemoveMatch drops the key from the image
    assert L.usn_remove_match(h, C.byref(w_conn), 2) == 1
    t, x, y, z, meta = _packed(w_conn)
    assert L.usn_debug_image_probe(h, t, x, y, z, meta) == 0
    # endpoint removal drops its rules
    assert L.usn_endpoint_remove(h, 1) == 0
    t, x, y, z, meta = _packed(w_listen)
    assert L.usn_debug_image_probe(h, t, x, y, z, meta) == 0
    t, x, y, z, meta = _packed(w_icmp)
    assert (L.usn_debug_image_probe(h, t, x, y, z, meta) >> 16) == 2
    # a NIC-owned rule (usn_table_build can install one) carries the NIC bit
    rules = np.zeros(1, lib.RULE_DTYPE)
    rules[0] = (lib.ip2int("10.0.0.2"), 0, 53, 0, 17, 1, 0)
    assert L.usn_table_build(h, rules.ctypes.data, 1) == 1
    got = L.usn_debug_image_probe(h, 1, lib.ip2int("10.0.0.2"), 0, 53, 17 | (1 << 8) | VALID)
    assert got & (1 << 12) and (got >> 16) == 0
    L.usn_ctx_destroy(h)


@pytest.mark.parametrize("n", [1, 2, 3, 17, 1000, 300000, 700000])
def test_image_bulk_sizes(n):
    """usn_table_build of n random connected 5-tuples and listening ports:
    every key found, load <= 0.51, displacement groups of ~10 (~5 above 128 K
    keys); 700000 rules put ~350K keys in each table: 8 shards of ~44K keys."""
    L, h = _ctx()
    assert L.usn_endpoint_add(h, 0, 0, -1) == 0
    for e in range(1, 9):
        assert L.usn_endpoint_add(h, e, 2, 0) == 0
    rng = np.random.default_rng(n)
    rules = np.zeros(n, lib.RULE_DTYPE)
    rules["dst_addr"] = rng.integers(0, 2 ** 32, n, dtype=np.uint64)
    conn = rng.random(n) < 0.5
    rules["src_addr"] = np.where(conn, rng.integers(0, 2 ** 32, n, dtype=np.uint64), 0)
    rules["dst_port"] = rng.integers(0, 65536, n)
    rules["src_port"] = np.where(conn, rng.integers(0, 65536, n), 0)
    rules["protocol"] = rng.choice([6, 17], n)
    rules["present"] = np.where(conn, 7, 1)
    rules["endpoint"] = rng.integers(1, 9, n)
    got_n = L.usn_table_build(h, rules.ctypes.data, n)
    assert got_n >= 1
    m0, g0, m1, g1, units, pmask = _info(L, h)
    n_conn, n_list = int(conn.sum()), int((~conn).sum())
    if n > 100:
        # tables above 64K keys are sharded: each shard sized for the largest
        # (up to ~1300 keys the load rises to 0.7 so that the image stays in LDS)
        lo = 0.71 if n <= 1400 else 0.51
        assert n_conn / lo <= m0 <= 1.05 * n_conn / 0.49 + 64
        assert n_list / lo <= m1 <= 1.05 * n_list / 0.49 + 64
        # ~10 keys per displacement; 5 beyond U's range (128 K keys: the image
        # is then read from L2 only, and small groups place twice as fast)
        per = 5 if n > 131072 else 10
        assert (n_conn + per - 1) // per <= g0 <= 1.05 * n_conn / per + 64
        assert (n_list + per - 1) // per <= g1 <= 1.05 * n_list / per + 64
    idx = rng.choice(n, min(n, 5000), replace=False)
    for i in idx:
        r = rules[i]
        p = int(r["present"])
        t = 0 if p == 7 else 1
        z = int(r["dst_port"]) | (int(r["src_port"]) << 16 if p == 7 else 0)
        meta = int(r["protocol"]) | (p << 8) | VALID
        got = L.usn_debug_image_probe(h, t, int(r["dst_addr"]), int(r["src_addr"]), z, meta)
        assert got, i
        # duplicates keep the first owner (HashMap::entry().or_insert)
        assert (got >> 16) in range(1, 9)
    L.usn_ctx_destroy(h)


def _rx_probe(L, h, dst, src, proto, has, dport, sport):
    out = (C.c_uint32 * 4)()
    r = L.usn_debug_image_probe_rx(h, dst, src, proto, has, dport, sport, out)
    return r, list(out)


HAS_PORTS = (6, 17, 33, 132, 136)


@pytest.mark.parametrize("seed", range(4))
def test_projection_image_equals_k1_k2(seed):
    """The projection table U (+ its overflow X) that the rx kernel reads
    answers get_endpoint's two lookups (endpoint.rs:317-327) exactly as the
    K1 / K2 tables do: every key1 / key2 of small address, port and protocol
    pools, against rules of every Want shape (several K1 rules per projection,
    K1 without K2 and the reverse, NIC-owned rules, shapes no frame matches)."""
    import random
    rng = random.Random(seed)
    L, h = _ctx()
    L.usn_debug_image_probe_rx.argtypes = [C.c_void_p] + [C.c_uint32] * 6 + [C.c_void_p]
    L.usn_debug_image_probe_rx.restype = C.c_int
    assert L.usn_endpoint_add(h, 0, 0, -1) == 0      # NIC
    assert L.usn_endpoint_add(h, 1, 1, 0) == 0       # host ring
    for e in range(2, 9):
        assert L.usn_endpoint_add(h, e, 2, 0) == 0
    assert L.usn_endpoint_add(h, 9, 0, -1) == 0      # a second NIC
    ips_s = ("10.0.0.1", "10.0.0.2", "0.0.0.0", "255.255.255.255")
    ips = [lib.ip2int(s) for s in ips_s]
    ports = [0, 22, 80, 443, 3333, 65535]
    protos = [6, 17, 1, 132, 50, 33, 136, 0]
    # usn_table_build: NIC owners are allowed there (AddMatch from a NIC panics, main.rs:287-289)
    nr = rng.choice([40, 400, 1500])
    rules = np.zeros(nr, lib.RULE_DTYPE)
    for i in range(nr):
        present = rng.choice([0, 1, 2, 7, 7, 7, 3, 5, 4])
        rules[i] = (rng.choice(ips), rng.choice(ips) if present & 2 else 0,
                    rng.choice(ports) if present & 1 else 0, rng.choice(ports) if present & 4 else 0,
                    rng.choice(protos), present, rng.choice(range(10)))
    assert L.usn_table_build(h, rules.ctypes.data, nr) > 10
    n = nic = 0
    for dst in ips:
        for src in ips:
            for proto in protos:
                combos = [(0, 0, 0)] + ([(1, d, s) for d in ports for s in ports] if proto in HAS_PORTS else [])
                for has, dport, sport in combos:
                    r, out = _rx_probe(L, h, dst, src, proto, has, dport, sport)
                    assert r == 1
                    assert out[:2] == out[2:], (dst, src, proto, has, dport, sport, out)
                    n += (out[2] != 0) + (out[3] != 0)
                    nic += (out[2] == 0x11FFE) + (out[3] == 0x11FFE)
    assert n > 10 and nic > 0
    _, _, _, _, _, pmask = _info(L, h)
    assert pmask & 4
    L.usn_ctx_destroy(h)


def test_projection_image_off(monkeypatch):
    """USN_NO_PROJ (A/B, the test build): no U is built; the K1 / K2 path
    answers alone."""
    monkeypatch.setenv("USN_NO_PROJ", "1")
    L, h = _ctx(test_build=True)
    L.usn_debug_image_probe_rx.argtypes = [C.c_void_p] + [C.c_uint32] * 6 + [C.c_void_p]
    assert L.usn_endpoint_add(h, 0, 0, -1) == 0
    assert L.usn_endpoint_add(h, 2, 2, 0) == 0
    w = lib.make_want("10.0.0.1", 6, 80)
    assert L.usn_add_match(h, C.byref(w), 2, 0) == 1
    r, out = _rx_probe(L, h, lib.ip2int("10.0.0.1"), 5, 6, 1, 80, 1234)
    assert r == 0 and out[3] == 0x10002 and out[0] == 0
    L.usn_ctx_destroy(h)


def test_projection_image_only_unmatchable_rules():
    """Rules no frame can hit (ports on a protocol without ports) leave U
    unbuilt: the K1 / K2 path answers (a miss), never an empty U table."""
    L, h = _ctx()
    L.usn_debug_image_probe_rx.argtypes = [C.c_void_p] + [C.c_uint32] * 6 + [C.c_void_p]
    assert L.usn_endpoint_add(h, 0, 0, -1) == 0
    assert L.usn_endpoint_add(h, 2, 2, 0) == 0
    w = lib.make_want("0.0.0.0", 50, 0)          # ESP has no ports: never matched
    assert L.usn_add_match(h, C.byref(w), 2, 0) == 1
    r, out = _rx_probe(L, h, 0, 0, 6, 1, 0, 0)
    assert r == 0 and out == [0, 0, 0, 0]
    _, _, _, _, _, pmask = _info(L, h)
    assert pmask & 4 == 0
    L.usn_ctx_destroy(h)


def _stats(L, h, refresh=1):
    f = L.usn_debug_image_stats
    f.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    out = (C.c_uint64 * 4)()
    assert f(h, refresh, out) == 0
    return list(out)


def _model_rx(reg, nics, dst, src, proto, has, dport, sport):
    """get_endpoint's two lookups (endpoint.rs:317-327) on a dict registry,
    normalised as usn_debug_image_probe_rx: 0 miss, 0x10000 | owner, 0x11FFE NIC."""
    def norm(k):
        if k not in reg:
            return 0
        o = reg[k]
        return 0x11FFE if o in nics else 0x10000 | o
    if has:
        k1 = (dst, src, dport, sport, proto, 7)
        k2 = (dst, 0, dport, 0, proto, 1)
    else:
        k1 = (dst, src, 0, 0, proto, 2)
        k2 = (dst, 0, 0, 0, proto, 0)
    return [norm(k1), norm(k2)]


@pytest.mark.parametrize("seed", range(3))
def test_incremental_image_follows_add_remove(seed):
    """AddMatch / RemoveMatch between batches update the image in place
    (a rebuild per change stalls the data path): after every
    change, U/X and K1/K2 answer get_endpoint's lookups exactly as the
    registry does, with small pools so that keys share projections (inline
    rule, X, the K2 owner), and almost no change rebuilds the image."""
    import random
    rng = random.Random(100 + seed)
    L, h = _ctx()
    L.usn_debug_image_probe_rx.argtypes = [C.c_void_p] + [C.c_uint32] * 6 + [C.c_void_p]
    L.usn_debug_image_probe_rx.restype = C.c_int
    assert L.usn_endpoint_add(h, 0, 0, -1) == 0      # NIC
    for e in range(1, 9):
        assert L.usn_endpoint_add(h, e, 2, 0) == 0
    ips = [lib.ip2int(s) for s in ("10.0.0.1", "10.0.0.2", "10.0.0.3", "0.0.0.0")]
    ports = [22, 80, 443, 3333, 5000, 65535]
    protos = [6, 17, 1, 132]
    reg = {}
    # a base table from usn_table_build (one full build), plus filler rules so
    # that groups are realistic
    base = np.zeros(3000, lib.RULE_DTYPE)
    for i in range(3000):
        base[i] = (rng.getrandbits(32), rng.getrandbits(32), rng.randrange(65536), rng.randrange(65536),
                   6, 7, rng.randrange(1, 9))
    L.usn_table_build(h, base.ctypes.data, 3000)
    for r in base:
        reg.setdefault((int(r[0]), int(r[1]), int(r[2]), int(r[3]), int(r[4]), 7), int(r[6]))
    b0, u0, _, _ = _stats(L, h)
    nops = 400
    for op in range(nops):
        proto = rng.choice(protos)
        has = proto in HAS_PORTS and rng.random() < 0.8
        dst, src = rng.choice(ips), rng.choice(ips)
        dport, sport = rng.choice(ports), rng.choice(ports)
        conn = rng.random() < 0.6
        w = lib.make_want(dst, proto, dport if has else None, src if conn else None,
                          sport if (has and conn) else None)
        key = (dst, src if conn else 0, dport if has else 0, sport if (has and conn) else 0, proto,
               (1 if has else 0) | (2 if conn else 0) | (4 if has and conn else 0))
        owner = rng.randrange(1, 9)
        if key in reg and rng.random() < 0.7:
            rc = L.usn_remove_match(h, C.byref(w), reg[key])
            assert rc == 1
            del reg[key]
        else:
            rc = L.usn_add_match(h, C.byref(w), owner, 0)
            assert rc == (0 if key in reg else 1)
            reg.setdefault(key, owner)
        _stats(L, h)                        # a batch after each control message: image up to date
        if op % 20 == 0 or op == nops - 1:
            for dst2 in ips:
                for src2 in ips:
                    for proto2 in protos:
                        combos = [(0, 0, 0)] + ([(1, d, s2) for d in ports for s2 in ports]
                                                if proto2 in HAS_PORTS else [])
                        for hs, dp, sp in combos:
                            r, out = _rx_probe(L, h, dst2, src2, proto2, hs, dp, sp)
                            want = _model_rx(reg, {0}, dst2, src2, proto2, hs, dp, sp)
                            assert out[2:] == want, (op, dst2, src2, proto2, hs, dp, sp, out, want)
                            if r == 1:
                                assert out[:2] == want, (op, dst2, src2, proto2, hs, dp, sp, out, want)
    b1, u1, pending, _ = _stats(L, h)
    assert pending == 0
    assert u1 - u0 > 250                    # the changes went in place
    # rebuilds: a table's first key, and each ~20 % growth of the small K2
    # and X tables these pools fill (tables of a few dozen keys: microseconds)
    assert b1 - b0 <= 20, (b1 - b0, u1 - u0)
    L.usn_ctx_destroy(h)


def test_incremental_image_c5_scale():
    """c5's 65 536 rules, then 2000 new connected rules and 1000 removals one
    control message at a time: every key answers as the registry says, and
    the image was rebuilt at most a few times (usn_table_build's once)."""
    L, h = _ctx()
    L.usn_debug_image_probe_rx.argtypes = [C.c_void_p] + [C.c_uint32] * 6 + [C.c_void_p]
    L.usn_debug_image_probe_rx.restype = C.c_int
    cfg = traffic.config("c5", n=16)
    for eid, kind, for_nic in cfg.endpoints:
        assert L.usn_endpoint_add(h, eid, kind, -1 if for_nic is None else for_nic) == 0
    rules = np.zeros(len(cfg.rules), lib.RULE_DTYPE)
    for i, (w, owner, sticky) in enumerate(cfg.rules):
        want = lib.make_want(w["dst"], w["proto"], w["dport"], w["src"], w["sport"])
        rules[i] = (want.dst_addr, want.src_addr, want.dst_port, want.src_port, want.protocol,
                    want.present, owner)
    assert L.usn_table_build(h, rules.ctypes.data, len(rules)) == len(rules)
    b0, u0, _, _ = _stats(L, h)
    rng = np.random.default_rng(5)
    eps = [e for e, kind, _ in cfg.endpoints if kind != 0]
    added = []
    for i in range(2000):
        r = rules[int(rng.integers(0, len(rules)))]
        w = lib.make_want(int(r["dst_addr"]), 6, int(r["dst_port"]), int(rng.integers(1, 2 ** 32)),
                          int(rng.integers(1024, 65536)))
        o = int(rng.choice(eps))
        if L.usn_add_match(h, C.byref(w), o, 0) == 1:
            added.append((w, o))
        if i % 50 == 0:
            _stats(L, h)                    # a batch would bring the image up to date here
    removed = added[:1000]
    for w, o in removed:
        assert L.usn_remove_match(h, C.byref(w), o) == 1
    b1, u1, _, _ = _stats(L, h)
    for j, (w, o) in enumerate(added):
        r, out = _rx_probe(L, h, w.dst_addr, w.src_addr, 6, 1, w.dst_port, w.src_port)
        want = 0 if j < 1000 else 0x10000 | o
        assert r == 1 and out[0] == want and out[2] == want, (j, out)
    for i in range(0, len(rules), 97):      # the installed table still answers
        r0 = rules[i]
        if r0["present"] == 7:
            r, out = _rx_probe(L, h, int(r0["dst_addr"]), int(r0["src_addr"]), int(r0["protocol"]), 1,
                               int(r0["dst_port"]), int(r0["src_port"]))
            assert out[0] == out[2] == 0x10000 | int(r0["endpoint"])
    assert b1 - b0 <= 3, (b1 - b0, u1 - u0)
    L.usn_ctx_destroy(h)
