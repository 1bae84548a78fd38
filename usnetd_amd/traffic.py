"""Synthetic workloads of the BASELINE.json configurations (numpy, vectorized).

  c1  4-rule table (DEBUG_PORTS TCP:22 + 3 static pipes, eval/enp6s0f0config),
      64 B UDP to 169.254.137.191:3333 (eval/Makefile:18); variants "fixed"
      (pkt-gen: one 5-tuple) and "rand" (random source port)
  c2  64 B IPv4/UDP, 16 listening rules, 90 % hit                (bench workload)
  c3  IMIX 64/576/1500 B (7:4:1), TCP/UDP/ICMP 45/45/10, 1024 rules
      (512 listening + 512 connected), 2048 B stride (netmap slots)
  c4  IPv4 70 % / IPv6 10 % / ARP 10 % / 802.1Q 10 %, 4096 rules
  c5  64 B, 65536 rules (16 IPs x 2048 listening ports + 32768 connected)
  c5x c5 with the connected rules on 64 of the listening ports (overflow-heavy)

Frames are generated directly into their HBM layout (fixed stride); every
frame start has 64 readable bytes.  Data is synthetic (no captures).  A
config's rule table is fixed (its own seed); `seed` varies only the traffic,
so every rx queue of a bench hits the one installed table.
"""
from __future__ import annotations

import dataclasses

import numpy as np

LOCAL = 0xA9FE89BF            # 169.254.137.191 (eval/Makefile:18)
NICMAC = bytes.fromhex("001b214b508c")
REMMAC = bytes.fromhex("001b214b508d")
EP_NIC, EP_HOST, EP_PIPE = 0, 1, 2
TCP, UDP, ICMP = 6, 17, 1


@dataclasses.dataclass
class Config:
    name: str
    n: int
    frames: np.ndarray        # flat uint8, n * stride (+ 64 pad)
    lens: np.ndarray          # uint16
    stride: int
    src: int                  # source endpoint (0 = the NIC: rx direction)
    endpoints: list           # (id, kind, for_nic)
    rules: list               # (want dict, owner, sticky)
    bridge: list = dataclasses.field(default_factory=list)

    def window(self, i):
        return bytes(self.frames[i * self.stride:i * self.stride + int(self.lens[i])])


def _want(dst, proto, dport=None, src=None, sport=None):
    return {"dst": int(dst), "proto": int(proto), "dport": dport, "src": src, "sport": sport}


def _u16be(H, col, v):
    v = np.asarray(v, dtype=np.uint32)
    H[:, col] = (v >> 8) & 0xFF
    H[:, col + 1] = v & 0xFF


def _u32be(H, col, v):
    v = np.asarray(v, dtype=np.uint64)
    for k in range(4):
        H[:, col + k] = (v >> (24 - 8 * k)) & 0xFF


def _layout(H, lens, stride, pad=64):
    n = H.shape[0]
    buf = np.zeros(n * stride + pad, dtype=np.uint8)
    view = buf[:n * stride].reshape(n, stride)
    view[:, :H.shape[1]] = H
    return buf


def build_ipv4(n, dst, src, proto, sport, dport, lens, ident=None, ff=0x4000, rng=None,
               dmac=NICMAC, smac=REMMAC, hdr=64):
    """IPv4 frames: header window (n, hdr) with TCP/UDP ports where proto has them."""
    H = np.zeros((n, hdr), dtype=np.uint8)
    H[:, 0:6] = np.frombuffer(dmac, np.uint8)
    H[:, 6:12] = np.frombuffer(smac, np.uint8)
    _u16be(H, 12, 0x0800)
    H[:, 14] = 0x45
    tl = np.asarray(lens, dtype=np.uint32) - 14
    _u16be(H, 16, tl)
    _u16be(H, 18, np.arange(n, dtype=np.uint32) & 0xFFFF if ident is None else ident)
    _u16be(H, 20, ff)
    H[:, 22] = 64
    H[:, 23] = np.asarray(proto, dtype=np.uint8) if np.ndim(proto) else proto
    _u32be(H, 26, src)
    _u32be(H, 30, dst)
    proto_a = np.broadcast_to(np.asarray(proto), (n,))
    has = (proto_a == TCP) | (proto_a == UDP)
    _u16be(H, 34, np.where(has, sport, 0x0800))          # ICMP: type 8 code 0
    _u16be(H, 36, np.where(has, dport, 0))
    is_udp = proto_a == UDP
    _u16be(H, 38, np.where(is_udp, tl - 20, 0))
    is_tcp = proto_a == TCP
    H[:, 46] = np.where(is_tcp, 0x50, H[:, 46])
    H[:, 47] = np.where(is_tcp, 0x10, H[:, 47])
    return H


def _base_endpoints(n_pipes):
    eps = [(0, EP_NIC, None), (1, EP_HOST, 0)]
    eps += [(2 + k, EP_PIPE, 0) for k in range(n_pipes)]
    return eps


def c1(n=1 << 16, variant="rand", seed=1):
    rng = np.random.default_rng(seed)
    rules = [(_want(LOCAL, TCP, 22), 1, True), (_want(LOCAL, UDP, 3333), 2, True),
             (_want(LOCAL, UDP, 3334), 3, True), (_want(LOCAL, UDP, 3335), 4, True)]
    sport = np.full(n, 1234, np.uint32) if variant == "fixed" else rng.integers(1024, 65536, n)
    lens = np.full(n, 64, np.uint16)
    src = np.full(n, 0xA9FE89BE, np.uint64)   # 169.254.137.190
    H = build_ipv4(n, LOCAL, src, UDP, sport, 3333, lens,
                   ident=np.zeros(n, np.uint32) if variant == "fixed" else None)
    return Config("c1-" + variant, n, _layout(H, lens, 64), lens, 64, 0, _base_endpoints(3), rules)


def c2(n=1 << 20, seed=2):
    """1M x 64 B IPv4/UDP, 16 rules (UDP 3333..3348 -> pipes 2..17), 90 % hit."""
    rng = np.random.default_rng(seed)
    rules = [(_want(LOCAL, UDP, 3333 + k), 2 + k, False) for k in range(16)]
    hit = rng.random(n) < 0.9
    dport = np.where(hit, 3333 + rng.integers(0, 16, n), rng.integers(20000, 30000, n))
    sport = rng.integers(1024, 65536, n)
    src = (10 << 24) | rng.integers(0, 1 << 16, n).astype(np.uint64)
    lens = np.full(n, 64, np.uint16)
    H = build_ipv4(n, LOCAL, src, UDP, sport, dport, lens)
    return Config("c2", n, _layout(H, lens, 64), lens, 64, 0, _base_endpoints(16), rules)


def _listen_conn_rules(rng, n_listen, n_conn, n_ips, n_ep, protos=(TCP, UDP), icmp=True,
                       conn_ports=(40000, 50000)):
    ips = LOCAL - np.arange(n_ips, dtype=np.int64)
    rules, listen, conn = [], [], []
    seen = set()
    if icmp:
        for j in range(n_ips):
            rules.append((_want(ips[j], ICMP), 2 + (j % n_ep), False))
    k = 0
    while len(listen) < n_listen:
        ip = int(ips[k % n_ips])
        proto = protos[(k // n_ips) % len(protos)]
        port = 1000 + k // (n_ips * len(protos))
        k += 1
        key = (ip, proto, port)
        if key in seen:
            continue
        seen.add(key)
        listen.append(key)
        rules.append((_want(ip, proto, port), 2 + int(rng.integers(0, n_ep)), False))
    while len(conn) < n_conn:
        ip = int(ips[rng.integers(0, n_ips)])
        proto = protos[int(rng.integers(0, len(protos)))]
        port = int(rng.integers(*conn_ports))
        rsrc = (10 << 24) | int(rng.integers(0, 1 << 20))
        rsport = int(rng.integers(1024, 65536))
        key = (ip, proto, port, rsrc, rsport)
        if key in seen:
            continue
        seen.add(key)
        conn.append(key)
        rules.append((_want(ip, proto, port, rsrc, rsport), 2 + int(rng.integers(0, n_ep)), False))
    return ips, rules, listen, conn


def _ipv4_mix(rng, n, ips, listen, conn, p_icmp, hit_rate=0.9):
    """Per-frame (dst, src, proto, sport, dport) hitting listen/conn rules at hit_rate."""
    listen = np.array(listen, dtype=np.int64).reshape(-1, 3)
    conn = np.array(conn, dtype=np.int64).reshape(-1, 5)
    kind = rng.random(n)
    icmp = kind < p_icmp
    hit = rng.random(n) < hit_rate
    use_conn = rng.random(n) < (len(conn) / max(1, len(conn) + len(listen)))
    li = rng.integers(0, max(1, len(listen)), n)
    ci = rng.integers(0, max(1, len(conn)), n)
    dst = np.where(use_conn, conn[ci, 0], listen[li, 0]).astype(np.uint64)
    proto = np.where(use_conn, conn[ci, 1], listen[li, 1]).astype(np.uint32)
    dport = np.where(use_conn, conn[ci, 2], listen[li, 2]).astype(np.uint32)
    src = np.where(use_conn, conn[ci, 3], (10 << 24) | rng.integers(0, 1 << 20, n)).astype(np.uint64)
    sport = np.where(use_conn, conn[ci, 4], rng.integers(1024, 65536, n)).astype(np.uint32)
    miss = ~hit
    dport = np.where(miss, rng.integers(20000, 30000, n), dport).astype(np.uint32)
    proto = np.where(icmp, ICMP, proto).astype(np.uint32)
    dst = np.where(icmp, ips[rng.integers(0, len(ips), n)], dst).astype(np.uint64)
    return dst, src, proto, sport, dport


def c3(n=1 << 18, seed=3, stride=2048):
    rng = np.random.default_rng(seed)
    ips, rules, listen, conn = _listen_conn_rules(np.random.default_rng(3), 504, 512, 8, 64)
    dst, src, proto, sport, dport = _ipv4_mix(rng, n, ips, listen, conn, p_icmp=0.10)
    sizes = rng.choice(np.array([64, 576, 1500]), size=n, p=[7 / 12, 4 / 12, 1 / 12])
    lens = sizes.astype(np.uint16)
    H = build_ipv4(n, dst, src, proto, sport, dport, lens)
    return Config("c3", n, _layout(H, lens, stride), lens, stride, 0, _base_endpoints(64), rules)


def c4(n=1 << 18, seed=4):
    rng = np.random.default_rng(seed)
    ips, rules, listen, conn = _listen_conn_rules(np.random.default_rng(4), 2048 - 32, 2048, 32, 256)
    dst, src, proto, sport, dport = _ipv4_mix(rng, n, ips, listen, conn, p_icmp=0.1)
    lens = np.full(n, 64, np.uint16)
    H = build_ipv4(n, dst, src, proto, sport, dport, lens)
    kind = rng.random(n)
    v6 = (kind >= 0.70) & (kind < 0.80)
    arp = (kind >= 0.80) & (kind < 0.90)
    vlan = kind >= 0.90
    H[v6, 12], H[v6, 13] = 0x86, 0xDD
    H[v6, 14] = 0x60
    H[arp, 12], H[arp, 13] = 0x08, 0x06
    H[arp, 0:6] = 0xFF
    # 802.1Q: tag then the IPv4 packet shifted by 4 bytes
    if vlan.any():
        inner = H[vlan, 12:60].copy()
        H[vlan, 12], H[vlan, 13] = 0x81, 0x00
        H[vlan, 14], H[vlan, 15] = 0x00, 0x05
        H[vlan, 16:64] = inner
    return Config("c4", n, _layout(H, lens, 64), lens, 64, 0, _base_endpoints(256), rules)


def c5(n=1 << 23, seed=5, n_ep=1000):
    """n_ep: endpoints owning the rules (4093 fills the 12-bit netmap pipe id
    space, USN_MAX_ENDPOINTS)."""
    rng = np.random.default_rng(seed)
    ips, rules, listen, conn = _listen_conn_rules(np.random.default_rng(5), 16 * 2048, 32768, 16, n_ep,
                                                  icmp=False)
    dst, src, proto, sport, dport = _ipv4_mix(rng, n, ips, listen, conn, p_icmp=0.0)
    lens = np.full(n, 64, np.uint16)
    H = build_ipv4(n, dst, src, proto, sport, dport, lens)
    return Config("c5", n, _layout(H, lens, 64), lens, 64, 0, _base_endpoints(n_ep), rules)


def c5x(n=1 << 23, seed=5, n_ep=1000):
    """c5 with the connected rules on the listening ports 1000..1063 (a server's
    accepted connections): ~16 connected rules share each of those projections
    with a listening rule, so most frames of the projection table's path also
    read its overflow table X (its worst case, not a BASELINE config)."""
    rng = np.random.default_rng(seed)
    ips, rules, listen, conn = _listen_conn_rules(np.random.default_rng(5), 16 * 2048, 32768, 16, n_ep,
                                                  icmp=False, conn_ports=(1000, 1064))
    dst, src, proto, sport, dport = _ipv4_mix(rng, n, ips, listen, conn, p_icmp=0.0)
    lens = np.full(n, 64, np.uint16)
    H = build_ipv4(n, dst, src, proto, sport, dport, lens)
    return Config("c5x", n, _layout(H, lens, 64), lens, 64, 0, _base_endpoints(n_ep), rules)


def c4tx(n=1 << 18, seed=6, host_at=None, host_src=0):
    """c4's mix SENT by the host endpoint (tx: find_forward with incoming ==
    false, endpoint.rs:194-256), the "ADD_MACS learned-MAC path" of
    BASELINE.json configs[3]: the bridge is prefilled with 64 endpoint MACs
    (main.rs:450-462); a quarter of the unicast source MACs are not yet in it
    (learned), some are multicast (never learned); half of the frames go to a
    bridged MAC (rule lookup), half to the gateway (Target::Nic); every new flow
    learns its answer rule (to_want); 30 % of frames repeat the previous one
    (decision cache).  host_at: frame indices replaced by a DHCP request (its
    effect on the NIC is ordered host work) from IPv4 source host_src (any
    0.0.0.0/8 address is unspecified in smoltcp 0.7.0, pkt.rs:46; another
    source makes the frame an ordinary one that learns its answer rule)."""
    cfg = c4(n, seed)
    rng = np.random.default_rng(seed + 100)
    stride = cfg.stride
    V = cfg.frames[:n * stride].reshape(n, stride)
    to_bridge = rng.random(n) < 0.5
    # to the gateway: the local side sends (swap addresses and ports); to a
    # bridged MAC: endpoint-to-endpoint traffic addressed to the rules' side
    ip = (V[:, 12] == 0x08) & (V[:, 13] == 0x00) & ~to_bridge
    a, b = V[ip, 26:30].copy(), V[ip, 30:34].copy()
    V[ip, 26:30], V[ip, 30:34] = b, a
    a, b = V[ip, 34:36].copy(), V[ip, 36:38].copy()
    V[ip, 34:36], V[ip, 36:38] = b, a
    bridged = np.zeros((64, 6), np.uint8)
    bridged[:, 0] = 0x02
    bridged[:, 5] = np.arange(64)
    bridged[:, 4] = 0xB0
    pool = np.zeros((256, 6), np.uint8)
    pool[:, 0] = 0x02
    pool[:, 4] = 0xC0
    pool[:, 5] = np.arange(256)
    pool[:192] = np.concatenate([bridged, bridged, bridged])[:192]   # in the bridge
    pool[250:, 0] = 0x03                                             # multicast: never learned
    arp = (V[:, 12] == 0x08) & (V[:, 13] == 0x06)
    dmac = np.where(to_bridge[:, None], bridged[rng.integers(0, 64, n)],
                    np.frombuffer(REMMAC, np.uint8)[None, :])
    dmac[arp] = 0xFF
    V[:, 0:6] = dmac
    V[:, 6:12] = pool[rng.integers(0, 256, n)]
    rep = rng.random(n) < 0.3
    rep[0] = False
    idx = np.arange(n)
    idx[rep] = 0
    idx = np.maximum.accumulate(np.where(rep, 0, idx))
    V[:] = V[idx]
    lens = cfg.lens[idx].copy()
    if host_at:
        req = build_ipv4(1, 0xFFFFFFFF, host_src, UDP, 68, 67, np.array([64], np.uint16),
                         dmac=b"\xff" * 6, smac=bytes(pool[3]))
        for i in host_at:
            V[i, :64] = req[0]
            lens[i] = 64
    return Config("c4tx", n, cfg.frames, lens, stride, 1, cfg.endpoints, cfg.rules,
                  bridge=[bytes(m) for m in bridged])


def c1fixed(n=1 << 16, seed=1):
    """c1 with one 5-tuple (pkt-gen style): nearly every frame is a cache hit."""
    return c1(n=n, variant="fixed", seed=seed)


CONFIGS = {"c1": c1, "c1fixed": c1fixed, "c2": c2, "c3": c3, "c4": c4, "c5": c5, "c4tx": c4tx, "c5x": c5x}


def config(name, n=None, seed=None, **kw):
    f = CONFIGS[name]
    if n is not None:
        kw["n"] = n
    if seed is not None:
        kw["seed"] = seed
    return f(**kw)


def extra_nics(cfg: Config, k: int, ctx=None):
    """Ids of k more NIC endpoints (further rx queues) after the config's own;
    registers them in ctx when given.  The rule table is shared: get_endpoint
    does not check which NIC a rule's owner belongs to (endpoint.rs:307-338)."""
    first = max(e[0] for e in cfg.endpoints) + 1
    ids = list(range(first, first + k))
    if ctx is not None:
        for i in ids:
            ctx.endpoint_add(i, EP_NIC, None)
    return ids


def install_ctx(ctx, cfg: Config):
    from .lib import make_want
    for eid, kind, for_nic in cfg.endpoints:
        ctx.endpoint_add(eid, kind, for_nic)
    for w, owner, sticky in cfg.rules:
        ctx.add_match(make_want(w["dst"], w["proto"], w["dport"], w["src"], w["sport"]), owner, sticky)
    for m in cfg.bridge:
        ctx.bridge_add(m)
