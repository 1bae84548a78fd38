"""Seeded random event streams for differential tests (small, pure Python).

Addresses and ports are drawn from small pools so that exact matches, cache
hits, fragments, DHCP steering, bridge learning and auto-learned answer rules
all happen often.  Used to compare the two CPU restatements with each other
and the GPU path with the C oracle.
"""
from __future__ import annotations

import random
import struct

IPS = ["169.254.137.191", "10.0.0.2", "10.0.0.3", "10.0.0.4", "127.0.0.1",
       "0.0.0.0", "255.255.255.255", "10.0.0.1", "0.1.2.3", "1.0.0.0", "10.0.0.255"]
PORTS = [22, 67, 68, 80, 443, 3333, 3334, 5555, 9999, 40000]
PROTOS = [6, 17, 17, 1, 132, 33, 136, 50]
MACS = ["00:1b:21:4b:50:8c", "00:1b:21:4b:50:8d", "02:00:00:00:00:02", "02:00:00:00:00:03",
        "02:00:00:00:00:04", "03:00:00:00:00:05", "ff:ff:ff:ff:ff:ff", "00:00:5e:00:01:01"]


def ipb(s):
    return bytes(int(x) for x in s.split("."))


def macb(s):
    return bytes(int(x, 16) for x in s.split(":"))


def rand_frame(rng: random.Random, idents) -> bytes:
    dmac, smac = macb(rng.choice(MACS)), macb(rng.choice(MACS))
    r = rng.random()
    if r < 0.04:
        return dmac + smac + b"\x08\x06" + bytes(28)
    if r < 0.06:
        return dmac + smac + b"\x88\x8e" + bytes(8)
    if r < 0.08:
        return dmac + smac + b"\x86\xdd" + bytes(40)
    if r < 0.10:
        return dmac + smac + b"\x81\x00" + bytes(30)
    if r < 0.11:
        return bytes(rng.randrange(0, 40))
    proto = rng.choice(PROTOS)
    src, dst = rng.choice(IPS), rng.choice(IPS)
    l4 = struct.pack(">HH", rng.choice(PORTS), rng.choice(PORTS))
    l4 += bytes(rng.choice([0, 0, 1, 4, 10, 20]))
    ihl = 5
    x = rng.random()
    if x < 0.05:
        ihl = rng.randrange(0, 16)
    hdr_len = max(ihl * 4, 20)
    ff = rng.choice([0x4000, 0x4000, 0x4000, 0x4000, 0x0000, 0x2000, 0x6000, 185, 0x2000 | 370])
    ident = rng.choice(idents)
    tl = hdr_len + len(l4)
    y = rng.random()
    if y < 0.03:
        tl = rng.randrange(0, tl + 30)
    h = bytearray(hdr_len)
    h[0] = (rng.choice([4, 4, 4, 6]) << 4) | ihl
    struct.pack_into(">HHH", h, 2, tl, ident, ff)
    h[9] = proto
    h[12:16] = ipb(src)
    h[16:20] = ipb(dst)
    body = bytes(h) + l4 + bytes(rng.choice([0, 0, 6]))
    return dmac + smac + b"\x08\x00" + body


def rand_want(rng):
    w = {"dst": rng.choice(IPS[:4]), "proto": rng.choice([6, 17, 1, 132, 50]),
         "dport": None, "src": None, "sport": None}
    if rng.random() < 0.8:
        w["dport"] = rng.choice(PORTS)
    if rng.random() < 0.3:
        w["src"] = rng.choice(IPS[:4])
        if w["dport"] is not None and rng.random() < 0.8:
            w["sport"] = rng.choice(PORTS)
    return w


def make_stream(seed: int, n_events: int = 400, tx_frac: float = 0.3, ops=True, n_rules=None,
                switch_p: float = 0.15, ops_p: float = 0.02):
    """Returns a fixture-shaped dict {endpoints, bridge, steps} without expectations.
    n_rules: how many initial rules (default 3..11); switch_p: chance per
    frame of a new source (runs of about 1/switch_p frames); ops_p: chance
    per event of a control op (each also ends the run)."""
    rng = random.Random(seed)
    endpoints = [[0, 0, -1], [1, 1, 0], [2, 2, 0], [3, 2, 0], [4, 3, 0], [5, 0, -1], [6, 2, 5]]
    live = {1, 2, 3, 4, 6}
    steps = []
    for _ in range(n_rules if n_rules is not None else rng.randrange(3, 12)):
        owner = rng.choice(sorted(live))
        steps.append({"op": "add_match", "want": rand_want(rng), "owner": owner, "sticky": False})
    idents = [1, 2, 3]
    src = 0
    last = None
    # DHCP requests from 0.0.0.0/8 (smoltcp 0.7.0's is_unspecified range,
    # pkt.rs:46) and, as a near miss that is an ordinary flow, from 1.0.0.0
    dhcp_reqs = [(macb("ff:ff:ff:ff:ff:ff") + macb("02:00:00:00:00:04") + b"\x08\x00" +
                  bytes([0x45, 0, 0, 48, 0, 9, 0x40, 0, 64, 17, 0, 0]) + ipb(s) +
                  ipb(d) + struct.pack(">HHHH", 68, 67, 28, 0) + bytes(20))
                 for s, d in (("0.0.0.0", "255.255.255.255"), ("0.0.0.0", "255.255.255.255"),
                              ("0.1.2.3", "10.0.0.255"), ("1.0.0.0", "255.255.255.255"))]
    dhcp_ans = (macb("ff:ff:ff:ff:ff:ff") + macb("00:1b:21:4b:50:8d") + b"\x08\x00" +
                bytes([0x45, 0, 0, 48, 0, 9, 0x40, 0, 64, 17, 0, 0]) + ipb("10.0.0.1") +
                ipb("255.255.255.255") + struct.pack(">HHHH", 67, 68, 28, 0) + bytes(20))
    for _ in range(n_events):
        if ops and rng.random() < ops_p:
            k = rng.random()
            if k < 0.5:
                steps.append({"op": "add_match", "want": rand_want(rng),
                              "owner": rng.choice(sorted(live)), "sticky": False})
            elif k < 0.8:
                steps.append({"op": "remove_match", "want": rand_want(rng),
                              "requester": rng.choice(sorted(live))})
            elif k < 0.9:
                steps.append({"op": "frag_clear"})
            elif len(live) > 2:
                victim = rng.choice(sorted(live - {1}))
                live.discard(victim)
                steps.append({"op": "remove_endpoint", "id": victim})
                if src == victim:
                    src = 0
            continue
        if rng.random() < switch_p:  # switch source endpoint (new batch)
            if rng.random() < tx_frac:
                src = rng.choice(sorted(live))
            else:
                src = rng.choice([0, 0, 0, 5])
        q = rng.random()
        if last is not None and q < 0.2:
            f = last                     # repeats exercise the decision cache
        elif q < 0.23:
            f = rng.choice(dhcp_reqs) if src not in (0, 5) else dhcp_ans
        else:
            f = rand_frame(rng, idents)
        last = f
        steps.append({"op": "frame", "src": src, "frame": f.hex()})
    bridge = ["02:00:00:00:00:03"] if rng.random() < 0.5 else []
    return {"name": "rand%d" % seed, "endpoints": endpoints, "bridge": bridge, "steps": steps}


def run_stream(stream, backend):
    """Feed a stream (no expectations) and return the per-frame decision list
    plus control-op return codes, in order."""
    for eid, kind, for_nic in stream["endpoints"]:
        backend.add_endpoint(eid, kind, None if for_nic < 0 else for_nic)
    from katrun import mac2bytes
    for m in stream.get("bridge", []):
        backend.bridge_add(mac2bytes(m))
    out = []
    steps = stream["steps"]
    i = 0
    while i < len(steps):
        st = steps[i]
        if st["op"] == "frame":
            j = i
            while j < len(steps) and steps[j]["op"] == "frame" and steps[j]["src"] == st["src"]:
                j += 1
            out.extend(backend.forward_run(st["src"], [bytes.fromhex(s["frame"]) for s in steps[i:j]]))
            i = j
            continue
        if st["op"] == "add_match":
            out.append(("add", backend.add_match(st["want"], st["owner"], st["sticky"])))
        elif st["op"] == "remove_match":
            out.append(("rm", backend.remove_match(st["want"], st["requester"])))
        elif st["op"] == "remove_endpoint":
            backend.remove_endpoint(st["id"])
        elif st["op"] == "frag_clear":
            backend.frag_clear()
        i += 1
    return out
