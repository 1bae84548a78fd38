#!/usr/bin/env python3
"""Generate tests/golden/kat_*.json: hand-derived known-answer frames.

The reference (ANLAB-KAIST/usnetd) ships no tests and no fixtures, and it
cannot be built in this image (no Rust toolchain; smoltcp 0.7.0 and
usnet_devices are not vendored).  These vectors are therefore derived BY HAND
from the reference source: every expected decision below is written literally
(never computed by an oracle) with the reference line that produces it.
Vectors that rest on recalled smoltcp 0.7.0 behaviour (no IP-version check,
IHL < 5 accepted) carry the tag "smoltcp-recall".

Fixture schema:
  endpoints: [[id, kind, for_nic]]        kind 0 NIC, 1 HOST, 2 PIPE, 3 UDS
  bridge:    ["02:..", ...]               ADD_MACS prefill (main.rs:450-462)
  steps: list of
    {"op": "frame", "src": id, "frame": hex, "expect": [cls, ep, reason], "why": str, "tags": [..]}
    {"op": "add_match", "want": W, "owner": id, "sticky": bool, "expect": 1|0}
    {"op": "remove_match", "want": W, "requester": id, "expect": 1|0|-1}
    {"op": "remove_endpoint", "id": id}
    {"op": "frag_clear"}
  W = {"dst": "a.b.c.d", "dport": int|null, "src": "a.b.c.d"|null, "sport": int|null, "proto": int}
  cls: 0 DROP, 1 EP, 2 NIC, 3 FLOOD; reason: 0 none, 1 PARSE, 2 LOOPBACK,
  3 NOMATCH, 4 EXCLUDED, 5 FRAGMISS, 6 DHCP_NONE; ep 65535 = none.

Run:  python tests/golden/make_golden.py   (rewrites the JSON next to it)
"""
import json
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))

DROP, EP, NIC, FLOOD = 0, 1, 2, 3
NONE, PARSE, LOOPBACK, NOMATCH, EXCLUDED, FRAGMISS, DHCP_NONE = range(7)
NOEP = 0xFFFF
K_NIC, K_HOST, K_PIPE, K_UDS = 0, 1, 2, 3


def ip(s):
    a, b, c, d = (int(x) for x in s.split("."))
    return bytes([a, b, c, d])


def mac(s):
    return bytes(int(x, 16) for x in s.split(":"))


def eth(dmac, smac, et, payload):
    return mac(dmac) + mac(smac) + struct.pack(">H", et) + payload


def ipv4(src, dst, proto, l4, ihl=5, tl=None, ident=1, flags_off=0x4000,
         ver=4, opt_fill=0x01, trunc_to=None):
    hl = ihl * 4
    hdr_len = max(hl, 20)
    if tl is None:
        tl = hdr_len + len(l4) if hl >= 20 else 20 + len(l4)
    h = bytearray(hdr_len)
    h[0] = (ver << 4) | ihl
    h[1] = 0
    struct.pack_into(">HHH", h, 2, tl, ident, flags_off)
    h[8] = 64
    h[9] = proto
    h[12:16] = ip(src)
    h[16:20] = ip(dst)
    for i in range(20, hdr_len):
        h[i] = opt_fill  # NOP options
    body = bytes(h) + l4
    if trunc_to is not None:
        body = body[:trunc_to]
    return body


def udp(sport, dport, payload=b"\x00" * 10):
    return struct.pack(">HHHH", sport, dport, 8 + len(payload), 0) + payload


def tcp(sport, dport):
    return struct.pack(">HHIIHHHH", sport, dport, 1, 0, 0x5002, 1024, 0, 0)


L = "169.254.137.191"     # eval/Makefile:18 target IP
R = "10.0.0.2"
R2 = "10.0.0.3"
NICMAC = "00:1b:21:4b:50:8c"   # eval/Makefile:18 dst MAC
REMMAC = "00:1b:21:4b:50:8d"
GW = "00:00:5e:00:01:01"
MAC2 = "02:00:00:00:00:02"
MAC3 = "02:00:00:00:00:03"
MAC4 = "02:00:00:00:00:04"
MAC9 = "02:00:00:00:00:09"
BCAST = "ff:ff:ff:ff:ff:ff"


def W(dst, proto, dport=None, src=None, sport=None):
    return {"dst": dst, "dport": dport, "src": src, "sport": sport, "proto": proto}


def rx(frame, cls, ep, reason, why, tags=()):
    return {"op": "frame", "src": 0, "frame": frame.hex(), "expect": [cls, ep, reason],
            "why": why, "tags": list(tags)}


def tx(src, frame, cls, ep, reason, why, tags=()):
    return {"op": "frame", "src": src, "frame": frame.hex(), "expect": [cls, ep, reason],
            "why": why, "tags": list(tags)}


def udp_rx(sport, dport, src=R, dst=L, **kw):
    return eth(NICMAC, REMMAC, 0x0800, ipv4(src, dst, 17, udp(sport, dport), **kw))


def kat_main():
    # Endpoints: NIC 0 with host ring 1, pipes 2/3, UDS 4; second NIC 5 with pipe 6.
    endpoints = [[0, K_NIC, -1], [1, K_HOST, 0], [2, K_PIPE, 0], [3, K_PIPE, 0],
                 [4, K_UDS, 0], [5, K_NIC, -1], [6, K_PIPE, 5]]
    s = []
    add = lambda w, owner, sticky=False, expect=1: s.append(
        {"op": "add_match", "want": w, "owner": owner, "sticky": sticky, "expect": expect})
    add(W(L, 6, 22), 1, True)                  # DEBUG_PORTS=...:TCP:22 (main.rs:510-522)
    add(W(L, 17, 3333), 2)
    add(W(L, 17, 3334), 3)
    add(W(L, 6, 80, R, 5555), 4)               # a connected 5-tuple
    add(W(L, 6, 80), 2)                        # listening on 80
    add(W(L, 1), 3)                            # ICMP, no ports
    add(W(L, 6, 23, R), 4)                     # DEBUG_PORTS with remote: sport None
    add(W(L, 17), 4)                           # UDP without port
    add(W(L, 132, 9), 3)                       # SCTP
    add(W(L, 50, None, R), 2)                  # ESP from R (key1 form, no ports)
    add(W(L, 17, 35263), 3)                    # for the IHL=4 quirk below
    add(W(L, 17, 28), 2)                       # for the IHL=0 quirk below
    add(W(L, 17, 3333), 3, expect=0)           # duplicate key -> "ER" (main.rs:272-274)

    # --- A.3.1 length checks -------------------------------------------------
    s.append(rx(bytes(13), DROP, NOEP, PARSE, "len<14: EthernetFrame::new_checked fails (pkt.rs:165)"))
    s.append(rx(eth(NICMAC, REMMAC, 0x0800, b""), DROP, NOEP, PARSE,
                "IPv4 payload 0 < 20 (Ipv4Packet::new_checked, pkt.rs:171)"))
    s.append(rx(eth(NICMAC, REMMAC, 0x0800, bytes(19)), DROP, NOEP, PARSE,
                "IPv4 payload 19 < 20 (pkt.rs:171)"))
    s.append(rx(udp_rx(1000, 3333), EP, 2, NONE, "key2 {L,3333,UDP} -> 2 (endpoint.rs:322)"))
    s.append(rx(udp_rx(1000, 3333), EP, 2, NONE, "identical PacketInfo: cache hit (endpoint.rs:186-191)"))
    s.append(rx(udp_rx(1000, 3334), EP, 3, NONE, "key2 -> 3"))
    s.append(rx(udp_rx(1000, 9999), DROP, NOEP, NOMATCH, "no rule (endpoint.rs:274-277)"))
    s.append(rx(eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 6, tcp(40000, 22))), EP, 1, NONE,
                "TCP:22 -> host ring"))
    s.append(rx(eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 6, tcp(5555, 80))), EP, 4, NONE,
                "key1 {L,80,R,5555,TCP} hit first (endpoint.rs:317-320)"))
    s.append(rx(eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 6, tcp(5556, 80))), EP, 2, NONE,
                "key1 miss, key2 {L,80,TCP} -> 2"))
    s.append(rx(eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 1, bytes(12))), EP, 3, NONE,
                "ICMP: no ports, key1 miss, key2 {L,None,None,None,1} -> 3"))
    s.append(rx(eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 6, tcp(40001, 23))), DROP, NOEP, NOMATCH,
                "A.3.6: rule {L,23,Some(R),None} never equals key1 (sport Some)"))
    s.append(rx(udp_rx(1000, 4444), DROP, NOEP, NOMATCH,
                "A.3.6: rule {L,None,UDP} never matches a UDP frame with ports"))
    # L4 exactly 4 bytes: ports None -> key2 {L,None,None,None,17} = rule -> 4
    f = eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 17, struct.pack(">HH", 1000, 3333)))
    s.append(rx(f, EP, 4, NONE, "A.3.4: payload.len()==4 is not >4 -> no ports (pkt.rs:179)"))
    f = eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 17, struct.pack(">HHB", 1000, 3333, 0)))
    s.append(rx(f, EP, 2, NONE, "A.3.4: payload.len()==5 -> ports read"))
    f = eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 132, udp(7, 9)))
    s.append(rx(f, EP, 3, NONE, "SCTP has ports (pkt.rs:131)"))
    f = eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 33, udp(7, 3333)))
    s.append(rx(f, DROP, NOEP, NOMATCH, "DCCP has ports; rule is UDP -> no match"))
    f = eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 0x88, udp(7, 3333)))
    s.append(rx(f, DROP, NOEP, NOMATCH, "UDPLite (136) has ports; rule is UDP"))
    f = eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 50, bytes(16)))
    s.append(rx(f, EP, 2, NONE, "ESP: key1 {L,None,Some(R),None,50} hits"))
    f = eth(NICMAC, REMMAC, 0x0800, ipv4(R2, L, 50, bytes(16)))
    s.append(rx(f, DROP, NOEP, NOMATCH, "ESP from R2: key1 and key2 miss"))
    # --- A.3.8 ethertypes ------------------------------------------------------
    s.append(rx(eth(BCAST, REMMAC, 0x0806, bytes(28)), FLOOD, NOEP, NONE, "ARP -> mirror_to_all (endpoint.rs:199-204)"))
    s.append(rx(eth(NICMAC, REMMAC, 0x888E, bytes(10)), FLOOD, NOEP, NONE, "EAPOL 0x888e (pkt.rs:206-213)"))
    s.append(rx(eth(NICMAC, REMMAC, 0x86DD, bytes(60)), DROP, NOEP, PARSE, "IPv6 -> None (pkt.rs:205)"))
    vlan = struct.pack(">HH", 5, 0x0800) + ipv4(R, L, 17, udp(1000, 3333))
    s.append(rx(eth(NICMAC, REMMAC, 0x8100, vlan), DROP, NOEP, PARSE, "802.1Q is Unknown(0x8100) -> None"))
    qinq = struct.pack(">HH", 5, 0x8100) + struct.pack(">HH", 6, 0x0800) + ipv4(R, L, 17, udp(1000, 3333))
    s.append(rx(eth(NICMAC, REMMAC, 0x88A8, qinq), DROP, NOEP, PARSE, "QinQ 0x88a8 -> None"))
    # --- A.3.9 loopback ------------------------------------------------------------
    s.append(rx(udp_rx(1000, 3333, dst="127.0.0.1"), DROP, NOEP, LOOPBACK, "dst 127/8 (endpoint.rs:205-208)"))
    s.append(rx(udp_rx(1000, 3333, src="127.0.0.1"), EP, 2, NONE, "src 127/8 is not special"))
    # --- A.3.1 header/total length -----------------------------------------------
    s.append(rx(udp_rx(1000, 3333, ihl=15, tl=40), DROP, NOEP, PARSE, "header_len 60 > total_len 40"))
    f = eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 17, udp(1000, 3333), tl=100))
    s.append(rx(f, DROP, NOEP, PARSE, "buffer shorter than total_len (truncated)"))
    f = eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 17, udp(1000, 3334)) + bytes(20))
    s.append(rx(f, EP, 3, NONE, "Ethernet padding after total_len ignored (payload = [hl..tl])"))
    # --- A.3.2/3 smoltcp-recall quirks ---------------------------------------------------
    f = eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 17, bytes(10), ihl=4, tl=30))
    s.append(rx(f, EP, 3, NONE, "IHL=4: ports read at ip[16..20] = dst bytes a9fe/89bf -> dport 35263",
                ["smoltcp-recall"]))
    f = eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 17, bytes(8), ihl=0, tl=28))
    s.append(rx(f, EP, 2, NONE, "IHL=0: ports = ip[0..4] = 0x4000, tl=28 -> dport 28",
                ["smoltcp-recall"]))
    s.append(rx(udp_rx(1001, 3333, ver=6), EP, 2, NONE, "version nibble 6 with ethertype IPv4 still parsed",
                ["smoltcp-recall"]))
    # --- A.3.5 IHL 12..15: ports beyond the 64-byte window ------------------------------
    s.append(rx(udp_rx(1002, 3334, ihl=15), EP, 3, NONE, "IHL=15: ports at frame[74..78]"))
    s.append(rx(udp_rx(1003, 3333, ihl=12), EP, 2, NONE, "IHL=12: ports at frame[62..66]"))
    # --- A.3.12 fragments -------------------------------------------------------------
    first = udp_rx(1004, 3333, ident=77, flags_off=0x2000)
    s.append(rx(first, EP, 2, NONE, "first fragment MF=1 DF=0 off=0: remembered (pkt.rs:198-202)"))
    s.append(rx(udp_rx(1004, 3334), EP, 3, NONE, "other flow in between (resets the cache)"))
    later = eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 17, bytes(24), ident=77, flags_off=185))
    s.append(rx(later, EP, 2, NONE, "later fragment: info from frag map (pkt.rs:172-176)"))
    s.append(rx(eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 17, bytes(24), ident=78, flags_off=185)),
                DROP, NOEP, FRAGMISS, "later fragment, no first seen -> None"))
    s.append(rx(udp_rx(1005, 3333, ident=88, flags_off=0x6000), EP, 2, NONE,
                "DF=1 and MF=1: not remembered"))
    s.append(rx(eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 17, bytes(24), ident=88, flags_off=185)),
                DROP, NOEP, FRAGMISS, "so its later fragment misses"))
    s.append(rx(eth(NICMAC, GW, 0x0800, ipv4(R, L, 17, bytes(24), ident=77, flags_off=185)),
                DROP, NOEP, FRAGMISS, "frag key includes the MACs (pkt.rs:136-143)"))
    s.append(rx(eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 17, bytes(24), ident=77, flags_off=0x2000 | 370)),
                EP, 2, NONE, "middle fragment (MF=1, off>0): lookup, not insert"))
    s.append({"op": "frag_clear"})
    s.append(rx(later, DROP, NOEP, FRAGMISS, "map cleared by the 90 s cleanup (main.rs Cleanup)"))

    # --- DHCP steering (A.3.10) ----------------------------------------------------------
    req = eth(BCAST, MAC4, 0x0800, ipv4("0.0.0.0", "255.255.255.255", 17, udp(68, 67, bytes(40))))
    s.append(tx(4, req, NIC, 0, NONE,
                "tx DHCP request: NIC.next_dhcp=4 (endpoint.rs:217-228); dmac bcast not in bridge -> NIC"))
    ans = eth(BCAST, REMMAC, 0x0800, ipv4("10.0.0.1", "255.255.255.255", 17, udp(67, 68, bytes(40))))
    s.append(rx(ans, EP, 4, NONE, "DHCP answer, no rule: next_dhcp.take() (endpoint.rs:262-268)"))
    s.append(rx(ans, DROP, NOEP, DHCP_NONE, "steering cleared last_pkt; next_dhcp now None"))
    s.append(rx(ans, DROP, NOEP, DHCP_NONE, "cache hit on the dropped answer"))

    # --- tx direction -----------------------------------------------------------------
    f = eth(GW, MAC2, 0x0800, ipv4(L, R, 17, udp(3333, 1000)))
    s.append(tx(2, f, NIC, 0, NONE, "tx: MAC2 learned; listening has (L,17,3333) -> no auto rule; dmac GW -> NIC"))
    f = eth(GW, MAC2, 0x0800, ipv4(L, R, 6, tcp(40000, 443)))
    s.append(tx(2, f, NIC, 0, NONE, "tx client flow: auto-learn {L,40000,R,443,TCP}->2 (endpoint.rs:229-249)"))
    f = eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 6, tcp(443, 40000)))
    s.append(rx(f, EP, 2, NONE, "answer matches the learned key1"))
    f = eth(MAC2, MAC3, 0x0800, ipv4(L, L, 17, udp(3334, 3333)))
    s.append(tx(3, f, EP, 2, NONE, "tx to a bridged MAC (MAC2) -> lookup key2 {L,3333,UDP} -> 2"))
    f = eth(MAC2, MAC2, 0x0800, ipv4(L, L, 17, udp(3333, 3333)))
    s.append(tx(2, f, DROP, NOEP, EXCLUDED, "lookup hits the source itself -> None (endpoint.rs:328-336)"))
    f = eth(MAC2, MAC4, 0x0800, ipv4(R, L, 6, tcp(5555, 80)))
    s.append(tx(4, f, DROP, NOEP, EXCLUDED,
                "A.3.7: key1 hits self-owned {L,80,R,5555}; no retry with key2 {L,80}->2"))
    s.append(tx(3, eth(BCAST, MAC3, 0x0806, bytes(28)), FLOOD, NOEP, NONE, "tx ARP -> flood"))
    a = eth(GW, MAC3, 0x0800, ipv4(L, R, 17, udp(3334, 2000)))
    s.append(tx(3, a, NIC, 0, NONE, "tx to gateway -> NIC"))
    b = eth(MAC2, MAC3, 0x0800, ipv4(L, R, 17, udp(3334, 2000)))
    s.append(tx(3, b, NIC, 0, NONE, "same PacketInfo, dmac now bridged: cache ignores MACs -> NIC"))
    c = eth(GW, MAC9, 0x0800, ipv4(L, R, 17, udp(3334, 2000)))
    s.append(tx(3, c, NIC, 0, NONE, "cache hit again: MAC9 is NOT learned (learning is after the cache)"))
    d = eth(MAC9, MAC2, 0x0800, ipv4(L, "10.1.1.1", 17, udp(3333, 1)))
    s.append(tx(2, d, NIC, 0, NONE, "dmac MAC9 not in bridge -> NIC"))

    # --- stale cache (A.3.11) ----------------------------------------------------------
    f7 = udp_rx(7, 3334)
    s.append(rx(f7, EP, 3, NONE, "cached decision 3"))
    s.append({"op": "remove_match", "want": W(L, 17, 3334), "requester": 3, "expect": 1})
    s.append(rx(f7, EP, 3, NONE, "RemoveMatch does not clear the cache: stale hit (main.rs:608-625)"))
    s.append(rx(udp_rx(8, 3333), EP, 2, NONE, "different flow"))
    s.append(rx(f7, DROP, NOEP, NOMATCH, "now the removal is visible"))
    f8 = udp_rx(8, 5000)
    s.append(rx(f8, DROP, NOEP, NOMATCH, "no rule yet; cached as None"))
    s.append({"op": "add_match", "want": W(L, 17, 5000), "owner": 2, "sticky": False, "expect": 1})
    s.append(rx(f8, EP, 2, NONE, "AddMatch cleared the NIC cache (main.rs:280-286)"))
    s.append({"op": "remove_match", "want": W(L, 6, 22), "requester": 2, "expect": -1})
    s.append(rx(eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 6, tcp(40000, 22))), EP, 1, NONE,
                "removal by a non-owner is refused (main.rs:612-616)"))
    f9 = udp_rx(9, 3333)
    s.append(rx(f9, EP, 2, NONE, "cached decision 2"))
    s.append({"op": "remove_endpoint", "id": 2})
    s.append(rx(f9, EP, 2, NONE, "stale hit even after the endpoint and its rules are gone"))
    s.append(rx(udp_rx(10, 3333), DROP, NOEP, NOMATCH, "rules of 2 were removed (main.rs:1063-1069)"))
    # second NIC: its rules are independent of NIC 0's endpoints only through the table
    s.append({"op": "frame", "src": 5, "frame": udp_rx(11, 3333).hex(), "expect": [DROP, NOEP, NOMATCH],
              "why": "NIC 5 rx: table is global; 3333 rule belonged to 2 (removed)", "tags": []})
    s.append({"op": "add_match", "want": W(L, 17, 6000), "owner": 6, "sticky": False, "expect": 1})
    s.append({"op": "frame", "src": 0, "frame": udp_rx(12, 6000).hex(), "expect": [EP, 6, NONE],
              "why": "lookup does not check the endpoint's NIC (A.2 note)", "tags": []})
    return {"name": "main", "endpoints": endpoints, "bridge": [], "steps": s}


def kat_bridge():
    """ADD_MACS prefill and tx-direction bridge semantics (endpoint.rs:195-197, 254-255)."""
    endpoints = [[0, K_NIC, -1], [1, K_HOST, 0], [2, K_PIPE, 0], [3, K_PIPE, 0]]
    s = [{"op": "add_match", "want": W(L, 17, 3333), "owner": 2, "sticky": True, "expect": 1},
         {"op": "add_match", "want": W(L, 17, 3334), "owner": 3, "sticky": True, "expect": 1}]
    f = eth(MAC3, MAC2, 0x0800, ipv4(L, L, 17, udp(3333, 3334)))
    s.append(tx(2, f, EP, 3, NONE, "dmac MAC3 prefilled by ADD_MACS -> lookup -> 3"))
    f = eth("03:00:00:00:00:07", "03:00:00:00:00:05", 0x0800, ipv4(L, R, 17, udp(3333, 9)))
    s.append(tx(2, f, NIC, 0, NONE, "multicast smac is not learned; dmac not bridged -> NIC"))
    f = eth("03:00:00:00:00:05", MAC2, 0x0800, ipv4(L, R, 17, udp(3333, 10)))
    s.append(tx(2, f, NIC, 0, NONE, "so a frame to that multicast MAC still goes to the NIC"))
    f = eth(MAC2, MAC3, 0x0800, ipv4(L, L, 17, udp(3334, 3333)))
    s.append(tx(3, f, EP, 2, NONE, "MAC2 was learned from its first tx frame"))
    f = eth(NICMAC, REMMAC, 0x0800, ipv4(R, L, 17, udp(1, 3334)))
    s.append(rx(f, EP, 3, NONE, "rx is never bridge-tested"))
    return {"name": "bridge", "endpoints": endpoints, "bridge": [MAC3], "steps": s}


def kat_dhcp():
    """is_dhcp_request's source test (pkt.rs:36-58): src_addr.is_unspecified()
    (pkt.rs:46) is smoltcp 0.7.0's range test self.0[0] == 0, i.e. 0.0.0.0/8
    (recalled: tag smoltcp-recall).  A request sets the NIC's next_dhcp and
    clears both caches (endpoint.rs:217-228) and learns NO answer rule; a frame
    from outside 0/8 is an ordinary client flow and learns one (:229-249)."""
    endpoints = [[0, K_NIC, -1], [1, K_HOST, 0], [2, K_PIPE, 0], [4, K_UDS, 0]]
    s = [{"op": "add_match", "want": W(L, 17, 3333), "owner": 2, "sticky": False, "expect": 1}]
    rec = ["smoltcp-recall"]

    def req(src, dst="10.0.0.255"):
        return eth(BCAST, MAC4, 0x0800, ipv4(src, dst, 17, udp(68, 67, bytes(40))))

    def ans(to, frm="10.0.0.255"):
        return eth(BCAST, REMMAC, 0x0800, ipv4(frm, to, 17, udp(67, 68, bytes(40))))

    for k, src in enumerate(("0.1.2.3", "0.0.0.0")):
        f = udp_rx(1000 + k, 3333)
        s.append(rx(f, EP, 2, NONE, "NIC caches decision 2"))
        s.append({"op": "remove_match", "want": W(L, 17, 3333), "requester": 2, "expect": 1})
        s.append(rx(f, EP, 2, NONE, "RemoveMatch leaves the NIC cache: stale hit (main.rs:608-625)"))
        s.append(tx(4, req(src), NIC, 0, NONE,
                    "tx UDP 68->67 to x.x.x.255 from %s: is_unspecified (0/8) -> DHCP request: "
                    "NIC.next_dhcp=4, caches cleared, no answer rule (endpoint.rs:217-228); "
                    "dmac bcast not bridged -> NIC" % src, rec))
        s.append(rx(f, DROP, NOEP, NOMATCH, "the request cleared the NIC cache (endpoint.rs:223)", rec))
        s.append(rx(ans(src), EP, 4, NONE, "answer: no rule, next_dhcp.take() -> 4 (endpoint.rs:262-268)", rec))
        s.append(rx(ans(src), DROP, NOEP, DHCP_NONE,
                    "again: no answer rule was learned and next_dhcp is None "
                    "(a learned rule would hit 4 via key1)", rec))
        s.append({"op": "add_match", "want": W(L, 17, 3333), "owner": 2, "sticky": False, "expect": 1})
    # 1.0.0.0 is outside 0/8: an ordinary client flow, the answer key is learned
    s.append(tx(4, req("1.0.0.0"), NIC, 0, NONE,
                "src 1.0.0.0 is not unspecified: auto-learn {1.0.0.0,68,10.0.0.255,67,UDP}->4 "
                "(endpoint.rs:229-249)", rec))
    s.append(rx(ans("1.0.0.0"), EP, 4, NONE, "key1 hits the learned answer rule (endpoint.rs:317-320)", rec))
    s.append(rx(ans("1.0.0.0"), EP, 4, NONE, "cache hit (a steered answer would have cleared it)", rec))
    s.append(rx(ans("0.9.9.9"), DROP, NOEP, DHCP_NONE,
                "next_dhcp was not set by the 1.0.0.0 frame (endpoint.rs:269-272)", rec))
    # 0/8 source but dst[3] != 255: not a request, the answer key is learned
    s.append(tx(4, req("0.7.7.7", "10.0.0.1"), NIC, 0, NONE,
                "0/8 source to 10.0.0.1 (dst[3]!=255): not a DHCP request -> learns", rec))
    s.append(rx(ans("0.7.7.7", "10.0.0.1"), EP, 4, NONE, "the learned answer rule", rec))
    s.append(rx(ans("0.7.7.7", "10.0.0.1"), EP, 4, NONE, "cache hit", rec))
    return {"name": "dhcp", "endpoints": endpoints, "bridge": [], "steps": s}


def main():
    for kat in (kat_main(), kat_bridge(), kat_dhcp()):
        path = os.path.join(HERE, "kat_%s.json" % kat["name"])
        with open(path, "w") as fh:
            json.dump(kat, fh, indent=1)
            fh.write("\n")
        n = sum(1 for st in kat["steps"] if st["op"] == "frame")
        print("wrote %s (%d frames)" % (path, n))


if __name__ == "__main__":
    main()
