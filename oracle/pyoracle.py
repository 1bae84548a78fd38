"""Independent pure-Python restatement of usnetd's match path.

TEST INFRASTRUCTURE ONLY -- used by tests/ to cross-check the C oracle
(oracle/usn_oracle.c) on small cases.  It is written from the reference
source directly (not from the C file), with Python's own dict/list types
standing in for hashbrown's HashMap and Vec:

  PacketInfo / extract_pkt_info   /root/reference/src/pkt.rs:11-218
  Want                            /root/reference/src/pkt.rs:220-258
  Endpoint::find_forward          /root/reference/src/endpoint.rs:172-296
  get_endpoint                    /root/reference/src/endpoint.rs:307-338
  add_listening_match             /root/reference/src/main.rs:266-298
  RemoveMatch / endpoint removal  /root/reference/src/main.rs:608-625, 1063-1069

PARITY UNPINNED: the reference has no tests or fixtures and cannot be built
here; this file and the C oracle agree with each other and with the
hand-derived known-answer frames in tests/golden/.

Decision words use the shared encoding documented in oracle/usn_oracle.h.
"""
from __future__ import annotations

import struct

DROP, EP, NIC, FLOOD = 0, 1, 2, 3
R_NONE, R_PARSE, R_LOOPBACK, R_NOMATCH, R_EXCLUDED, R_FRAGMISS, R_DHCP_NONE = range(7)
KIND_NIC, KIND_HOST, KIND_PIPE, KIND_UDS = 0, 1, 2, 3
PORT_PROTOS = (6, 17, 0x21, 0x84, 0x88)  # pkt.rs:128-133


def dec(cls: int, reason: int = 0, ep: int = 0xFFFF) -> int:
    return (ep & 0xFFFF) | (cls << 16) | (reason << 20)


# PacketInfo: ("ipv4", src, dst, proto, sport|None, dport|None) | ("arp",) | ("eapol",)
def _parse(frame: bytes, frag_map: dict):
    """extract_pkt_info -> (info, smac, dmac) or an int drop reason."""
    if len(frame) < 14:
        return R_PARSE
    dmac, smac = bytes(frame[0:6]), bytes(frame[6:12])
    (et,) = struct.unpack_from(">H", frame, 12)
    if et == 0x0806:
        return ("arp",), smac, dmac
    if et == 0x0800:
        ip = frame[14:]
        if len(ip) < 20:
            return R_PARSE
        header_len = (ip[0] & 0x0F) * 4
        (total_len,) = struct.unpack_from(">H", ip, 2)
        if len(ip) < header_len or header_len > total_len or len(ip) < total_len:
            return R_PARSE
        ident, flags_off = struct.unpack_from(">HH", ip, 4)
        proto = ip[9]
        src, dst = struct.unpack_from(">II", ip, 12)
        key = (ident, src, dst, proto, smac, dmac)
        if ((flags_off << 3) & 0xFFFF) > 0:
            got = frag_map.get(key)
            return got if got is not None else R_FRAGMISS
        payload = ip[header_len:total_len]
        if proto in PORT_PROTOS and len(payload) > 4:
            sport, dport = struct.unpack_from(">HH", payload, 0)
        else:
            sport = dport = None
        ret = (("ipv4", src, dst, proto, sport, dport), smac, dmac)
        dont_frag = bool(flags_off & 0x4000)
        more_frags = bool(flags_off & 0x2000)
        if not dont_frag and more_frags:
            frag_map[key] = ret
        return ret
    if et == 0x888E:
        return ("eapol",), smac, dmac
    return R_PARSE


class Endpoint:
    def __init__(self, kind: int, for_nic):
        self.kind = kind
        self.for_nic = for_nic
        self.listening = []  # Vec<(Ipv4Address, u8, Option<u16>)>
        self.next_dhcp = None
        self.last_pkt = None
        self.last_dst = None  # decision word (DROP == None target)


class Switch:
    def __init__(self):
        self.eps: dict[int, Endpoint] = {}
        self.match_register: dict[tuple, tuple] = {}  # Want tuple -> (sticky, owner)
        self.bridge: list[bytes] = []
        self.frag_map: dict = {}

    # --- control plane ---------------------------------------------------
    def add_endpoint(self, eid, kind, for_nic=None):
        self.eps[eid] = Endpoint(kind, for_nic)

    def remove_endpoint(self, eid):
        self.match_register = {k: v for k, v in self.match_register.items() if v[1] != eid}
        del self.eps[eid]

    @staticmethod
    def want(dst, proto, dport=None, src=None, sport=None):
        return (dst, dport, src, sport, proto)

    def add_match(self, want, owner, sticky=False):
        if want in self.match_register:
            return False
        ep = self.eps[owner]
        ep.listening.append((want[0], want[4], want[1]))
        self.eps[ep.for_nic].last_pkt = None
        self.match_register[want] = (sticky, owner)
        return True

    def remove_match(self, want, requester):
        got = self.match_register.get(want)
        if got is not None and got[1] != requester:
            return -1
        return 1 if self.match_register.pop(want, None) is not None else 0

    # --- data path -------------------------------------------------------
    def _get_endpoint(self, src_id, info):
        _, src, dst, proto, sport, dport = info
        hit = self.match_register.get((dst, dport, src, sport, proto))
        if hit is None:
            hit = self.match_register.get((dst, dport, None, None, proto))
        if hit is not None:
            owner = hit[1]
            if self.eps[owner].kind == KIND_NIC or owner == src_id:
                return None, True
            return owner, False
        return None, False

    def forward(self, src_id: int, frame: bytes) -> int:
        me = self.eps[src_id]
        incoming = me.kind == KIND_NIC
        got = _parse(frame, self.frag_map)
        if isinstance(got, int):
            return dec(DROP, got)
        info, smac, dmac = got
        if me.last_pkt is not None and me.last_pkt == info:
            return me.last_dst
        me.last_pkt = None
        if not incoming and (smac[0] & 1) == 0 and smac not in self.bridge:
            self.bridge.append(smac)
        if info[0] in ("arp", "eapol"):
            return dec(FLOOD)
        if (info[2] >> 24) == 127:
            return dec(DROP, R_LOOPBACK)
        me.last_pkt = info
        _, src, dst, proto, sport, dport = info
        if not incoming:
            want = (src, sport, dst, dport, proto)  # to_want: reversed tuple
            if (want[0], want[4], want[1]) not in me.listening:
                # src_addr.is_unspecified() (pkt.rs:46): smoltcp 0.7.0 tests the
                # 0.0.0.0/8 range, self.0[0] == 0 (smoltcp-recall)
                is_dhcp_req = (proto == 17 and (src >> 24) == 0 and sport == 68 and dport == 67
                               and (dst & 0xFF) == 255)
                if is_dhcp_req:
                    if me.for_nic is not None:
                        nic = self.eps[me.for_nic]
                        nic.next_dhcp = src_id
                        nic.last_pkt = None
                        me.last_pkt = None
                else:
                    if want not in self.match_register:
                        self.eps[me.for_nic].last_pkt = None
                        self.match_register[want] = (False, src_id)
        if not incoming and dmac not in self.bridge:
            d = dec(NIC, 0, me.for_nic)
        else:
            owner, excluded = self._get_endpoint(src_id, info)
            if owner is None:
                if proto == 17 and sport == 67 and dport == 68:
                    if me.next_dhcp is not None:
                        d = dec(EP, 0, me.next_dhcp)
                        me.next_dhcp = None
                        me.last_pkt = None
                    else:
                        d = dec(DROP, R_DHCP_NONE)
                else:
                    d = dec(DROP, R_EXCLUDED if excluded else R_NOMATCH)
            else:
                d = dec(EP, 0, owner)
        me.last_dst = d
        return d
