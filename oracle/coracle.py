"""ctypes binding of the C oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product (usnetd_amd/).
PARITY UNPINNED (see usn_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

KIND_NIC, KIND_HOST, KIND_PIPE, KIND_UDS = 0, 1, 2, 3


class Want(C.Structure):
    _fields_ = [("dst_addr", C.c_uint32), ("src_addr", C.c_uint32),
                ("dst_port", C.c_uint16), ("src_port", C.c_uint16),
                ("protocol", C.c_uint8), ("mask", C.c_uint8), ("_pad", C.c_uint16)]


def ip2int(s: str) -> int:
    a, b, c, d = (int(x) for x in s.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def make_want(dst, proto, dport=None, src=None, sport=None) -> Want:
    w = Want()
    w.dst_addr = ip2int(dst) if isinstance(dst, str) else dst
    w.protocol = proto
    m = 0
    if dport is not None:
        m |= 1
        w.dst_port = dport
    if src is not None:
        m |= 2
        w.src_addr = ip2int(src) if isinstance(src, str) else src
    if sport is not None:
        m |= 4
        w.src_port = sport
    w.mask = m
    return w


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.uso_create.restype = P
        L.uso_destroy.argtypes = [P]
        L.uso_add_endpoint.argtypes = [P, C.c_int, C.c_int, C.c_int]
        L.uso_remove_endpoint.argtypes = [P, C.c_int]
        L.uso_add_match.argtypes = [P, C.POINTER(Want), C.c_int, C.c_int]
        L.uso_remove_match.argtypes = [P, C.POINTER(Want), C.c_int]
        L.uso_lookup.argtypes = [P, C.POINTER(Want)]
        L.uso_rule_count.argtypes = [P]
        L.uso_rules.argtypes = [P, P, P, P, C.c_int]
        L.uso_bridge_add.argtypes = [P, C.c_char_p]
        L.uso_bridge_count.argtypes = [P]
        L.uso_frag_clear.argtypes = [P]
        L.uso_get_cache.argtypes = [P, C.c_int, C.POINTER(C.c_uint32), C.c_char_p]
        L.uso_get_next_dhcp.argtypes = [P, C.c_int]
        L.uso_forward.argtypes = [P, C.c_int, C.c_char_p, C.c_uint32]
        L.uso_forward.restype = C.c_uint32
        L.uso_forward_batch.argtypes = [P, C.c_int, P, C.c_uint64, P, P, C.c_uint64, P]
        _lib = L
    return _lib


class Oracle:
    """Sequential reference restatement (one usnetd daemon's match state)."""

    def __init__(self):
        self.L = lib()
        self.h = self.L.uso_create()

    def close(self):
        if self.h:
            self.L.uso_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_endpoint(self, eid, kind, for_nic=-1):
        rc = self.L.uso_add_endpoint(self.h, eid, kind, -1 if for_nic is None else for_nic)
        assert rc == 0, (eid, kind, for_nic)

    def remove_endpoint(self, eid):
        return self.L.uso_remove_endpoint(self.h, eid)

    def add_match(self, want: Want, owner: int, sticky=False) -> int:
        return self.L.uso_add_match(self.h, C.byref(want), owner, int(bool(sticky)))

    def remove_match(self, want: Want, requester: int) -> int:
        return self.L.uso_remove_match(self.h, C.byref(want), requester)

    def lookup(self, want: Want) -> int:
        return self.L.uso_lookup(self.h, C.byref(want))

    def rule_count(self) -> int:
        return self.L.uso_rule_count(self.h)

    def rules(self):
        """[(dst, src, dport, sport, proto, mask, owner)] with absent fields zeroed."""
        n = self.rule_count()
        ws = (Want * max(n, 1))()
        owners = np.zeros(max(n, 1), np.int32)
        sticky = np.zeros(max(n, 1), np.uint8)
        got = self.L.uso_rules(self.h, C.cast(ws, C.c_void_p), owners.ctypes.data,
                               sticky.ctypes.data, n)
        return [(w.dst_addr, w.src_addr if w.mask & 2 else 0, w.dst_port if w.mask & 1 else 0,
                 w.src_port if w.mask & 4 else 0, w.protocol, w.mask, int(owners[i]))
                for i, w in enumerate(ws[:got])]

    def bridge_count(self) -> int:
        return self.L.uso_bridge_count(self.h)

    def bridge_add(self, mac: bytes):
        self.L.uso_bridge_add(self.h, bytes(mac))

    def frag_clear(self):
        self.L.uso_frag_clear(self.h)

    def forward(self, src: int, frame: bytes) -> int:
        return self.L.uso_forward(self.h, src, bytes(frame), len(frame))

    def cache(self, eid):
        d = C.c_uint32()
        buf = C.create_string_buffer(16)
        if not self.L.uso_get_cache(self.h, eid, C.byref(d), buf):
            return None
        return d.value, buf.raw

    def next_dhcp(self, eid):
        return self.L.uso_get_next_dhcp(self.h, eid)

    def forward_batch(self, src: int, frames: np.ndarray, lens: np.ndarray,
                      stride: int = 0, offsets: np.ndarray | None = None) -> np.ndarray:
        """frames: uint8 buffer; stride>0 or offsets (uint64) selects the layout."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        n = lens.shape[0]
        out = np.empty(n, dtype=np.uint32)
        offp = None
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            offp = offsets.ctypes.data
        self.L.uso_forward_batch(self.h, src, frames.ctypes.data, stride, offp,
                                 lens.ctypes.data, n, out.ctypes.data)
        return out


def install_oracle(o: "Oracle", cfg) -> None:
    """Install a usnetd_amd.traffic.Config (endpoints, rules, bridge) into an oracle."""
    for eid, kind, for_nic in cfg.endpoints:
        o.add_endpoint(eid, kind, -1 if for_nic is None else for_nic)
    for w, owner, sticky in cfg.rules:
        o.add_match(make_want(w["dst"], w["proto"], w["dport"], w["src"], w["sport"]), owner, sticky)
    for m in cfg.bridge:
        o.bridge_add(m)
