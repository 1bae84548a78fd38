"""Known-answer fixture runner shared by the oracle tests and the GPU tests.

A backend implements:
  add_endpoint(id, kind, for_nic) / remove_endpoint(id)
  add_match(want_dict, owner, sticky) -> 1|0 / remove_match(want_dict, requester) -> 1|0|-1
  bridge_add(mac_bytes) / frag_clear()
  forward_run(src, [frame_bytes, ...]) -> [decision_word, ...]
Consecutive frames from one source with no control op in between form one
run, i.e. one drained rx batch (endpoint.rs:128-169).
"""
from __future__ import annotations

import glob
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PARITY_MASK = 0x00FFFFFF


def load_kats():
    out = []
    for p in sorted(glob.glob(os.path.join(HERE, "golden", "kat_*.json"))):
        with open(p) as fh:
            out.append(json.load(fh))
    return out


def ip2int(s):
    if s is None:
        return None
    a, b, c, d = (int(x) for x in s.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def mac2bytes(s):
    return bytes(int(x, 16) for x in s.split(":"))


def expect_word(cls, ep, reason):
    return (ep & 0xFFFF) | (cls << 16) | (reason << 20)


def run_kat(kat, backend):
    """Returns list of (step_index, got_word, expected_word, why) mismatches."""
    for eid, kind, for_nic in kat["endpoints"]:
        backend.add_endpoint(eid, kind, None if for_nic < 0 else for_nic)
    for m in kat.get("bridge", []):
        backend.bridge_add(mac2bytes(m))
    bad = []
    steps = kat["steps"]
    i = 0
    while i < len(steps):
        st = steps[i]
        op = st["op"]
        if op == "frame":
            j = i
            while j < len(steps) and steps[j]["op"] == "frame" and steps[j]["src"] == st["src"]:
                j += 1
            run = steps[i:j]
            got = backend.forward_run(st["src"], [bytes.fromhex(s["frame"]) for s in run])
            for k, (s, g) in enumerate(zip(run, got)):
                exp = expect_word(*s["expect"])
                if (g & PARITY_MASK) != exp:
                    bad.append((i + k, g & PARITY_MASK, exp, s["why"]))
            i = j
            continue
        if op == "add_match":
            rc = backend.add_match(st["want"], st["owner"], st["sticky"])
            if rc != st["expect"]:
                bad.append((i, rc, st["expect"], "add_match"))
        elif op == "remove_match":
            rc = backend.remove_match(st["want"], st["requester"])
            if rc != st["expect"]:
                bad.append((i, rc, st["expect"], "remove_match"))
        elif op == "remove_endpoint":
            backend.remove_endpoint(st["id"])
        elif op == "frag_clear":
            backend.frag_clear()
        else:
            raise ValueError(op)
        i += 1
    return bad


class COracleBackend:
    def __init__(self):
        import coracle
        self.o = coracle.Oracle()
        self.make_want = coracle.make_want

    def _w(self, w):
        return self.make_want(w["dst"], w["proto"], w["dport"], w["src"], w["sport"])

    def add_endpoint(self, eid, kind, for_nic):
        self.o.add_endpoint(eid, kind, -1 if for_nic is None else for_nic)

    def remove_endpoint(self, eid):
        self.o.remove_endpoint(eid)

    def add_match(self, w, owner, sticky):
        return self.o.add_match(self._w(w), owner, sticky)

    def remove_match(self, w, requester):
        return self.o.remove_match(self._w(w), requester)

    def bridge_add(self, mac):
        self.o.bridge_add(mac)

    def frag_clear(self):
        self.o.frag_clear()

    def forward_run(self, src, frames):
        return [self.o.forward(src, f) for f in frames]


class PyOracleBackend:
    def __init__(self):
        import pyoracle
        self.s = pyoracle.Switch()

    @staticmethod
    def _w(w):
        return (ip2int(w["dst"]), w["dport"], ip2int(w["src"]), w["sport"], w["proto"])

    def add_endpoint(self, eid, kind, for_nic):
        self.s.add_endpoint(eid, kind, for_nic)

    def remove_endpoint(self, eid):
        self.s.remove_endpoint(eid)

    def add_match(self, w, owner, sticky):
        return int(self.s.add_match(self._w(w), owner, sticky))

    def remove_match(self, w, requester):
        return self.s.remove_match(self._w(w), requester)

    def bridge_add(self, mac):
        self.s.bridge.append(bytes(mac))

    def frag_clear(self):
        self.s.frag_map.clear()

    def forward_run(self, src, frames):
        return [self.s.forward(src, f) for f in frames]
