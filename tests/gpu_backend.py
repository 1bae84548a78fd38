"""katrun/randtraffic backend that drives the product through the C ABI on a GPU.

Each run of consecutive frames from one source becomes one device-resident
batch (fixed 128-byte slots), classified by usn_classify and completed by
usn_finalize -- the same sequence a host daemon performs per drained ring.
"""
from __future__ import annotations

import numpy as np

from usnetd_amd import lib

SLOT = 128


class GpuBackend:
    def __init__(self, ctx: lib.Ctx | None = None, check_order=True):
        self.ctx = ctx or lib.Ctx(0)
        self.check_order = check_order
        self.stream = self.ctx.stream()
        self.kinds = {}

    def add_endpoint(self, eid, kind, for_nic):
        self.kinds[eid] = kind
        self.ctx.endpoint_add(eid, kind, for_nic)

    def remove_endpoint(self, eid):
        self.ctx.endpoint_remove(eid)

    def add_match(self, w, owner, sticky):
        return self.ctx.add_match(lib.want_from_dict(w), owner, sticky)

    def remove_match(self, w, requester):
        return self.ctx.remove_match(lib.want_from_dict(w), requester)

    def bridge_add(self, mac):
        self.ctx.bridge_add(mac)

    def frag_clear(self):
        self.ctx.frag_clear()

    def forward_run(self, src, frames):
        n = len(frames)
        buf = np.zeros(n * SLOT, dtype=np.uint8)
        lens = np.zeros(n, dtype=np.uint16)
        for i, f in enumerate(frames):
            f = f[:SLOT]
            buf[i * SLOT:i * SLOT + len(f)] = np.frombuffer(f, np.uint8)
            lens[i] = len(f)
        b = lib.DeviceBatch(self.ctx, buf, lens, src, stride=SLOT)
        r = lib.DeviceResult(self.ctx, n)
        try:
            self.ctx.classify(b, r, self.stream)
            self.ctx.finalize(b, r, self.stream)
            d = r.decisions()
            if self.check_order:
                check_order(r, d)
        finally:
            # the device chain of this source points at r: keep it alive
            self._keep = (b, r)
        return [int(x) for x in d]


def check_order(r: lib.DeviceResult, d: np.ndarray):
    """order/runs must be the stable per-tile sort of the decisions' bins."""
    tiles = r.tiles()
    order = r.order()
    runs = r.runs()
    n = r.n
    n_ep = None
    for t in range(r.ntiles):
        nf = int(tiles[t]["n_frames"])
        seg = d[t * lib.USN_TILE:t * lib.USN_TILE + nf]
        cls = (seg >> 16) & 0xF
        assert int(tiles[t]["class_count"][0]) == int((cls == 0).sum())
        assert int(tiles[t]["class_count"][1]) == int((cls == 1).sum())
        o = order[t * lib.USN_TILE:t * lib.USN_TILE + nf].astype(np.int64)
        assert sorted(o.tolist()) == list(range(nf)), "order is not a permutation"
        nr = int(tiles[t]["n_runs"])
        rr = runs[t * lib.USN_TILE:t * lib.USN_TILE + nr]
        starts = (rr & 0xFFFF).astype(np.int64)
        bins = (rr >> 16).astype(np.int64)
        assert nr >= 1 and starts[0] == 0 and (np.diff(starts) > 0).all()
        assert (np.diff(bins) > 0).all(), "runs not sorted by bin"
        ends = np.append(starts[1:], nf)
        for b, s, e in zip(bins, starts, ends):
            idx = o[s:e]
            assert (np.diff(idx) > 0).all(), "order within a bin is not stable"
            sd = seg[idx]
            c = (sd >> 16) & 0xF
            # every member maps to bin b
            if n_ep is None:
                pass
            assert len(set(((sd & 0xFFFF) * (c == 1) + (c != 1) * (1 << 20) + c).tolist())) == 1, \
                "mixed decisions inside one run"
    return True
