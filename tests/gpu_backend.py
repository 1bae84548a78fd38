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
    def __init__(self, ctx: lib.Ctx | None = None, check_order=True, split_tx_seed=None):
        """split_tx_seed: a sending endpoint's run of frames goes to the
        device as 2-8 consecutive rings in one usn_classify_multi launch (one
        tx grid), split at seeded random frames"""
        self.ctx = ctx or lib.Ctx(0)
        self.check_order = check_order
        self.stream = self.ctx.stream()
        self.kinds = {}
        self.split_rng = None
        if split_tx_seed is not None:
            import random
            self.split_rng = random.Random(split_tx_seed)

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

    def _batch(self, src, frames):
        n = len(frames)
        buf = np.zeros(n * SLOT, dtype=np.uint8)
        lens = np.zeros(n, dtype=np.uint16)
        for i, f in enumerate(frames):
            f = f[:SLOT]
            buf[i * SLOT:i * SLOT + len(f)] = np.frombuffer(f, np.uint8)
            lens[i] = len(f)
        return lib.DeviceBatch(self.ctx, buf, lens, src, stride=SLOT), lib.DeviceResult(self.ctx, n)

    def forward_run(self, src, frames):
        n = len(frames)
        if self.split_rng is not None and self.kinds.get(src) != lib.EP_NIC and n >= 2:
            m = self.split_rng.randint(2, min(8, n))
            cuts = [0] + sorted(self.split_rng.sample(range(1, n), m - 1)) + [n]
            parts = [self._batch(src, frames[x:y]) for x, y in zip(cuts, cuts[1:])]
            try:
                self.ctx.classify_multi([p[0] for p in parts], [p[1] for p in parts], self.stream)
                out = []
                for b, r in parts:
                    self.ctx.finalize(b, r, self.stream)
                    d = r.decisions()
                    if self.check_order:
                        check_order(r, d)
                    out += [int(x) for x in d]
            finally:
                self._keep = parts
            return out
        b, r = self._batch(src, frames)
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
    """The per-endpoint lists (usn_result.index / bin_off) must be the stable
    scatter of the final decisions by bin, and the tile headers' class counts
    must count them."""
    n_ep = int(r.summary()["n_ep"])
    got = r.lists(d.shape[0])
    want = lib.expected_lists(d, n_ep)
    assert sorted(got) == sorted(want), "bins differ"
    for b in want:
        assert np.array_equal(got[b], want[b]), "list of bin %d differs" % b
    tiles = r.tiles()
    for t in range(r.ntiles):
        nf = int(tiles[t]["n_frames"])
        seg = d[t * lib.USN_TILE:t * lib.USN_TILE + nf]
        cls = (seg >> 16) & 0xF
        for c in range(4):
            assert int(tiles[t]["class_count"][c]) == int((cls == c).sum())
    return True
