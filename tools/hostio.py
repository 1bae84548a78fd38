#!/usr/bin/env python3
"""PCIe-inclusive rate of the match path: frames start and end in host memory.

The loop a host runs per drained ring: pinned-host header
windows + lengths -> hipMemcpyAsync H2D -> usn_classify -> usn_finalize (the
ordered host stage: it reads the batch summary and tile headers, and patches
results when a batch needs it) -> D2H of the decisions and the per-endpoint
lists (index + bin_off, ABI v3).  Batches go round-robin over S streams, one NIC rx queue each; a
stream's previous batch is finalized and copied back right before its next
batch is enqueued, so the copies and host stage of one stream overlap the
kernels of the others.  At the end every batch's returned decisions are
compared with the C oracle (bits [23:0]) and its returned lists with the
stable sort of the oracle's decisions by bin.  Reported in DESIGN.md; never the
bench value.  usage: hostio.py [config] [frames] [batches] [streams] [rounds]"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
from usnetd_amd import lib, shard, traffic  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    nb = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    S = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 6
    ctx = lib.Ctx(0)
    L = ctx.L
    cfgs = [traffic.config(name, n=n, seed=shard.queue_seed(k, 0)) for k in range(nb)]
    cfg0 = cfgs[0]
    traffic.install_ctx(ctx, cfg0)
    nics = [cfg0.src] + traffic.extra_nics(cfg0, S - 1, ctx)
    W = cfg0.stride
    fbytes, lbytes = n * W, n * 2
    n_ep = max(max(e[0] for e in cfg0.endpoints), max(nics)) + 1   # the extra NICs are endpoints too
    obytes = n * 4 + n * 4 + (n_ep + 4) * 4   # decisions | index | bin_off
    host = []
    for cfg in cfgs:
        hp = C.c_void_p()
        lib.check(L.usn_host_alloc_pinned(ctx.h, fbytes + lbytes + obytes, C.byref(hp)))
        C.memmove(hp.value, cfg.frames.ctypes.data, fbytes)
        C.memmove(hp.value + fbytes, cfg.lens.ctypes.data, lbytes)
        host.append(hp.value)
    streams = [ctx.stream() for _ in range(S)]
    # two device batch/result sets per stream: the carried cache reads the previous result
    dev = [[(lib.DeviceBatch(ctx, cfg0.frames, cfg0.lens, nics[si], stride=W), lib.DeviceResult(ctx, n))
            for _ in range(2)] for si in range(S)]
    pending = [None] * S      # (k, set) classified on stream si, not yet finalized
    flip = [0] * S
    host_frames = [0]

    def drain(si):
        if pending[si] is None:
            return
        k, j = pending[si]
        b, r = dev[si][j]
        s = streams[si]
        info = ctx.finalize(b, r, s)
        host_frames[0] += info.n_host
        hp = host[k]
        lib.check(L.usn_memcpy_d2h(ctx.h, hp + fbytes + lbytes, r.desc.decisions, n * 4, s))
        lib.check(L.usn_memcpy_d2h(ctx.h, hp + fbytes + lbytes + n * 4, r.desc.index, n * 4, s))
        lib.check(L.usn_memcpy_d2h(ctx.h, hp + fbytes + lbytes + n * 8, r.desc.bin_off, (n_ep + 4) * 4, s))
        pending[si] = None

    def one(k, si):
        drain(si)
        j = flip[si] = flip[si] ^ 1
        b, r = dev[si][j]
        s = streams[si]
        hp = host[k % nb]
        lib.check(L.usn_memcpy_h2d(ctx.h, b.buf.ptr, hp, fbytes, s))
        lib.check(L.usn_memcpy_h2d(ctx.h, b.lbuf.ptr, hp + fbytes, lbytes, s))
        lib.check(L.usn_classify(ctx.h, C.byref(b.desc), C.byref(r.desc), s))
        pending[si] = (k % nb, j)

    def finish():
        for si in range(S):
            drain(si)
        ctx.sync()

    for k in range(2 * S):
        one(k, k % S)
    finish()
    rates = []
    for _ in range(rounds):
        K = 4 * nb
        t0 = time.perf_counter()
        for k in range(K):
            one(k, k % S)
        finish()
        rates.append(K * n / (time.perf_counter() - t0) / 1e6)
    # every batch's decisions made the round trip and equal the oracle's
    import coracle
    coracle.build()
    bad = bad_lists = 0
    for k, cfg in enumerate(cfgs):
        o = coracle.Oracle()
        coracle.install_oracle(o, cfg0)
        want = o.forward_batch(cfg0.src, cfg.frames, cfg.lens, stride=W)
        got = np.frombuffer((C.c_uint8 * (n * 4)).from_address(host[k] + fbytes + lbytes), np.uint32)
        bad += int(((got ^ want) & lib.PARITY_MASK).astype(bool).sum())
        bins = lib.dec_bin(want, n_ep)
        idx = np.frombuffer((C.c_uint8 * (n * 4)).from_address(host[k] + fbytes + lbytes + n * 4), np.uint32)
        off = np.frombuffer((C.c_uint8 * ((n_ep + 4) * 4)).from_address(host[k] + fbytes + lbytes + n * 8),
                            np.uint32)
        want_off = np.concatenate([[0], np.cumsum(np.bincount(bins, minlength=n_ep + 3))])
        bad_lists += int(not np.array_equal(idx, np.argsort(bins, kind="stable").astype(np.uint32)))
        bad_lists += int(not np.array_equal(off.astype(np.int64), want_off))
    res = {"config": name, "mpps_median": round(float(np.median(rates)), 1),
           "mpps_all": [round(x, 1) for x in rates], "frames_per_batch": n, "streams": S,
           "h2d_bytes_per_frame": W + 2, "d2h_bytes_per_frame": 8,
           "pcie_gbs_equiv": round(float(np.median(rates)) * (W + 10) / 1e3, 1),
           "host_stage_frames": host_frames[0], "decisions_checked": nb * n,
           "decisions_differing_from_oracle": bad, "batches_with_lists_differing": bad_lists,
           "loop": "H2D windows+lens, usn_classify, usn_finalize, D2H decisions+index+bin_off; "
                   "%d streams, a stream's previous batch finalized before its next" % S}
    print(json.dumps(res))
    assert bad == 0 and bad_lists == 0


if __name__ == "__main__":
    main()
