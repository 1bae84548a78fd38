#!/usr/bin/env python3
"""PCIe-inclusive rate of the match path: frames start and end in host memory.

Per batch (one drained ring): pinned-host frames + lengths -> hipMemcpyAsync
H2D -> usn_classify -> D2H of the decisions and the per-endpoint order.
Batches go round-robin over S streams (one rx queue each), so copies of one
batch overlap the kernel of another.  Reported for DESIGN.md; never the bench
value.  usage: hostio.py [frames] [batches] [streams] [rounds]"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from usnetd_amd import lib, traffic  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 6
    ctx = lib.Ctx(0)
    L = ctx.L
    cfg0 = traffic.config("c2", n=n, seed=2)
    traffic.install_ctx(ctx, cfg0)
    nics = [0] + traffic.extra_nics(cfg0, S - 1, ctx)
    fbytes, lbytes = n * 64, n * 2
    host = []
    for k in range(nb):
        cfg = cfg0 if k == 0 else traffic.config("c2", n=n, seed=17 * k + 2)
        hp = C.c_void_p()
        lib.check(L.usn_host_alloc_pinned(ctx.h, fbytes + lbytes + n * 6, C.byref(hp)))
        C.memmove(hp.value, cfg.frames.ctypes.data, fbytes)
        C.memmove(hp.value + fbytes, cfg.lens.ctypes.data, lbytes)
        host.append(hp.value)
    streams = [ctx.stream() for _ in range(S)]
    dev = []
    for si in range(S):
        b = lib.DeviceBatch(ctx, cfg0.frames, cfg0.lens, nics[si], stride=64)
        r = lib.DeviceResult(ctx, n)
        dev.append((b, r))

    def one(k, si):
        b, r = dev[si]
        s = streams[si]
        hp = host[k % nb]
        lib.check(L.usn_memcpy_h2d(ctx.h, b.buf.ptr, hp, fbytes, s))
        lib.check(L.usn_memcpy_h2d(ctx.h, b.lbuf.ptr, hp + fbytes, lbytes, s))
        lib.check(L.usn_classify(ctx.h, C.byref(b.desc), C.byref(r.desc), s))
        lib.check(L.usn_memcpy_d2h(ctx.h, hp + fbytes + lbytes, r.desc.decisions, n * 4, s))
        lib.check(L.usn_memcpy_d2h(ctx.h, hp + fbytes + lbytes + n * 4, r.desc.order, n * 2, s))

    for k in range(2 * S):
        one(k, k % S)
    ctx.sync()
    rates = []
    for _ in range(rounds):
        K = 4 * nb
        t0 = time.perf_counter()
        for k in range(K):
            one(k, k % S)
        ctx.sync()
        rates.append(K * n / (time.perf_counter() - t0) / 1e6)
    # the decisions of one batch made the round trip intact
    out = np.frombuffer((C.c_uint8 * (n * 4)).from_address(host[0] + fbytes + lbytes), np.uint32)
    assert (out >> 16 & 0xF).max() <= 3
    res = {"mpps_median": round(float(np.median(rates)), 1), "mpps_all": [round(x, 1) for x in rates],
           "frames_per_batch": n, "streams": S,
           "h2d_bytes_per_frame": 66, "d2h_bytes_per_frame": 6,
           "pcie_gbs_equiv": round(float(np.median(rates)) * 72 / 1e3, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
