#!/usr/bin/env python3
"""Phase timeline of the classify kernel from the diagnostic build
(build/abl/stamps: -DUSN_STAMPS=1).  Wave 0 of each workgroup stamps the
global 100 MHz clock at 12 phase boundaries; this prints, over workgroups,
the median / p90 of each phase and the spread of start and end times.
Only the SHARES are meaningful (the stamps add waits of their own)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from usnetd_amd import lib, traffic  # noqa: E402

NAMES = ["start", "loads issued", "table+zero barrier", "carry", "round0 decided / probes issued",
         "all rounds decided", "stores+hostlist+lastreduce", "-", "-", "-",
         "tile_order+cls", "header"]
# c4tx: the one-launch tx kernel (stamps indexed by tile)
TX_NAMES = ["start", "header loads + bridge", "parse, flags, probes", "LAST out",
            "hits, HEAD/INS out, walk back", "look-back", "decisions", "fill, host list", "-", "-",
            "tile_order+cls", "header"]
TX_STEPS = [1, 2, 3, 4, 5, 6, 7, 10, 11]


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    rings = int(sys.argv[3]) if len(sys.argv) > 3 else 1   # c4tx: consecutive rings per grid
    path = os.path.join(ROOT, "build", "abl", os.environ.get("STAMPS_BUILD", "stamps"), "libusn.so")
    ctx = lib.Ctx(0, libpath=path)
    # tx: one ring replayed (steady state: its answer rules are learned by the first pass)
    if cfgname == "c4tx":   # one ring's frames (seed 6) in 8 device buffers
        cfgs = [traffic.config(cfgname, n=n, seed=6)] * 8
    else:
        cfgs = [traffic.config(cfgname, n=n, seed=17 * k + 2) for k in range(5)]
    traffic.install_ctx(ctx, cfgs[0])
    bs = [lib.DeviceBatch(ctx, c.frames, c.lens, c.src, stride=c.stride) for c in cfgs]
    rs = [lib.DeviceResult(ctx, n) for _ in cfgs]
    s = ctx.stream()
    tx = cfgname == "c4tx"
    if rings > 1:   # c4tx: one grid of `rings` consecutive rings (one ring's frames in 5 buffers)
        assert tx and rings <= 8
        rs2 = [lib.DeviceResult(ctx, n) for _ in range(2 * rings)]
        for i in range(12):
            grp = [(i * rings + k) % 8 for k in range(rings)]
            res = [rs2[(i % 2) * rings + k] for k in range(rings)]
            ctx.classify_multi([bs[g] for g in grp], res, s)
            for g, r in zip(grp, res):
                ctx.finalize(bs[g], r, s)
    else:
        for i in range(40):
            lib.check(ctx.L.usn_classify(ctx.h, C.byref(bs[i % 5].desc), C.byref(rs[i % 5].desc), s))
            if tx:
                ctx.finalize(bs[i % 5], rs[i % 5], s)
    ctx.sync(s)
    ntiles = rings * ((n + 1023) // 1024)
    buf = np.zeros(16384 * 16, np.uint64)
    # the build that ran: the 512-thread one (every config now) or the 256-thread
    # one (STAMPS512=0 forces it); the other's buffer is all zero
    names_fn = ["usn_debug_stamps"] if os.environ.get("STAMPS512") == "0" else ["usn_debug_stamps512",
                                                                               "usn_debug_stamps"]
    for nm in names_fn:
        fn = getattr(ctx.L, nm)
        fn.argtypes = [C.c_void_p, C.c_size_t]
        rc = fn(buf.ctypes.data, buf.nbytes)
        assert rc == 0, rc
        if buf.any():
            break
    st = buf.reshape(16384, 16)[:ntiles, :12].astype(np.int64)
    t0 = st[:, 0].min()
    us = lambda x: x / 100.0   # 100 MHz ticks -> us
    print("%s n=%d tiles=%d  kernel span %.2f us" % (cfgname, n, ntiles, us(st[:, 11].max() - t0)))
    print("start offset: median %.2f p90 %.2f max %.2f us" % tuple(
        us(np.percentile(st[:, 0] - t0, q)) for q in (50, 90, 100)))
    print("end   offset: median %.2f p90 %.2f max %.2f us" % tuple(
        us(np.percentile(st[:, 11] - t0, q)) for q in (50, 90, 100)))
    names, steps = (TX_NAMES, TX_STEPS) if tx else (NAMES, [1, 2, 3, 4, 5, 6, 10, 11])
    for i, k in enumerate(steps):
        prev = steps[i - 1] if i else 0
        d = st[:, k] - st[:, prev]
        print("  %-28s median %6.2f  p90 %6.2f  max %6.2f us" % (
            names[k], us(np.median(d)), us(np.percentile(d, 90)), us(d.max())))
        e = st[:, k] - t0
        print("  %-28s   (at: median %6.2f  p90 %6.2f  max %6.2f us)" % (
            "", us(np.median(e)), us(np.percentile(e, 90)), us(e.max())))
    tot = st[:, 11] - st[:, 0]
    print("  %-28s median %6.2f  p90 %6.2f  max %6.2f us" % ("TOTAL per block", us(np.median(tot)),
                                                        us(np.percentile(tot, 90)), us(tot.max())))
    # workgroups in flight: the stamped part of every block over the span.  Below
    # what the chip holds, the rest is dispatch, prologue and the stamp flush.
    span = st[:, 11].max() - t0
    print("  workgroups in flight (stamped part): mean %.1f; mean block %.2f us, %.1f blocks per slot"
          % (tot.sum() / span, us(tot.mean()), ntiles / max(1.0, tot.sum() / span)))


if __name__ == "__main__":
    main()
