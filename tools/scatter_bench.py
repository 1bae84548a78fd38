#!/usr/bin/env python3
"""Device time of the per-endpoint scatter alone (scan_agg + scan_chunks +
scatter kernels, usn_debug_scatter) on classified batches of a config, per
A/B build (build/abl/<name>/libusn.so; "base" = the in-tree library).

usage: python tools/scatter_bench.py [--config c5] [--frames N] [--multi 2] [--launches 50] [variants...]
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from usnetd_amd import lib, traffic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--frames", type=int, default=1 << 23)
    ap.add_argument("--multi", type=int, default=2)
    ap.add_argument("--launches", type=int, default=50)
    ap.add_argument("--json", default="")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    names = a.variants or ["base"]
    cfgs = [traffic.config(a.config, n=a.frames, seed=17 * k + 2) for k in range(a.multi)]
    out = {}
    first_idx = None   # the first variant's lists: every other variant must equal them
    for nm in names:
        path = None if nm == "base" else os.path.join(ROOT, "build", "abl", nm, "libusn.so")
        ctx = lib.Ctx(0, libpath=path)
        traffic.install_ctx(ctx, cfgs[0])
        nics = [cfgs[0].src] + list(traffic.extra_nics(cfgs[0], a.multi - 1, ctx))
        bs = [lib.DeviceBatch(ctx, c.frames, c.lens, nics[k], stride=c.stride) for k, c in enumerate(cfgs)]
        rs = [lib.DeviceResult(ctx, a.frames) for _ in cfgs]
        ba = (lib.Batch * a.multi)(*[b.desc for b in bs])
        ra = (lib.Result * a.multi)(*[r.desc for r in rs])
        s = ctx.stream()
        lib.check(ctx.L.usn_classify_multi(ctx.h, C.cast(ba, C.c_void_p), C.cast(ra, C.c_void_p),
                                           a.multi, s), "classify")
        ctx.sync(s)
        ref = [r.index() for r in rs]
        f = ctx.L.usn_debug_scatter
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]
        evs = [(ctx.event(), ctx.event()) for _ in range(a.launches)]
        for i in range(5):
            f(ctx.h, C.cast(ba, C.c_void_p), C.cast(ra, C.c_void_p), a.multi, s)
        for x, y in evs:
            ctx.record(x, s)
            lib.check(f(ctx.h, C.cast(ba, C.c_void_p), C.cast(ra, C.c_void_p), a.multi, s), "scatter")
            ctx.record(y, s)
        ctx.sync(s)
        us = [ctx.elapsed_ms(x, y) * 1e3 for x, y in evs]
        same = all((r.index() == x).all() for r, x in zip(rs, ref))
        idx = [r.index() for r in rs]
        if first_idx is None:
            first_idx = idx
        same_first = all((x == y).all() for x, y in zip(idx, first_idx))
        med = statistics.median(us)
        out[nm] = dict(scatter_us=round(med, 2), min_us=round(min(us), 2), same_as_classify=same,
                       same_as_first_variant=same_first, frames=a.frames * a.multi)
        print("%-10s scatter %8.2f us (min %8.2f) per %d frames  %.1f GB/s of 12 B/frame  same=%s"
              " same_as_first=%s"
              % (nm, med, min(us), a.frames * a.multi, 12 * a.frames * a.multi / med / 1e3, same,
                 same_first), flush=True)
        if nm.startswith("stamps"):   # the diagnostic build: phase medians of the last launch
            import numpy as np
            buf = np.zeros(2 * 16384 * 16, np.uint64)   # the scatter's stamps: slots 16384..
            fn = ctx.L.usn_debug_stamps512
            fn.argtypes = [C.c_void_p, C.c_size_t]
            assert fn(buf.ctypes.data, buf.nbytes) == 0
            chunks = sum(rs[0].ntiles for _ in rs) // 8 or 1
            st = buf.reshape(2 * 16384, 16)[16384:16384 + min(chunks, 16384), :12].astype(np.int64)
            t0 = st[:, 0].min()
            names = ["start", "bases+barrier"] + ["tile %d" % k for k in range(8)] + ["loop end", "write-out"]
            for k in range(1, 12):
                dk = (st[:, k] - st[:, k - 1]) * 10 / 1000.0   # 100 MHz ticks -> us
                print("   %-14s median %7.2f us  p90 %7.2f" % (names[k], np.median(dk), np.percentile(dk, 90)))
            print("   span start %.2f..%.2f us, end %.2f..%.2f us, per chunk %.2f us" % (
                0, (st[:, 0].max() - t0) / 100, (st[:, 11].min() - t0) / 100, (st[:, 11].max() - t0) / 100,
                np.median(st[:, 11] - st[:, 0]) / 100), flush=True)
        for b in bs:
            b.free()
        for r in rs:
            r.free()
        ctx.close()
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(dict(config=a.config, variants=out), fh, indent=1)


if __name__ == "__main__":
    main()
