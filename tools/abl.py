#!/usr/bin/env python3
"""Interleaved A/B timing of kernel variants in ONE process (cdna guide §5.4
rule 24).  Each variant is a build of the same C ABI (make abl ->
build/abl/<name>/libusn.so).  Prints per-variant median kernel time per
launch (HIP events around each launch) and back-to-back time per step.

usage: python tools/abl.py [--config c2] [--frames N] [--rounds 5] [--launches 100] [variants...]
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from usnetd_amd import lib, traffic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--batches", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=100)
    ap.add_argument("--json", default="")
    ap.add_argument("--streams", type=int, default=1,
                    help="round-robin batches over S streams, one NIC rx queue (source) each")
    ap.add_argument("--multi", type=int, default=1,
                    help="classify Q batches of Q distinct rx queues per launch (usn_classify_multi)")
    ap.add_argument("--private", dest="shared", action="store_false",
                    help="each variant allocates its own batches (default: shared buffers)")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    names = a.variants or sorted(os.listdir(os.path.join(ROOT, "build", "abl")))
    cfgs = [traffic.config(a.config, n=a.frames, seed=17 * k + 2) for k in range(a.batches)]
    runs = {}
    first = None
    for nm in names:
        # "build@ENV=VAL,ENV2=VAL": the build's library with context knobs set
        # while its context is created (USN_PH_GROUP, USN_PH_LOAD, USN_T512)
        build, _, knobs = nm.partition("@")
        # "product": the in-tree library (usnetd_amd/libusn.so, always the tree
        # under test); other names: build/abl/<name>, built by `make abl` or
        # tools/abl_commit.sh (rebuild them with the tree they are to match)
        # "testlib": the test build of the tree (build/test/libusn.so), which
        # reads the context knobs after "@" (USN_RX_EV, USN_TIMING_EV, ...)
        path = None if build == "product" else lib.TEST_LIB_PATH if build == "testlib" else \
            os.path.join(ROOT, "build", "abl", build, "libusn.so")
        saved = {}
        for kv in filter(None, knobs.split(",")):
            k, v = kv.split("=", 1)
            saved[k] = os.environ.get(k)
            os.environ[k] = v
        ctx = lib.Ctx(0, libpath=path)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        traffic.install_ctx(ctx, cfgs[0])
        nq = max(a.streams, a.multi)
        nics = [0] + list(traffic.extra_nics(cfgs[0], nq - 1, ctx))
        # parity check: batch 0 into a private result of this variant
        print("variant %s: check launch" % nm, flush=True)
        chk_b = lib.DeviceBatch(ctx, cfgs[0].frames, cfgs[0].lens, nics[0], stride=cfgs[0].stride)
        chk_r = lib.DeviceResult(ctx, a.frames)
        cs = ctx.stream()
        lib.check(ctx.L.usn_classify(ctx.h, C.byref(chk_b.desc), C.byref(chk_r.desc), cs))
        ctx.sync(cs)
        chk = chk_r.decisions()
        if first is None or not a.shared:
            bs = [lib.DeviceBatch(ctx, c.frames, c.lens, nics[k % nq], stride=c.stride)
                  for k, c in enumerate(cfgs)]
            rs = [lib.DeviceResult(ctx, a.frames) for _ in cfgs]
            first = (bs, rs)
        else:
            # the same device buffers for every variant: a variant's speed must not
            # depend on where its own allocations landed in HBM
            bs, rs = first
        s = ctx.stream()
        ss = [s] + [ctx.stream() for _ in range(a.streams - 1)]
        evs = [(ctx.event(), ctx.event()) for _ in range(a.launches)]
        e0, e1 = ctx.event(), ctx.event()
        groups = []
        if a.multi > 1:
            assert a.batches % a.multi == 0
            for g in range(a.batches // a.multi):
                ba = (lib.Batch * a.multi)(*[bs[g * a.multi + j].desc for j in range(a.multi)])
                ra = (lib.Result * a.multi)(*[rs[g * a.multi + j].desc for j in range(a.multi)])
                groups.append((ba, ra))
        runs[nm] = dict(ctx=ctx, bs=bs, rs=rs, s=s, chk=chk, ss=ss, evs=evs, e0=e0, e1=e1, per=[], b2b=[],
                        ejoin=[ctx.event() for _ in ss], groups=groups)
    for rnd in range(a.rounds):
        for nm in names:
            R = runs[nm]
            ctx, s = R["ctx"], R["s"]
            L = ctx.L
            bd = [C.byref(b.desc) for b in R["bs"]]
            rd = [C.byref(r.desc) for r in R["rs"]]
            G = R["groups"]

            def launch(i, stream):
                if G:
                    ba, ra = G[i % len(G)]
                    return L.usn_classify_multi(ctx.h, C.cast(ba, C.c_void_p), C.cast(ra, C.c_void_p),
                                                a.multi, stream)
                return L.usn_classify(ctx.h, bd[i % len(bd)], rd[i % len(rd)], stream)
            for i in range(10):
                launch(i, s)
            for i, (x, y) in enumerate(R["evs"]):
                ctx.record(x, s)
                rc = launch(i, s)
                assert rc == 0, rc
                ctx.record(y, s)
            ctx.sync(s)
            R["per"] += [ctx.elapsed_ms(x, y) * 1e3 for x, y in R["evs"]]
            ss = R["ss"]
            ctx.record(R["e0"], s)
            for x in ss[1:]:
                ctx.wait_event(x, R["e0"])
            for i in range(a.launches):
                # batch k always goes to stream k % S (its rx queue): per-source order kept
                if G:
                    launch(i, ss[(i % len(G)) % len(ss)])
                else:
                    k = i % len(bd)
                    L.usn_classify(ctx.h, bd[k], rd[k], ss[k % len(ss)])
            for x, ej in zip(ss[1:], R["ejoin"]):
                ctx.record(ej, x)
                ctx.wait_event(s, ej)
            ctx.record(R["e1"], s)
            ctx.sync(s)
            R["b2b"].append(ctx.elapsed_ms(R["e0"], R["e1"]) * 1e3 / a.launches / max(1, a.multi))
    ref = None
    out = {}
    for nm in names:
        R = runs[nm]
        d = R["chk"]
        if ref is None:
            ref = d
        same = bool(((d ^ ref) & lib.PARITY_MASK).max() == 0) if d.shape == ref.shape else False
        med = statistics.median(R["per"]) / max(1, a.multi)   # per batch
        b2b = statistics.median(R["b2b"])
        gbs = 72 * a.frames / (med * 1e-6) / 1e9
        out[nm] = dict(kernel_us=round(med, 2), kernel_us_min=round(min(R["per"]), 2),
                       step_us=round(b2b, 2), gbs=round(gbs, 1),
                       mpps=round(a.frames / b2b, 1), same_as_first=same)
        print("%-12s kernel %8.2f us (min %8.2f)  step %8.2f us  %7.1f GB/s  %9.1f Mpkt/s  same=%s"
              % (nm, med, min(R["per"]), b2b, gbs, a.frames / b2b, same), flush=True)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(dict(config=a.config, frames=a.frames, variants=out), fh, indent=1)


if __name__ == "__main__":
    main()
