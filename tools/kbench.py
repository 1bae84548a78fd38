#!/usr/bin/env python3
"""Minimal driver for profiling: N back-to-back usn_classify launches of one
config (no oracle, no CPU baseline).  usage: kbench.py [config] [frames] [launches] [libpath]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from usnetd_amd import lib, traffic  # noqa: E402

cfgname = sys.argv[1] if len(sys.argv) > 1 else "c2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
launches = int(sys.argv[3]) if len(sys.argv) > 3 else 50
libpath = sys.argv[4] if len(sys.argv) > 4 else None
nb = 5
ctx = lib.Ctx(0, libpath=libpath)
cfgs = [traffic.config(cfgname, n=n, seed=17 * k + 2) for k in range(nb)]
traffic.install_ctx(ctx, cfgs[0])
bs = [lib.DeviceBatch(ctx, c.frames, c.lens, c.src, stride=c.stride) for c in cfgs]
rs = [lib.DeviceResult(ctx, n) for _ in cfgs]
s = ctx.stream()
for i in range(launches):
    lib.check(ctx.L.usn_classify(ctx.h, C.byref(bs[i % nb].desc), C.byref(rs[i % nb].desc), s))
ctx.sync(s)
print("kbench done", cfgname, n, launches)
