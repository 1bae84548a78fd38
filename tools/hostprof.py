#!/usr/bin/env python3
"""Host time of usn_classify_multi by checkpoint (the test build's
usn_debug_host_prof; HPROF in usn_host.cpp): the bench's launches of one
config (bench.Run) enqueued round after round, the device draining between
bursts so the queue never fills; prints mean microseconds per call for each
segment and the ctypes call's own wall time.

usage: python tools/hostprof.py [config=c3] [rounds=400]"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from usnetd_amd import lib  # noqa: E402

SEGMENTS = ["lock+checks", "table/bridge/chains", "fill_args", "rx state", "launch_classify",
            "events", "launch_scatter", "batch records"]


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    ctx = lib.Ctx(0, lib.TEST_LIB_PATH)
    L = ctx.L
    prof = L.usn_debug_host_prof
    prof.argtypes = [C.c_void_p, C.c_int]
    prof.restype = C.c_int
    run = bench.Run(L, ctx, name, bench.DEFAULT_FRAMES[name], 0, 1, bench.EXTRA_QUEUES.get(name, 0),
                    0, False)
    buf = (C.c_uint64 * 16)()
    for i in range(2 * run.RR):   # warm-up
        run.step(i)
    ctx.sync()
    prof(buf, 1)
    wall = 0.0
    for i in range(rounds):
        t = time.perf_counter()
        run.step(i)
        wall += time.perf_counter() - t
        if i % 8 == 7:
            ctx.sync()
    ctx.sync()
    prof(buf, 0)
    calls = buf[15]
    out = {"config": name, "calls": int(calls), "launches_per_round": len(run.launches),
           "us_per_call": {s: round(buf[k + 1] / calls / 1e3, 2) for k, s in enumerate(SEGMENTS)},
           "inside_us_per_call": round(sum(buf[1:9]) / calls / 1e3, 2),
           "python_wall_us_per_call": round(wall * 1e6 / calls, 2)}
    print(json.dumps(out))
    run.free()


if __name__ == "__main__":
    main()
