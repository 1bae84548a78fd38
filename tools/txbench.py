#!/usr/bin/env python3
"""tx-direction timing (c4tx): device time of the tx launch (HIP events on
the launch stream), usn_finalize wall time (it waits for the launch, then
applies the learned state and runs any host tail) and the classify call's
wall time (the table rebuild when the previous batch learned), per batch.

Usage: python tools/txbench.py [n] [batches] [distinct]
  distinct > 1 rotates over that many differently-seeded rings (new flows
  keep learning answer rules); 1 replays one ring (steady state: nothing new).
"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

from usnetd_amd import lib, traffic  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    distinct = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    libpath = sys.argv[4] if len(sys.argv) > 4 else None   # an A/B build (build/abl/<v>/libusn.so)
    cfgs = [traffic.c4tx(n=n, seed=6 + k) for k in range(distinct)]
    ctx = lib.Ctx(0, libpath) if libpath else lib.Ctx(0)
    traffic.install_ctx(ctx, cfgs[0])
    s = ctx.stream()
    batches = [lib.DeviceBatch(ctx, c.frames, c.lens, c.src, stride=c.stride) for c in cfgs]
    results = [lib.DeviceResult(ctx, n) for _ in range(2)]
    ev = [(ctx.event(), ctx.event()) for _ in range(nb)]
    rows = []
    for k in range(nb):
        b, r = batches[k % distinct], results[k % 2]
        t0 = time.perf_counter()
        ctx.record(ev[k][0], s)
        ctx.classify(b, r, s)
        ctx.record(ev[k][1], s)
        t1 = time.perf_counter()
        info = ctx.finalize(b, r, s)
        t2 = time.perf_counter()
        dbg = (C.c_uint32 * 10)()
        if hasattr(ctx.L, "usn_debug_tx_state"):
            ctx.L.usn_debug_tx_state.argtypes = [C.c_void_p, C.c_void_p]
        if hasattr(ctx.L, "usn_debug_tx_state") and ctx.L.usn_debug_tx_state(ctx.h, dbg) == 0:
            print("tx state", list(dbg), flush=True)
        rows.append({"batch": k, "device_ms": round(ctx.elapsed_ms(*ev[k]), 4),
                     "classify_call_ms": round((t1 - t0) * 1e3, 3),
                     "finalize_ms": round((t2 - t1) * 1e3, 3),
                     "n_learned": int(info.n_learned), "n_host": int(info.n_host),
                     "rules": ctx.rule_count()})
        print(json.dumps(rows[-1]), flush=True)
    dev = np.array([x["device_ms"] for x in rows[1:]])
    fin = np.array([x["finalize_ms"] for x in rows[1:]])
    cal = np.array([x["classify_call_ms"] for x in rows[1:]])
    out = {"n": n, "batches": nb, "distinct": distinct,
           "device_ms_median": float(np.median(dev)),
           "device_mpps": round(n / np.median(dev) / 1e3, 1),
           "classify_call_ms_median": float(np.median(cal)),
           "finalize_ms_median": float(np.median(fin)),
           # usn_finalize synchronises the stream first, so its wall time
           # holds the kernel's: a batch costs classify call + finalize
           "end_to_end_mpps": round(n / (np.median(fin) + np.median(cal)) / 1e3, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
