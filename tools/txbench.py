#!/usr/bin/env python3
"""tx-direction timing (c4tx): device time of one usn_classify call (the tx
launch plus the per-endpoint scatter; HIP events on the launch stream),
usn_finalize wall time (it waits for the launch, then applies the learned
state and runs any host tail) and the classify call's wall time (the table
rebuild when the previous batch learned), per batch.

Usage: python tools/txbench.py [n] [batches] [distinct] [libpath] [--rotate R] [--rings 2]
  distinct > 1 rotates over that many differently-seeded rings (new flows
  keep learning answer rules); 1 replays one ring (steady state: nothing new).
  --rotate R: the one ring's frames in R distinct device buffers used in turn
  (same flows, nothing new learned after the first batch, and R x the ring's
  bytes touched between two uses of a buffer: with R x 64 MiB > 256 MiB no
  batch is served from the Infinity Cache -- SURVEY §8d's anti-cache rule).
  --rings R: R consecutive rings per launch (one tx grid, usn_classify_multi);
  a row is then one launch (R x n frames).
  --concat K: each ring is K copies of the n generated frames (K x n frames,
  the same flows: the per-frame work of an n-frame ring in a larger grid).
"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("n", nargs="?", type=int, default=1 << 20)
    ap.add_argument("batches", nargs="?", type=int, default=8)
    ap.add_argument("distinct", nargs="?", type=int, default=1)
    ap.add_argument("libpath", nargs="?", default=None)
    ap.add_argument("--rotate", type=int, default=1)
    ap.add_argument("--rings", type=int, default=1, choices=range(1, 9))
    ap.add_argument("--concat", type=int, default=1)
    a = ap.parse_args()
    n, nb, distinct = a.n, a.batches, a.distinct
    cfgs = [traffic.c4tx(n=n, seed=6 + k) for k in range(distinct)]
    if a.concat > 1:
        for c in cfgs:
            c.frames = np.concatenate([c.frames[:n * c.stride]] * a.concat + [c.frames[n * c.stride:]])
            c.lens = np.concatenate([c.lens[:n]] * a.concat)
        n *= a.concat
    ctx = lib.Ctx(0, a.libpath) if a.libpath else lib.Ctx(0)
    traffic.install_ctx(ctx, cfgs[0])
    s = ctx.stream()
    batches = [lib.DeviceBatch(ctx, c.frames, c.lens, c.src, stride=c.stride) for c in cfgs]
    for _ in range(a.rotate - 1):   # the same ring again in another buffer
        batches.append(lib.DeviceBatch(ctx, cfgs[0].frames, cfgs[0].lens, cfgs[0].src,
                                       stride=cfgs[0].stride))
    R = a.rings
    results = [lib.DeviceResult(ctx, n) for _ in range(2 * R)]
    ev = [(ctx.event(), ctx.event()) for _ in range(nb)]
    rows = []
    for k in range(nb):
        bb = [batches[(R * k + q) % len(batches)] for q in range(R)]
        rr = [results[(R * k + q) % (2 * R)] for q in range(R)]
        t0 = time.perf_counter()
        ctx.record(ev[k][0], s)
        ctx.classify_multi(bb, rr, s)
        ctx.record(ev[k][1], s)
        t1 = time.perf_counter()
        infos = [ctx.finalize(b, r, s) for b, r in zip(bb, rr)]
        t2 = time.perf_counter()
        info = lib.FinalizeInfo()
        info.n_learned = sum(i.n_learned for i in infos)
        info.n_host = sum(i.n_host for i in infos)
        rows.append({"batch": k, "device_ms": round(ctx.elapsed_ms(*ev[k]), 4),
                     "classify_call_ms": round((t1 - t0) * 1e3, 3),
                     "finalize_ms": round((t2 - t1) * 1e3, 3),
                     "n_learned": int(info.n_learned), "n_host": int(info.n_host),
                     "rules": ctx.rule_count()})
        print(json.dumps(rows[-1]), flush=True)
    steady = rows[max(1, len(batches)):] or rows[1:]
    dev = np.array([x["device_ms"] for x in steady])
    fin = np.array([x["finalize_ms"] for x in steady])
    cal = np.array([x["classify_call_ms"] for x in steady])
    out = {"n": n, "rings_per_launch": R, "batches": nb, "distinct": distinct, "rotate_buffers": len(batches),
           "rotating_bytes": int(len(batches) * n * cfgs[0].stride),
           "device_ms_median": float(np.median(dev)),
           "device_mpps": round(R * n / np.median(dev) / 1e3, 1),
           "classify_call_ms_median": float(np.median(cal)),
           "finalize_ms_median": float(np.median(fin)),
           # usn_finalize synchronises the stream first, so its wall time
           # holds the kernel's: a batch costs classify call + finalize
           "end_to_end_mpps": round(R * n / (np.median(fin) + np.median(cal)) / 1e3, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
