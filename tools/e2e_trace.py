#!/usr/bin/env python3
"""Where bench.py's end-to-end loop (poll rounds with usn_finalize of every
ring) spends its host time, per config: per step, the calls' enqueue time,
and each usn_finalize call's time (the first of a round waits for the
round's launch).  Prints medians.
usage: e2e_trace.py [config=c3] [steps=200]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from usnetd_amd import lib  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
ctx = lib.Ctx(0)
n = bench.DEFAULT_FRAMES[name]
run = bench.Run(ctx.L, ctx, name, n, 0, 1, bench.extra_queues(name), 0, False)
for i in range(20):
    run.step(i)
run.finalize_all()
enq, fins, steps = [], [], []
t_prev = None
for i in range(K):
    t0 = time.perf_counter()
    run.step(i, e2e=True)
    t1 = time.perf_counter()
    enq.append(t1 - t0)
    if i:
        times = []
        run.finalize_round(i - 1, times)
        fins.append(times)
    t2 = time.perf_counter()
    if t_prev is not None:
        steps.append(t2 - t_prev)
    t_prev = t2
run.finalize_round(K - 1)
ctx.sync()
us = lambda v: round(statistics.median(v) * 1e6, 2)   # noqa: E731
per_pos = [us([f[k] for f in fins]) for k in range(len(fins[0]))]
print({"config": name, "rings_per_step": run.Q, "launches": [(s, list(q)) for s, q in run.launches],
       "step_us": us(steps), "enqueue_us": us(enq), "finalize_us_by_position": per_pos,
       "finalize_sum_us": round(sum(per_pos), 2)}, flush=True)
