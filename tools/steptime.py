#!/usr/bin/env python3
"""Where does a short timed run lose time?  bench.py's Run for c5, then
repeated timed runs of K steps (HIP events per step on the main stream).
usage: steptime.py [K] [repeats]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from usnetd_amd import lib  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
ctx = lib.Ctx(0)
run = bench.Run(ctx.L, ctx, "c5", 1 << 23, 0, 1, 0, 2, False)
for i in range(5):
    run.step(i)
kern, _ = run.launch_probe(20)
print("probe launch us", round(kern * 1e3, 1))
for rep in range(reps):
    wall, ev = run.timed(K, None)
    print("run %d: K=%d wall ms/step %.4f event ms/step %.4f" % (rep, K, wall * 1e3 / K, ev / K), flush=True)
wall, ev = run.timed(200, None)
print("K=200 wall ms/step %.4f event ms/step %.4f" % (wall * 1e3 / 200, ev / 200))
