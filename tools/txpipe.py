#!/usr/bin/env python3
"""c4tx alone, as bench.py measures it (measure_tx: sequential and pipelined
rings, end to end with usn_finalize), for A/B runs under library env knobs
(e.g. USN_TX_LISTS_SIDE=1).  Prints one JSON line.

usage: python tools/txpipe.py [--steps K] [--warmup W]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from usnetd_amd import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    a = ap.parse_args()
    ctx = lib.Ctx(0)
    a.no_cpu_baseline = True
    x = bench.measure_tx(ctx, a)
    keep = ("value", "pipelined_with_events_mpps", "sequential_mpps", "device_mpps", "ms_per_ring", "rings",
            "learned_in_timed_rings")
    print(json.dumps({k: x[k] for k in keep if k in x}))


if __name__ == "__main__":
    main()
