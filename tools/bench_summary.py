#!/usr/bin/env python3
"""One line per config of a bench.py JSON line: value, launch fraction of
the HBM roofline, launch median, frames per launch, steady-state GB/s.
usage: bench_summary.py <bench.log>"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k, x in [("c5", d)] + [(k, d[k]) for k in ("c2", "c3", "c4", "c4tx") if k in d]:
    r = x.get("roofline", {})
    print("%-5s %10.1f Mpkt/s  frac %.4f  launch %8.2f us  frames %9d  steady %s GB/s"
          % (k, x.get("value"), r.get("frac") or 0, r.get("kernel_us_median") or 0,
             r.get("frames_per_launch") or 0, r.get("achieved_steady_state")))
