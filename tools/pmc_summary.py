#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output (counter_collection.csv) per kernel:
mean value of each counter per dispatch.  usage: pmc_summary.py <dir>..."""
import csv
import glob
import os
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "?")
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print("  %-28s n=%4d mean=%.4g" % (c, len(v), sum(v) / len(v)))
