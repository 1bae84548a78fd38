#!/usr/bin/env python3
"""Per-kernel duration summary of a rocprofv3 --kernel-trace CSV, split by
grid size and by whether a dispatch overlapped another classify dispatch in
time (concurrent launches on two streams share the GPU, so their durations
are not per-launch costs).  usage: trace_summary.py <kernel_trace.csv>"""
import csv
import statistics
import sys
from collections import defaultdict

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                 int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])))
rows.sort()
g = defaultdict(list)
for i, (s, e, k, wg) in enumerate(rows):
    ov = any(s2 < e and s < e2 for j, (s2, e2, k2, _) in enumerate(rows[max(0, i - 8):i + 9])
             if (j + max(0, i - 8)) != i and "classify" in k2)
    g[(k, wg, "overlapped" if ov else "isolated")].append((e - s) / 1e3)
print("| kernel | workgroups | timing | dispatches | mean us | median us | min us | max us |")
print("|---|---|---|---|---|---|---|---|")
for (k, wg, kind), v in sorted(g.items(), key=lambda x: (x[0][0], -x[0][1], x[0][2])):
    print("| %s | %d | %s | %d | %.2f | %.2f | %.2f | %.2f |" % (
        k[:58], wg, kind, len(v), statistics.mean(v), statistics.median(v), min(v), max(v)))
