#!/usr/bin/env python3
"""HBM traffic per classify launch from two rocprofv3 PMC passes (FETCH_SIZE
and WRITE_SIZE collected in separate runs, MI355X_MICROARCH.md §HBM):
  bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024
FETCH_SIZE is doubled because on gfx950 it reports half of the bytes of a
16-byte-per-lane streaming read; our frame loads are 16 B per lane, and the
known read volume of a launch (64 B window + 2 B length per frame) checks the
factor (printed as fetch_vs_algorithmic).
usage: pmc_traffic.py <fetch_dir> <write_dir> <frames_per_launch> <out.json>"""
import csv
import glob
import json
import os
import statistics
import sys


def per_dispatch(d, counter, frames):
    """Counter values of the classify dispatches covering `frames` frames
    (1024-frame tiles: grid = frames / 4 threads for 256-thread workgroups,
    frames / 2 for the 512-thread build)."""
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if ("classify_rx_kernel" in r.get("Kernel_Name", "") and r["Counter_Name"] == counter
                    and int(r["Grid_Size"]) in (frames // 4, frames // 2)):
                vals.append(float(r["Counter_Value"]))
    return vals


fd, wd, frames, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
fetch = per_dispatch(fd, "FETCH_SIZE", frames)
write = per_dispatch(wd, "WRITE_SIZE", frames)
f_kb = statistics.median(fetch)
w_kb = statistics.median(write)
read_algo = frames * (64 + 2)
write_algo = frames * (4 + 2)
res = {
    "frames_per_launch": frames,
    "fetch_size_kb_median": f_kb, "write_size_kb_median": w_kb,
    "dispatches": [len(fetch), len(write)],
    "hbm_read_bytes_per_launch": int(2 * f_kb * 1024),
    "hbm_write_bytes_per_launch": int(w_kb * 1024),
    "hbm_bytes_per_launch": int((2 * f_kb + w_kb) * 1024),
    "algorithmic_bytes_per_launch": frames * 72,
    "fetch_vs_algorithmic": round(2 * f_kb * 1024 / read_algo, 4),
    "write_vs_algorithmic": round(w_kb * 1024 / write_algo, 4),
    "correction": "FETCH_SIZE x2 (gfx950, 16 B/lane loads), WRITE_SIZE x1",
}
os.makedirs(os.path.dirname(out), exist_ok=True)
with open(out, "w") as fh:
    json.dump(res, fh, indent=1)
print(json.dumps(res))
