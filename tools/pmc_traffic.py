#!/usr/bin/env python3
"""HBM traffic per classify call from two rocprofv3 PMC passes (FETCH_SIZE
and WRITE_SIZE collected in separate runs, MI355X_MICROARCH.md §HBM):
  bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024
FETCH_SIZE is doubled because on gfx950 it tallies the 128-byte requests of
coalesced streaming reads at 64 B; the known read volume of a call (64 B
window + 2 B length per frame) checks the factor (fetch_vs_algorithmic).

One usn_classify_multi call = classify_rx_kernel (or tx_kernel) + the
per-endpoint scatter (scan_kernel, scatter_kernel): the
counters of every dispatch of these kernels are summed per kernel name and
divided by the number of classify / tx dispatches covering `frames` frames
(every call of the run has that shape).
usage: pmc_traffic.py <fetch_dir> <write_dir> <frames_per_launch> <out.json> [KERNEL=F[+B] ...]
KERNEL=F: that kernel's FETCH_SIZE counted xF instead of x2.  KERNEL=1+B: a
kernel that mixes both kinds of read (the tx kernel: its header windows are
coalesced 128-byte requests, its rule probes scattered 64-byte ones) counted
x1 plus the B bytes per frame its coalesced reads' requests are short of
(the tx kernel's 64-byte header line and 2-byte length per frame, tallied at
32 and 1: tx_kernel=1+33; calibration: tools/tx_pmc_cal.hip under the TCC
request counters, profiles/r05/r05i/pmc_cal.json -- the header pattern 0.50
requests per frame tallied at 32 B, the lengths at 1 B, a scattered 16-byte
probe one request tallied at 64 B, a kernel mixing the three within 3 % of
its parts; the guide's x2 for the whole kernel is reported beside it as
hbm_bytes_per_launch_x2).  c3's classify
reads one window per 2048-byte slot inside the first 64-byte half of a line:
a 64-byte EA request, which FETCH_SIZE (= TCC_EA0_RDREQ x 64 B) counts
exactly, so c3 uses classify_rx_kernel=1 (calibration: tools/stride_floor.hip
under --pmc, profiles/r04/r04a/stride_floor_pmc.json)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ("classify_rx_kernel", "tx_kernel", "scan_kernel", "scatter_kernel", "txstate_kernel")
MAIN = ("classify_rx_kernel", "tx_kernel")


def per_kernel(d, counter, frames):
    """{kernel: summed counter}, and the number of classify dispatches
    covering `frames` frames (1024-frame tiles of 512 or 256 threads)."""
    tot = defaultdict(float)
    calls = 0
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = next((k for k in KERNELS if k in r.get("Kernel_Name", "")), None)
            if k is None:
                continue
            tot[k] += float(r["Counter_Value"])
            if k in MAIN and int(r["Grid_Size"]) in (frames // 4, frames // 2):
                calls += 1
    return tot, calls


def main():
    fd, wd, frames, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    factor, extra = {}, {}
    for kv in sys.argv[5:]:
        k, f = kv.split("=", 1)
        f, _, b = f.partition("+")
        factor[k] = float(f)
        if b:
            extra[k] = float(b)
    fetch, nf = per_kernel(fd, "FETCH_SIZE", frames)
    write, nw = per_kernel(wd, "WRITE_SIZE", frames)
    if not nf or not nw:
        sys.exit("no classify dispatch of %d frames in %s / %s" % (frames, fd, wd))
    rd = {k: factor.get(k, 2.0) * v * 1024 / nf + extra.get(k, 0.0) * frames for k, v in fetch.items()}
    wr = {k: v * 1024 / nw for k, v in write.items()}
    read_algo = frames * (64 + 2)
    write_algo = frames * (4 + 4)
    res = {
        "frames_per_launch": frames,
        "calls": [nf, nw],
        "hbm_read_bytes_per_launch": int(sum(rd.values())),
        "hbm_write_bytes_per_launch": int(sum(wr.values())),
        "hbm_bytes_per_launch": int(sum(rd.values()) + sum(wr.values())),
        "algorithmic_bytes_per_launch": frames * 74,
        "per_kernel_read_bytes": {k: int(v) for k, v in rd.items()},
        "per_kernel_write_bytes": {k: int(v) for k, v in wr.items()},
        "fetch_vs_algorithmic": round(sum(rd.values()) / read_algo, 4),
        "write_vs_algorithmic": round(sum(wr.values()) / write_algo, 4),
        "traffic_vs_algorithmic": round((sum(rd.values()) + sum(wr.values())) / (frames * 74), 4),
        # every kernel's FETCH_SIZE x2 (the guide's streaming correction), beside the model
        "hbm_bytes_per_launch_x2": int(sum(2.0 * v * 1024 / nf for v in fetch.values()) + sum(wr.values())),
        "correction": "FETCH_SIZE x2 (gfx950, 128-B requests tallied at 64 B), WRITE_SIZE x1" +
                      "".join("; %s FETCH_SIZE x%g%s" % (k, f, " + %g B/frame" % extra[k] if k in extra else "")
                              for k, f in sorted(factor.items())),
    }
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
