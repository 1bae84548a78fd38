#!/usr/bin/env python3
"""Per-unit TCC request counts of tools/tx_pmc_cal.hip's calibration kernels
and of the tx call's kernels (tools/txbench.py), from rocprofv3 --pmc passes
(counter CSVs under the given directories), and the tx kernel's read bytes
under each model:
  raw       FETCH_SIZE as reported
  x2        the guide's streaming correction applied to the whole kernel
  1+32      tools/pmc_traffic.py's model (FETCH_SIZE x1 + 32 B per frame)
  calibrated  headers at the bytes of their lines (64 B per frame, whatever
            cal_hdr's tally of that pattern is), lengths at 2 B per frame, the
            rest (probes, sets, learned lists) at cal_probe's tally
usage: pmc_cal_summary.py <frames_per_tx_launch> <out.json> <pass_dir> [...]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

COUNTERS = ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_BUBBLE_sum", "FETCH_SIZE",
            "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum", "WRITE_SIZE")


def short(name):
    for k in ("cal_hdr", "cal_lens", "cal_mixed", "tx_kernel", "scan_kernel", "scatter_kernel"):
        if k in name:
            return k
    m = re.search(r"cal_probe<(\d+)>", name)
    return "cal_probe_%s" % ("8MiB" if m and m.group(1) == "8" else "1GiB") if "cal_probe" in name else None


def median(v):
    v = sorted(v)
    return v[len(v) // 2]


def main():
    frames_tx, out = int(sys.argv[1]), sys.argv[2]
    vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> per dispatch
    grid = {}
    for d in sys.argv[3:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r.get("Kernel_Name", ""))
                if k is None or r["Counter_Name"] not in COUNTERS:
                    continue
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                grid[k] = int(r["Grid_Size"])
    res = {}
    for k, cs in vals.items():
        frames = grid[k] if k.startswith("cal_") else frames_tx
        row = {"frames": frames}
        for c, v in cs.items():
            x = median(v)
            if c in ("FETCH_SIZE", "WRITE_SIZE"):
                row[c.lower() + "_bytes_per_frame"] = round(x * 1024 / frames, 3)
            else:
                row[c[:-4].lower() + "_per_frame"] = round(x / frames, 4)
        res[k] = row
    cal = {}
    try:
        hdr = res["cal_hdr"]["fetch_size_bytes_per_frame"]
        lens = res["cal_lens"]["fetch_size_bytes_per_frame"]
        cal["hdr_tally_per_frame"] = hdr
        cal["hdr_factor"] = round(64.0 / hdr, 3) if hdr else None
        cal["lens_tally_per_frame"] = lens
        for t in ("cal_probe_8MiB", "cal_probe_1GiB"):
            if t in res:
                cal[t + "_tally_per_probe"] = round(res[t]["fetch_size_bytes_per_frame"] / 3, 2)
                cal[t + "_rdreq_per_probe"] = round(res[t].get("tcc_ea0_rdreq_per_frame", 0) / 3, 3)
        mix = res.get("cal_mixed", {}).get("fetch_size_bytes_per_frame")
        parts = hdr + lens + res["cal_probe_8MiB"]["fetch_size_bytes_per_frame"]
        if mix:
            cal["mixed_tally_vs_parts"] = round(mix / parts, 4)
        tx = res["tx_kernel"]["fetch_size_bytes_per_frame"]
        cal["tx_kernel_read_bytes_per_frame"] = {
            "raw": round(tx, 2), "x2": round(2 * tx, 2), "1+32": round(tx + 32, 2),
            "calibrated": round(64 + 2 + (tx - hdr - lens), 2)}
    except KeyError as e:
        cal["missing"] = str(e)
    res["calibration"] = cal
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
