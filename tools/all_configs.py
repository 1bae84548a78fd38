#!/usr/bin/env python3
"""BASELINE.md §3's comparison table: every config through bench.py (one
process each, device-resident, rotating batches > 256 MiB), with the 1-core
and N-core CPU baselines of the same config.

Usage: python tools/all_configs.py [--out profiles/r01_all_configs.json]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# name, frames per batch, rx queues, streams, steps
RUNS = [
    ("c1fixed", 1 << 20, 16, 2, 200),
    ("c1", 1 << 20, 16, 2, 200),
    ("c2", 1 << 20, 16, 2, 400),
    ("c3", 1 << 18, 16, 2, 400),     # IMIX at 2048 B stride: 512 MiB per rotation of 16 rings
    ("c4", 1 << 20, 16, 2, 200),
    ("c5", 1 << 23, 2, 1, 40),       # 8M frames (512 MiB) per batch, 2 rings in one launch (bench default)
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "all_configs.json"))
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--only", nargs="*")
    args = ap.parse_args()
    rows = []
    for name, n, q, st, steps in RUNS:
        if args.only and name not in args.only:
            continue
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", name, "--frames", str(n),
               "--queues", str(q), "--streams", str(st), "--steps", str(steps), "--warmup",
               str(max(4, steps // 8)), "--cpu-seconds", str(args.cpu_seconds), "--no-extra"]
        print("==", " ".join(cmd[1:]), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode or not line:
            print(r.stdout[-2000:], r.stderr[-2000:], flush=True)
            raise SystemExit("bench failed for %s" % name)
        d = json.loads(line[-1])
        rows.append({"config": name, "frames_per_batch": n, "gpu_mpps": d["value"],
                     "roofline_frac": d["roofline"]["frac"],
                     "achieved_gbs": d["roofline"]["achieved"],
                     "steady_state_gbs": d["roofline"].get("achieved_steady_state"),
                     "cpu_1core_mpps": d["cpu_baseline"]["value"],
                     "cpu_ncore_mpps": d["cpu_baseline_ncores"]["value"],
                     "cpu_ncores": d["cpu_baseline_ncores"]["cores"],
                     "host_stage_frames": d["config"]["host_stage_frames"],
                     "bench": d})
        print(json.dumps({k: v for k, v in rows[-1].items() if k != "bench"}), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rows, fh, indent=1)
    print("| config | CPU 1-core (Mpkts/s) | CPU N-core (Mpkts/s) | 1×MI355X (Mpkts/s) | HBM roofline fraction (isolated launch) | steady-state GB/s |")
    print("|---|---|---|---|---|---|")
    for r in rows:
        print("| %s | %.1f | %.1f (%d cores) | %.0f | %.3f | %s |" % (
            r["config"], r["cpu_1core_mpps"], r["cpu_ncore_mpps"], r["cpu_ncores"], r["gpu_mpps"],
            r["roofline_frac"], r["steady_state_gbs"]))


if __name__ == "__main__":
    main()
