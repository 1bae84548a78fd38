#!/usr/bin/env python3
"""Latency of the first batch after an AddMatch (a rule change
must not stall the data path for a whole image rebuild).  c5's 65 536-rule
table; each round: one AddMatch of a new connected rule (a server accepting
a connection, /root/reference/src/main.rs:266-298), then one 1M-frame rx
batch classified and finalized.  Reports the wall time of AddMatch + classify
+ finalize per round, and the same rounds with no AddMatch.  USN_IMG_FULL=1
makes every change rebuild the image (round 2's behaviour): only the test
build (build/test/libusn.so) reads that knob, so it is loaded then.
usage: python tools/addmatch_latency.py [rounds]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from usnetd_amd import lib, traffic  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    cfg = traffic.config("c5", n=1 << 20, seed=3)
    full = bool(os.environ.get("USN_IMG_FULL"))
    libpath = lib.TEST_LIB_PATH if full else None   # the product library ignores USN_IMG_FULL
    ctx = lib.Ctx(0, libpath=libpath)
    traffic.install_ctx(ctx, cfg)
    s = ctx.stream()
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, cfg.src, stride=cfg.stride)
    rs = [lib.DeviceResult(ctx, cfg.n) for _ in range(2)]
    owner = [e for e, kind, _ in cfg.endpoints if kind != 0][0]
    for k in range(5):
        ctx.classify(b, rs[k % 2], s)
        ctx.finalize(b, rs[k % 2], s)
    out = {}
    for mode in ("no_addmatch", "addmatch"):
        ms = []
        for k in range(rounds):
            t0 = time.perf_counter()
            if mode == "addmatch":
                w = lib.make_want("10.0.0.1", 6, 80, "192.168.%d.%d" % (k // 250, k % 250 + 1), 40000 + k)
                assert ctx.add_match(w, owner) == 1
            ctx.classify(b, rs[k % 2], s)
            ctx.finalize(b, rs[k % 2], s)
            ms.append((time.perf_counter() - t0) * 1e3)
        out[mode] = {"median_ms": round(statistics.median(ms), 3), "max_ms": round(max(ms), 3)}
    out["image_rebuild_every_change"] = full
    out["library"] = os.path.relpath(libpath or lib.LIB_PATH, ROOT)
    out["rules"] = ctx.rule_count()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
