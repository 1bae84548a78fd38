#!/usr/bin/env python3
"""bench.py -- device-resident usnetd match-path throughput on MI355X.

Metric (BASELINE.json): Mpkts/s of device-resident L4 classification of 64 B
frames, and the achieved HBM GB/s of the classify kernel against the gfx950
peak.  One step = one usn_classify pass over one batch of the configuration
the metric is quoted on (BASELINE.json configs[1] = "c2": 1M x 64 B IPv4/UDP
frames, 16-rule endpoint table), frames already resident in HBM.  Batches
rotate over --batches distinct buffers (> 256 MiB in total) so the Infinity
Cache cannot serve them.  Multi-GPU: one process per GPU, each classifying its
own batches with a replicated rule table ("replicas only", weak scaling; no
collective on the data path -- gloo carries only the timing barrier/max).

Usage: python bench.py [--gpus N --steps K --warmup W] (torchrun for N > 1)
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ALGO_BYTES = 64 + 2 + 4 + 2   # header window + length + decision + order index per frame
HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--frames", type=int, default=0, help="frames per batch (default: config's)")
    ap.add_argument("--batches", type=int, default=5, help="distinct rotating batches")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--launch-probe", type=int, default=100, help="per-launch event pairs")
    ap.add_argument("--queues", type=int, default=16,
                    help="NIC rx queues (sources) drained per poll round")
    ap.add_argument("--streams", type=int, default=2,
                    help="HIP streams; stream s owns queues [s*Q/S, (s+1)*Q/S) and classifies "
                         "their drained rings with one usn_classify_multi launch per round")
    return ap.parse_args()


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    from usnetd_amd import lib, shard, traffic
    L = lib.load()            # the HIP runtime is loaded here, before torch (if any)
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_mod
        dist_mod.init_process_group("gloo")
        dist = dist_mod

    defaults = {"c2": 1 << 20, "c5": 1 << 23, "c3": 1 << 18, "c4": 1 << 20, "c1": 1 << 20,
                "c1fixed": 1 << 20}
    n = args.frames or defaults[args.config]
    S = max(1, args.streams)
    Qt = max(S, args.queues - args.queues % S)   # rx queues in total
    P = min(8, Qt // S)                           # queues (batches) per launch
    Qt = P * S
    R = max(2, -(-args.batches // Qt))            # rounds of distinct batches rotated through
    nb = R * Qt
    device = local
    if world > 1:   # one rank per GPU; more ranks than GPUs (a rehearsal) share them round-robin
        import torch
        ndev = torch.cuda.device_count()   # counts without initialising the GPU
        if ndev > 0:
            device = local % ndev
    ctx = lib.Ctx(device)
    batches, results, cfg0 = [], [], None
    nics = None
    for k in range(nb):
        cfg = traffic.config(args.config, n=n, seed=shard.batch_seed(rank, k))
        if k == 0:
            cfg0 = cfg
            traffic.install_ctx(ctx, cfg)
            nics = [cfg.src] + traffic.extra_nics(cfg, Qt - 1, ctx)
        batches.append(lib.DeviceBatch(ctx, cfg.frames, cfg.lens, nics[k % Qt], stride=cfg.stride))
        results.append(lib.DeviceResult(ctx, n))
        if k:
            del cfg
    streams = [ctx.stream() for _ in range(S)]
    stream = streams[0]
    h = ctx.h
    # launch (round r, stream s): the batches of queues [sP, sP+P) of round r
    groups = {}
    for r in range(R):
        for si in range(S):
            ks = [r * Qt + si * P + j for j in range(P)]
            ba = (lib.Batch * P)(*[batches[k].desc for k in ks])
            ra = (lib.Result * P)(*[results[k].desc for k in ks])
            groups[(r, si)] = (C.cast(ba, C.c_void_p), C.cast(ra, C.c_void_p), ba, ra)
    multi = L.usn_classify_multi
    single = L.usn_classify
    bdesc = [C.byref(b.desc) for b in batches]
    rdesc = [C.byref(r.desc) for r in results]
    joins = [ctx.event() for _ in streams]

    def launch(i, per=P, count=None, one_queue=False):
        """Launch i on stream i % S: `count` (default per) batches of that
        stream's queues.  one_queue: the single-queue reference (stream 0,
        one batch per launch, batches in rotation)."""
        if one_queue:
            rc = single(h, bdesc[i % nb], rdesc[i % nb], stream)
        else:
            si = i % S
            r = (i // S) % R
            if per == 1:
                k = r * Qt + si * P
                rc = single(h, bdesc[k], rdesc[k], streams[si])
            else:
                g = groups[(r, si)]
                rc = multi(h, g[0], g[1], count or per, streams[si])
        if rc:
            lib.check(rc, "usn_classify")

    def timed(steps, per, one_queue=False):
        """Exactly `steps` batches, `per` per launch (the last launch takes the rest)."""
        full, rest = divmod(steps, per)
        for x in streams:
            ctx.sync(x)
        if dist:
            dist.barrier()
        ctx.sync()
        t0 = time.perf_counter()
        ctx.record(ev0, stream)
        for x in streams[1:]:
            ctx.wait_event(x, ev0)
        for i in range(full):
            launch(i, per, one_queue=one_queue)
        if rest:
            launch(full, per, rest, one_queue=one_queue)
        for x, ej in zip(streams[1:], joins[1:]):
            ctx.record(ej, x)
            ctx.wait_event(stream, ej)
        ctx.record(ev1, stream)
        ctx.sync(stream)
        ctx.sync()
        t1 = time.perf_counter()
        if dist:
            dist.barrier()
        return t1 - t0, ctx.elapsed_ms(ev0, ev1), steps

    ev0, ev1 = ctx.event(), ctx.event()
    for i in range(-(-args.warmup // P)):
        launch(i)
    wall, ev_ms, done = timed(args.steps, P)
    elapsed = shard.max_over_ranks(wall, dist)

    # every batch of the last rotation: the ordered host stage had nothing to do
    host_frames, flags = 0, 0
    cls = [0, 0, 0, 0]
    for x in streams:
        ctx.sync(x)
    for k in range(nb):
        info = ctx.finalize(batches[k], results[k], streams[(k % Qt) // P])
        host_frames += info.n_host
        flags |= info.flags
        cls = [x + y for x, y in zip(cls, info.class_count)]

    # per-launch kernel duration (HIP events on the launch stream): the same
    # launches back to back on ONE stream, so no launch shares the GPU with
    # another (stream order serialises them) and none starts from an idle GPU
    probe = []
    evs = [(ctx.event(), ctx.event()) for _ in range(args.launch_probe)]
    for x in streams:
        ctx.sync(x)
    for i, (ea, eb) in enumerate(evs):
        ctx.record(ea, stream)
        g = groups[((i // S) % R, i % S)]
        rc = multi(h, g[0], g[1], P, stream)
        if rc:
            lib.check(rc, "usn_classify_multi")
        ctx.record(eb, stream)
    ctx.sync(stream)
    for ea, eb in evs:
        probe.append(ctx.elapsed_ms(ea, eb))
    kern_ms = float(np.median(probe)) if probe else ev_ms / max(1, done // P)
    achieved = ALGO_BYTES * n * P / (kern_ms * 1e-3) / 1e9

    # the same batches one per launch (single rx queue), for reference
    single_mpps = None
    if P > 1 and args.steps >= 4:
        w1, _, d1 = timed(max(4, args.steps // 2), 1, one_queue=True)
        single_mpps = round(d1 * n / w1 / 1e6, 1)

    total_frames = world * done * n
    value = total_frames / elapsed / 1e6
    out = {
        "metric": "Mpkts/s device-resident L4 classify @64B frames; HBM GB/s vs roofline",
        "value": round(value, 2),
        "unit": "Mpkts/s",
        "n_gpus": world,
        "steps": done,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / done, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic frames generated on the host (no captures), resident in HBM",
        "config": {
            "workload": "%s: %d x 64B IPv4/UDP frames per batch (one drained rx ring), %d-rule "
                        "endpoint table, NIC rx; %d rx queues on %d streams, %d rings per launch"
                        % (args.config, n, len(cfg0.rules), Qt, S, P),
            "frames_per_batch": n,
            "rx_queues": Qt,
            "streams": S,
            "batches_per_launch": P,
            "rotating_batches": nb,
            "rotating_bytes": int(nb * (n * cfg0.stride + n * 2)),
            "parallelism": "replicas%d" % world,
            "host_stage_frames": int(host_frames),
            "summary_flags": int(flags),
            "class_count_last_rotation": [int(x) for x in cls],
            "event_ms_per_step": round(ev_ms / done, 5),
            "single_queue_mpps": single_mpps,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "kernel": "classify_rx_kernel",
            "kernel_us_median": round(kern_ms * 1e3, 3),
            "achieved_basis": "launches serialised on one stream (HIP events around each; no overlap)",
            # the timed region's launches overlap on two streams: per GPU, algorithmic
            # bytes of all its frames / the timed region's wall time
            "achieved_steady_state": round(ALGO_BYTES * done * n / elapsed / 1e9, 1),
            "batches_per_launch": P,
            "algo_bytes_per_frame": ALGO_BYTES,
        },
        "cpu_baseline": None,
    }
    pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
    if os.path.exists(pmc):
        try:
            with open(pmc) as fh:
                pm = json.load(fh)
            if int(pm.get("frames_per_launch", -1)) == n * P:
                out["roofline"]["traffic"] = pm.get("hbm_bytes_per_launch")
                out["roofline"]["traffic_source"] = os.path.relpath(pmc, ROOT)
        except Exception:
            pass
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg0, args.cpu_seconds)
        out["cpu_baseline_ncores"] = cpu_baseline_ncores(args.config, n, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    for b in batches:
        b.free()
    for r in results:
        r.free()
    ctx.close()
    if dist:
        dist.destroy_process_group()


def cpu_baseline(cfg, seconds):
    """The sequential C oracle (restatement of the reference matcher, one
    thread) timed on this host on the same batch, repeated for ~`seconds`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle
    coracle.build()
    o = coracle.Oracle()
    coracle.install_oracle(o, cfg)
    passes, t0 = 0, time.perf_counter()
    while True:
        o.forward_batch(cfg.src, cfg.frames, cfg.lens, stride=cfg.stride)
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(passes * cfg.n / el / 1e6, 3), "unit": "Mpkts/s", "cores": 1,
            "kind": "port",
            "sample": "%d passes over one %s batch (%d x 64B frames), sequential C restatement "
                      "with the 1-entry cache, %.1f s" % (passes, cfg.name, cfg.n, el)}


def _cpu_worker(arg):
    """One core: its own oracle, its own rx queue (batch), passes for ~seconds."""
    name, n, seed, seconds = arg
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle
    from usnetd_amd import traffic
    cfg = traffic.config(name, n=n, seed=seed)
    o = coracle.Oracle()
    coracle.install_oracle(o, cfg)
    passes, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        o.forward_batch(cfg.src, cfg.frames, cfg.lens, stride=cfg.stride)
        passes += 1
    return passes * cfg.n, time.perf_counter() - t0


def cpu_baseline_ncores(name, n, seconds):
    """SURVEY §8d's N-core variant: the sequential oracle sharded by rx queue,
    one process per core, N = the host CPUs this job may use (at most 16 on
    the GPU box).  Aggregate frames / slowest worker's time."""
    import multiprocessing as mp
    try:
        ncores = len(os.sched_getaffinity(0))
    except AttributeError:
        ncores = os.cpu_count() or 1
    ncores = max(1, min(ncores, int(os.environ.get("OMP_NUM_THREADS", ncores)), 16))
    nshard = min(n, 1 << 18)   # each core's queue: a quarter-size batch keeps memory small
    ctx = mp.get_context("spawn")
    with ctx.Pool(ncores) as pool:
        res = pool.map(_cpu_worker, [(name, nshard, 1000 + k, seconds) for k in range(ncores)])
    frames = sum(r[0] for r in res)
    el = max(r[1] for r in res)
    return {"value": round(frames / el / 1e6, 3), "unit": "Mpkts/s", "cores": ncores,
            "kind": "port",
            "sample": "%d processes, each the sequential C restatement over its own %s rx queue "
                      "(%d x 64B frames) for %.1f s" % (ncores, name, nshard, el)}


if __name__ == "__main__":
    main()
