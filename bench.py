#!/usr/bin/env python3
"""bench.py -- device-resident usnetd match-path throughput on MI355X.

Metric (BASELINE.json): Mpkts/s of device-resident L4 classification of 64 B
frames, and the classify kernel's achieved HBM GB/s against the gfx950 peak.

Workload: BASELINE.json configs[4] ("c5"), the configuration the north star
reports at 1, 2, 4 and 8 GPUs: 64 B IPv4 TCP/UDP frames, a 65 536-rule table
(16 IPs x 2048 listening ports + 32 768 connected 5-tuples, L2/MALL-resident),
1 000 endpoints, 8M frames per drained rx ring.  Frames are resident in HBM
when the timed region starts.  At N=1 the line also carries configs[1] ("c2":
1M x 64 B frames, 16 rules) under the key "c2", measured the same way.

One step = one poll round: every rx queue the rank owns is drained once (one
batch per queue, the reference's Endpoint::forward drain of each readable
ring, /root/reference/src/main.rs:1029-1046), classified on the device with
usn_classify_multi (up to 16M frames per launch).  c5: 2 queues of 8M frames
per rank = 16M frames per step, both in one launch on one stream; c2: 16
queues of 1M, 8 per launch on 2 HIP streams.

Multi-GPU: one process per GPU (torchrun), "replicas only": each rank owns a
disjoint block of the node's rx queues (usnetd_amd.shard.rank_queues) and a
replica of the rule table; no collective on the data path (gloo carries the
barrier and the max-over-ranks time).  --strong fixes the whole job's frames
per step at 64M (c5) and splits the queues over the ranks; the default is
weak scaling (fixed queues per rank).

Usage: python bench.py [--gpus N --steps K --warmup W]
For N > 1 under torch.distributed.run (WORLD_SIZE set) each process is one
rank and WORLD_SIZE must equal N.  Without a launcher, `--gpus N` starts N
rank processes itself (before anything touches the GPU: launch_ranks) and
prints rank 0's line; "n_gpus" is the number of ranks that joined the process
group, checked against N.
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

ALGO_BYTES = 64 + 2 + 4 + 4   # header window + length + decision + per-endpoint list entry per frame
HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
LAUNCH_FRAMES = 1 << 24       # frames per launch the rings are grouped to (8 x 1M, or 2 x 8M)
ROTATE_BYTES = 1 << 30        # distinct batch bytes per rank, > the 256 MiB Infinity Cache
STRONG_FRAMES = 1 << 26       # --strong: 64M frames per step for the whole job
PROBE_GROUP = 8               # calls per event pair of the per-call device-time probe
METRIC = "Mpkts/s device-resident L4 classify @64B frames; HBM GB/s vs roofline"
DEFAULT_FRAMES = {"c1": 1 << 20, "c1fixed": 1 << 20, "c2": 1 << 20, "c3": 1 << 18, "c4": 1 << 20,
                  "c5": 1 << 23}


def launch_frames(name, queues=0):
    """Frames per classify launch of a config in the bench's launch shape
    (Run: up to 8 rings of the config's batch size, at most 16M frames, the
    rings of `queues` rx queues dealt over the streams)."""
    n = DEFAULT_FRAMES[name]
    P = max(1, min(8, LAUNCH_FRAMES // n))
    S = 1 if P * n >= LAUNCH_FRAMES else 2
    Q = queues or P * S
    S = min(S, Q)
    return n * min(P, -(-Q // S))


def extra_queues(name):
    """rx queues per rank of a config measured under its own key at N=1"""
    return EXTRA_QUEUES.get(name, 0)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c5")
    ap.add_argument("--frames", type=int, default=0, help="frames per batch (default: config's)")
    ap.add_argument("--queues", type=int, default=0,
                    help="rx queues per rank (default: one launch's rings per stream)")
    ap.add_argument("--streams", type=int, default=0,
                    help="streams (default: 1 when one launch covers a poll round's 16M frames, else 2)")
    ap.add_argument("--rings-per-launch", type=int, default=0,
                    help="rx rings per usn_classify_multi launch (default: 8M frames' worth, <= 8)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: 64M frames per step for the whole job")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the other configs' keys at N=1")
    ap.add_argument("--extras", default="c2,c3,c4,c4tx",
                    help="configs measured under their own keys at N=1")
    ap.add_argument("--launch-probe", type=int, default=150, help="per-launch event pairs")
    ap.add_argument("--ramp", type=int, default=200,
                    help="untimed poll rounds between the probe and the timed steps (clock ramp)")
    ap.add_argument("--lists-async", type=int, default=0,
                    help="1: per-endpoint lists on the library's side stream (usn_set_lists_async): "
                         "a round's scatter overlaps the next round's classify")
    ap.add_argument("--result-rounds", type=int, default=2,
                    help="rounds of result buffers (>= 2: the end-to-end loop finalizes round i - 1 "
                         "while round i is queued)")
    ap.add_argument("--rotate-mib", type=int, default=ROTATE_BYTES >> 20,
                    help="distinct batch bytes per rank (default 1024: past the 256 MiB Infinity Cache)")
    ap.add_argument("--tx-launches", type=int, default=TX_LAUNCHES,
                    help="c4tx: timed multi-ring launches at least")
    ap.add_argument("--tx-rings", type=int, default=8, choices=range(1, 9),
                    help="c4tx: consecutive rings of the sending endpoint per tx launch (one grid)")
    ap.add_argument("--host-inclusive", default="c5,c2",
                    help="configs whose PCIe-inclusive rate is measured at N=1 ('' for none)")
    ap.add_argument("--launch-check", action="store_true",
                    help="launcher self-test: ranks join the process group and report, no GPU")
    return ap.parse_args(argv)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_envs(n, port, base_env=None):
    """The environment of each of the n rank processes launch_ranks starts
    (torch.distributed.run's variables, rendezvous on 127.0.0.1)."""
    envs = []
    for r in range(n):
        e = dict(base_env if base_env is not None else os.environ)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: start N rank processes of this
    script (this process never touches the GPU) and exit with the worst exit
    status.  Rank 0 prints the JSON line."""
    import subprocess
    port = _free_port()
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=e)
             for e in rank_envs(n, port)]
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


class Run:
    """The rank's rx queues of one config, resident in HBM, and the launches
    of one poll round."""

    def __init__(self, L, ctx, name, n, rank, world, queues, streams, strong, rings_per_launch=0,
                 rotate_bytes=ROTATE_BYTES, result_rounds=2):
        from usnetd_amd import shard, traffic
        self.L, self.ctx, self.name, self.n = L, ctx, name, n
        P = rings_per_launch or max(1, min(8, LAUNCH_FRAMES // n))   # rings per launch
        # c4/c5 (8M-frame rings): both rings of a poll round in ONE launch on one
        # stream, as the daemon's usn_classify_multi does (A/B, profiles/r02cg:
        # 64.9-65.6 Gpkt/s against 64.8-65.9 for one ring per launch on two
        # streams, with no dependence on how two streams' launches overlap;
        # two 2-ring launches on two streams: 61.1-62.0)
        S = max(1, streams) if streams else (1 if P * n >= LAUNCH_FRAMES else 2)
        mine, _ = shard.step_queues(n, world, rank, strong, queues or P * S, STRONG_FRAMES)
        self.queues = mine                                # global queue ids of this rank
        Q = len(mine)
        S = min(S, Q)
        P = min(P, -(-Q // S))
        self.P, self.S, self.Q = P, S, Q
        # launches of one poll round: stream s takes queues s, s+S, ... in groups of P
        per_stream = [list(range(s, Q, S)) for s in range(S)]
        self.launches = []                                # (stream index, [local queue])
        for s in range(S):
            qs = per_stream[s]
            for k in range(0, len(qs), P):
                self.launches.append((s, qs[k:k + P]))
        # rotation: R rounds of distinct batches per queue (> 256 MiB in all)
        cfg0 = None
        self.batches, self.results = [], []
        frame_bytes = None
        R = 1
        for rnd in range(64):
            if rnd >= R:
                break
            for j, gq in enumerate(mine):
                cfg = traffic.config(name, n=n, seed=shard.queue_seed(gq, rnd))
                if cfg0 is None:
                    cfg0 = cfg
                    traffic.install_ctx(ctx, cfg)
                    self.nics = [cfg.src] + traffic.extra_nics(cfg, Q - 1, ctx)
                    frame_bytes = n * cfg.stride
                    R = max(1, -(-rotate_bytes // (frame_bytes * Q)))
                self.batches.append(_batch(ctx, cfg, self.nics[j]))
                self.results.append(_result(ctx, n))
                del cfg
        self.R = R
        # results: RR >= 2 rounds of result sets per queue, as the daemon binds
        # them (two per source, daemon/usnetd.cpp: round i - 1 is delivered
        # while round i is classified; the reference writes each frame into its
        # target's ring and never overwrites one in place,
        # /root/reference/src/endpoint.rs:61-74).  The value loop, the launch
        # probe and the end-to-end loop all rotate over them, so no round's
        # outputs are still in the Infinity Cache when they are written again.
        # value_single_result_set (one set per queue, rewritten every round:
        # ~170 MB of c5 outputs stay MALL-resident) is reported beside it
        self.RR = max(R, result_rounds)
        for _ in range(self.RR - R):
            for j in range(Q):
                self.results.append(_result(ctx, n))
        self.cfg0 = cfg0
        self.rotating_bytes = int(R * Q * (frame_bytes + 2 * n))
        self.streams = [ctx.stream() for _ in range(S)]
        self.joins = [ctx.event() for _ in range(S)]
        self.ev0, self.ev1 = ctx.event(), ctx.event()
        self.groups = []                                  # per round, per launch: (stream, ptrs)
        for rnd in range(self.RR):
            gl = []
            for s, qs in self.launches:
                kb = [(rnd % R) * Q + j for j in qs]
                kr = [rnd * Q + j for j in qs]
                ba = (_lib().Batch * len(kb))(*[self.batches[k].desc for k in kb])
                ra = (_lib().Result * len(kr))(*[self.results[k].desc for k in kr])
                gl.append((s, C.cast(ba, C.c_void_p), C.cast(ra, C.c_void_p), len(kb), ba, ra))
            self.groups.append(gl)
        self.h = ctx.h

    def frames_per_step(self):
        return self.Q * self.n

    def step(self, i, stream_override=None, single=False):
        """poll round i: its launches, into round i's result sets (i mod RR;
        `single`: one result set per queue, i mod R)"""
        multi = self.L.usn_classify_multi
        for s, ba, ra, cnt, _, _ in self.groups[i % (self.R if single else self.RR)]:
            st = self.streams[s] if stream_override is None else stream_override
            rc = multi(self.h, ba, ra, cnt, st)
            if rc:
                _lib().check(rc, "usn_classify_multi")

    def timed(self, steps, dist, single=False):
        ctx = self.ctx
        for x in self.streams:
            ctx.sync(x)
        if dist:
            dist.barrier()
        ctx.sync()
        t0 = time.perf_counter()
        main = self.streams[0]
        ctx.record(self.ev0, main)
        for x in self.streams[1:]:
            ctx.wait_event(x, self.ev0)
        for i in range(steps):
            self.step(i, single=single)
        self.enqueue_s = time.perf_counter() - t0     # host time to enqueue the steps
        for x, ej in zip(self.streams[1:], self.joins[1:]):
            ctx.record(ej, x)
            ctx.wait_event(main, ej)
        ctx.record(self.ev1, main)
        ctx.sync(main)
        ctx.sync()
        t1 = time.perf_counter()
        if dist:
            dist.barrier()
        return t1 - t0, ctx.elapsed_ms(self.ev0, self.ev1)

    def finalize_round(self, i, times=None):
        """usn_finalize of every ring of poll round i, on the stream its call
        ran on (the ordered host stage, /root/reference/src/endpoint.rs:128-169:
        the reference decides and delivers every frame of a drain before the
        next); `times` collects each call's wall time"""
        if not hasattr(self, "_fin_args"):   # ctypes arguments built once (the loop times the library)
            from usnetd_amd import lib as _l
            self._fin_info = _l.FinalizeInfo()
            ib = C.byref(self._fin_info)
            self._fin_args = [[(self.h, C.byref(self.batches[(r % self.R) * self.Q + j].desc),
                                C.byref(self.results[r * self.Q + j].desc), self.streams[s], ib)
                               for s, qs in self.launches for j in qs] for r in range(self.RR)]
        fin = self.L.usn_finalize
        for a in self._fin_args[i % self.RR]:
            t = time.perf_counter()
            rc = fin(*a)
            if rc:
                _lib().check(rc, "usn_finalize")
            if times is not None:
                times.append(time.perf_counter() - t)

    def end_to_end(self, steps, dist):
        """Poll rounds with the ordered host stage in the timed loop: round i's
        calls, then usn_finalize of every ring of round i - 1 (a daemon
        finalizes and delivers round i - 1 while round i runs on the GPU),
        the last round finalized before the clock stops.  Returns (wall s,
        finalize call times)."""
        ctx = self.ctx
        for x in self.streams:
            ctx.sync(x)
        if dist:
            dist.barrier()
        times = []
        t0 = time.perf_counter()
        t1 = None
        for i in range(steps):
            self.step(i)
            if i:
                self.finalize_round(i - 1, times)
                if i == 1:
                    t1 = time.perf_counter()   # round 0 out: the pipeline is full
        self.finalize_round(steps - 1, times)
        for x in self.streams:
            ctx.sync(x)
        t2 = time.perf_counter()
        if dist:
            dist.barrier()
        # (wall of all rounds; and rounds 1.. after round 0's finalize, without
        # the pipeline's fill)
        return t2 - t0, times, (t2 - t1 if t1 is not None else t2 - t0)

    def finalize_host_us(self, rounds=3):
        """usn_finalize's own host time per ring: the rounds' GPU work done
        first, so the call waits for nothing"""
        times = []
        for i in range(rounds):
            self.step(i)
            for x in self.streams:
                self.ctx.sync(x)
            self.finalize_round(i, times)
        return float(np.median(times)) * 1e6

    def lists_wait(self, ra, cnt, stream):
        """the stream waits for the lists of one launch (side-stream mode)"""
        for j in range(cnt):
            rc = self.L.usn_lists_wait(self.h, C.byref(ra[j]), stream)
            if rc:
                _lib().check(rc, "usn_lists_wait")

    def launch_probe(self, count):
        """Median duration of one launch (HIP events on the stream it runs on):
        the first launch group of the round, back to back on one stream, so no
        launch shares the GPU with another and none starts from an idle GPU."""
        ctx = self.ctx
        st = self.streams[0]
        # an event pair around every PROBE_GROUP calls, not around each: each
        # event is a marker packet of its own between two calls (2-3 us of a
        # c3 call of 40 us, profiles/r06)
        G = PROBE_GROUP
        evs = [(ctx.event(), ctx.event()) for _ in range(max(1, count // G))]
        for x in self.streams:
            ctx.sync(x)
        i = 0
        for ea, eb in evs:
            ctx.record(ea, st)
            for _ in range(G):
                _, ba, ra, cnt, _, ral = self.groups[i % self.RR][0]
                i += 1
                rc = self.L.usn_classify_multi(self.h, ba, ra, cnt, st)
                if rc:
                    _lib().check(rc, "usn_classify_multi")
                self.lists_wait(ral, cnt, st)     # the call's lists, wherever they were built
            ctx.record(eb, st)
        ctx.sync(st)
        ms = [ctx.elapsed_ms(a, b) / G for a, b in evs]
        frames = self.groups[0][0][3] * self.n
        return float(np.median(ms)), frames

    def finalize_all(self):
        """usn_finalize of every batch of the last rotation (result rounds
        0 .. RR - 1): the ordered host stage has nothing to do on these configs
        (no fragments, DHCP, stale caches); counted and reported."""
        host_frames, flags, cls = 0, 0, [0, 0, 0, 0]
        for x in self.streams:
            self.ctx.sync(x)
        for r in range(self.RR):
            for j in range(self.Q):
                info = self.ctx.finalize(self.batches[(r % self.R) * self.Q + j],
                                         self.results[r * self.Q + j], self.streams[0])
                host_frames += info.n_host
                flags |= info.flags
                cls = [x + y for x, y in zip(cls, info.class_count)]
        return host_frames, flags, cls

    def free(self):
        for b in self.batches:
            b.free()
        for r in self.results:
            r.free()


def _lib():
    from usnetd_amd import lib
    return lib


def _batch(ctx, cfg, src):
    return _lib().DeviceBatch(ctx, cfg.frames, cfg.lens, src, stride=cfg.stride)


def _result(ctx, n):
    return _lib().DeviceResult(ctx, n)


def measure(run, args, dist, world):
    from usnetd_amd import shard
    for i in range(args.warmup):
        run.step(i)
    # The GPU reaches its steady rate only after many poll rounds on both
    # streams: untimed ramp rounds, the per-launch probe, ramp rounds again
    # (config.untimed_ramp_steps counts both), then the timed steps.  With the probe after the timed
    # steps and no ramp, K = 20 read 53.2 Gpkt/s against 58.1 at 100 steps
    # (tools/steptime.py: 0.301 -> 0.292 -> 0.280 ms per step over the first
    # three runs of 20 steps); K = 20 after 2 x 40 / 100 / 200 ramp rounds:
    # 58.7-58.8 / 59.1-60.0 / 59.6-59.8 Gpkt/s against 60.5 at 400 steps
    # (profiles/r02aq; 200 rounds cost ~0.1 s).
    for i in range(args.ramp):
        run.step(args.warmup + i)
    kern_ms, probe_frames = run.launch_probe(args.launch_probe) if args.launch_probe else (None, 0)
    for i in range(args.ramp):      # again: the one-stream probe lets the rate drop
        run.step(args.warmup + args.ramp + i)
    wall, ev_ms = run.timed(args.steps, dist)
    elapsed = shard.max_over_ranks(wall, dist)
    enqueue_s = run.enqueue_s
    # the same K rounds with one result set per queue rewritten every round
    # (rounds 0 .. R - 1 only; round 5's value basis), reported beside the value
    wall1, _ = run.timed(args.steps, dist, single=True)
    elapsed1 = shard.max_over_ranks(wall1, dist)
    run.enqueue_s = enqueue_s
    host_frames, flags, cls = run.finalize_all()
    # the same poll rounds with usn_finalize of every ring in the timed loop
    # (what the reference does per drain)
    e2e_wall, fin_times, e2e_steady = run.end_to_end(args.steps, dist)
    e2e_elapsed = shard.max_over_ranks(e2e_wall, dist)
    e2e_steady = shard.max_over_ranks(e2e_steady, dist)
    fin_host_us = run.finalize_host_us()
    frames = world * args.steps * run.frames_per_step()
    achieved = ALGO_BYTES * probe_frames / (kern_ms * 1e-3) / 1e9 if kern_ms else None
    roof = {
        "bound": "hbm",
        "achieved": round(achieved, 1) if achieved else None,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
        "traffic": None,
        "kernel": "classify_rx_kernel + per-endpoint scatter (scan_kernel unless the launch "
                  "self-scans, scatter_kernel)",
        "kernel_us_median": round(kern_ms * 1e3, 3) if kern_ms else None,
        "frames_per_launch": probe_frames,
        "algo_bytes_per_frame": ALGO_BYTES,
        "achieved_basis": "algorithmic bytes of one usn_classify_multi call (its three kernels) / "
                          "its median duration (HIP events on its stream around groups of %d "
                          "back-to-back calls on one stream)" % PROBE_GROUP,
        # the timed region (launches overlapping on the streams): per GPU,
        # algorithmic bytes of all its frames / the timed region's wall time
        "achieved_steady_state": round(ALGO_BYTES * args.steps * run.frames_per_step() / elapsed
                                       / 1e9, 1),
    }
    pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % run.name)
    if os.path.exists(pmc):
        try:
            with open(pmc) as fh:
                pm = json.load(fh)
            if int(pm.get("frames_per_launch", -1)) == probe_frames:
                roof["traffic"] = pm.get("hbm_bytes_per_launch")
                roof["traffic_source"] = os.path.relpath(pmc, ROOT)
        except (OSError, ValueError):
            pass
    return {
        "value": round(frames / elapsed / 1e6, 2),
        "value_basis": "K poll rounds, round i into result set i mod %d of each queue (the daemon's "
                       "double-buffered results), no usn_finalize in the loop" % run.RR,
        "value_single_result_set": round(frames / elapsed1 / 1e6, 2),
        "end_to_end_mpps": round(frames / e2e_elapsed / 1e6, 2),
        "end_to_end": {
            "basis": "poll rounds with usn_finalize of every ring in the timed loop (round i-1's "
                     "rings finalized after round i's calls are enqueued), wall clock, max over ranks",
            "ms_per_step": round(e2e_elapsed * 1e3 / args.steps, 5),
            # rounds 1..K-1 after round 0's usn_finalize returned (the pipeline full)
            "steady_mpps": round(frames * (args.steps - 1) / args.steps / e2e_steady / 1e6, 2)
            if args.steps > 1 else None,
            "finalize_call_us_per_ring_median": round(float(np.median(fin_times)) * 1e6, 2),
            "finalize_host_us_per_ring": round(fin_host_us, 2),
            "rings_per_step": run.Q,
        },
        "ms_per_step": round(elapsed * 1e3 / args.steps, 5),
        "event_ms_per_step": round(ev_ms / args.steps, 5),
        # the host's own time to enqueue a step's calls (close to ms_per_step: host-bound)
        "enqueue_ms_per_step": round(run.enqueue_s * 1e3 / args.steps, 5),
        "frames_per_step_per_gpu": run.frames_per_step(),
        "host_stage_frames": int(host_frames),
        "summary_flags": int(flags),
        "class_count_last_rotation": [int(x) for x in cls],
        "roofline": roof,
    }


# c3: 8 rx rings of 256K IMIX frames in 2 KiB slots (4 GiB), two calls of 4
# rings on two streams.  With 4 rings in two calls of 2 the step was bound by
# the host's enqueue (3 launches per call, ~6 us each): 17-28 Gpkt/s between
# runs; 8 rings in calls of 4: 29.2, enqueue 0.043 of a 0.072 ms step
# (profiles/r03/r03r)
EXTRA_QUEUES = {"c3": 8}
EXTRA_MIN_STEPS = {"c3": 200}   # c3's poll round is ~55 us: 200 rounds time ~11 ms, not ~2
TX_ROTATE = 8              # c4tx: the ring in 8 device buffers (512 MiB > the 256 MiB Infinity Cache;
                           # 7 others, 448 MiB, between two uses of one at 4 or 8 rings per launch)
TX_RINGS = 100             # c4tx: timed rings (and device event pairs) at least
TX_LAUNCHES = 50           # c4tx: timed multi-ring launches at least (400 rings, ~15 ms: the
                           # loop's fill and drain < 1 %; at 13 launches 5-10 %, profiles/r06/r06r)


def measure_tx(ctx, args):
    """configs[3] in the tx direction (c4tx, traffic.c4tx): 1M frames sent by
    the host endpoint, with ADD_MACS bridge MACs, MAC learning and answer-rule
    learning (/root/reference/src/endpoint.rs:194-253).  One ring's frames
    in TX_ROTATE device buffers used in turn: the first pass learns every
    flow's answer rule, the timed passes learn nothing new, and no pass is
    served from the Infinity Cache.  A tx launch changes shared state: launch
    j + 1 may be enqueued before launch j's rings are finalized (at most two
    launches in flight; launch j + 1 is decided again on the host when a
    finalize of launch j changed what it started from).  value = frames /
    wall time of that pipelined loop with --tx-rings (8) consecutive rings per
    launch (one tx grid, usn_classify_multi), one ring per launch beside it; the
    device time of the call (tx kernel + per-endpoint scatter, HIP events)
    gives the roofline."""
    from usnetd_amd import lib, traffic
    n = DEFAULT_FRAMES["c4"]
    cfg = traffic.c4tx(n=n, seed=6)
    traffic.install_ctx(ctx, cfg)
    s = ctx.stream()
    bufs = [lib.DeviceBatch(ctx, cfg.frames, cfg.lens, cfg.src, stride=cfg.stride)
            for _ in range(TX_ROTATE)]
    res = [lib.DeviceResult(ctx, n) for _ in range(2)]
    learn_us, learn_n, next_us = None, 0, None
    for k in range(TX_ROTATE + args.warmup):          # learning pass + warm-up
        ctx.sync()
        t = time.perf_counter()
        ctx.classify(bufs[k % TX_ROTATE], res[k % 2], s)
        nl = ctx.finalize(bufs[k % TX_ROTATE], res[k % 2], s).n_learned
        if k == 0:   # the first ring learns every flow's answer rule (and the bridge MACs)
            learn_us, learn_n = (time.perf_counter() - t) * 1e6, nl
        elif k == 1:   # its classify brings the rule image up to date with what ring 0 learned
            next_us = (time.perf_counter() - t) * 1e6
    # >= 100 rings (about 8 ms) and as many event pairs for the device median
    # (the anti-cache rule of BASELINE.md: >= 100 launches)
    K = max(args.steps, TX_RINGS)
    evs = [(ctx.event(), ctx.event()) for _ in range(K)]
    # sequential (each ring finalized before the next is enqueued), for reference
    learned = 0
    ctx.sync()
    t0 = time.perf_counter()
    for k in range(K):
        b, r = bufs[k % TX_ROTATE], res[k % 2]
        ctx.classify(b, r, s)
        learned += ctx.finalize(b, r, s).n_learned
    wall_seq = time.perf_counter() - t0
    # pipelined (the value): ring k + 1 enqueued before ring k's usn_finalize,
    # as a sending endpoint's next ring is drained while the previous one is
    # finalized; usn_finalize of ring k waits for ring k's launches only.
    # Timed without events in the loop; a second pass with an event pair
    # around every call gives the device time per call (the roofline).
    def pipelined(with_events):
        def launch(k):
            if with_events:
                ctx.record(evs[k][0], s)
            ctx.classify(bufs[k % TX_ROTATE], res[k % 2], s)
            if with_events:
                ctx.record(evs[k][1], s)
        nl = 0
        ctx.sync()
        t = time.perf_counter()
        launch(0)
        for k in range(K):
            if k + 1 < K:
                launch(k + 1)
            nl += ctx.finalize(bufs[k % TX_ROTATE], res[k % 2], s).n_learned
        return time.perf_counter() - t, nl
    wall, nl = pipelined(False)
    learned += nl
    wall_ev, nl = pipelined(True)
    learned += nl
    dev_ms = float(np.median([ctx.elapsed_ms(a, e) for a, e in evs]))
    # P consecutive rings per usn_classify_multi launch (one tx grid: ring
    # k's header loads overlap the chain of the rings before), launch j + 1
    # enqueued before launch j's rings are finalized
    P = args.tx_rings
    res2 = res + [lib.DeviceResult(ctx, n) for _ in range(2 * P - 2)]
    K2 = max(-(-K // P), args.tx_launches)
    evs2 = [(ctx.event(), ctx.event()) for _ in range(K2)]

    # the loop's ctypes arguments built once (the loop times the library, not
    # the binding): launch j takes buffers Pj .. Pj + P - 1 (mod TX_ROTATE)
    # and results Pj .. (mod 2P), a cycle of PER launches
    PER = TX_ROTATE
    margs, fargs = [], []
    finfo = lib.FinalizeInfo()
    for j in range(PER):
        ks = [P * j + q for q in range(P)]
        ba = (lib.Batch * P)(*[bufs[k % TX_ROTATE].desc for k in ks])
        ra = (lib.Result * P)(*[res2[k % (2 * P)].desc for k in ks])
        margs.append((ctx.h, C.cast(ba, C.c_void_p), C.cast(ra, C.c_void_p), P, s, ba, ra))
        fargs.append([(ctx.h, C.byref(bufs[k % TX_ROTATE].desc), C.byref(res2[k % (2 * P)].desc), s,
                       C.byref(finfo)) for k in ks])
    multi, fin = ctx.L.usn_classify_multi, ctx.L.usn_finalize

    def pipelined2(with_events, K2=K2):
        def launch(j):
            if with_events:
                ctx.record(evs2[j][0], s)
            rc = multi(*margs[j % PER][:5])
            if rc:
                lib.check(rc, "usn_classify_multi")
            if with_events:
                ctx.record(evs2[j][1], s)
        nl = 0
        ctx.sync()
        t = time.perf_counter()
        launch(0)
        for j in range(K2):
            if j + 1 < K2:
                launch(j + 1)
            for a in fargs[j % PER]:
                rc = fin(*a)
                if rc:
                    lib.check(rc, "usn_finalize")
                nl += finfo.n_learned
        return time.perf_counter() - t, nl
    # untimed: the tx scratch grows to P rings' frames and tiles once
    ctx.classify_multi(bufs[:P], res2[:P], s)
    for q in range(P):
        learned += ctx.finalize(bufs[q], res2[q], s).n_learned
    wall2, nl = pipelined2(False)
    learned += nl
    wall2_ev, nl = pipelined2(True)
    learned += nl
    # the same loop over only the launches the timed rings fill (13 at the
    # defaults): its fill (the first launch's enqueue) and drain (the last
    # launch's finalizes) are a visible share of it (profiles/r06/r06r)
    K2s = -(-K // P)
    wall2s, nl = pipelined2(False, K2s)
    learned += nl
    dev2_ms = float(np.median([ctx.elapsed_ms(a, e) for a, e in evs2]))
    # the value: P rings per launch (its device time gives the roofline);
    # one ring per launch beside it
    F2 = P * n
    achieved = ALGO_BYTES * F2 / (dev2_ms * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": "tx_kernel (%d rings per grid) + per-endpoint scatter" % P,
            "kernel_us_median": round(dev2_ms * 1e3, 3),
            "frames_per_launch": F2, "algo_bytes_per_frame": ALGO_BYTES}
    pmc = os.path.join(ROOT, "profiles", "pmc_c4tx.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as fh:
                pm = json.load(fh)
            if int(pm.get("frames_per_launch", -1)) == F2:
                roof["traffic"] = pm.get("hbm_bytes_per_launch")
                roof["traffic_x2"] = pm.get("hbm_bytes_per_launch_x2")   # the guide's x2 throughout
                roof["traffic_model"] = pm.get("correction")
                roof["traffic_source"] = os.path.relpath(pmc, ROOT)
        except (OSError, ValueError):
            pass
    x = {"value": round(P * K2 * n / wall2 / 1e6, 2), "unit": "Mpkts/s",
         "value_basis": "end to end: every ring classified and finalized; %d consecutive rings "
                        "per usn_classify_multi launch (one tx grid), launch j + 1 enqueued "
                        "before launch j's usn_finalize calls (no events in the timed loop), "
                        "%d launches timed (the first one's enqueue and the last one's "
                        "finalizes inside the timed region)" % (P, K2),
         "rings_per_launch": P,
         "launches": K2,
         "short_loop": {"launches": K2s, "mpps": round(P * K2s * n / wall2s / 1e6, 2)},
         "ms_per_ring": round(wall2 * 1e3 / (P * K2), 4),
         "device_mpps": round(F2 / (dev2_ms * 1e-3) / 1e6, 2),
         "pipelined_with_events_mpps": round(P * K2 * n / wall2_ev / 1e6, 2),
         "one_ring_launches": {"mpps": round(K * n / wall / 1e6, 2),
                               "sequential_mpps": round(K * n / wall_seq / 1e6, 2),
                               "ms_per_ring": round(wall * 1e3 / K, 4),
                               "device_us_per_launch_median": round(dev_ms * 1e3, 3),
                               "device_mpps": round(n / (dev_ms * 1e-3) / 1e6, 2),
                               "with_events_mpps": round(K * n / wall_ev / 1e6, 2),
                               "basis": "one ring per launch, ring k + 1 enqueued before ring "
                                        "k's usn_finalize (sequential: each ring finalized "
                                        "before the next is enqueued)"},
         "rings": P * K2, "learned_in_timed_rings": int(learned),
         "learning_ring_us": round(learn_us, 1), "learning_ring_learned": int(learn_n),
         "after_learning_ring_us": round(next_us, 1),
         "learning_ring_basis": "wall time of the first ring (classify call + usn_finalize, "
                                "which applies what it learned: answer rules into the registry, "
                                "the rule image brought up to date by the next ring's classify: "
                                "after_learning_ring_us)",
         "workload": "c4tx: %d x 64B frames per ring sent by the host endpoint, %d rules after "
                     "learning, ADD_MACS bridge; ring in %d rotating buffers (%d MiB)"
                     % (n, ctx.rule_count(), TX_ROTATE, TX_ROTATE * n * cfg.stride >> 20),
         "roofline": roof}
    if not args.no_cpu_baseline:
        x["cpu_baseline"] = cpu_baseline(cfg, min(args.cpu_seconds, 3.0))
    for b in bufs:
        b.free()
    for r in res2:
        r.free()
    return x


HOST_INCLUSIVE = {"c5": (1 << 23, 4, 2, 3), "c2": (1 << 20, 8, 4, 4)}   # frames, batches, streams, rounds


def measure_host_inclusive(ctx, name):
    """The PCIe-inclusive rate (north_star): frames start and end
    in pinned host memory.  Per drained ring: hipMemcpyAsync H2D of the header
    windows + lengths, usn_classify, usn_finalize, D2H of the decisions and the
    per-endpoint lists (index + bin_off).  Rings go round-robin over S
    streams, one NIC rx queue each, two device buffer sets per stream; a
    stream's previous ring is finalized and copied back right before its next
    ring is enqueued, so one stream's copies overlap the others' kernels.
    Every returned decision and list is checked against the same ring
    classified device-resident before the timed rounds (the device path,
    itself parity-tested against the oracle in tests/).  Never the value."""
    from usnetd_amd import lib, shard, traffic
    n, nb, S, rounds = HOST_INCLUSIVE[name]
    L = ctx.L
    cfgs = [traffic.config(name, n=n, seed=shard.queue_seed(100 + k, 0)) for k in range(nb)]
    cfg0 = cfgs[0]
    traffic.install_ctx(ctx, cfg0)
    nics = [cfg0.src] + traffic.extra_nics(cfg0, S - 1, ctx)
    W = cfg0.stride
    fbytes, lbytes = n * W, n * 2
    n_ep = max(max(e[0] for e in cfg0.endpoints), max(nics)) + 1
    obytes = n * 8 + (n_ep + 4) * 4            # decisions | index | bin_off
    host = []
    for cfg in cfgs:
        hp = C.c_void_p()
        lib.check(L.usn_host_alloc_pinned(ctx.h, fbytes + lbytes + obytes, C.byref(hp)))
        C.memmove(hp.value, cfg.frames.ctypes.data, fbytes)
        C.memmove(hp.value + fbytes, cfg.lens.ctypes.data, lbytes)
        host.append(hp.value)
    streams = [ctx.stream() for _ in range(S)]
    dev = [[(lib.DeviceBatch(ctx, cfg0.frames, cfg0.lens, nics[si], stride=W), lib.DeviceResult(ctx, n))
            for _ in range(2)] for si in range(S)]
    # the device-resident decisions and lists of every ring (the check)
    ref = []
    b0, r0 = dev[0][0]
    for cfg in cfgs:
        b0.buf.upload(cfg.frames)
        b0.lbuf.upload(cfg.lens)
        ctx.classify(b0, r0, streams[0])
        ctx.finalize(b0, r0, streams[0])
        ref.append((r0.decisions().copy(), r0.index().copy(), r0.bin_off(n_ep + 3).copy()))
    pending = [None] * S
    flip = [0] * S
    host_frames = [0]
    out_of = lambda k, off, cnt: np.frombuffer((C.c_uint8 * (cnt * 4)).from_address(host[k] + fbytes + lbytes + off),
                                              np.uint32)

    def drain(si):
        if pending[si] is None:
            return
        k, j = pending[si]
        b, r = dev[si][j]
        s = streams[si]
        host_frames[0] += ctx.finalize(b, r, s).n_host
        hp = host[k] + fbytes + lbytes
        lib.check(L.usn_memcpy_d2h(ctx.h, hp, r.desc.decisions, n * 4, s))
        lib.check(L.usn_memcpy_d2h(ctx.h, hp + n * 4, r.desc.index, n * 4, s))
        lib.check(L.usn_memcpy_d2h(ctx.h, hp + n * 8, r.desc.bin_off, (n_ep + 4) * 4, s))
        pending[si] = None

    def one(k, si):
        drain(si)
        j = flip[si] = flip[si] ^ 1
        b, r = dev[si][j]
        s = streams[si]
        hp = host[k % nb]
        lib.check(L.usn_memcpy_h2d(ctx.h, b.buf.ptr, hp, fbytes, s))
        lib.check(L.usn_memcpy_h2d(ctx.h, b.lbuf.ptr, hp + fbytes, lbytes, s))
        lib.check(L.usn_classify(ctx.h, C.byref(b.desc), C.byref(r.desc), s))
        pending[si] = (k % nb, j)

    def finish():
        for si in range(S):
            drain(si)
        ctx.sync()

    for k in range(2 * S):                   # warm-up: every stream and buffer set used
        one(k, k % S)
    finish()
    rates = []
    K = 2 * nb
    for _ in range(rounds):
        for k in range(nb):                  # poison the host copies: the check sees this round's
            out_of(k, 0, n)[:] = 0xFFFFFFFF
        t0 = time.perf_counter()
        for k in range(K):
            one(k, k % S)
        finish()
        rates.append(K * n / (time.perf_counter() - t0) / 1e6)
    bad = bad_lists = 0
    for k in range(nb):
        d, idx, off = ref[k]
        bad += int(((out_of(k, 0, n) ^ d) & lib.PARITY_MASK).astype(bool).sum())
        bad_lists += int(not np.array_equal(out_of(k, n * 4, n), idx))
        bad_lists += int(not np.array_equal(out_of(k, n * 8, n_ep + 4)[:n_ep + 4], off[:n_ep + 4]))
    for si in range(S):
        for b, r in dev[si]:
            r.free()
            b.free()
    for hp in host:
        L.usn_host_free_pinned(ctx.h, C.c_void_p(hp))
    med = float(np.median(rates))
    return {"mpps_median": round(med, 1), "mpps_all": [round(x, 1) for x in rates], "unit": "Mpkts/s",
            "frames_per_ring": n, "rings_per_round": K, "streams": S,
            "h2d_bytes_per_frame": W + 2, "d2h_bytes_per_frame": 8,
            "pcie_gbs_equiv": round(med * (W + 10) / 1e3, 1),
            "host_stage_frames": host_frames[0], "decisions_checked": nb * n,
            "decisions_differing": bad, "rings_with_lists_differing": bad_lists,
            "check": "each ring's round-tripped decisions and lists against the same ring "
                     "classified device-resident before the timed rounds",
            "loop": "pinned H2D windows+lens, usn_classify, usn_finalize, D2H decisions+index+bin_off; "
                    "%d streams, a stream's previous ring finalized before its next" % S}


def workload(run, strong):
    cfg = run.cfg0
    sizes = sorted(set(int(x) for x in np.unique(cfg.lens)))
    fr = ("%dB frames" % sizes[0]) if len(sizes) == 1 else \
         ("IMIX frames (%s B) in %d-byte slots" % ("/".join(str(x) for x in sizes[:4]), cfg.stride))
    return ("%s: %d x %s per drained rx ring, %d-rule endpoint table, %d endpoints, NIC rx; "
            "step = one poll round of %d rx queues per GPU (%d rings per launch, %d streams)%s"
            % (run.name, run.n, fr, len(cfg.rules), len(cfg.endpoints), run.Q, run.P,
               run.S, "; strong scaling: 64M frames per step in all" if strong else ""))


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d: refusing to report a different GPU count"
                 % (args.gpus, world))
    if args.launch_check:
        return launch_check(rank, world)
    from usnetd_amd import lib, shard
    L = lib.load()            # the HIP runtime is loaded here, before torch (if any)
    dist = None
    device = local
    if world > 1:
        import torch
        import torch.distributed as dist_mod
        dist_mod.init_process_group("gloo")
        dist = dist_mod
        # counts without initialising the GPU; more ranks than GPUs (a
        # rehearsal): round-robin
        device = shard.rank_device(local, torch.cuda.device_count())
    ctx = lib.Ctx(device)
    if args.lists_async:
        ctx.set_lists_async(True)
    joined = joined_ranks(dist, rank, device)   # every rank is in the group, on its device
    n = args.frames or DEFAULT_FRAMES[args.config]
    run = Run(L, ctx, args.config, n, rank, world, args.queues, args.streams, args.strong,
              args.rings_per_launch, args.rotate_mib << 20, args.result_rounds)
    res = measure(run, args, dist, world)
    out = {
        "metric": METRIC,
        "value": res["value"],
        "unit": "Mpkts/s",
        "value_basis": res["value_basis"],
        "value_single_result_set": res["value_single_result_set"],
        "end_to_end_mpps": res["end_to_end_mpps"],
        "end_to_end": res["end_to_end"],
        "n_gpus": len(joined),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": res["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic frames generated on the host (no captures), resident in HBM",
        "config": {
            "workload": workload(run, args.strong),
            "frames_per_batch": n,
            "rx_queues_per_gpu": run.Q,
            "streams": run.S,
            "batches_per_launch": run.P,
            "rotating_bytes_per_gpu": run.rotating_bytes,
            "result_rounds": run.RR,
            "parallelism": "replicas%d" % world,
            "rank_devices": [d for _, d in joined],
            "event_ms_per_step": res["event_ms_per_step"],
            "enqueue_ms_per_step": res["enqueue_ms_per_step"],
            "lists_async": bool(args.lists_async),
            "untimed_ramp_steps": 2 * args.ramp,
            "frames_per_step_per_gpu": res["frames_per_step_per_gpu"],
            "host_stage_frames": res["host_stage_frames"],
            "summary_flags": res["summary_flags"],
            "class_count_last_rotation": res["class_count_last_rotation"],
        },
        "roofline": res["roofline"],
        "cpu_baseline": None,
    }
    cfg0 = run.cfg0
    run.free()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # pinned like configs[0] (/root/reference/eval/Makefile:22
        # runs the matcher under `taskset -c 6`): one spawned process on one
        # CPU, and one pinned process per CPU of the job's share
        out["cpu_baseline"] = cpu_pinned_1core(args.config, args.cpu_seconds, nshard=1 << 20)
        out["cpu_baseline_ncores"] = cpu_baseline_ncores(args.config, args.cpu_seconds, pin=True)
    del cfg0
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.no_extra:
        # configs[0], the CPU-only config, in both traffic variants
        for name in ("c1", "c1fixed"):
            out[name] = measure_c1(name, min(args.cpu_seconds, 3.0))
    if world == 1 and not args.no_extra:
        # the other BASELINE configs, each measured the same way, under its own
        # key: configs[1] (c2), configs[2] (c3: IMIX in 2048-byte slots) and
        # configs[3] in both directions (c4 rx, c4tx: the ADD_MACS learned-MAC
        # path of a sending endpoint)
        for name in [x for x in args.extras.split(",") if x and x != args.config]:
            ctx.close()
            ctx = lib.Ctx(device)
            if args.lists_async:
                ctx.set_lists_async(True)
            if name == "c4tx":
                x = measure_tx(ctx, args)
            else:
                rx = Run(L, ctx, name, DEFAULT_FRAMES[name], 0, 1, EXTRA_QUEUES.get(name, 0),
                         args.streams, False, result_rounds=args.result_rounds)
                xa = argparse.Namespace(**vars(args))
                xa.steps = max(args.steps, EXTRA_MIN_STEPS.get(name, 0))
                x = measure(rx, xa, None, 1)
                x["workload"] = workload(rx, False)
                if not args.no_cpu_baseline:
                    x["cpu_baseline"] = cpu_pinned_1core(name, min(args.cpu_seconds, 3.0))
                rx.free()
            out[name] = x
    if world == 1 and not args.no_extra and args.host_inclusive:
        # the PCIe-inclusive rate of c5 and c2 (frames and results in pinned
        # host memory), beside the device-resident value
        out["host_inclusive"] = {}
        for name in args.host_inclusive.split(","):
            ctx.close()
            ctx = lib.Ctx(device)
            out["host_inclusive"][name] = measure_host_inclusive(ctx, name)
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


def joined_ranks(dist, rank, device):
    """(rank, HIP device) of every rank in the process group, checked: each
    rank 0..WORLD_SIZE-1 exactly once (so n_gpus counts ranks that ran)."""
    from usnetd_amd import shard
    got = shard.gather_objects((rank, device), dist)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if sorted(r for r, _ in got) != list(range(world)):
        raise SystemExit("bench.py: ranks %s joined, expected 0..%d" % (got, world - 1))
    return got


def launch_check(rank, world):
    """--launch-check: the ranks rendezvous over gloo and rank 0 prints who
    joined (CPU test of launch_ranks; no GPU call)."""
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    joined = joined_ranks(dist, rank, -1)
    if rank == 0:
        print(json.dumps({"n_gpus": len(joined), "ranks": [r for r, _ in joined],
                          "pid": os.getpid()}), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def frames_desc(cfg):
    """What a config's frames are, for the CPU baselines' sample strings."""
    sizes = sorted(set(int(x) for x in np.unique(cfg.lens)))
    if len(sizes) == 1:
        return "%dB frames" % sizes[0]
    return "IMIX frames (%s B) in %d-byte slots" % ("/".join(str(x) for x in sizes[:4]), cfg.stride)


def cpu_baseline(cfg, seconds):
    """The sequential C oracle (restatement of the reference matcher, one
    thread) timed on this host on the rank's first batch, repeated for about
    `seconds` (at least one pass)."""
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
            "sample": "%d passes over one %s batch (%d x %s), sequential C restatement "
                      "with the 1-entry cache, %.1f s" % (passes, cfg.name, cfg.n, frames_desc(cfg), el)}


def _cpu_worker(arg):
    """One core: its own oracle, its own rx queue (batch), passes for ~seconds;
    pinned to `core` when one is given (taskset-style, os.sched_setaffinity)."""
    name, n, seed, seconds, core = arg
    if core is not None:
        os.sched_setaffinity(0, {core})
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
    aff = sorted(os.sched_getaffinity(0))
    return passes * cfg.n, time.perf_counter() - t0, frames_desc(cfg), aff


def host_cpus():
    """The CPUs this job may run on (its affinity set; the GPU box gives a
    share of a larger machine)."""
    try:
        return sorted(os.sched_getaffinity(0))
    except AttributeError:
        return list(range(os.cpu_count() or 1))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline_ncores(name, seconds, pin=False, nshard=1 << 18):
    """SURVEY §8d's N-core variant: the sequential oracle sharded by rx queue,
    one process per core, N = the host CPUs this job may use (at most 16 on
    the GPU box); with `pin`, worker k runs on the k-th of those CPUs only.
    Aggregate frames / slowest worker's time."""
    import multiprocessing as mp
    cpus = host_cpus()
    ncores = max(1, min(len(cpus), int(os.environ.get("OMP_NUM_THREADS", len(cpus))), 16))
    ctx = mp.get_context("spawn")
    with ctx.Pool(ncores) as pool:
        res = pool.map(_cpu_worker, [(name, nshard, 1000 + k, seconds, cpus[k] if pin else None)
                                     for k in range(ncores)])
    frames = sum(r[0] for r in res)
    el = max(r[1] for r in res)
    return {"value": round(frames / el / 1e6, 3), "unit": "Mpkts/s", "cores": ncores,
            "kind": "port", "pinned": bool(pin),
            "sample": "%d processes%s, each the sequential C restatement over its own %s rx queue "
                      "(%d x %s) for %.1f s" % (ncores, " (one per CPU, pinned)" if pin else "", name,
                                                nshard, res[0][2], el)}


def cpu_pinned_1core(name, seconds, nshard=1 << 18):
    """BASELINE configs[0] as the reference measured it: the matcher on ONE
    pinned core (`taskset -c 6`, /root/reference/eval/Makefile:22).  One
    spawned process pinned with os.sched_setaffinity to one CPU of this job's
    set (CPU 6 when the set holds it)."""
    import multiprocessing as mp
    cpus = host_cpus()
    core = 6 if 6 in cpus else cpus[min(len(cpus) - 1, 6)]
    ctx = mp.get_context("spawn")
    with ctx.Pool(1) as pool:
        frames, el, desc, aff = pool.map(_cpu_worker, [(name, nshard, 1000, seconds, core)])[0]
    return {"value": round(frames / el / 1e6, 3), "unit": "Mpkts/s", "cores": 1, "kind": "port",
            "pinned_cpu": core, "affinity_seen_by_worker": aff,
            "sample": "one process pinned to CPU %d, the sequential C restatement (1-entry cache) "
                      "over one %s rx queue (%d x %s) for %.1f s" % (core, name, nshard, desc, el)}


C1_KEYS = {"c1": "random UDP source port per frame (smolbench-style flood)",
           "c1fixed": "fixed 5-tuple (pkt-gen -f tx), every frame a 1-entry-cache hit"}


def measure_c1(name, seconds):
    """configs[0] ("CPU reference, no GPU"): the reference's own CPU
    measurement setup -- 64 B UDP to UDP:3333 of the host, the 4-rule table
    of DEBUG_PORTS TCP:22 + 3 pipes (/root/reference/eval/enp6s0f0config:1-6,
    eval/Makefile:11-28) -- timed on this host, 1 core pinned and N cores,
    with the host CPU named."""
    cpus = host_cpus()
    one = cpu_pinned_1core(name, seconds)
    return {"value": one["value"], "unit": "Mpkts/s", "device": "cpu",
            "traffic": C1_KEYS[name],
            "workload": "%s: 64B IPv4/UDP frames to the host's UDP:3333, 4-rule table "
                        "(DEBUG_PORTS TCP:22 + 3 static pipes)" % name,
            "cpu_model": cpu_model(), "host_cpus": len(cpus),
            "cpu_baseline": one,
            "cpu_baseline_ncores": cpu_baseline_ncores(name, seconds, pin=True)}


if __name__ == "__main__":
    main()
