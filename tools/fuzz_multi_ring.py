#!/usr/bin/env python3
"""Differential fuzz of multi-ring tx launches on the GPU: random streams
(tests/randtraffic.py) through tests/gpu_backend.GpuBackend with every
sending run split into 2-8 rings of one usn_classify_multi launch, against
the C oracle.  Stops at the first mismatch.
usage: fuzz_multi_ring.py first_seed n_seeds [n_events=3000] [filler=0]
  filler > 0: that many rules no frame hits first (tests/test_gpu_parity.py
  _filler), so the image is past LDS and the rx kernel probes U and X."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import coracle  # noqa: E402
import katrun  # noqa: E402
import randtraffic  # noqa: E402
from gpu_backend import GpuBackend  # noqa: E402

coracle.build()
s0, ns = int(sys.argv[1]), int(sys.argv[2])
n_events = int(sys.argv[3]) if len(sys.argv) > 3 else 3000
n_filler = int(sys.argv[4]) if len(sys.argv) > 4 else 0
if n_filler:
    from test_gpu_parity import _filler
frames = 0
t0 = time.time()
for seed in range(s0, s0 + ns):
    # alternate short runs with many ops and long runs spanning tiles
    long_runs = seed % 2
    stream = randtraffic.make_stream(seed, n_events=n_events, tx_frac=0.3 + 0.5 * ((seed >> 1) % 2),
                                     switch_p=0.0008 if long_runs else 0.1,
                                     ops_p=0.0005 if long_runs else 0.02,
                                     n_rules=40 if n_filler else None)
    if n_filler:
        stream["steps"] = _filler(n_filler) + stream["steps"]
    want = randtraffic.run_stream(stream, katrun.COracleBackend())
    got = randtraffic.run_stream(stream, GpuBackend(split_tx_seed=seed))
    assert len(want) == len(got), (seed, len(want), len(got))
    for i, (x, y) in enumerate(zip(want, got)):
        if isinstance(x, tuple):
            ok = x == y
        else:
            ok = (x & katrun.PARITY_MASK) == (y & katrun.PARITY_MASK)
        if not ok:
            print("MISMATCH seed %d event %d: want %r got %r" % (seed, i, x, y), flush=True)
            sys.exit(1)
    frames += sum(1 for x in want if not isinstance(x, tuple))
    if seed % 10 == 9 or seed == s0 + ns - 1:
        print("seeds %d..%d ok, %d frames, %.0f s" % (s0, seed, frames, time.time() - t0), flush=True)
print({"fuzz": "multi_ring", "filler": n_filler, "seeds": ns, "frames": frames, "mismatches": 0})
