"""CPU tests: pin the oracle before trusting it.

Both CPU restatements (C: oracle/usn_oracle.c, Python: oracle/pyoracle.py)
are checked against the hand-derived known-answer frames in tests/golden/
(the reference ships no tests or fixtures: parity unpinned),
then against each other on seeded random event streams.
"""
import numpy as np
import pytest

import katrun
import randtraffic


@pytest.fixture(scope="module", autouse=True)
def _build_oracle():
    import coracle
    coracle.build()


@pytest.mark.parametrize("kat", katrun.load_kats(), ids=lambda k: k["name"])
@pytest.mark.parametrize("backend", ["c", "py"])
def test_kat(kat, backend):
    be = katrun.COracleBackend() if backend == "c" else katrun.PyOracleBackend()
    bad = katrun.run_kat(kat, be)
    assert not bad, "\n".join("step %d: got %#x want %#x (%s)" % b for b in bad)


def test_kat_covers_every_quirk():
    kats = {k["name"]: k for k in katrun.load_kats()}
    frames = [s for k in kats.values() for s in k["steps"] if s["op"] == "frame"]
    reasons = {s["expect"][2] for s in frames}
    classes = {s["expect"][0] for s in frames}
    assert reasons == set(range(7)), reasons
    assert classes == {0, 1, 2, 3}
    assert any("smoltcp-recall" in s["tags"] for s in frames)
    assert len(frames) >= 60


@pytest.mark.parametrize("seed", range(12))
def test_c_vs_python_random(seed):
    stream = randtraffic.make_stream(seed, n_events=600)
    a = randtraffic.run_stream(stream, katrun.COracleBackend())
    b = randtraffic.run_stream(stream, katrun.PyOracleBackend())
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        if isinstance(x, tuple):
            assert x == y, (i, x, y)
        else:
            assert (x & katrun.PARITY_MASK) == (y & katrun.PARITY_MASK), (i, hex(x), hex(y))


def test_batch_api_matches_single():
    import coracle
    from usnetd_amd import traffic
    cfg = traffic.config("c2", n=4096)
    o1, o2 = coracle.Oracle(), coracle.Oracle()
    for o in (o1, o2):
        coracle.install_oracle(o, cfg)
    d1 = o1.forward_batch(cfg.src, cfg.frames, cfg.lens, stride=cfg.stride)
    d2 = np.array([o2.forward(cfg.src, cfg.window(i))
                   for i in range(cfg.n)], dtype=np.uint32)
    assert (d1 == d2).all()
