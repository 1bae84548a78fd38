"""usn_result_release of an rx result that was classified but not finalized
(ADVICE r05, medium): the release is the step before the caller frees or
re-binds the memory, so it must wait for that batch's classify and lists
(on the caller's stream, or on the side stream with usn_set_lists_async)
before it returns.  After the release nothing of the launch may still run,
and what the result holds is the oracle's."""
import ctypes as C

import numpy as np
import pytest

import katrun

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def coracle_mod():
    import coracle
    coracle.build()
    return coracle


def _hip():
    from usnetd_amd import lib
    lib.load()                       # libamdhip64 is already mapped by libusn.so
    h = C.CDLL("libamdhip64.so")
    h.hipStreamQuery.argtypes = [C.c_void_p]
    h.hipStreamQuery.restype = C.c_int
    return h


@pytest.mark.parametrize("lists_async", [0, 1])
def test_release_waits_for_unfinalized_rx(lists_async, coracle_mod):
    from usnetd_amd import lib, traffic
    n = 1 << 22                      # ~60 us of device work: far longer than the release call
    cfg = traffic.config("c5", n=n, seed=11)
    ctx = lib.Ctx(0)
    traffic.install_ctx(ctx, cfg)
    if lists_async:
        ctx.set_lists_async(True)
    s = ctx.stream()
    b = lib.DeviceBatch(ctx, cfg.frames, cfg.lens, cfg.src, stride=cfg.stride)
    r = lib.DeviceResult(ctx, n)
    ctx.sync()
    ctx.classify(b, r, s)
    lib.check(ctx.L.usn_result_release(ctx.h, C.byref(r.desc)), "usn_result_release")
    assert _hip().hipStreamQuery(s) == 0, "the batch's launch still runs after usn_result_release"
    o = coracle_mod.Oracle()
    coracle_mod.install_oracle(o, cfg)
    want = o.forward_batch(cfg.src, cfg.frames, cfg.lens, stride=cfg.stride)
    got = r.decisions()
    assert np.array_equal(got & katrun.PARITY_MASK, want & katrun.PARITY_MASK)
    n_ep = int(r.summary()["n_ep"])
    ref = lib.expected_lists(want, n_ep)
    lists = r.lists()
    assert sorted(lists) == sorted(ref)
    assert all(np.array_equal(lists[k], ref[k]) for k in ref)
    r.free()                         # a second release of the same result is harmless
    b.free()
    ctx.close()
