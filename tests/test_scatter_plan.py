"""CPU tests of how a launch's per-endpoint lists are planned (usn_host.cpp
scatter_plan, through the test hook usn_debug_scatter_plan; no GPU call):
the chunk length, the scan threads' chunks, and when the scan launch is
skipped -- for the bench's launch shapes."""
import ctypes
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CUS = 256   # MI355X


def plan(ntiles, nbins, cus=CUS):
    from usnetd_amd import lib
    L = ctypes.CDLL(lib.LIB_PATH)
    f = L.usn_debug_scatter_plan
    f.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                  ctypes.POINTER(ctypes.c_uint32)]
    f.restype = ctypes.c_int
    nt = (ctypes.c_uint32 * len(ntiles))(*ntiles)
    out = (ctypes.c_uint32 * 4)()
    rc = f(nt, len(ntiles), nbins, cus, out)
    assert rc == 0, rc
    return {"tc": out[0], "cpt": out[1], "noscan": bool(out[2]), "selfscan": bool(out[3])}


@pytest.mark.parametrize("name,ntiles,nbins,want", [
    # c5: two 8M rings, 1005 bins -- 8-tile chunks, the scan at 4 chunks per thread
    ("c5", [8192, 8192], 1005, {"tc": 8, "cpt": 4, "noscan": False, "selfscan": False}),
    # c2: eight 1M rings, 19 bins -- 1024 chunks, too many to self-scan
    ("c2", [1024] * 8, 19, {"tc": 8, "cpt": 1, "noscan": False, "selfscan": False}),
    # c4 rx: eight 1M rings, 259 bins
    ("c4", [1024] * 8, 259, {"tc": 8, "cpt": 1, "noscan": False, "selfscan": False}),
    # c3: four 256K rings, 67 bins -- a chunk per CU, 9.4 MB of rows: self-scan
    ("c3", [256] * 4, 67, {"tc": 4, "cpt": 1, "noscan": False, "selfscan": True}),
    # a tx ring (c4tx): 1024 tiles, 261 bins -- 4-tile chunks, 138 MB of rows: the scan
    ("c4tx", [1024], 261, {"tc": 4, "cpt": 1, "noscan": False, "selfscan": False}),
    # one 1M c2 ring (the daemon's): self-scan
    ("c2ring", [1024], 19, {"tc": 4, "cpt": 1, "noscan": False, "selfscan": True}),
    # a drained ring of 8K frames: one chunk, no scan at all
    ("small", [8], 19, {"tc": 8, "cpt": 1, "noscan": True, "selfscan": False}),
])
def test_plan_of_the_bench_shapes(name, ntiles, nbins, want):
    got = plan(ntiles, nbins)
    assert got == want, (name, got)


def test_chunks_per_cu():
    """About one chunk per CU: the chunk length halves as the launch shrinks,
    never below one tile, never above the LDS shape's."""
    for tiles, tc in ((16384, 8), (2048, 8), (1024, 4), (512, 2), (300, 1), (64, 1)):
        assert plan([tiles], 19)["tc"] == tc, tiles
    assert plan([1024], 19, cus=128)["tc"] == 8
    # c5's bins at 4 tiles per CU: the LDS shape caps the chunk at 8 tiles anyway
    assert plan([4096], 1005)["tc"] == 8


def test_self_scan_needs_a_resident_launch_and_few_rows():
    assert plan([256] * 4, 67)["selfscan"]
    assert plan([256] * 4, 67, cus=128) == {"tc": 8, "cpt": 1, "noscan": False, "selfscan": True}
    assert not plan([300] * 4, 67)["selfscan"]                  # 4 x 75 chunks > 256 CUs
    assert not plan([1024], 1005)["selfscan"]                   # 2 KiB rows: 512 MB read
    assert not plan([2048] * 4, 67)["selfscan"]                 # 1024 chunks
