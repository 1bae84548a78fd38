"""CPU tests of the drop-in boundary: the library builds for gfx950, loads,
and exports every entry point include/usn_classify.h declares (no GPU calls)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(ROOT, "include", "usn_classify.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(usn_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_api():
    names = declared()
    for must in ("usn_ctx_create", "usn_classify", "usn_finalize", "usn_add_match",
                 "usn_remove_match", "usn_result_bind", "usn_endpoint_add"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from usnetd_amd import lib
    L = ctypes.CDLL(lib.LIB_PATH)
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing
    assert set(declared()) <= set(lib.EXPORTED)
    assert L.usn_abi_version() == 3


def test_device_code_is_gfx950():
    from usnetd_amd import lib
    blob = open(lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob      # the embedded offload bundle
    assert b"amdgcn-amd-amdhsa--gfx942" not in blob


def test_result_layout():
    from usnetd_amd import lib
    L = lib.load()
    n = 5000
    nbytes = L.usn_result_bytes(n)
    buf = ctypes.create_string_buffer(nbytes + 256)
    base = (ctypes.addressof(buf) + 255) & ~255
    r = lib.Result()
    assert L.usn_result_bind(base, nbytes, n, ctypes.byref(r)) == 0
    ptrs = [r.decisions, r.index, r.bin_off, r.tiles, r.summary, r.host_list, r.scratch]
    assert ptrs == sorted(ptrs) and all(p % 256 == 0 for p in ptrs)
    assert r.index - r.decisions >= 4 * n and r.bin_off - r.index >= 4 * n
    assert r.max_bins == lib.USN_MAX_BINS            # usn_result_bytes: any endpoint count
    # sized for endpoint ids < 1002 (c5): a smaller scratch, max_bins 1005
    small = L.usn_result_bytes_ep(n, 1002)
    assert small < nbytes
    assert L.usn_result_bind(base, small, n, ctypes.byref(r)) == 0 and 1005 <= r.max_bins < 1016
    assert L.usn_result_bind(base, L.usn_result_bytes_ep(n, 0) - 1, n, ctypes.byref(r)) == -34


def test_ab_only_knobs_refused_in_product_builds():
    """the ablation knobs that give wrong results on purpose
    compile only with USN_AB_BUILD=1 (the Makefile's `abl` builds); a product
    build that sets one stops at usn_device.hip's static_assert."""
    import shutil
    import subprocess
    import pytest
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc) and not shutil.which("hipcc"):
        pytest.skip("no hipcc")
    src = os.path.join(ROOT, "usnetd_amd", "csrc", "usn_device.hip")
    base = [hipcc, "-std=c++17", "--offload-arch=gfx950", "-fsyntax-only", "-DUSN_NTHREADS=512",
            "-DUSN_NS=usn_t512", src]
    bad = subprocess.run(base + ["-DUSN_ABL_NOPROBE=1"], capture_output=True, text=True)
    assert bad.returncode != 0 and "A/B-only knob" in bad.stderr, bad.stderr[-2000:]
    ok = subprocess.run(base + ["-DUSN_ABL_NOPROBE=1", "-DUSN_AB_BUILD=1"], capture_output=True,
                        text=True)
    assert ok.returncode == 0, ok.stderr[-2000:]
