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
    assert L.usn_abi_version() == 5


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
    """the one knob that breaks the kernel on purpose (the ISA
    test's USN_ISA_PERTURB) compiles only with USN_AB_BUILD=1; a product build
    that sets it stops at usn_device.hip's static_assert.  (The wrong-result
    ablation knobs left the device source in round 6, VERDICT r05 #9.)"""
    import shutil
    import subprocess
    import pytest
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc) and not shutil.which("hipcc"):
        pytest.skip("no hipcc")
    src = os.path.join(ROOT, "usnetd_amd", "csrc", "usn_device.hip")
    with open(src) as fh:
        assert "USN_ABL_" not in fh.read()
    base = [hipcc, "-std=c++17", "--offload-arch=gfx950", "-fsyntax-only", "-DUSN_NTHREADS=512",
            "-DUSN_NS=usn_t512", src]
    bad = subprocess.run(base + ["-DUSN_ISA_PERTURB=1"], capture_output=True, text=True)
    assert bad.returncode != 0 and "perturbation" in bad.stderr, bad.stderr[-2000:]
    ok = subprocess.run(base + ["-DUSN_ISA_PERTURB=1", "-DUSN_AB_BUILD=1"], capture_output=True,
                        text=True)
    assert ok.returncode == 0, ok.stderr[-2000:]


KNOBS = [b"USN_DEBUG_CORRUPT", b"USN_SCATTER_SLOW_RANK", b"USN_SCATTER_TC", b"USN_SCAN_CPT",
         b"USN_SELFSCAN_KB", b"USN_NO_PROJ", b"USN_IMG_FULL", b"USN_PH_LOAD", b"USN_PH_GROUP",
         b"USN_T512", b"USN_TX_T512", b"USN_PROFILE_HOST", b"USN_RX_EV", b"USN_RX_STATE",
         b"USN_TIMING_EV"]


def test_product_library_reads_no_environment_knob():
    """the test and A/B hooks (USN_DEBUG_CORRUPT corrupts count
    rows or decisions; the others move the list plan or the image geometry)
    are compiled only into the test build (build/test/libusn.so,
    USN_TEST_HOOKS): the product library holds none of their names and does
    not call getenv at all; the test build holds every one."""
    import subprocess
    from usnetd_amd import lib
    prod = open(lib.LIB_PATH, "rb").read()
    test = open(lib.TEST_LIB_PATH, "rb").read()
    for k in KNOBS:
        assert k not in prod, k
        assert k in test, k
    nm = subprocess.run(["nm", "-D", "--undefined-only", lib.LIB_PATH], capture_output=True, text=True)
    if nm.returncode == 0:
        assert not re.search(r"\bgetenv\b", nm.stdout), "the product library imports getenv"


def test_result_release_without_gpu():
    """usn_result_release on a registry-only context: the records of a result
    are dropped (nothing to release is fine); a null result is refused."""
    from usnetd_amd import lib
    L = lib.load()
    h = ctypes.c_void_p()
    assert L.usn_ctx_create(-1, ctypes.byref(h)) == 0   # USN_HOST_ONLY
    n = 4096
    nbytes = L.usn_result_bytes(n)
    buf = ctypes.create_string_buffer(nbytes + 256)
    base = (ctypes.addressof(buf) + 255) & ~255
    r = lib.Result()
    assert L.usn_result_bind(base, nbytes, n, ctypes.byref(r)) == 0
    assert L.usn_result_release(h, ctypes.byref(r)) == 0
    assert L.usn_result_release(h, None) == -22
    L.usn_ctx_destroy(h)
