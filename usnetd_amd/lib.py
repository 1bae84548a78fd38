"""ctypes binding of the C ABI in include/usn_classify.h (usnetd_amd/libusn.so).

This is thin plumbing for tests, bench.py and the control plane; the product is
the native library.  Loading fails loudly when the library is missing or when
no gfx950 device is present: there is no CPU fallback for the match path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libusn.so")
# the test build (Makefile: the product's device code, a host object that
# reads the A/B and test knobs of the environment); only tests that force
# failures and A/B tools load it -- the product library reads no environment
TEST_LIB_PATH = os.path.join(os.path.dirname(HERE), "build", "test", "libusn.so")

USN_TILE = 1024
USN_WINDOW = 64
USN_WINDOW_MAX = 80
USN_MAX_ENDPOINTS = 4095
USN_MAX_BINS = USN_MAX_ENDPOINTS + 3
R_WINDOW = 7
PARITY_MASK = 0x00FFFFFF
EP_NIC, EP_HOST, EP_PIPE, EP_UDS = 0, 1, 2, 3
CLS_DROP, CLS_EP, CLS_NIC, CLS_FLOOD = 0, 1, 2, 3
F_CACHE, F_FRAG1, F_FRAGN, F_DHCP, F_HOST, F_LEARN = (1 << 24, 1 << 25, 1 << 26, 1 << 27,
                                                      1 << 28, 1 << 29)
S_STALE, S_STALE_EXTENDS, S_COUT = 1, 2, 8
STATUS = {0: "ok", -22: "EINVAL", -12: "ENOMEM", -17: "EEXIST", -2: "ENOENT", -1: "EPERM",
          -5: "EHIP", -19: "ENODEV", -34: "ERANGE", -16: "EBUSY", -74: "ELIST"}
USN_EBUSY = -16
USN_EINVAL = -22
USN_ELIST = -74


class UsnError(RuntimeError):
    pass


class Want(C.Structure):
    _fields_ = [("dst_addr", C.c_uint32), ("src_addr", C.c_uint32), ("dst_port", C.c_uint16),
                ("src_port", C.c_uint16), ("protocol", C.c_uint8), ("present", C.c_uint8),
                ("_reserved", C.c_uint16)]


class Batch(C.Structure):
    _fields_ = [("frames", C.c_void_p), ("stride", C.c_uint64), ("offsets", C.c_void_p),
                ("lens", C.c_void_p), ("n", C.c_uint64), ("src_endpoint", C.c_uint16),
                ("window", C.c_uint16), ("_reserved", C.c_uint16 * 2)]


# int (*usn_frame_reader)(void *user, uint16_t src, uint64_t index, uint8_t *out, uint32_t cap)
FRAME_READER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint16, C.c_uint64, C.POINTER(C.c_uint8),
                           C.c_uint32)


class Result(C.Structure):
    _fields_ = [("decisions", C.c_void_p), ("index", C.c_void_p), ("bin_off", C.c_void_p),
                ("tiles", C.c_void_p), ("summary", C.c_void_p), ("host_list", C.c_void_p),
                ("scratch", C.c_void_p), ("n", C.c_uint64), ("max_bins", C.c_uint32),
                ("bind_tag", C.c_uint32)]


class FinalizeInfo(C.Structure):
    _fields_ = [("n_host", C.c_uint32), ("n_patched", C.c_uint32), ("n_learned", C.c_uint32),
                ("flags", C.c_uint32), ("class_count", C.c_uint32 * 4)]


TILE_HDR_DTYPE = np.dtype([("n_frames", "<u2"), ("_r0", "<u2"), ("n_host", "<u2"),
                           ("bin_nic", "<u2"), ("class_count", "<u2", (4,)), ("last_state", "<u4"),
                           ("last_dst", "<u4"), ("last_idx", "<u4"), ("last_info", "<u4", (4,)),
                           ("_pad", "<u4")])
SUMMARY_DTYPE = np.dtype([("flags", "<u4"), ("first_break", "<u4"), ("n_frames", "<u4"),
                          ("n_tiles", "<u4"), ("cin_state", "<u4"), ("cin_dst", "<u4"),
                          ("cin_info", "<u4", (4,)), ("cout_state", "<u4"), ("cout_dst", "<u4"),
                          ("cout_info", "<u4", (4,)), ("n_ep", "<u4"), ("n_bins", "<u4"),
                          ("host_epoch", "<u4"), ("_pad", "<u4")])
RULE_DTYPE = np.dtype([("dst_addr", "<u4"), ("src_addr", "<u4"), ("dst_port", "<u2"),
                       ("src_port", "<u2"), ("protocol", "u1"), ("present", "u1"),
                       ("endpoint", "<u2")])
assert TILE_HDR_DTYPE.itemsize == 48 and SUMMARY_DTYPE.itemsize == 80 and RULE_DTYPE.itemsize == 16

_libs: dict = {}


def load(path: str | None = None):
    """Load libusn.so (raises if it was not built).  `path` selects another
    build of the same ABI (A/B experiments in tools/)."""
    path = path or LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise UsnError("%s is missing: run `make` (or __graft_entry__.build()) first; "
                       "the match path has no CPU fallback" % path)
    L = C.CDLL(path)
    P, I, U16, U32, U64, SZ = C.c_void_p, C.c_int, C.c_uint16, C.c_uint32, C.c_uint64, C.c_size_t
    sig = {
        "usn_abi_version": ([], I), "usn_strerror": ([I], C.c_char_p),
        "usn_last_hip_error": ([], I),
        "usn_ctx_create": ([I, C.POINTER(P)], I), "usn_ctx_destroy": ([P], None),
        "usn_endpoint_add": ([P, U16, I, C.c_int32], I), "usn_endpoint_remove": ([P, U16], I),
        "usn_add_match": ([P, C.POINTER(Want), U16, I], I),
        "usn_remove_match": ([P, C.POINTER(Want), U16], I),
        "usn_rule_count": ([P], I),
        "usn_rules_get": ([P, P, P, P, U32], I),
        "usn_lookup": ([P, C.POINTER(Want)], I),
        "usn_bridge_add": ([P, C.c_char_p], I), "usn_bridge_count": ([P], I),
        "usn_bridge_set": ([P, P, U32], I), "usn_table_build": ([P, P, U32], I),
        "usn_frag_clear": ([P], I), "usn_cache_clear": ([P, U16], I),
        "usn_result_bytes": ([U64], SZ), "usn_result_bytes_ep": ([U64, U32], SZ),
        "usn_result_bind": ([P, SZ, U64, C.POINTER(Result)], I),
        "usn_result_release": ([P, C.POINTER(Result)], I),
        "usn_classify": ([P, C.POINTER(Batch), C.POINTER(Result), P], I),
        "usn_finalize": ([P, C.POINTER(Batch), C.POINTER(Result), P, C.POINTER(FinalizeInfo)], I),
        "usn_dev_alloc": ([P, SZ, C.POINTER(P)], I), "usn_dev_free": ([P, P], I),
        "usn_host_alloc_pinned": ([P, SZ, C.POINTER(P)], I), "usn_host_free_pinned": ([P, P], I),
        "usn_memcpy_h2d": ([P, P, P, SZ, P], I), "usn_memcpy_d2h": ([P, P, P, SZ, P], I),
        "usn_memset_d": ([P, P, I, SZ, P], I),
        "usn_stream_create": ([P, C.POINTER(P)], I), "usn_stream_destroy": ([P, P], I),
        "usn_stream_sync": ([P, P], I), "usn_device_sync": ([P], I),
        "usn_event_create": ([P, C.POINTER(P)], I), "usn_event_destroy": ([P, P], I),
        "usn_event_record": ([P, P, P], I),
        "usn_event_elapsed_ms": ([P, P, P, C.POINTER(C.c_float)], I),
        "usn_stream_wait_event": ([P, P, P], I),
        "usn_classify_multi": ([P, P, P, U32, P], I),
        "usn_set_frame_reader": ([P, FRAME_READER, P], I),
        "usn_ctx_create_group": ([P, U32, C.POINTER(P)], I),
        "usn_ctx_replicas": ([P], I), "usn_replica_select": ([P, U32], I),
        "usn_replica_device": ([P, U32], I),
        "usn_set_lists_async": ([P, I], I), "usn_lists_wait": ([P, C.POINTER(Result), P], I),
    }
    optional = {"usn_set_frame_reader", "usn_ctx_create_group", "usn_ctx_replicas",
                "usn_replica_select", "usn_replica_device", "usn_result_bytes_ep",
                "usn_set_lists_async", "usn_lists_wait", "usn_result_release"}   # A/B builds of older ABI versions lack these
    for name, (args, res) in sig.items():
        if name in optional and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _libs[path] = L
    return L


EXPORTED = ["usn_abi_version", "usn_strerror", "usn_last_hip_error", "usn_ctx_create",
            "usn_ctx_destroy", "usn_endpoint_add", "usn_endpoint_remove", "usn_add_match",
            "usn_remove_match", "usn_rule_count", "usn_rules_get", "usn_lookup", "usn_bridge_add",
            "usn_bridge_count", "usn_frag_clear", "usn_cache_clear", "usn_result_bytes", "usn_result_bytes_ep",
            "usn_result_bind", "usn_classify", "usn_finalize", "usn_dev_alloc", "usn_dev_free",
            "usn_host_alloc_pinned", "usn_host_free_pinned", "usn_memcpy_h2d", "usn_memcpy_d2h",
            "usn_memset_d", "usn_stream_create", "usn_stream_destroy", "usn_stream_sync",
            "usn_device_sync", "usn_event_create", "usn_event_destroy", "usn_event_record",
            "usn_event_elapsed_ms", "usn_stream_wait_event", "usn_classify_multi",
            "usn_bridge_set", "usn_table_build", "usn_set_frame_reader", "usn_ctx_create_group",
            "usn_ctx_replicas", "usn_replica_select", "usn_replica_device", "usn_set_lists_async",
            "usn_lists_wait", "usn_result_release"]


def check(rc, what=""):
    if rc < 0:
        L = load() if LIB_PATH in _libs or not _libs else next(iter(_libs.values()))
        extra = ""
        if rc == -5:
            extra = " (hipError %d)" % L.usn_last_hip_error()
        raise UsnError("%s failed: %s%s" % (what, STATUS.get(rc, rc), extra))
    return rc


def ip2int(s):
    if s is None:
        return None
    if isinstance(s, int):
        return s
    a, b, c, d = (int(x) for x in s.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def make_want(dst, proto, dport=None, src=None, sport=None) -> Want:
    w = Want()
    w.dst_addr = ip2int(dst)
    w.protocol = proto
    p = 0
    if dport is not None:
        p |= 1
        w.dst_port = dport
    if src is not None:
        p |= 2
        w.src_addr = ip2int(src)
    if sport is not None:
        p |= 4
        w.src_port = sport
    w.present = p
    return w


def want_from_dict(d) -> Want:
    return make_want(d["dst"], d["proto"], d.get("dport"), d.get("src"), d.get("sport"))


class DevBuf:
    """A device allocation owned by a Ctx."""

    def __init__(self, ctx: "Ctx", nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        check(ctx.L.usn_dev_alloc(ctx.h, max(self.nbytes, 16), C.byref(p)), "usn_dev_alloc")
        self.ptr = p.value

    def free(self):
        if self.ptr:
            self.ctx.L.usn_dev_free(self.ctx.h, self.ptr)
            self.ptr = None

    def upload(self, arr: np.ndarray, stream=None, offset=0):
        arr = np.ascontiguousarray(arr)
        assert offset + arr.nbytes <= self.nbytes
        check(self.ctx.L.usn_memcpy_h2d(self.ctx.h, self.ptr + offset, arr.ctypes.data,
                                        arr.nbytes, stream), "h2d")
        if stream is None:
            self.ctx.sync()

    def download(self, dtype, count, offset=0, stream=None) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        check(self.ctx.L.usn_memcpy_d2h(self.ctx.h, out.ctypes.data, self.ptr + offset,
                                        out.nbytes, stream), "d2h")
        self.ctx.sync(stream)
        return out


class Ctx:
    """One usn_ctx bound to one gfx950 device (the daemon's match state)."""

    def __init__(self, device: int = 0, libpath: str | None = None, devices=None):
        """devices: a list of HIP devices -> one registry with a device
        replica per entry (usn_ctx_create_group); replica 0 is selected."""
        self.L = load(libpath)
        h = C.c_void_p()
        if devices is not None:
            arr = (C.c_int * len(devices))(*devices)
            check(self.L.usn_ctx_create_group(C.cast(arr, C.c_void_p), len(devices), C.byref(h)),
                  "usn_ctx_create_group")
            device = devices[0]
        else:
            check(self.L.usn_ctx_create(device, C.byref(h)), "usn_ctx_create")
        self.h = h.value
        self.device = device

    def replicas(self) -> int:
        return check(self.L.usn_ctx_replicas(self.h), "usn_ctx_replicas")

    def select(self, replica: int):
        """Classify and device plumbing act on this replica from now on."""
        check(self.L.usn_replica_select(self.h, replica), "usn_replica_select")
        self.device = check(self.L.usn_replica_device(self.h, replica), "usn_replica_device")

    def close(self):
        if self.h:
            self.L.usn_ctx_destroy(self.h)
            self.h = None

    # --- control plane --------------------------------------------------------
    def endpoint_add(self, eid, kind, for_nic=None):
        return check(self.L.usn_endpoint_add(self.h, eid, kind, -1 if for_nic is None else for_nic),
                     "usn_endpoint_add")

    def endpoint_remove(self, eid):
        return check(self.L.usn_endpoint_remove(self.h, eid), "usn_endpoint_remove")

    def add_match(self, want: Want, owner: int, sticky=False) -> int:
        rc = self.L.usn_add_match(self.h, C.byref(want), owner, int(bool(sticky)))
        return rc if rc in (0, 1) else check(rc, "usn_add_match")

    def remove_match(self, want: Want, requester: int) -> int:
        rc = self.L.usn_remove_match(self.h, C.byref(want), requester)
        return -1 if rc == -1 else check(rc, "usn_remove_match")

    def rule_count(self):
        return check(self.L.usn_rule_count(self.h), "usn_rule_count")

    def rules(self):
        n = self.rule_count()
        ws = (Want * max(n, 1))()
        owners = np.zeros(max(n, 1), np.uint16)
        sticky = np.zeros(max(n, 1), np.uint8)
        got = check(self.L.usn_rules_get(self.h, C.cast(ws, C.c_void_p), owners.ctypes.data,
                                         sticky.ctypes.data, n), "usn_rules_get")
        return [(ws[i], int(owners[i]), bool(sticky[i])) for i in range(got)]

    def lookup(self, want: Want) -> int:
        rc = self.L.usn_lookup(self.h, C.byref(want))
        return -1 if rc == -2 else check(rc, "usn_lookup")

    def bridge_add(self, mac: bytes):
        check(self.L.usn_bridge_add(self.h, bytes(mac)), "usn_bridge_add")

    def table_build(self, rules) -> int:
        """rules: [(Want, owner, sticky)] -> usn_table_build (bulk replace)."""
        arr = np.zeros(len(rules), RULE_DTYPE)
        for i, (w, owner, sticky) in enumerate(rules):
            arr[i] = (w.dst_addr, w.src_addr, w.dst_port, w.src_port, w.protocol,
                      (w.present & 7) | (0x80 if sticky else 0), owner)
        return check(self.L.usn_table_build(self.h, arr.ctypes.data, len(rules)),
                     "usn_table_build")

    def bridge_set(self, macs) -> None:
        arr = np.frombuffer(b"".join(bytes(m) for m in macs), np.uint8) if macs else np.zeros(6, np.uint8)
        check(self.L.usn_bridge_set(self.h, arr.ctypes.data, len(macs)), "usn_bridge_set")

    def bridge_count(self) -> int:
        return check(self.L.usn_bridge_count(self.h), "usn_bridge_count")

    def frag_clear(self):
        check(self.L.usn_frag_clear(self.h), "usn_frag_clear")

    def cache_clear(self, eid):
        check(self.L.usn_cache_clear(self.h, eid), "usn_cache_clear")

    def set_frame_reader(self, fn):
        """fn(src_endpoint, index) -> bytes of that frame of the batch being
        finalized (the host copy, whole or its first USN_WINDOW_MAX bytes);
        None unregisters.  The ctypes callback is kept alive on the Ctx."""
        if fn is None:
            self._reader = None
            check(self.L.usn_set_frame_reader(self.h, FRAME_READER(), None), "usn_set_frame_reader")
            return

        def cb(user, src, index, out, cap):
            try:
                data = bytes(fn(int(src), int(index)))[:cap]
            except Exception:
                return -1
            C.memmove(out, data, len(data))
            return len(data)
        self._reader = FRAME_READER(cb)
        check(self.L.usn_set_frame_reader(self.h, self._reader, None), "usn_set_frame_reader")

    # --- plumbing ---------------------------------------------------------------
    def alloc(self, nbytes) -> DevBuf:
        return DevBuf(self, nbytes)

    def sync(self, stream=None):
        if stream is None:
            check(self.L.usn_device_sync(self.h), "usn_device_sync")
        else:
            check(self.L.usn_stream_sync(self.h, stream), "usn_stream_sync")

    def stream(self):
        s = C.c_void_p()
        check(self.L.usn_stream_create(self.h, C.byref(s)), "usn_stream_create")
        return s.value

    def event(self):
        e = C.c_void_p()
        check(self.L.usn_event_create(self.h, C.byref(e)), "usn_event_create")
        return e.value

    def record(self, ev, stream):
        check(self.L.usn_event_record(self.h, ev, stream), "usn_event_record")

    def wait_event(self, stream, ev):
        check(self.L.usn_stream_wait_event(self.h, stream, ev), "usn_stream_wait_event")

    def elapsed_ms(self, a, b) -> float:
        ms = C.c_float()
        check(self.L.usn_event_elapsed_ms(self.h, a, b, C.byref(ms)), "usn_event_elapsed_ms")
        return ms.value

    # --- hot path -----------------------------------------------------------------
    def classify(self, batch: "DeviceBatch", result: "DeviceResult", stream=None):
        check(self.L.usn_classify(self.h, C.byref(batch.desc), C.byref(result.desc), stream),
              "usn_classify")

    def classify_multi(self, batches, results, stream=None):
        """One launch over several batches (usn_classify_multi): rx rings of
        distinct NIC sources, or up to eight consecutive rings of a sending
        endpoint (in one tx grid)."""
        n = len(batches)
        ba = (Batch * n)(*[b.desc for b in batches])
        ra = (Result * n)(*[r.desc for r in results])
        check(self.L.usn_classify_multi(self.h, C.cast(ba, C.c_void_p), C.cast(ra, C.c_void_p), n,
                                        stream), "usn_classify_multi")

    def set_lists_async(self, on=True):
        """Build the per-endpoint lists on a side stream (usn_set_lists_async)."""
        check(self.L.usn_set_lists_async(self.h, int(bool(on))), "usn_set_lists_async")

    def scatter_fallbacks(self) -> int:
        """Scatter chunks (on this replica's device, since the library was
        loaded) whose optimistic ranks were not stably sorted and were ranked
        again the ballot way (expected 0; usn_debug_scatter_fallbacks)."""
        f = self.L.usn_debug_scatter_fallbacks
        f.argtypes = [C.c_void_p]
        f.restype = C.c_int64
        return check(f(self.h), "usn_debug_scatter_fallbacks")

    def lists_wait(self, result: "DeviceResult", stream=None):
        check(self.L.usn_lists_wait(self.h, C.byref(result.desc), stream), "usn_lists_wait")

    def finalize(self, batch: "DeviceBatch", result: "DeviceResult", stream=None) -> FinalizeInfo:
        info = FinalizeInfo()
        check(self.L.usn_finalize(self.h, C.byref(batch.desc), C.byref(result.desc), stream,
                                  C.byref(info)), "usn_finalize")
        return info


class DeviceBatch:
    """Frames + lengths resident in HBM (one drained rx ring)."""

    def __init__(self, ctx: Ctx, frames: np.ndarray, lens: np.ndarray, src: int,
                 stride: int = 0, offsets: np.ndarray | None = None, pad: int = USN_WINDOW,
                 window: int | None = None):
        """window: readable bytes of each frame at its start (usn_batch.window);
        default min(stride, 2048) for strided layouts, USN_WINDOW for offsets."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8).reshape(-1)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        self.n = int(lens.shape[0])
        self.buf = ctx.alloc(frames.nbytes + pad)
        self.buf.upload(frames)
        self.lbuf = ctx.alloc(lens.nbytes)
        self.lbuf.upload(lens)
        self.obuf = None
        self.desc = Batch()
        self.desc.frames = self.buf.ptr
        self.desc.lens = self.lbuf.ptr
        self.desc.n = self.n
        self.desc.src_endpoint = src
        if window is None:
            window = min(int(stride), 2048) if offsets is None and stride else USN_WINDOW
        self.desc.window = window
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            self.obuf = ctx.alloc(offsets.nbytes)
            self.obuf.upload(offsets)
            self.desc.offsets = self.obuf.ptr
            self.desc.stride = 0
        else:
            self.desc.stride = stride

    def set_src(self, src):
        self.desc.src_endpoint = src

    def free(self):
        for b in (self.buf, self.lbuf, self.obuf):
            if b is not None:
                b.free()


class DeviceResult:
    """One usn_result: decisions, the per-endpoint lists (index, bin_off),
    tile headers, summary.  max_endpoints sizes the scatter scratch for
    endpoint ids below it (default: any id, USN_MAX_ENDPOINTS)."""

    def __init__(self, ctx: Ctx, n: int, max_endpoints: int | None = None):
        self.ctx = ctx
        self.n = int(n)
        if max_endpoints is None:
            nbytes = ctx.L.usn_result_bytes(self.n)
        else:
            nbytes = ctx.L.usn_result_bytes_ep(self.n, int(max_endpoints))
        self.buf = ctx.alloc(nbytes)
        self.desc = Result()
        check(ctx.L.usn_result_bind(self.buf.ptr, nbytes, self.n, C.byref(self.desc)),
              "usn_result_bind")
        self.ntiles = (self.n + USN_TILE - 1) // USN_TILE

    def _off(self, ptr):
        return ptr - self.buf.ptr

    def decisions(self, n=None) -> np.ndarray:
        return self.buf.download(np.uint32, n or self.n, self._off(self.desc.decisions))

    def index(self, n=None) -> np.ndarray:
        return self.buf.download(np.uint32, n or self.n, self._off(self.desc.index))

    def bin_off(self, nbins=None) -> np.ndarray:
        nb = int(self.summary()["n_bins"]) if nbins is None else nbins
        return self.buf.download(np.uint32, nb + 1, self._off(self.desc.bin_off))

    def lists(self, n=None) -> dict:
        """{bin: frame indices in frame order} of the device-wide scatter
        (bins: endpoint ids, then n_ep = NIC, n_ep + 1 = FLOOD, n_ep + 2 = DROP)."""
        off = self.bin_off()
        idx = self.index(n)
        return {b: idx[off[b]:off[b + 1]] for b in range(off.size - 1) if off[b + 1] > off[b]}

    def tiles(self) -> np.ndarray:
        raw = self.buf.download(np.uint8, self.ntiles * TILE_HDR_DTYPE.itemsize,
                                self._off(self.desc.tiles))
        return raw.view(TILE_HDR_DTYPE)

    def summary(self) -> np.ndarray:
        raw = self.buf.download(np.uint8, SUMMARY_DTYPE.itemsize, self._off(self.desc.summary))
        return raw.view(SUMMARY_DTYPE)[0]

    def free(self):
        """usn_result_release (the context's records of this result), then the memory"""
        if self.buf is None:
            return
        if hasattr(self.ctx.L, "usn_result_release") and self.ctx.h:
            check(self.ctx.L.usn_result_release(self.ctx.h, C.byref(self.desc)), "usn_result_release")
        self.buf.free()
        self.buf = None


def dec_bin(dec: np.ndarray, n_ep: int) -> np.ndarray:
    """bin of each decision word: its endpoint id (class EP), else NIC / FLOOD / DROP after the
    endpoints (usn_classify.h, usn_result.index)."""
    cls = (dec >> 16) & 0xF
    ep = dec & 0xFFFF
    other = n_ep + ((cls + 2) & 3)
    return np.where(cls == CLS_EP, ep, other).astype(np.int64)


def expected_lists(dec: np.ndarray, n_ep: int) -> dict:
    """{bin: frame indices} a stable scatter of these decisions must produce."""
    bins = dec_bin(np.asarray(dec, np.uint32), n_ep)
    order = np.argsort(bins, kind="stable")
    sb = bins[order]
    cuts = np.flatnonzero(np.diff(sb)) + 1
    return {int(sb[g[0]]): order[g].astype(np.uint32) for g in np.split(np.arange(sb.size), cuts)
            if g.size}
