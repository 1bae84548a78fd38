"""usnetd_amd -- MI355X-native implementation of usnetd's per-frame L4 match path.

The product is the native library usnetd_amd/libusn.so (HIP kernels for gfx950
plus the C++ host behind the C ABI in include/usn_classify.h).  This package
holds its ctypes binding (lib.py), the synthetic workload generator of the
BASELINE.json configurations (traffic.py) and the sharding helpers used by the
multi-GPU bench (shard.py).
"""
from . import lib  # noqa: F401
