"""fastclick_amd -- MI355X-native FastClick receive-path hot path.

IPv4/IPv6 header validation with the Internet checksum, 5-tuple flow-ID hashing
and per-output classification with stable per-port partition, run by
hand-written HIP kernels for gfx950 behind a C ABI (include/fastclick_gpu.h) and
a Click-shaped BatchElement host harness (include/fcclick.h).

Python here is plumbing (ctypes bindings, torch device buffers, synthetic
batches); packet processing happens in libfcgpu.so.
"""
from . import _native  # noqa: F401
from ._native import Context, make_cfg, load  # noqa: F401

__all__ = ["Context", "make_cfg", "load"]
