"""Host-resident (PCIe-inclusive) rates, for DESIGN.md.

1. fcgpu_process_host on a 1M-packet C2 batch: gather first min(len,128) B of
   every frame into pinned staging, H2D, kernels, D2H of verdict/hash/perm.
2. The GPUIPCheckClassify element behind a BURST-32 source (Click-shaped
   packets, linked-list batches, annotation scatter, per-port relinking) at
   several BATCH (accumulation) sizes.
Prints one JSON line.
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from fastclick_amd import synth, click as K, _native as N  # noqa: E402


def raw_host(n):
    b = synth.c2(n)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    ctx = N.Context(0, n, cfg)
    base = b.arena.ctypes.data
    ptrs = (C.c_void_p * n)(*[base + int(o) for o in b.desc[:, 0]])
    lens = np.ascontiguousarray(b.desc[:, 1], dtype=np.uint32)
    v = np.zeros(n, np.uint16); h = np.zeros(n, np.uint32); p = np.zeros(n, np.uint32)
    st = np.zeros(18, np.uint32)
    kw = dict(verdict=v.ctypes.data, hash=h.ctypes.data, perm=p.ctypes.data, port_start=st.ctypes.data)
    ctx.process_host(ptrs, lens.ctypes.data, n, **kw)
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.process_host(ptrs, lens.ctypes.data, n, **kw)
    dt = time.perf_counter() - t0
    ctx.close()
    return n * reps / dt / 1e6


def main():
    out = {"process_host_mpps_1M": round(raw_host(1 << 20), 2)}
    b = synth.c2(1 << 20)
    for batch in (4096, 65536, 262144):
        conf = f"GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash, BATCH {batch})"
        out[f"element_mpps_batch{batch}"] = round(K.bench_element(conf, b, burst=32, reps=3) / 1e6, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
