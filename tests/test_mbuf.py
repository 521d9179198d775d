"""mbuf ingress (fcgpu_pool_register / fcgpu_process_mbufs).

A DPDK-style mempool is emulated in page-locked host memory: elements of
128-B mbuf header (rte_mbuf layout: buf_addr @0, data_off @16, data_len @40)
+ 128-B headroom + 2048-B data room. The batch handed to the device is the
array of mbuf pointers in rx-burst order (here: shuffled over the pool, as
a mempool hands buffers out), including pointers outside the pool and a
frame running past it, which must read as empty frames. The device verdicts,
hashes and tile partition must equal the oracle's on the same frames.
"""
import mmap

import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N
from tests.helpers import compare

ELEM = 128 + 128 + 2048


def make_pool(frames, rng):
    """(pool bytes, mbuf pointers in rx order, frames in rx order) for the
    given frames, one mbuf each, placed at shuffled pool slots."""
    n = len(frames)
    size = ((n + 8) * ELEM + 4095) & ~4095
    buf = mmap.mmap(-1, size)
    arr = np.frombuffer(buf, np.uint8)
    base = arr.ctypes.data
    slots = rng.permutation(n + 8)[:n]
    ptrs = np.zeros(n, np.uint64)
    for k, (f, s_) in enumerate(zip(frames, slots)):
        e = int(s_) * ELEM
        hdr = arr[e:e + 128]
        hdr[0:8] = np.frombuffer(np.uint64(base + e + 128).tobytes(), np.uint8)      # buf_addr
        hdr[16:18] = np.frombuffer(np.uint16(128).tobytes(), np.uint8)               # data_off
        hdr[40:42] = np.frombuffer(np.uint16(len(f)).tobytes(), np.uint8)            # data_len
        arr[e + 256:e + 256 + len(f)] = np.frombuffer(f, np.uint8)
        ptrs[k] = base + e
    return buf, arr, base, size, ptrs


@pytest.mark.gpu
def test_gpu_mbuf_ingress_vs_oracle(oracle):
    import torch
    from fastclick_amd.device import DeviceOutputs
    rng = np.random.default_rng(90)
    b = synth.c4(20_000, seed=91)
    synth.add_ip_options(b, 0.1, seed=92)
    synth.inject_errors(b, 0.02, seed=93)
    frames = b.frames()
    buf, arr, base, size, ptrs = make_pool(frames, rng)
    # bad pointers: outside the pool, inside but with a frame past its end
    bad_out = [5, 77, 19_999]
    for i in bad_out:
        ptrs[i] = base + size + 4096 * (i + 1)
    i_edge = 1234
    e = int(ptrs[i_edge] - base)
    arr[e:e + 8] = np.frombuffer(np.uint64(base + size - 100).tobytes(), np.uint8)   # buf_addr near the end
    arr[e + 16:e + 18] = np.frombuffer(np.uint16(0).tobytes(), np.uint8)
    exp_frames = list(frames)
    for i in bad_out + [i_edge]:
        exp_frames[i] = b""
    exp_b = synth.from_frames(exp_frames)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16, badsrc=[N.raw_addr("192.0.2.255")])
    exp = oracle.process_batch(cfg, exp_b)
    ctx = N.Context(0, b.n, cfg)
    try:
        ctx.pool_register(base, size)
        outs = DeviceOutputs(b.n, 16, device="cuda:0", anno=True, perm=True, partition=N.PART_TILE)
        ctx.process_mbufs(ptrs.ctypes.data, b.n, **outs.ptrs())
        torch.cuda.synchronize()
        got = outs.numpy()
        compare(got, exp, anno=True, perm=True, ctx="mbuf")
        assert (got["reason"][bad_out + [i_edge]] == N.R_MINISCULE).all()
        assert np.array_equal(np.array(ctx.counters(), np.uint64), exp["counters"])
    finally:
        ctx.close()          # unregisters the pool before the mapping goes away
