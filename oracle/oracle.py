"""TEST INFRASTRUCTURE ONLY: ctypes front-end of the C oracle (fc_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as a checker / reported CPU baseline. The product path
(fastclick_amd/) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(BUILD, "liboracle.so")
CPU_BASELINE = os.path.join(BUILD, "fc_cpu_baseline")

_lib = None


def build(force=False):
    """Compile the C restatement (gcc) and the CPU-baseline pipeline (g++)."""
    subprocess.check_call(["make", "-s", "-C", HERE] + (["-B"] if force else []))


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    from fastclick_amd import _native as N  # struct layouts only (no device code)
    lib = C.CDLL(LIB)
    lib.fco_in_cksum.restype = C.c_uint16
    lib.fco_in_cksum.argtypes = [C.c_void_p, C.c_int]
    lib.fco_ipflowid_hash.restype = C.c_uint32
    lib.fco_ipflowid_hash.argtypes = [C.c_uint32, C.c_uint16, C.c_uint32, C.c_uint16]
    lib.fco_ip6flowid_hash.restype = C.c_uint32
    lib.fco_ip6flowid_hash.argtypes = [C.c_void_p, C.c_uint16, C.c_void_p, C.c_uint16]
    lib.fco_lb_hash_port.restype = C.c_int
    lib.fco_lb_hash_port.argtypes = [C.c_uint32, C.c_int]
    lib.fco_crc32c_u32.restype = C.c_uint32
    lib.fco_crc32c_u32.argtypes = [C.c_uint32, C.c_uint32]
    lib.fco_process_batch2.restype = None
    lib.fco_process_batch2.argtypes = [C.POINTER(N.fcgpu_cfg), C.c_void_p, C.c_void_p, C.c_uint32,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.fco_set_program.restype = None
    lib.fco_lb_hash_ring.restype = None
    lib.fco_lb_hash_ring.argtypes = [C.c_uint32, C.c_uint32, C.c_void_p]
    lib.fco_set_lb_table.restype = None
    lib.fco_set_lb_table.argtypes = [C.c_void_p, C.c_uint32]
    lib.fco_set_program.argtypes = [C.c_uint32, C.POINTER(N.fcgpu_step), C.c_uint32, C.c_int32]
    lib.fco_process_batch.restype = None
    lib.fco_process_batch.argtypes = [C.POINTER(N.fcgpu_cfg), C.c_void_p, C.c_void_p, C.c_uint32,
                                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p]
    lib.fco_flow_new.restype = C.c_void_p
    lib.fco_flow_new.argtypes = [C.c_uint32]
    lib.fco_flow_free.restype = None
    lib.fco_flow_free.argtypes = [C.c_void_p]
    lib.fco_flow_count.restype = C.c_uint32
    lib.fco_flow_count.argtypes = [C.c_void_p]
    lib.fco_flow_batch.restype = None
    lib.fco_flow_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                   C.c_void_p, C.c_void_p]
    lib.fco_imp_new.restype = C.c_void_p
    lib.fco_imp_new.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
    lib.fco_imp_free.restype = None
    lib.fco_imp_free.argtypes = [C.c_void_p]
    lib.fco_imp_batch.restype = None
    lib.fco_imp_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                  C.c_void_p, C.c_uint32, C.c_void_p]
    lib.fco_imp_maintain.restype = C.c_uint32
    lib.fco_imp_maintain.argtypes = [C.c_void_p, C.c_uint32]
    lib.fco_imp_stats.restype = None
    lib.fco_imp_stats.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    _lib = lib
    return lib


def _p(a):
    return a.ctypes.data if a is not None else None


def set_program(kind, steps, output_everything=-1):
    """Install the decision program the oracle uses for CLS_PROGRAM (global)."""
    from fastclick_amd import _native as N
    lib = load()
    arr = (N.fcgpu_step * max(len(steps), 1))()
    for i, st in enumerate(steps):
        arr[i] = st if isinstance(st, N.fcgpu_step) else N.fcgpu_step(*[int(x) for x in st])
    lib.fco_set_program(kind, arr, len(steps), output_everything)


def lb_hash_ring(nsel, size=None):
    """LoadBalancer::build_hash_ring over the selector [0, nsel): the
    constant_hash_agg table (CST_BUCKETS size, default 100 per destination)."""
    size = 100 * nsel if size is None else size
    ring = np.zeros(size, np.uint32)
    load().fco_lb_hash_ring(nsel, size, _p(ring))
    return ring


def set_lb_table(table):
    """Install the CLS_LB_TABLE table the oracle uses (global)."""
    t = np.ascontiguousarray(table, dtype=np.uint8)
    load().fco_set_lb_table(_p(t), len(t))


def process_batch(cfg, batch, program=None, lb_table=None):
    """Run the oracle over a synth.Batch; returns the same dict as the device path.
    program: optional (kind, steps, output_everything) for CLS_PROGRAM;
    lb_table: the bucket -> output table for CLS_LB_TABLE."""
    from fastclick_amd import _native as N
    lib = load()
    if program is not None:
        set_program(*program)
    if lb_table is not None:
        set_lb_table(lb_table)
    n = batch.n
    arena = np.ascontiguousarray(batch.arena)
    desc = np.ascontiguousarray(batch.desc, dtype=np.uint32)
    verdict = np.zeros(n, np.uint16)
    hsh = np.zeros(n, np.uint32)
    anno = np.zeros(n, N.anno_dtype())
    perm = np.zeros(n, np.uint32)
    start = np.zeros(cfg.nports + 2, np.uint32)
    ctr = np.zeros(N.NCOUNTERS, np.uint64)
    ntiles = (n + N.TILE - 1) // N.TILE
    perm_tile = np.zeros(n, np.uint32)
    tile_count = np.zeros(ntiles * (cfg.nports + 1), np.uint16)
    ip_rw = np.zeros(n, np.uint32)
    lib.fco_process_batch2(C.byref(cfg), _p(arena), _p(desc), n, _p(verdict), _p(hsh), _p(anno),
                           _p(perm), _p(start), _p(perm_tile), _p(tile_count), _p(ctr), _p(ip_rw))
    return dict(verdict=verdict, reason=(verdict & 0xFF).astype(np.uint8),
                port=(verdict >> 8).astype(np.uint8), hash=hsh, anno=anno, perm=perm,
                port_start=start, perm_tile=perm_tile, tile_count=tile_count, counters=ctr, ip_rw=ip_rw)


class FlowTable:
    """FlowIPManagerHMP restatement (fc_oracle.c fco_flow_*): IDs in order of
    first appearance, kept across batches."""

    def __init__(self, max_flows):
        self.lib = load()
        self.t = self.lib.fco_flow_new(max_flows)

    def batch(self, batch, res):
        """res: this batch's process_batch() result (verdict, anno)."""
        flowid = np.zeros(batch.n, np.uint32)
        arena = np.ascontiguousarray(batch.arena)
        desc = np.ascontiguousarray(batch.desc, dtype=np.uint32)
        self.lib.fco_flow_batch(self.t, _p(arena), _p(desc), batch.n, _p(res["verdict"]),
                                _p(np.ascontiguousarray(res["anno"])), _p(flowid))
        return flowid

    def count(self):
        return self.lib.fco_flow_count(self.t)

    def __del__(self):
        if getattr(self, "t", None):
            self.lib.fco_flow_free(self.t)
            self.t = None


class ImpFlowTable:
    """VirtualFlowManagerIMP restatement (fc_oracle.c fco_imp_*): IDs popped
    from a free-ID stack, idle flows expired by a timer wheel. Times in ms."""

    def __init__(self, capacity, timeout_s=0, recycle_ms=1000):
        self.lib = load()
        self.t = self.lib.fco_imp_new(capacity, timeout_s, recycle_ms)

    def batch(self, batch, res, now_ms):
        flowid = np.zeros(batch.n, np.uint32)
        arena = np.ascontiguousarray(batch.arena)
        desc = np.ascontiguousarray(batch.desc, dtype=np.uint32)
        self.lib.fco_imp_batch(self.t, _p(arena), _p(desc), batch.n, _p(res["verdict"]),
                               _p(np.ascontiguousarray(res["anno"])), now_ms & 0xFFFFFFFF, _p(flowid))
        return flowid

    def maintain(self, now_ms):
        return self.lib.fco_imp_maintain(self.t, now_ms & 0xFFFFFFFF)

    def stats(self):
        v = (C.c_uint32 * 3)()
        self.lib.fco_imp_stats(self.t, C.byref(v, 0), C.byref(v, 4), C.byref(v, 8))
        return dict(count=v[0], free_ids=v[1], pending=v[2])

    def __del__(self):
        if getattr(self, "t", None):
            self.lib.fco_imp_free(self.t)
            self.t = None


def in_cksum(data: bytes) -> int:
    lib = load()
    buf = C.create_string_buffer(bytes(data), len(data) or 1)
    return lib.fco_in_cksum(buf, len(data))
