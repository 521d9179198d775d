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
    lib.fco_process_batch2.restype = None
    lib.fco_process_batch2.argtypes = [C.POINTER(N.fcgpu_cfg), C.c_void_p, C.c_void_p, C.c_uint32,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_void_p]
    lib.fco_process_batch.restype = None
    lib.fco_process_batch.argtypes = [C.POINTER(N.fcgpu_cfg), C.c_void_p, C.c_void_p, C.c_uint32,
                                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p]
    _lib = lib
    return lib


def _p(a):
    return a.ctypes.data if a is not None else None


def process_batch(cfg, batch):
    """Run the oracle over a synth.Batch; returns the same dict as the device path."""
    from fastclick_amd import _native as N
    lib = load()
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
    lib.fco_process_batch2(C.byref(cfg), _p(arena), _p(desc), n, _p(verdict), _p(hsh), _p(anno),
                           _p(perm), _p(start), _p(perm_tile), _p(tile_count), _p(ctr))
    return dict(verdict=verdict, reason=(verdict & 0xFF).astype(np.uint8),
                port=(verdict >> 8).astype(np.uint8), hash=hsh, anno=anno, perm=perm,
                port_start=start, perm_tile=perm_tile, tile_count=tile_count, counters=ctr)


def in_cksum(data: bytes) -> int:
    lib = load()
    buf = C.create_string_buffer(bytes(data), len(data) or 1)
    return lib.fco_in_cksum(buf, len(data))
