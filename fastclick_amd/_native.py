"""ctypes binding of the C ABI in include/fastclick_gpu.h (libfcgpu.so).

The shared library is built in-tree by ``fastclick_amd.build`` (hipcc, gfx950)
into ``fastclick_amd/lib/``. Loading fails loudly when it is missing: there is
no CPU fallback for the product path.
"""
from __future__ import annotations

import ctypes as C
import os

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
# FCGPU_LIB: another build of the library (same-box A/B measurements only)
LIBFCGPU = os.environ.get("FCGPU_LIB") or os.path.join(LIB_DIR, "libfcgpu.so")
LIBFCCLICK = os.path.join(LIB_DIR, "libfcclick.so")

# ---- constants mirrored from include/fastclick_gpu.h -----------------------
ABI_VERSION = 25
SPAN_SLOTS = 3
SPAN_COPY = 0
SPAN_ZEROCOPY = 1
SPAN_AUTO = 2
OK, EINVAL, ENODEV, ENOMEM, ERUNTIME = 0, -1, -2, -3, -4
R_MINISCULE, R_BAD_VERSION, R_BAD_HLEN, R_BAD_IP_LEN, R_BAD_CKSUM, R_BAD_SADDR, R_OK, \
    R_BAD_IP6, R_VLAN_REJECT, R_NO_MATCH, R_L4_PROTO, R_L4_LENGTH, R_L4_CKSUM, \
    R_TTL_EXPIRED, R_SETCKSUM_BAD = range(15)
NREASON_SLOTS = 14
RW_DECTTL, RW_SETCKSUM, RW_INPLACE = 1, 2, 4
L4_NONE, L4_UDP, L4_TCP = 0, 1, 2


def reason_slot(r: int) -> int:
    """Counter slot of reason r (reasons 0-5, 7-14; 6 = valid has none)."""
    return r if r < 6 else r - 1
CHECK_IP4, MARK_IP4, CHECK_AUTO, MARK_IP6 = 0, 1, 2, 3
HASH_NONE, HASH_FLOWID, HASH_FLOW5ID = 0, 1, 2
CLS_NONE, CLS_LB_HASH, CLS_HASH_IP, CLS_HASHSWITCH, CLS_PROGRAM, CLS_LB_CRC, CLS_LB_TABLE = 0, 1, 2, 3, 4, 5, 6
PROG_IPFILTER, PROG_CLASSIFIER = 0, 1
STEP_SHORT_YES = 1
MAX_STEPS = 8192
MAX_PORTS = 64
LB_TABLE_MAX = 1 << 24
MAX_ADDRS = 16
CTR_COUNT, CTR_DROPS, CTR_REASON, CTR_PORT = 0, 1, 2, 16
NCOUNTERS = CTR_PORT + MAX_PORTS + 1
CTR_SHARDS = 64
PART_GLOBAL, PART_TILE = 0, 1
OUT_VERDICT, OUT_HASH, OUT_ANNO, OUT_PERM, OUT_PORT_START, OUT_TILE_COUNT, OUT_TILE_PERM, OUT_FLOWID, \
    OUT_IP_RW, OUT_ANNO8 = (1 << k for k in range(10))
SUBMIT_COPY = 1 << 31
SUBMIT_DESC32 = 1 << 30
FAULT_SUBMIT, FAULT_WAIT, FAULT_LAUNCH, FAULT_ALLOC = 0, 1, 2, 3
OUT_ABSENT = (1 << 64) - 1
TILE = 256

REASON_TEXTS = ["tiny packet", "bad IPv4 version", "bad IPv4 header length",
                "bad IPv4 length", "bad IPv4 checksum", "bad source address"]


class fcgpu_cfg(C.Structure):
    _fields_ = [
        ("size", C.c_uint32),
        ("check_mode", C.c_uint32),
        ("offset", C.c_int32),
        ("checksum", C.c_uint32),
        ("hash_mode", C.c_uint32),
        ("classify", C.c_uint32),
        ("nports", C.c_uint32),
        ("hs_offset", C.c_int32),
        ("hs_length", C.c_int32),
        ("native_vlan", C.c_int32),
        ("nbadsrc", C.c_uint32),
        ("ngooddst", C.c_uint32),
        ("badsrc", C.c_uint32 * MAX_ADDRS),
        ("gooddst", C.c_uint32 * MAX_ADDRS),
        ("nbad6", C.c_uint32),
        ("bad6", (C.c_uint8 * 16) * MAX_ADDRS),
        ("process_eh", C.c_uint32),
        ("l4_mode", C.c_uint32),
        ("l4_checksum", C.c_uint32),
        ("rewrite", C.c_uint32),
        ("ttl_multicast", C.c_uint32),
        ("vlan_ethertype", C.c_uint32),
    ]


class fcgpu_anno(C.Structure):
    _fields_ = [
        ("dst_ip", C.c_uint32),
        ("length", C.c_uint16),
        ("vlan_tci", C.c_uint16),
        ("nh", C.c_uint16),
        ("th", C.c_uint16),
        ("ip6_nxt", C.c_uint8),
        ("ipver", C.c_uint8),
        ("reserved", C.c_uint16),
    ]


class fcgpu_anno8(C.Structure):
    _fields_ = [("dst_ip", C.c_uint32), ("length", C.c_uint16), ("nh", C.c_uint8), ("thl", C.c_uint8)]


class fcgpu_xmeta(C.Structure):
    _fields_ = [("off", C.c_uint32), ("length", C.c_uint32), ("src_index", C.c_uint32), ("src_rank", C.c_uint32)]


ANNO_DTYPE = None   # numpy structured dtype, set lazily (numpy import is optional here)


def anno_dtype():
    global ANNO_DTYPE
    if ANNO_DTYPE is None:
        import numpy as np
        ANNO_DTYPE = np.dtype([("dst_ip", "<u4"), ("length", "<u2"), ("vlan_tci", "<u2"),
                               ("nh", "<u2"), ("th", "<u2"), ("ip6_nxt", "u1"), ("ipver", "u1"),
                               ("reserved", "<u2")])
        assert ANNO_DTYPE.itemsize == C.sizeof(fcgpu_anno) == 16
    return ANNO_DTYPE


FLOW_NONE = 0xFFFFFFFF
FLOW_FULL = 0xFFFFFFFE
FLOW_MAX_BATCH = 64 * ((1 << 14) + 64)   # FCGPU_FLOW_MAX_BATCH
MAX_FLOWS = 1 << 23
FLOW_MGR_HMP = 0
FLOW_MGR_IMP = 1


class fcgpu_flow_config(C.Structure):
    _fields_ = [("manager", C.c_uint32), ("capacity", C.c_uint32), ("timeout_s", C.c_uint32),
                ("recycle_ms", C.c_uint32)]


class fcgpu_flow_stat(C.Structure):
    _fields_ = [(k, C.c_uint32) for k in ("manager", "capacity", "count", "free_ids", "pending", "epochs")]


class fcgpu_out(C.Structure):
    _fields_ = [
        ("verdict", C.c_void_p),
        ("hash", C.c_void_p),
        ("anno", C.c_void_p),
        ("perm", C.c_void_p),
        ("port_start", C.c_void_p),
        ("tile_count", C.c_void_p),
        ("partition", C.c_uint32),
        ("reserved", C.c_uint32),
        ("tile_perm", C.c_void_p),
        ("flowid", C.c_void_p),
        ("ip_rw", C.c_void_p),
    ]


class fcgpu_job(C.Structure):
    _fields_ = [
        ("arena", C.c_void_p),
        ("desc", C.c_void_p),
        ("n", C.c_uint32),
        ("reserved", C.c_uint32),
        ("stream", C.c_void_p),
        ("out", fcgpu_out),
    ]


class fcgpu_block_layout(C.Structure):
    _fields_ = [(k, C.c_size_t) for k in ("verdict", "hash", "anno", "perm", "port_start", "tile_count",
                                          "tile_perm", "flowid", "ip_rw", "bytes")]


class fcgpu_mbuf_layout(C.Structure):
    _fields_ = [("buf_addr", C.c_uint32), ("data_off", C.c_uint32), ("data_len", C.c_uint32),
                ("header_bytes", C.c_uint32)]


MBUF_LAYOUT_DPDK = (0, 16, 40, 64)      # FCGPU_MBUF_LAYOUT_DPDK (rte_mbuf, DPDK >= 20.11)


class fcgpu_step(C.Structure):
    _fields_ = [
        ("offset", C.c_int32),
        ("value", C.c_uint32),
        ("mask", C.c_uint32),
        ("yes", C.c_int32),
        ("no", C.c_int32),
        ("flags", C.c_uint32),
    ]


# Every symbol include/fastclick_gpu.h declares (checked by tests/test_abi.py).
FCGPU_SYMBOLS = {
    "fcgpu_abi_version": (C.c_int, []),
    "fcgpu_device_count": (C.c_int, []),
    "fcgpu_default_cfg": (None, [C.POINTER(fcgpu_cfg)]),
    "fcgpu_open": (C.c_int, [C.c_int, C.c_uint32, C.POINTER(C.c_void_p)]),
    "fcgpu_configure": (C.c_int, [C.c_void_p, C.POINTER(fcgpu_cfg)]),
    "fcgpu_close": (None, [C.c_void_p]),
    "fcgpu_process": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                C.POINTER(fcgpu_out), C.c_void_p]),
    "fcgpu_process_jobs": (C.c_int, [C.c_void_p, C.POINTER(fcgpu_job), C.c_uint32, C.c_void_p]),
    "fcgpu_process_host": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_void_p, C.c_uint32,
                                     C.POINTER(fcgpu_out)]),
    "fcgpu_set_program": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(fcgpu_step), C.c_uint32,
                                    C.c_int32]),
    "fcgpu_set_lb_table": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    "fcgpu_lb_hash_ring": (C.c_int, [C.c_uint32, C.c_uint32, C.c_void_p]),
    "fcgpu_set_host_threads": (C.c_int, [C.c_void_p, C.c_uint32]),
    "fcgpu_span_submit": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t, C.c_void_p, C.c_uint32,
                                    C.POINTER(fcgpu_out)]),
    "fcgpu_span_wait": (C.c_int, [C.c_void_p, C.c_uint32]),
    "fcgpu_span_poll": (C.c_int, [C.c_void_p, C.c_uint32]),
    "fcgpu_span_mode": (C.c_int, [C.c_void_p, C.c_uint32]),
    "fcgpu_span_reserve": (C.c_int, [C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint32]),
    "fcgpu_span_zerocopy_active": (C.c_int, [C.c_void_p]),
    "fcgpu_inject_fault": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32]),
    "fcgpu_launch_guard_selftest": (C.c_int, []),
    "fcgpu_block_layout_for": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]),
    "fcgpu_span_submit_block": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t,
                                          C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32]),
    "fcgpu_flow_enable": (C.c_int, [C.c_void_p, C.c_uint32]),
    "fcgpu_flow_reset": (C.c_int, [C.c_void_p]),
    "fcgpu_flow_count": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32)]),
    "fcgpu_flow_configure": (C.c_int, [C.c_void_p, C.POINTER(fcgpu_flow_config)]),
    "fcgpu_program_jit": (C.c_int, [C.c_void_p, C.c_int]),
    "fcgpu_program_jit_active": (C.c_int, [C.c_void_p]),
    "fcgpu_flow_set_time": (C.c_int, [C.c_void_p, C.c_uint32]),
    "fcgpu_flow_maintain": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "fcgpu_flow_stats": (C.c_int, [C.c_void_p, C.POINTER(fcgpu_flow_stat)]),
    "fcgpu_host_alloc": (C.c_void_p, [C.c_size_t]),
    "fcgpu_host_free": (None, [C.c_void_p]),
    "fcgpu_pool_register": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "fcgpu_process_mbufs": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(fcgpu_mbuf_layout),
                                      C.POINTER(fcgpu_out), C.c_void_p]),
    "fcgpu_host_register": (C.c_int, [C.c_void_p, C.c_size_t, C.c_int]),
    "fcgpu_host_unregister": (C.c_int, [C.c_void_p]),
    "fcgpu_read_counters": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]),
    "fcgpu_counters_derive": (None, [C.c_void_p]),
    "fcgpu_reset_counters": (C.c_int, [C.c_void_p]),
    "fcgpu_counters_device": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "fcgpu_use_counters": (C.c_int, [C.c_void_p, C.c_void_p]),
    "fcgpu_set_timing": (C.c_int, [C.c_void_p, C.c_int]),
    "fcgpu_read_timing": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_uint32),
                                    C.c_int]),
    "fcgpu_exchange_plan": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                      C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]),
    "fcgpu_exchange_pack": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p]),
    "fcgpu_exchange_unpack": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64), C.c_uint32,
                                        C.c_void_p, C.c_void_p]),
    "fcgpu_exchange_build": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                       C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                       C.c_void_p]),
    "fcgpu_exchange_build_fixed": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                             C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, C.c_void_p,
                                             C.c_void_p, C.c_void_p]),
    "fcgpu_exchange_unpack_fixed": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64,
                                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                              C.c_void_p]),
    "fcgpu_process_counted": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                        C.POINTER(fcgpu_out), C.c_void_p]),
    "fcgpu_last_error": (C.c_char_p, [C.c_void_p]),
}

_lib = None


class NativeMissing(RuntimeError):
    pass


def load(path: str = LIBFCGPU):
    """Load libfcgpu.so (after torch, so one HIP runtime serves both)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NativeMissing(
            f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    try:
        import torch  # noqa: F401  (share torch's HIP runtime: same soname)
    except Exception:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in FCGPU_SYMBOLS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.fcgpu_abi_version() != ABI_VERSION:
        raise NativeMissing("libfcgpu.so ABI version mismatch")
    _lib = lib
    return lib


def lb_hash_ring(nsel: int, size: int | None = None):
    """The constant_hash_agg ring (fcgpu_lb_hash_ring: LoadBalancer::
    build_hash_ring over [0, nsel), size CST_BUCKETS or 100 per output) as a
    uint8 array, the table Context.set_lb_table takes. Host-only."""
    import numpy as np
    size = 100 * nsel if size is None else size
    out = np.zeros(size, np.uint8)
    rc = load().fcgpu_lb_hash_ring(nsel, size, out.ctypes.data)
    if rc != OK:
        raise ValueError(f"fcgpu_lb_hash_ring({nsel}, {size}) failed ({rc})")
    return out


def default_cfg() -> fcgpu_cfg:
    cfg = fcgpu_cfg()
    lib = _lib
    if lib is not None:
        lib.fcgpu_default_cfg(C.byref(cfg))
    else:
        # same values as fcgpu_default_cfg (fcgpu_context.hip)
        cfg.size = C.sizeof(fcgpu_cfg)
        cfg.check_mode = CHECK_IP4
        cfg.hash_mode = HASH_FLOWID
        cfg.classify = CLS_NONE
        cfg.nports = 1
        cfg.hs_length = 1
        cfg.nbad6 = 1
        cfg.l4_checksum = 1
        for j in range(16):
            cfg.bad6[0][j] = 0xFF
    return cfg


def make_cfg(*, check_mode=CHECK_IP4, offset=0, checksum=False, hash_mode=HASH_FLOWID,
             classify=CLS_NONE, nports=1, hs_offset=0, hs_length=1, native_vlan=0,
             badsrc=(), gooddst=(), bad6=None, process_eh=False, l4_mode=L4_NONE,
             l4_checksum=True, rewrite=0, ttl_multicast=True, vlan_ethertype=0) -> fcgpu_cfg:
    """Build an fcgpu_cfg. Addresses are raw network-order words (bytes a.b.c.d
    -> little-endian u32 of those bytes), as IPAddress stores them."""
    cfg = default_cfg()
    cfg.check_mode = check_mode
    cfg.offset = offset
    cfg.checksum = 1 if checksum else 0
    cfg.hash_mode = hash_mode
    cfg.classify = classify
    cfg.nports = nports
    cfg.hs_offset = hs_offset
    cfg.hs_length = hs_length
    cfg.native_vlan = native_vlan
    cfg.nbadsrc = len(badsrc)
    for j, a in enumerate(badsrc):
        cfg.badsrc[j] = a
    cfg.ngooddst = len(gooddst)
    for j, a in enumerate(gooddst):
        cfg.gooddst[j] = a
    cfg.process_eh = 1 if process_eh else 0
    cfg.l4_mode = l4_mode
    cfg.l4_checksum = 1 if l4_checksum else 0
    cfg.rewrite = rewrite
    cfg.ttl_multicast = 1 if ttl_multicast else 0
    cfg.vlan_ethertype = vlan_ethertype
    if bad6 is not None:
        cfg.nbad6 = len(bad6)
        for j, a in enumerate(bad6):
            for k in range(16):
                cfg.bad6[j][k] = a[k]
    return cfg


def derive_counters(vec):
    """fcgpu_counters_derive on a summed counter vector (numpy / list of
    NCOUNTERS): drops = checker reason slots, count = all packets - drops."""
    import numpy as np
    v = np.array(vec, dtype=np.uint64).copy()
    drops = int(v[CTR_REASON:CTR_REASON + reason_slot(R_NO_MATCH)].sum())
    total = int(v[CTR_PORT:CTR_PORT + MAX_PORTS + 1].sum())
    v[CTR_DROPS] = drops
    v[CTR_COUNT] = total - drops
    return v


def raw_addr(dotted: str) -> int:
    """'a.b.c.d' -> raw s_addr word as read little-endian from packet bytes."""
    b = bytes(int(x) for x in dotted.split("."))
    return int.from_bytes(b, "little")


class Context:
    """Owning wrapper over an fcgpu_ctx (one per thread x stream)."""

    def __init__(self, device: int = 0, max_batch: int = 1 << 20, cfg: fcgpu_cfg | None = None):
        self.lib = load()
        h = C.c_void_p()
        rc = self.lib.fcgpu_open(device, max_batch, C.byref(h))
        if rc != OK:
            raise RuntimeError(f"fcgpu_open failed ({rc}): {self.lib.fcgpu_last_error(None).decode()}")
        self.h = h
        self.max_batch = max_batch
        self.cfg = None
        if cfg is not None:
            self.configure(cfg)

    def _chk(self, rc, what):
        if rc != OK:
            raise RuntimeError(f"{what} failed ({rc}): {self.lib.fcgpu_last_error(self.h).decode()}")

    def configure(self, cfg: fcgpu_cfg):
        self._chk(self.lib.fcgpu_configure(self.h, C.byref(cfg)), "fcgpu_configure")
        self.cfg = cfg

    def process(self, arena_ptr, desc_ptr, n, *, verdict=0, hash=0, anno=0, perm=0,
                port_start=0, tile_count=0, partition=PART_GLOBAL, tile_perm=0, flowid=0, ip_rw=0,
                stream=0):
        out = fcgpu_out(verdict or None, hash or None, anno or None, perm or None,
                        port_start or None, tile_count or None, partition, 0, tile_perm or None,
                        flowid or None, ip_rw or None)
        self._chk(self.lib.fcgpu_process(self.h, arena_ptr, desc_ptr, n, C.byref(out),
                                         stream or None), "fcgpu_process")

    def process_counted(self, arena_ptr, desc_ptr, n_max, count_ptr, base=0, *, verdict=0, hash=0, anno=0,
                        perm=0, port_start=0, tile_count=0, partition=PART_TILE, tile_perm=0, flowid=0, ip_rw=0,
                        stream=0):
        """fcgpu_process_counted: the first *count_ptr - base packets (a device word) of
        at most n_max; the launch covers n_max, nothing is read back to the host."""
        out = fcgpu_out(verdict or None, hash or None, anno or None, perm or None, port_start or None,
                        tile_count or None,
                        partition, 0, tile_perm or None, flowid or None, ip_rw or None)
        self._chk(self.lib.fcgpu_process_counted(self.h, arena_ptr, desc_ptr, n_max, count_ptr, base,
                                                 C.byref(out), stream or None), "fcgpu_process_counted")

    def jobs(self, specs):
        """Prepare an fcgpu_job array from (arena_ptr, desc_ptr, n, stream, outputs-dict)
        tuples; run it with run_jobs (no per-job Python work on the launch path)."""
        arr = (fcgpu_job * max(len(specs), 1))()
        for k, (arena, desc, n, stream, o) in enumerate(specs):
            arr[k].arena = arena
            arr[k].desc = desc
            arr[k].n = n
            arr[k].stream = stream or None
            arr[k].out = fcgpu_out(o.get("verdict") or None, o.get("hash") or None, o.get("anno") or None,
                                   o.get("perm") or None, o.get("port_start") or None,
                                   o.get("tile_count") or None, o.get("partition", PART_GLOBAL), 0,
                                   o.get("tile_perm") or None, o.get("flowid") or None, o.get("ip_rw") or None)
        return arr, len(specs)

    def run_jobs(self, prepared, stream=0):
        arr, n = prepared
        self._chk(self.lib.fcgpu_process_jobs(self.h, arr, n, stream or None), "fcgpu_process_jobs")

    def pool_register(self, base: int, nbytes: int):
        """Register a packet-buffer pool (mbuf headers + data rooms) for fcgpu_process_mbufs."""
        self._chk(self.lib.fcgpu_pool_register(self.h, base, nbytes), "fcgpu_pool_register")

    def process_mbufs(self, ptrs_addr: int, n: int, layout=MBUF_LAYOUT_DPDK, stream=0, **outs):
        """ptrs_addr: host array of n mbuf pointers (uint64) inside the registered pool."""
        lay = fcgpu_mbuf_layout(*layout)
        o = fcgpu_out(outs.get("verdict") or None, outs.get("hash") or None, outs.get("anno") or None,
                      outs.get("perm") or None, outs.get("port_start") or None, outs.get("tile_count") or None,
                      outs.get("partition", PART_GLOBAL), 0, outs.get("tile_perm") or None,
                      outs.get("flowid") or None, outs.get("ip_rw") or None)
        self._chk(self.lib.fcgpu_process_mbufs(self.h, ptrs_addr, n, C.byref(lay), C.byref(o), stream or None),
                  "fcgpu_process_mbufs")

    def process_host(self, frames, lens_ptr, n, *, verdict=0, hash=0, anno=0, perm=0,
                     port_start=0, tile_count=0, partition=PART_GLOBAL, tile_perm=0, flowid=0, ip_rw=0):
        out = fcgpu_out(verdict or None, hash or None, anno or None, perm or None,
                        port_start or None, tile_count or None, partition, 0, tile_perm or None,
                        flowid or None, ip_rw or None)
        self._chk(self.lib.fcgpu_process_host(self.h, frames, lens_ptr, n, C.byref(out)),
                  "fcgpu_process_host")

    def span_submit(self, slot, span_ptr, span_bytes, desc_ptr, n, *, verdict=0, hash=0, anno=0, perm=0,
                    port_start=0, tile_count=0, partition=PART_GLOBAL, tile_perm=0, flowid=0, ip_rw=0):
        """Asynchronous: frames already contiguous in host memory (pinned for DMA)."""
        out = fcgpu_out(verdict or None, hash or None, anno or None, perm or None,
                        port_start or None, tile_count or None, partition, 0, tile_perm or None,
                        flowid or None, ip_rw or None)
        self._chk(self.lib.fcgpu_span_submit(self.h, slot, span_ptr, span_bytes, desc_ptr, n, C.byref(out)),
                  "fcgpu_span_submit")

    def span_wait(self, slot):
        self._chk(self.lib.fcgpu_span_wait(self.h, slot), "fcgpu_span_wait")

    def set_program(self, kind, steps, output_everything=-1):
        """steps: sequence of (offset, value, mask, yes, no, flags) or fcgpu_step."""
        arr = (fcgpu_step * max(len(steps), 1))()
        for i, st in enumerate(steps):
            arr[i] = st if isinstance(st, fcgpu_step) else fcgpu_step(*[int(x) for x in st])
        self._chk(self.lib.fcgpu_set_program(self.h, kind, arr, len(steps), output_everything),
                  "fcgpu_set_program")

    def set_lb_table(self, table):
        """The bucket -> output table of CLS_LB_TABLE (uint8 sequence)."""
        import numpy as np
        t = np.ascontiguousarray(table, dtype=np.uint8)
        self._chk(self.lib.fcgpu_set_lb_table(self.h, t.ctypes.data, len(t)), "fcgpu_set_lb_table")

    def program_jit(self, enable=True):
        """Compile the installed (and later) decision programs to code (hiprtc)."""
        self._chk(self.lib.fcgpu_program_jit(self.h, int(enable)), "fcgpu_program_jit")

    def program_jit_active(self) -> bool:
        return bool(self.lib.fcgpu_program_jit_active(self.h))

    def flow_enable(self, max_flows: int):
        """Device flow table (FlowIPManagerHMP semantics); 0 disables it."""
        self._chk(self.lib.fcgpu_flow_enable(self.h, max_flows), "fcgpu_flow_enable")

    def flow_configure(self, manager=FLOW_MGR_IMP, capacity=65536, timeout_s=0, recycle_ms=1000):
        """Flow manager: FLOW_MGR_HMP (IDs 0, 1, ...) or FLOW_MGR_IMP (free-ID
        stack, timeouts on a timer wheel); capacity 0 disables the table."""
        fc = fcgpu_flow_config(manager, capacity, timeout_s, recycle_ms)
        self._chk(self.lib.fcgpu_flow_configure(self.h, C.byref(fc)), "fcgpu_flow_configure")

    def flow_set_time(self, now_ms: int):
        self._chk(self.lib.fcgpu_flow_set_time(self.h, now_ms & 0xFFFFFFFF), "fcgpu_flow_set_time")

    def flow_maintain(self, now_ms: int, stream=None):
        self._chk(self.lib.fcgpu_flow_maintain(self.h, now_ms & 0xFFFFFFFF, stream), "fcgpu_flow_maintain")

    def flow_stats(self) -> dict:
        st = fcgpu_flow_stat()
        self._chk(self.lib.fcgpu_flow_stats(self.h, C.byref(st)), "fcgpu_flow_stats")
        return {k: getattr(st, k) for k, _ in fcgpu_flow_stat._fields_}

    def flow_reset(self):
        self._chk(self.lib.fcgpu_flow_reset(self.h), "fcgpu_flow_reset")

    def flow_count(self) -> int:
        v = C.c_uint32()
        self._chk(self.lib.fcgpu_flow_count(self.h, C.byref(v)), "fcgpu_flow_count")
        return v.value

    def set_host_threads(self, n: int):
        self._chk(self.lib.fcgpu_set_host_threads(self.h, n), "fcgpu_set_host_threads")

    def counters(self, n=NCOUNTERS):
        buf = (C.c_uint64 * n)()
        self._chk(self.lib.fcgpu_read_counters(self.h, buf, n), "fcgpu_read_counters")
        return list(buf)

    def reset_counters(self):
        self._chk(self.lib.fcgpu_reset_counters(self.h), "fcgpu_reset_counters")

    def counters_device_ptr(self) -> int:
        p = C.c_void_p()
        self._chk(self.lib.fcgpu_counters_device(self.h, C.byref(p)), "fcgpu_counters_device")
        return p.value

    def use_counters(self, dptr: int):
        self._chk(self.lib.fcgpu_use_counters(self.h, dptr or None), "fcgpu_use_counters")

    def set_timing(self, every):
        """every: bracket every k-th launch with events (True = 1, False/0 = off)."""
        self._chk(self.lib.fcgpu_set_timing(self.h, int(every)), "fcgpu_set_timing")

    def read_timing(self):
        ms = (C.c_double * 3)()
        cnt = (C.c_uint32 * 3)()
        self._chk(self.lib.fcgpu_read_timing(self.h, ms, cnt, 3), "fcgpu_read_timing")
        return list(ms), list(cnt)

    def exchange_plan(self, desc, perm, port_start, n, world, rank, meta, seg_bytes, stream=0):
        """fcgpu_exchange_plan on device pointers (flow re-shard, one record per leaving packet)."""
        self._chk(self.lib.fcgpu_exchange_plan(self.h, desc, perm, port_start, n, world, rank, meta, seg_bytes,
                                               stream or None), "fcgpu_exchange_plan")

    def exchange_pack(self, arena, port_start, meta, seg_bytes, n, world, send, send_cap, stream=0):
        """fcgpu_exchange_pack: the leaving frames into their owners' segments of send
        (after exchange_plan of the same batch on this context)."""
        self._chk(self.lib.fcgpu_exchange_pack(self.h, arena, port_start, meta, seg_bytes, n, world,
                                               send or None, send_cap, stream or None), "fcgpu_exchange_pack")

    def exchange_build(self, arena, desc, verdict, n, world, rank, meta, seg_n, seg_bytes, send, send_cap,
                       stream=0):
        """fcgpu_exchange_build on device pointers: records and send buffer from the owner pass's verdicts."""
        self._chk(self.lib.fcgpu_exchange_build(self.h, arena, desc, verdict, n, world, rank, meta, seg_n,
                                                seg_bytes, send or None, send_cap, stream or None),
                  "fcgpu_exchange_build")

    def exchange_build_fixed(self, arena, desc, verdict, n, world, rank, seg_recs, seg_bytes, meta, send,
                             stream=0):
        """fcgpu_exchange_build_fixed on device pointers: every owner's segment at its
        fixed place (header + seg_recs records; seg_bytes frame bytes)."""
        self._chk(self.lib.fcgpu_exchange_build_fixed(self.h, arena, desc, verdict, n, world, rank, seg_recs,
                                                      seg_bytes, meta, send, stream or None),
                  "fcgpu_exchange_build_fixed")

    def exchange_unpack_fixed(self, rmeta, world, seg_recs, seg_bytes, desc, count, stall, step, total=0,
                              stream=0):
        """fcgpu_exchange_unpack_fixed: received fixed segments -> descriptors, *count, *stall
        (and *total += count when total is given)."""
        self._chk(self.lib.fcgpu_exchange_unpack_fixed(self.h, rmeta, world, seg_recs, seg_bytes, desc, count,
                                                       stall, total or None, step, stream or None),
                  "fcgpu_exchange_unpack_fixed")

    def exchange_unpack(self, meta, n, src_displ, desc, stream=0):
        """fcgpu_exchange_unpack: received records -> descriptors (src_displ: per-source segment starts)."""
        arr = (C.c_uint64 * max(len(src_displ), 1))(*[int(x) for x in src_displ])
        self._chk(self.lib.fcgpu_exchange_unpack(self.h, meta, n, arr, len(src_displ), desc, stream or None),
                  "fcgpu_exchange_unpack")

    def close(self):
        if getattr(self, "h", None):
            self.lib.fcgpu_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
