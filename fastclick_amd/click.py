"""ctypes binding of the Click-shaped host harness (include/fcclick.h).

    run_element("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16)", batch,
                burst=32, nsinks=17)

pushes the batch through the element in BURST-packet PacketBatches and returns,
per input packet, the output it left on, its departure order and its
annotations -- the observable behaviour a Click graph sees.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _native as N

_lib = None


class fcclick_result(C.Structure):
    _fields_ = [("out_port", C.c_void_p), ("out_seq", C.c_void_p), ("out_agg", C.c_void_p),
                ("out_dst", C.c_void_p), ("out_len", C.c_void_p), ("out_nh", C.c_void_p),
                ("out_batches", C.c_void_p), ("handlers", C.c_char_p), ("handlers_cap", C.c_size_t),
                ("out_paint", C.c_void_p), ("out_flow", C.c_void_p), ("out_ip8", C.c_void_p),
                ("out_parked", C.c_void_p), ("out_batch", C.c_void_p)]


def load():
    global _lib
    if _lib is not None:
        return _lib
    N.load()   # libfcgpu.so first (same HIP runtime as torch), then the harness
    path = os.environ.get("FCCLICK_LIB", N.LIBFCCLICK)   # FCCLICK_LIB: an A/B build of the harness
    if not os.path.exists(path):
        raise N.NativeMissing(f"{path} not built (run __graft_entry__.build())")
    lib = C.CDLL(path)
    lib.fcclick_check_config.restype = C.c_int
    lib.fcclick_check_config.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t]
    lib.fcclick_element_cfg.restype = C.c_int
    lib.fcclick_element_cfg.argtypes = [C.c_char_p, C.POINTER(N.fcgpu_cfg), C.c_char_p, C.c_size_t]
    lib.fcclick_parse_program.restype = C.c_int
    lib.fcclick_parse_program.argtypes = [C.c_char_p, C.POINTER(N.fcgpu_step), C.c_uint32,
                                          C.POINTER(C.c_uint32), C.POINTER(C.c_int32), C.c_char_p,
                                          C.c_size_t]
    lib.fcclick_run.restype = C.c_int
    lib.fcclick_run.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                C.POINTER(fcclick_result), C.c_char_p, C.c_size_t]
    lib.fcclick_run_ex.restype = C.c_int
    lib.fcclick_run_ex.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                   C.c_uint32, C.POINTER(fcclick_result), C.c_char_p, C.c_size_t]
    lib.fcclick_run_clocked.restype = C.c_int
    lib.fcclick_run_clocked.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                        C.c_void_p, C.POINTER(fcclick_result), C.c_char_p, C.c_size_t]
    if hasattr(lib, "fcclick_stage_compact"):      # absent from older A/B builds of the harness
        lib.fcclick_stage_compact.restype = C.c_int
        lib.fcclick_stage_compact.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                              C.c_size_t, C.c_void_p, C.POINTER(C.c_size_t), C.c_char_p, C.c_size_t]
    lib.fcclick_bench.restype = C.c_int
    lib.fcclick_bench.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                  C.POINTER(C.c_double), C.c_char_p, C.c_size_t]
    lib.fcclick_bench_threads.restype = C.c_int
    lib.fcclick_bench_threads.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                          C.c_uint32, C.c_uint32, C.POINTER(C.c_double), C.c_char_p, C.c_size_t]
    if hasattr(lib, "fcclick_bench_timed"):        # absent from older A/B builds of the harness
        lib.fcclick_bench_timed.restype = C.c_int
        lib.fcclick_bench_timed.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                            C.c_double, C.c_uint32, C.POINTER(C.c_double), C.c_char_p, C.c_size_t]
    _lib = lib
    return lib


class ConfigError(ValueError):
    pass


def check_config(conf: str):
    lib = load()
    err = C.create_string_buffer(512)
    if lib.fcclick_check_config(conf.encode(), err, 512) != 0:
        raise ConfigError(err.value.decode())


def element_cfg(conf: str):
    """The fcgpu_cfg a GPUIPCheckClassify configuration string produces (no GPU)."""
    lib = load()
    cfg = N.fcgpu_cfg()
    err = C.create_string_buffer(512)
    if lib.fcclick_element_cfg(conf.encode(), C.byref(cfg), err, 512) != 0:
        raise ConfigError(err.value.decode())
    return cfg


def parse_program(text: str):
    """Reference `program` handler text -> (steps: list[fcgpu_step], output_everything)."""
    lib = load()
    cap = N.MAX_STEPS
    steps = (N.fcgpu_step * cap)()
    n = C.c_uint32()
    oe = C.c_int32()
    err = C.create_string_buffer(512)
    if lib.fcclick_parse_program(text.encode(), steps, cap, C.byref(n), C.byref(oe), err, 512) != 0:
        raise ConfigError(err.value.decode())
    return [steps[i] for i in range(n.value)], oe.value


def stage_compact(conf: str, batch, fill=None):
    """The element's compact staging of `batch` (include/fcclick.h
    fcclick_stage_compact) as a Batch: frame byte b of packet i at
    arena[desc[i, 0] + b] for every byte the chain reads; the rest of the
    arena is `fill` (default zeros), e.g. random bytes to make sure nothing
    outside the staged range decides anything. None when the chain stages
    whole captures."""
    from . import synth
    lib = load()
    n = batch.n
    cap = 256 + 128 * n + synth.ARENA_PAD
    out = np.zeros(cap, np.uint8) if fill is None else np.ascontiguousarray(fill[:cap], dtype=np.uint8).copy()
    desc = np.zeros((n, 2), np.uint32)
    used = C.c_size_t()
    err = C.create_string_buffer(512)
    arena = np.ascontiguousarray(batch.arena)
    src = np.ascontiguousarray(batch.desc, dtype=np.uint32)
    rc = lib.fcclick_stage_compact(conf.encode(), arena.ctypes.data, src.ctypes.data, n, out.ctypes.data, cap,
                                   desc.ctypes.data, C.byref(used), err, 512)
    if rc == -2:
        return None
    if rc != 0:
        raise ConfigError(err.value.decode())
    return synth.Batch(arena=out, desc=desc)


PER_PACKET = 0xFFFFFFFF   # burst value: the source calls push(0, p) per packet (fcclick.h)
TIMER_FLUSH = 1           # fcclick_run_ex flag: end with the element's timer, not flush()


def run_element(conf: str, batch, *, burst: int = 32, nsinks: int = 1, timer_flush: bool = False,
                burst_ns=None, allow_error: bool = False):
    """Source(batch, BURST) -> conf => sinks. burst_ns: the element's clock (ns)
    at each burst (fcclick_run_clocked), for time-driven behaviour.
    allow_error: a run whose element reported a GPU runtime error (packets a
    failed batch cost) returns its results with the message in out["error"]
    instead of raising."""
    lib = load()
    n = batch.n
    arena = np.ascontiguousarray(batch.arena)
    desc = np.ascontiguousarray(batch.desc, dtype=np.uint32)
    out = {k: np.zeros(n, dt) for k, dt in (("port", np.uint32), ("seq", np.uint32), ("agg", np.uint32),
                                            ("dst", np.uint32), ("len", np.uint32), ("nh", np.int32),
                                            ("paint", np.uint8), ("flow", np.uint32), ("ip8", np.uint32),
                                            ("batch", np.uint32))}
    nb = np.zeros(1, np.uint32)
    parked = np.zeros(1, np.uint32)
    hbuf = C.create_string_buffer(4096)
    res = fcclick_result(out["port"].ctypes.data, out["seq"].ctypes.data, out["agg"].ctypes.data,
                         out["dst"].ctypes.data, out["len"].ctypes.data, out["nh"].ctypes.data,
                         nb.ctypes.data, C.cast(hbuf, C.c_char_p), 4096, out["paint"].ctypes.data,
                         out["flow"].ctypes.data, out["ip8"].ctypes.data, parked.ctypes.data,
                         out["batch"].ctypes.data)
    err = C.create_string_buffer(512)
    if burst_ns is not None:
        clock = np.ascontiguousarray(burst_ns, dtype=np.uint64)
        assert len(clock) >= -(-n // burst) and not timer_flush
        rc = lib.fcclick_run_clocked(conf.encode(), arena.ctypes.data, desc.ctypes.data, n, burst, nsinks,
                                     clock.ctypes.data, C.byref(res), err, 512)
    else:
        rc = lib.fcclick_run_ex(conf.encode(), arena.ctypes.data, desc.ctypes.data, n, burst, nsinks,
                                TIMER_FLUSH if timer_flush else 0, C.byref(res), err, 512)
    if rc == -1:
        raise ConfigError(err.value.decode())
    if rc != 0 and not allow_error:
        raise RuntimeError(f"element runtime error: {err.value.decode()}")
    out["error"] = err.value.decode() if rc != 0 else ""
    handlers = {}
    name = None
    for line in hbuf.value.decode().splitlines():
        if "=" in line and line.split("=", 1)[0] in ("count", "drops", "drop_details", "port_counts",
                                                                "flow_count", "flow_drops", "gpu_errors",
                                                                "gpu_retries", "error"):
            name, val = line.split("=", 1)
            handlers[name] = val
        elif name is not None:
            handlers[name] += "\n" + line
    out["batches"] = int(nb[0])
    out["parked"] = int(parked[0])
    out["handlers"] = handlers
    return out


def bench_element(conf: str, batch, *, burst: int = 32, reps: int = 5, threads: int = 1,
                  seconds: float | None = None) -> float:
    """Packets/s through the element (threads > 1: that many instances, one
    per thread, each with its own GPU context, their timed loops started
    together after every set-up; all packets over the union of the windows).
    seconds: push for that long instead of `reps` passes (fcclick_bench_timed)."""
    lib = load()
    arena = np.ascontiguousarray(batch.arena)
    desc = np.ascontiguousarray(batch.desc, dtype=np.uint32)
    pps = C.c_double()
    err = C.create_string_buffer(512)
    if seconds is not None:
        rc = lib.fcclick_bench_timed(conf.encode(), arena.ctypes.data, desc.ctypes.data, batch.n, burst,
                                     float(seconds), threads, C.byref(pps), err, 512)
    else:
        rc = lib.fcclick_bench_threads(conf.encode(), arena.ctypes.data, desc.ctypes.data, batch.n, burst, reps,
                                       threads, C.byref(pps), err, 512)
    if rc != 0:
        raise RuntimeError(err.value.decode())
    return pps.value
