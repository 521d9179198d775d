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


class fcclick_event(C.Structure):
    _fields_ = [("t_ns", C.c_uint64), ("kind", C.c_uint32), ("count", C.c_uint32)]


EV_BURST, EV_READ = 0, 1
HANDLERS = ("count", "drops", "drop_details", "port_counts", "flow_count", "flow_count_fids", "flow_drops",
            "gpu_errors", "gpu_retries", "error")


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
    if hasattr(lib, "fcclick_run_events"):         # absent from older A/B builds of the harness
        lib.fcclick_run_events.restype = C.c_int
        lib.fcclick_run_events.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                           C.POINTER(fcclick_event), C.c_uint32, C.POINTER(fcclick_result),
                                           C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
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
    if hasattr(lib, "fcclick_run_threads"):        # absent from older A/B builds of the harness
        lib.fcclick_run_threads.restype = C.c_int
        lib.fcclick_run_threads.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                            C.c_uint32, C.c_uint32, C.c_void_p, C.c_char_p, C.c_size_t, C.c_char_p,
                                            C.c_size_t]
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
    # a record holds at most max(frame, OFFSET + 60-B header + 16-B L4 tail)
    # bytes plus its 16-B packing slack (capture.hh stage_record_size): room
    # for every frame whatever the chain (OFFSET < 300 here)
    lens = np.asarray(batch.desc[:, 1], dtype=np.int64) if n else np.zeros(0, np.int64)
    cap = 256 + int((np.maximum(lens, 384) + 32).sum()) + synth.ARENA_PAD
    out = np.zeros(cap, np.uint8)
    if fill is not None:
        f = np.asarray(fill, dtype=np.uint8).ravel()[:cap]
        out[:len(f)] = f
    desc = np.zeros((n, 2), np.uint32)
    used = C.c_size_t()
    err = C.create_string_buffer(512)
    arena = np.ascontiguousarray(batch.arena)
    src = np.ascontiguousarray(batch.desc, dtype=np.uint32)
    rc = lib.fcclick_stage_compact(conf.encode(), arena.ctypes.data, src.ctypes.data, n, out.ctypes.data, out.size,
                                   desc.ctypes.data, C.byref(used), err, 512)
    if rc == -2:
        return None
    if rc != 0:
        raise ConfigError(err.value.decode())
    return synth.Batch(arena=out, desc=desc)


PER_PACKET = 0xFFFFFFFF   # burst value: the source calls push(0, p) per packet (fcclick.h)
TIMER_FLUSH = 1           # fcclick_run_ex flag: end with the element's timer, not flush()


def parse_handlers(text: str) -> dict:
    """"name=value" lines (a value may span lines) -> {name: value}."""
    handlers = {}
    name = None
    for line in text.splitlines():
        if "=" in line and line.split("=", 1)[0] in HANDLERS:
            name, val = line.split("=", 1)
            handlers[name] = val
        elif name is not None:
            handlers[name] += "\n" + line
    return handlers


class _Run:
    """The per-packet result arrays one harness run fills (fcclick_result)."""

    def __init__(self, batch):
        n = batch.n
        self.n = n
        self.arena = np.ascontiguousarray(batch.arena)
        self.desc = np.ascontiguousarray(batch.desc, dtype=np.uint32)
        self.out = {k: np.zeros(n, dt) for k, dt in (("port", np.uint32), ("seq", np.uint32), ("agg", np.uint32),
                                                     ("dst", np.uint32), ("len", np.uint32), ("nh", np.int32),
                                                     ("paint", np.uint8), ("flow", np.uint32),
                                                     ("ip8", np.uint32), ("batch", np.uint32))}
        self.nb = np.zeros(1, np.uint32)
        self.parked = np.zeros(1, np.uint32)
        self.hbuf = C.create_string_buffer(4096)
        o = self.out
        self.res = fcclick_result(o["port"].ctypes.data, o["seq"].ctypes.data, o["agg"].ctypes.data,
                                  o["dst"].ctypes.data, o["len"].ctypes.data, o["nh"].ctypes.data,
                                  self.nb.ctypes.data, C.cast(self.hbuf, C.c_char_p), 4096,
                                  o["paint"].ctypes.data, o["flow"].ctypes.data, o["ip8"].ctypes.data,
                                  self.parked.ctypes.data, o["batch"].ctypes.data)
        self.err = C.create_string_buffer(512)

    def finish(self, rc: int, allow_error: bool) -> dict:
        if rc == -1:
            raise ConfigError(self.err.value.decode())
        if rc != 0 and not allow_error:
            raise RuntimeError(f"element runtime error: {self.err.value.decode()}")
        out = self.out
        out["error"] = self.err.value.decode() if rc != 0 else ""
        out["batches"] = int(self.nb[0])
        out["parked"] = int(self.parked[0])
        out["handlers"] = parse_handlers(self.hbuf.value.decode())
        return out


def run_element(conf: str, batch, *, burst: int = 32, nsinks: int = 1, timer_flush: bool = False,
                burst_ns=None, allow_error: bool = False):
    """Source(batch, BURST) -> conf => sinks. burst_ns: the element's clock (ns)
    at each burst (fcclick_run_clocked), for time-driven behaviour.
    allow_error: a run whose element reported a GPU runtime error (packets a
    failed batch cost) returns its results with the message in out["error"]
    instead of raising."""
    lib = load()
    r = _Run(batch)
    if burst_ns is not None:
        clock = np.ascontiguousarray(burst_ns, dtype=np.uint64)
        assert len(clock) >= -(-r.n // burst) and not timer_flush
        rc = lib.fcclick_run_clocked(conf.encode(), r.arena.ctypes.data, r.desc.ctypes.data, r.n, burst, nsinks,
                                     clock.ctypes.data, C.byref(r.res), r.err, 512)
    else:
        rc = lib.fcclick_run_ex(conf.encode(), r.arena.ctypes.data, r.desc.ctypes.data, r.n, burst, nsinks,
                                TIMER_FLUSH if timer_flush else 0, C.byref(r.res), r.err, 512)
    return r.finish(rc, allow_error)


def run_element_events(conf: str, batch, events, *, nsinks: int = 1, allow_error: bool = False):
    """A scripted run on a virtual clock (fcclick_run_events): `events` is a
    list of ("burst", t_ns, count) -- the next `count` packets as one
    PacketBatch at time t_ns -- and ("read", t_ns) -- the element's Timer fires
    at t_ns, then every handler is read. Returns run_element's dict plus
    out["reads"]: one {handler: value} dict per read, in order."""
    lib = load()
    r = _Run(batch)
    ev = (fcclick_event * len(events))()
    for k, e in enumerate(events):
        if e[0] == "burst":
            ev[k] = fcclick_event(int(e[1]), EV_BURST, int(e[2]))
        elif e[0] == "read":
            ev[k] = fcclick_event(int(e[1]), EV_READ, 0)
        else:
            raise ValueError(f"unknown event {e!r}")
    cap = 4096 * (1 + sum(1 for e in events if e[0] == "read"))
    rbuf = C.create_string_buffer(cap)
    rc = lib.fcclick_run_events(conf.encode(), r.arena.ctypes.data, r.desc.ctypes.data, r.n, nsinks, ev,
                                len(events), C.byref(r.res), rbuf, cap, r.err, 512)
    out = r.finish(rc, allow_error)
    out["reads"] = [parse_handlers(block) for block in rbuf.value.decode().split("--\n")[:-1]]
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


def run_element_threads(conf: str, batch, *, threads: int, reps: int = 1, burst: int = 32, nsinks: int = 1):
    """`threads` element instances (one GPU context each) set up, then each
    pushing `batch` `reps` times and flushing, all at once
    (fcclick_run_threads). Returns (port_pkts [threads, nsinks]: the packets
    each thread's outputs received, [one handler dict per thread])."""
    lib = load()
    arena = np.ascontiguousarray(batch.arena)
    desc = np.ascontiguousarray(batch.desc, dtype=np.uint32)
    pk = np.zeros((threads, nsinks), np.uint64)
    cap = 4096 * threads
    hbuf = C.create_string_buffer(cap)
    err = C.create_string_buffer(512)
    rc = lib.fcclick_run_threads(conf.encode(), arena.ctypes.data, desc.ctypes.data, batch.n, burst, reps, threads,
                                 nsinks, pk.ctypes.data, hbuf, cap, err, 512)
    if rc != 0:
        raise RuntimeError(err.value.decode())
    return pk, [parse_handlers(b) for b in hbuf.value.decode().split("--\n")[:-1]]
