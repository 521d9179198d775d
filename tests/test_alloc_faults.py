"""Allocation failures leave no partial state (FCGPU_FAULT_ALLOC,
include/fastclick_gpu.h).

Every device or pinned buffer the library makes after fcgpu_open -- scratch
made on first use, span and staging blocks, flow tables, programs -- is made
through one all-or-nothing group (fastclick_amd/csrc/fcgpu_internal.hh
alloc_group): a call whose allocation fails returns an error, and the next
call retries and gives the oracle's results. Before this, a failure part way
through a group left its first pointer set, so the next call skipped the
allocation and launched on null pointers (a GPU fault instead of an error),
and fcgpu_set_program / fcgpu_set_lb_table freed the old buffer before making
the new one (the device configuration then named freed memory).

Each case injects one failure at every allocation index of its group in
turn (fcgpu_inject_fault ALLOC, skip k, count 1) on a fresh context, checks
that the call fails, then checks the same context's next calls against the
oracle (tests/test_exchange.py, tests/test_flow.py and tests/test_program.py
hold the unfaulted parity of the same paths)."""
import ctypes as C

import numpy as np
import pytest

from fastclick_amd import _native as N
from fastclick_amd import synth

torch = pytest.importorskip("torch")


def test_alloc_fault_kind_arguments():
    lib = N.load()
    assert N.FAULT_ALLOC == 3
    assert lib.fcgpu_inject_fault(N.FAULT_ALLOC, 0, 0) == N.OK
    assert lib.fcgpu_inject_fault(N.FAULT_ALLOC + 1, 0, 1) == N.EINVAL


@pytest.fixture
def alloc_fault():
    lib = N.load()
    lib.fcgpu_inject_fault(N.FAULT_ALLOC, 0, 0)

    def arm(skip):
        assert lib.fcgpu_inject_fault(N.FAULT_ALLOC, skip, 1) == N.OK

    yield arm
    lib.fcgpu_inject_fault(N.FAULT_ALLOC, 0, 0)


def _clear():
    N.load().fcgpu_inject_fault(N.FAULT_ALLOC, 0, 0)


def _cfg(**kw):
    base = dict(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    base.update(kw)
    return N.make_cfg(**base)


def _batch(n=5000, seed=3):
    b = synth.c4(n, seed=seed)
    synth.inject_errors(b, 0.03, seed=seed + 1)
    return b


def _run(ctx, b, cfg, partition=N.PART_TILE, flowid=False):
    from fastclick_amd import device as D
    db = D.DeviceBatch.upload(b)
    outs = D.DeviceOutputs(b.n, cfg.nports, anno=False, perm=True, port_start=True, partition=partition,
                           flowid=flowid)
    D.run_device(ctx, db, outs)
    torch.cuda.synchronize()
    return outs.numpy()


def _check(got, exp, what):
    assert np.array_equal(got["verdict"], exp["verdict"]), what
    assert np.array_equal(got["hash"], exp["hash"]), what


@pytest.mark.gpu
@pytest.mark.parametrize("skip", range(4))
def test_gpu_alloc_fault_exchange_build(alloc_fault, skip):
    """fcgpu_exchange_build's scratch (4 buffers): a failure at any of them
    is an error; the retry on the same context equals the restatement."""
    from oracle import exchange as X
    from tests.test_exchange import _build_gpu, _ragged
    world, n = 4, 3000
    arena, desc = _ragged(n, 21)
    owner = np.random.default_rng(22).integers(-1, world, n)
    perm, ps = X.partition(owner, world)
    emeta, eseg = X.plan(desc, perm, ps, world, 1)
    ctx = N.Context(0, n)
    try:
        alloc_fault(skip)
        with pytest.raises(RuntimeError, match="scratch"):
            _build_gpu(ctx, arena, desc, owner, world, 1)
        _clear()
        send, meta, seg_n, seg_b = _build_gpu(ctx, arena, desc, owner, world, 1)
    finally:
        ctx.close()
    assert np.array_equal(seg_b, eseg) and np.array_equal(meta, emeta)
    assert np.array_equal(send[:int(eseg.sum())], X.pack(arena, desc, emeta, ps, eseg, world))


@pytest.mark.gpu
@pytest.mark.parametrize("skip", range(4))
def test_gpu_alloc_fault_exchange_plan(alloc_fault, skip):
    """fcgpu_exchange_plan's scratch (4 buffers), then plan + pack again."""
    from oracle import exchange as X
    from tests.test_exchange import _pack_gpu, _ragged
    world, n = 3, 3000
    arena, desc = _ragged(n, 23)
    owner = np.random.default_rng(24).integers(-1, world, n)
    perm, ps = X.partition(owner, world)
    emeta, eseg = X.plan(desc, perm, ps, world, 2)
    ctx = N.Context(0, n)
    try:
        alloc_fault(skip)
        with pytest.raises(RuntimeError, match="scratch"):
            _pack_gpu(ctx, arena, desc, perm, ps, world, 2)
        _clear()
        send, meta, seg_n, seg_b = _pack_gpu(ctx, arena, desc, perm, ps, world, 2)
    finally:
        ctx.close()
    assert np.array_equal(seg_b, eseg) and np.array_equal(meta, emeta)
    assert np.array_equal(send[:int(eseg.sum())], X.pack(arena, desc, emeta, ps, eseg, world))


@pytest.mark.gpu
@pytest.mark.parametrize("manager,timeout,skips", [(N.FLOW_MGR_HMP, 0, (0, 4, 9)),
                                                  (N.FLOW_MGR_IMP, 0, (10,)),
                                                  (N.FLOW_MGR_IMP, 2, (11, 15, 18))])
def test_gpu_alloc_fault_flow_table(oracle, alloc_fault, manager, timeout, skips):
    """A flow table whose allocation fails part way is absent, not partial:
    batches on the context run without one (no flow IDs, no fault); the next
    configure makes the whole table and its IDs equal the oracle's."""
    from tests.test_flow import oracle_flows
    cfg = _cfg()
    bs = [synth.c3(4000, nflows=500, seed=31), synth.c3(3000, nflows=500, seed=32)]
    if manager == N.FLOW_MGR_HMP:
        exp_ids, _ = oracle_flows(oracle, cfg, bs, 1 << 12)
    else:
        t = oracle.ImpFlowTable(1 << 12, timeout, 100)
        exp_ids = np.concatenate([t.batch(b, oracle.process_batch(cfg, b), 0) for b in bs])
    for skip in skips:
        ctx = N.Context(0, 4096, cfg)
        try:
            alloc_fault(skip)
            with pytest.raises(RuntimeError, match="out of memory"):
                ctx.flow_configure(manager=manager, capacity=1 << 12, timeout_s=timeout, recycle_ms=100)
            _clear()
            r = _run(ctx, bs[0], cfg)
            _check(r, oracle.process_batch(cfg, bs[0]), f"no table after skip {skip}")
            assert ctx.flow_count() == 0
            ctx.flow_configure(manager=manager, capacity=1 << 12, timeout_s=timeout, recycle_ms=100)
            ctx.flow_set_time(0)
            ids = np.concatenate([_run(ctx, b, cfg, flowid=True)["flowid"] for b in bs])
        finally:
            ctx.close()
        assert np.array_equal(ids, exp_ids), f"skip {skip}"


@pytest.mark.gpu
def test_gpu_alloc_fault_program_and_lb_table_kept(oracle, alloc_fault):
    """fcgpu_set_program / fcgpu_set_lb_table uploading a replacement that
    cannot be allocated keep the installed one: the batch after the failed
    call is classified by the previous program / table."""
    b = _batch()
    cfg = _cfg(classify=N.CLS_PROGRAM, nports=4)
    prog_a, prog_b = (N.PROG_IPFILTER, [], 1), (N.PROG_IPFILTER, [], 3)
    ctx = N.Context(0, b.n, cfg)
    try:
        ctx.set_program(*prog_a)
        alloc_fault(0)
        with pytest.raises(RuntimeError, match="fcgpu_set_program"):
            ctx.set_program(*prog_b)
        _clear()
        _check(_run(ctx, b, cfg), oracle.process_batch(cfg, b, program=prog_a), "program kept")
        ctx.set_program(*prog_b)
        _check(_run(ctx, b, cfg), oracle.process_batch(cfg, b, program=prog_b), "program replaced")
    finally:
        ctx.close()

    cfg = _cfg(classify=N.CLS_LB_TABLE, nports=8)
    ring_a = oracle.lb_hash_ring(8, 800).astype(np.uint8)
    ring_b = oracle.lb_hash_ring(5, 5000).astype(np.uint8)
    ctx = N.Context(0, b.n, cfg)
    try:
        ctx.set_lb_table(ring_a)
        alloc_fault(0)
        with pytest.raises(RuntimeError, match="fcgpu_set_lb_table"):
            ctx.set_lb_table(ring_b)
        _clear()
        _check(_run(ctx, b, cfg), oracle.process_batch(cfg, b, lb_table=ring_a), "table kept")
        ctx.set_lb_table(ring_b)
        _check(_run(ctx, b, cfg), oracle.process_batch(cfg, b, lb_table=ring_b), "table replaced")
    finally:
        ctx.close()


def _host_call(ctx, b, partition):
    frames = b.frames()
    bufs = [C.create_string_buffer(f, len(f)) for f in frames]
    ptrs = (C.c_void_p * b.n)(*[C.addressof(x) for x in bufs])
    lens = np.ascontiguousarray(b.desc[:, 1], dtype=np.uint32)
    verdict = np.zeros(b.n, np.uint16)
    hsh = np.zeros(b.n, np.uint32)
    perm = np.zeros(b.n, np.uint32)
    start = np.zeros(18, np.uint32)
    tc = np.zeros(((b.n + 255) // 256) * 17, np.uint16)
    if partition == N.PART_GLOBAL:
        ctx.process_host(ptrs, lens.ctypes.data, b.n, verdict=verdict.ctypes.data, hash=hsh.ctypes.data,
                         perm=perm.ctypes.data, port_start=start.ctypes.data)
    else:
        ctx.process_host(ptrs, lens.ctypes.data, b.n, verdict=verdict.ctypes.data, hash=hsh.ctypes.data,
                         perm=perm.ctypes.data, tile_count=tc.ctypes.data, partition=N.PART_TILE)
    return dict(verdict=verdict, hash=hsh, perm=perm)


@pytest.mark.gpu
@pytest.mark.parametrize("partition,skips", [(N.PART_GLOBAL, (0, 5, 8, 9, 10)),
                                             (N.PART_TILE, (0, 7, 15, 16, 31))])
def test_gpu_alloc_fault_host_path(oracle, alloc_fault, partition, skips):
    """fcgpu_process_host: the whole-batch path's staging (9 buffers) and
    arena (2), the pipelined path's slots (16 buffers each): every failure an
    error, the retry equal to the oracle."""
    b = _batch(6000, seed=41)
    cfg = _cfg()
    exp = oracle.process_batch(cfg, b)
    for skip in skips:
        ctx = N.Context(0, b.n, cfg)
        try:
            alloc_fault(skip)
            with pytest.raises(RuntimeError, match="out of memory"):
                _host_call(ctx, b, partition)
            _clear()
            got = _host_call(ctx, b, partition)
        finally:
            ctx.close()
        _check(got, exp, f"host path, skip {skip}")
        if partition == N.PART_GLOBAL:
            assert np.array_equal(got["perm"], exp["perm"])
        else:
            assert np.array_equal(got["perm"], exp["perm_tile"])


def _span_check(got, exp, what):
    assert np.array_equal(got["verdict"] & 0xff, exp["reason"].astype(np.uint16)), what
    ok = exp["reason"] == N.R_OK
    assert np.array_equal(got["hash"][ok], exp["hash"][ok]), what


@pytest.mark.gpu
@pytest.mark.parametrize("via,skip", [("submit_block", 0), ("submit_block", 1), ("reserve", 0), ("reserve", 1)])
def test_gpu_alloc_fault_span_blocks(oracle, alloc_fault, via, skip):
    """The element's block path in copy mode: the slot's input and result
    blocks (2), made by fcgpu_span_reserve at the element's initialize or by
    the first fcgpu_span_submit_block; the retry's result block equals the
    oracle's."""
    from tests.test_span_modes import Block, OUTS, _cfg as span_cfg
    b = _batch(3000, seed=51)
    cfg = span_cfg()
    exp = oracle.process_batch(cfg, b)
    lib = N.load()
    ctx = N.Context(0, 4096, cfg)
    blk = Block(lib, ctx.h, b, 4096)
    try:
        assert lib.fcgpu_span_mode(ctx.h, N.SPAN_COPY) == N.OK
        alloc_fault(skip)
        if via == "reserve":
            rc = lib.fcgpu_span_reserve(ctx.h, blk.in_bytes, OUTS, N.PART_TILE)
        else:
            rc = lib.fcgpu_span_submit_block(ctx.h, 0, blk.pin, blk.in_bytes, 0, blk.frames_off, b.n, blk.out,
                                             OUTS, N.PART_TILE)
        assert rc == N.ENOMEM, (rc, lib.fcgpu_last_error(ctx.h))
        _clear()
        if via == "reserve":
            assert lib.fcgpu_span_reserve(ctx.h, blk.in_bytes, OUTS, N.PART_TILE) == N.OK
        got = blk.run(ctx.h)
    finally:
        blk.free()
        ctx.close()
    _span_check(got, exp, f"{via}, skip {skip}")


@pytest.mark.gpu
@pytest.mark.parametrize("skip", [0, 9, 10])
def test_gpu_alloc_fault_span_submit(oracle, alloc_fault, skip):
    """fcgpu_span_submit in copy mode: the slot's device outputs (10 buffers)
    and its span block; the retry equals the oracle."""
    from tests.test_span_modes import Block, _cfg as span_cfg
    b = _batch(3000, seed=52)
    cfg = span_cfg()
    exp = oracle.process_batch(cfg, b)
    lib = N.load()
    ctx = N.Context(0, 4096, cfg)
    blk = Block(lib, ctx.h, b, 4096)
    verdict = np.zeros(b.n, np.uint16)
    hsh = np.zeros(b.n, np.uint32)
    tc = np.zeros(((b.n + 255) // 256) * 17, np.uint16)
    tp = np.zeros(b.n, np.uint8)

    def submit():
        ctx.span_submit(0, blk.pin + blk.frames_off, b.n * 64, blk.pin, b.n, verdict=verdict.ctypes.data,
                        hash=hsh.ctypes.data, tile_count=tc.ctypes.data, tile_perm=tp.ctypes.data,
                        partition=N.PART_TILE)
        ctx.span_wait(0)

    try:
        assert lib.fcgpu_span_mode(ctx.h, N.SPAN_COPY) == N.OK
        alloc_fault(skip)
        with pytest.raises(RuntimeError, match="out of memory"):
            submit()
        _clear()
        submit()
    finally:
        blk.free()
        ctx.close()
    _span_check(dict(verdict=verdict, hash=hsh), exp, f"span submit, skip {skip}")
    assert np.array_equal(tp, (exp["perm_tile"] % 256).astype(np.uint8))


@pytest.mark.gpu
def test_gpu_span_slot_block_then_span_submit(oracle):
    """One slot used first by the element's block path and then by
    fcgpu_span_submit: the slot's stream exists from the first, its device
    output buffers only from the second -- the second makes them (the guard
    is the buffers, not the stream) and both results equal the oracle."""
    from tests.test_span_modes import Block, _cfg as span_cfg
    b = _batch(2000, seed=53)
    cfg = span_cfg()
    exp = oracle.process_batch(cfg, b)
    lib = N.load()
    ctx = N.Context(0, 4096, cfg)
    blk = Block(lib, ctx.h, b, 4096)
    verdict = np.zeros(b.n, np.uint16)
    hsh = np.zeros(b.n, np.uint32)
    try:
        assert lib.fcgpu_span_mode(ctx.h, N.SPAN_COPY) == N.OK
        _span_check(blk.run(ctx.h), exp, "block path")
        ctx.span_submit(0, blk.pin + blk.frames_off, b.n * 64, blk.pin, b.n, verdict=verdict.ctypes.data,
                        hash=hsh.ctypes.data)
        ctx.span_wait(0)
    finally:
        blk.free()
        ctx.close()
    _span_check(dict(verdict=verdict, hash=hsh), exp, "span submit after the block path")


@pytest.mark.gpu
@pytest.mark.parametrize("skip", [0, 1])
def test_gpu_alloc_fault_pool_register(oracle, alloc_fault, skip):
    """fcgpu_pool_register's descriptor scratch (2 buffers) is made before the
    pool is pinned: a failure registers nothing (fcgpu_process_mbufs then
    refuses, no launch), the next registration works and the mbuf batch
    equals the oracle."""
    from fastclick_amd.device import DeviceOutputs
    from tests.test_mbuf import make_pool
    b = _batch(3000, seed=61)
    buf, arr, base, size, ptrs = make_pool(b.frames(), np.random.default_rng(62))
    cfg = _cfg()
    exp = oracle.process_batch(cfg, b)
    ctx = N.Context(0, b.n, cfg)
    try:
        alloc_fault(skip)
        with pytest.raises(RuntimeError, match="out of memory"):
            ctx.pool_register(base, size)
        _clear()
        outs = DeviceOutputs(b.n, 16, device="cuda:0", perm=True, partition=N.PART_TILE)
        with pytest.raises(RuntimeError, match="no pool registered"):
            ctx.process_mbufs(ptrs.ctypes.data, b.n, **outs.ptrs())
        ctx.pool_register(base, size)
        ctx.process_mbufs(ptrs.ctypes.data, b.n, **outs.ptrs())
        torch.cuda.synchronize()
        got = outs.numpy()
    finally:
        ctx.close()
    _check(got, exp, f"mbufs, skip {skip}")


@pytest.mark.gpu
def test_gpu_alloc_fault_reconfigure_keeps_config(oracle, alloc_fault):
    """fcgpu_configure to LB_MODE hash_crc makes the CRC tables before it
    touches the context's configuration: a failed allocation leaves the
    previous configuration in force (no launch with a null table), the next
    configure switches."""
    b = _batch(4000, seed=71)
    cfg_a, cfg_b = _cfg(), _cfg(classify=N.CLS_LB_CRC)
    ctx = N.Context(0, b.n, cfg_a)
    try:
        alloc_fault(0)
        with pytest.raises(RuntimeError, match="CRC table"):
            ctx.configure(cfg_b)
        _clear()
        _check(_run(ctx, b, cfg_a), oracle.process_batch(cfg_a, b), "previous configuration kept")
        ctx.configure(cfg_b)
        _check(_run(ctx, b, cfg_b), oracle.process_batch(cfg_b, b), "hash_crc after the retry")
    finally:
        ctx.close()
