"""Block submissions in every span mode (fcgpu_span_mode): COPY, ZEROCOPY and
AUTO (zero-copy while >= 4 AUTO contexts share the device) give the same
result blocks, equal to the oracle's verdicts, hashes and tile partition.

The element path (fcgpu_span_submit_block) of include/fastclick_gpu.h, driven
through ctypes with pinned blocks from fcgpu_host_alloc, as RxCore stages
them: [descriptors: cap x 8 B][64-B records] in, the fcgpu_block_layout_for
arrays out.
"""
import ctypes as C

import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N

OUTS = 0x1 | 0x2 | 0x20 | 0x40          # verdict, hash, tile_count, tile_perm


def _cfg():
    return N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16,
                      badsrc=[N.raw_addr("192.0.2.255")])


class Block:
    """A pinned input block holding batch b as 64-B records, and a result block."""

    def __init__(self, lib, ctx, b, cap, place=None):
        """place[i]: the 64-B record slot packet i is staged in (default i, as
        RxCore stages; the ABI allows any placement)."""
        self.lib = lib
        n = b.n
        self.n = n
        self.frames_off = (cap * 8 + 255) & ~255
        rec = 64
        self.in_bytes = self.frames_off + n * rec
        self.pin = lib.fcgpu_host_alloc(self.in_bytes + 65536)
        assert self.pin
        buf = np.ctypeslib.as_array(C.cast(self.pin, C.POINTER(C.c_uint8)), shape=(self.in_bytes + 65536,))
        buf[:] = 0
        desc = buf[:cap * 8].view(np.uint32).reshape(cap, 2)
        place = np.arange(n) if place is None else place
        for i in range(n):
            off, ln = int(b.desc[i, 0]), int(b.desc[i, 1])
            cp = min(ln, 64)
            r = int(place[i]) * rec
            buf[self.frames_off + r:self.frames_off + r + cp] = b.arena[off:off + cp]
            desc[i] = (r, ln)
        self.L = N.fcgpu_block_layout()
        assert lib.fcgpu_block_layout_for(ctx, n, OUTS, N.PART_TILE, C.byref(self.L)) == N.OK
        self.out = lib.fcgpu_host_alloc(self.L.bytes)
        assert self.out
        self.res = np.ctypeslib.as_array(C.cast(self.out, C.POINTER(C.c_uint8)), shape=(self.L.bytes,))

    def run(self, ctx, slot=0):
        self.res[:] = 0xEE
        rc = self.lib.fcgpu_span_submit_block(ctx, slot, self.pin, self.in_bytes, 0, self.frames_off, self.n,
                                              self.out, OUTS, N.PART_TILE)
        assert rc == N.OK, self.lib.fcgpu_last_error(ctx)
        assert self.lib.fcgpu_span_wait(ctx, slot) == N.OK
        n = self.n
        return {"verdict": self.res[self.L.verdict:self.L.verdict + 2 * n].view(np.uint16).copy(),
                "hash": self.res[self.L.hash:self.L.hash + 4 * n].view(np.uint32).copy(),
                "tile_perm": self.res[self.L.tile_perm:self.L.tile_perm + n].copy()}

    def free(self):
        self.lib.fcgpu_host_free(self.pin)
        self.lib.fcgpu_host_free(self.out)


def test_span_mode_arguments():
    """Mode values beyond AUTO are rejected without a device call."""
    lib = N.load()
    assert lib.fcgpu_span_mode(None, N.SPAN_COPY) == N.EINVAL
    assert N.SPAN_AUTO == 2


@pytest.mark.gpu
def test_gpu_span_modes_copy_zerocopy_auto(oracle):
    lib = N.load()
    b = synth.c4(5000 + 37, seed=601)
    synth.inject_errors(b, 0.03, seed=602)
    cfg = _cfg()
    exp = oracle.process_batch(cfg, b)
    cap = 8192
    ctxs = []
    for _ in range(4):
        h = C.c_void_p()
        assert lib.fcgpu_open(0, cap, C.byref(h)) == N.OK
        assert lib.fcgpu_configure(h, C.byref(cfg)) == N.OK
        ctxs.append(h)
    blk = Block(lib, ctxs[0], b, cap)
    try:
        def check(got):
            assert np.array_equal(got["verdict"] & 0xff, exp["reason"].astype(np.uint16))
            ok = exp["reason"] == N.R_OK
            assert np.array_equal(got["hash"][ok], exp["hash"][ok])
            return got
        assert lib.fcgpu_span_mode(ctxs[0], 7) == N.EINVAL
        copy = check(blk.run(ctxs[0]))                       # COPY (default)
        assert lib.fcgpu_span_mode(ctxs[0], N.SPAN_ZEROCOPY) == N.OK
        zc = check(blk.run(ctxs[0], slot=1))
        # an empty batch in zero-copy mode: no buffers needed, nothing queued
        assert lib.fcgpu_span_submit_block(ctxs[0], 0, None, 0, 0, 0, 0, None, OUTS, N.PART_TILE) == N.OK
        assert lib.fcgpu_span_wait(ctxs[0], 0) == N.OK
        for k in copy:
            assert np.array_equal(copy[k], zc[k]), k
        # AUTO: three AUTO contexts -> copies; a fourth -> zero-copy; back to three -> copies
        for h in ctxs[:3]:
            assert lib.fcgpu_span_mode(h, N.SPAN_AUTO) == N.OK
        a3 = check(blk.run(ctxs[0], slot=2))
        assert lib.fcgpu_span_mode(ctxs[3], N.SPAN_AUTO) == N.OK
        a4 = check(blk.run(ctxs[0]))
        lib.fcgpu_close(ctxs.pop())
        a3b = check(blk.run(ctxs[0], slot=1))
        for got in (a3, a4, a3b):
            for k in copy:
                assert np.array_equal(copy[k], got[k]), k
    finally:
        blk.free()
        for h in ctxs:
            lib.fcgpu_close(h)


def _pinned(lib, nbytes, dtype):
    p = lib.fcgpu_host_alloc(nbytes)
    assert p
    arr = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(nbytes,)).view(dtype)
    return p, arr


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["copy", "zerocopy"])
def test_gpu_span_submit_modes(oracle, mode):
    """fcgpu_span_submit (frames already contiguous in host memory: the pcap
    ingress, a host-resident ring) in COPY and ZEROCOPY mode: verdicts, hashes,
    annotations and the tile partition equal the oracle's; ZEROCOPY reads the
    pinned span in place and writes the pinned output arrays."""
    lib = N.load()
    b = synth.c3(20_000 + 11, seed=611)
    synth.inject_errors(b, 0.02, seed=612)
    cfg = _cfg()
    exp = oracle.process_batch(cfg, b)
    n = b.n
    ctx = N.Context(0, 32768, cfg)
    ptrs = []
    try:
        span_bytes = b.arena.size
        ps, span = _pinned(lib, span_bytes + 4096, np.uint8)
        span[:] = 0
        span[:span_bytes] = b.arena
        pd, desc = _pinned(lib, 8 * n, np.uint32)
        desc[:] = np.ascontiguousarray(b.desc, dtype=np.uint32).reshape(-1)
        pv, verdict = _pinned(lib, 2 * n, np.uint16)
        ph, hsh = _pinned(lib, 4 * n, np.uint32)
        pa, anno = _pinned(lib, 16 * n, np.uint8)
        ntiles = -(-n // 256)
        ptc, tc = _pinned(lib, 2 * 17 * ntiles, np.uint16)
        ptp, tp = _pinned(lib, n + 256, np.uint8)
        ptrs = [ps, pd, pv, ph, pa, ptc, ptp]
        want = N.SPAN_ZEROCOPY if mode == "zerocopy" else N.SPAN_COPY
        assert lib.fcgpu_span_mode(ctx.h, want) == N.OK
        for slot in range(2):
            verdict[:] = 0xEEEE
            ctx.span_submit(slot, ps, span_bytes, pd, n, verdict=pv, hash=ph, anno=pa, tile_count=ptc,
                            tile_perm=ptp, partition=N.PART_TILE)
            ctx.span_wait(slot)
            assert np.array_equal(verdict & 0xff, exp["reason"].astype(np.uint16))
            assert np.array_equal(verdict >> 8, exp["port"].astype(np.uint16))
            ok = exp["reason"] == N.R_OK
            assert np.array_equal(hsh[ok], exp["hash"][ok])
            # the tile partition: each tile's packets in output order, input order within an output
            port = exp["port"].astype(np.int64)
            for t in (0, ntiles // 2, ntiles - 1):
                lo, hi = t * 256, min(n, t * 256 + 256)
                order = lo + tp[lo:hi].astype(np.int64)
                assert np.array_equal(order, lo + np.argsort(port[lo:hi], kind="stable"))
    finally:
        for p in ptrs:
            lib.fcgpu_host_free(p)
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["reversed", "few_swapped"])
def test_gpu_zerocopy_records_out_of_order(oracle, layout):
    """Zero-copy blocks whose 64-B records fill the block end to end but are not
    in packet order (all of them, or a few swapped): the descriptors place
    every window, in both modes -- the oracle's results and the copy mode's."""
    lib = N.load()
    b = synth.c4(3000 + 5, seed=621)
    synth.inject_errors(b, 0.03, seed=622)
    cfg = _cfg()
    exp = oracle.process_batch(cfg, b)
    n = b.n
    place = np.arange(n)[::-1].copy() if layout == "reversed" else np.arange(n)
    if layout == "few_swapped":
        rng = np.random.default_rng(623)
        for a, c in rng.integers(0, n, (5, 2)):
            place[[a, c]] = place[[c, a]]
    h = C.c_void_p()
    assert lib.fcgpu_open(0, 4096, C.byref(h)) == N.OK
    assert lib.fcgpu_configure(h, C.byref(cfg)) == N.OK
    blk = Block(lib, h, b, 4096, place=place)
    try:
        copy = blk.run(h)
        assert lib.fcgpu_span_mode(h, N.SPAN_ZEROCOPY) == N.OK
        zc = blk.run(h, slot=1)
        for got in (copy, zc):
            assert np.array_equal(got["verdict"] & 0xff, exp["reason"].astype(np.uint16))
            ok = exp["reason"] == N.R_OK
            assert np.array_equal(got["hash"][ok], exp["hash"][ok])
        for k in copy:
            assert np.array_equal(copy[k], zc[k]), k
    finally:
        blk.free()
        lib.fcgpu_close(h)


@pytest.mark.gpu
def test_gpu_span_zerocopy_strided_slots(oracle):
    """A ring of 64-B slots end to end (span bytes = 64 n, nothing past the
    last frame but the pinned allocation's slack) read in place, against the
    oracle."""
    lib = N.load()
    b = synth.c4(8192 + 64, seed=631)
    synth.inject_errors(b, 0.02, seed=632)
    cfg = _cfg()
    exp = oracle.process_batch(cfg, b)
    n = b.n
    assert np.array_equal(b.desc[:, 0].astype(np.int64), 64 * np.arange(n))
    ctx = N.Context(0, 16384, cfg)
    ptrs = []
    try:
        ps, span = _pinned(lib, 64 * n + 4096, np.uint8)
        span[:] = 0
        span[:64 * n] = b.arena[:64 * n]
        pd, desc = _pinned(lib, 8 * n, np.uint32)
        desc[:] = np.ascontiguousarray(b.desc, dtype=np.uint32).reshape(-1)
        pv, verdict = _pinned(lib, 2 * n, np.uint16)
        ph, hsh = _pinned(lib, 4 * n, np.uint32)
        ptrs = [ps, pd, pv, ph]
        assert lib.fcgpu_span_mode(ctx.h, N.SPAN_ZEROCOPY) == N.OK
        ctx.span_submit(0, ps, 64 * n, pd, n, verdict=pv, hash=ph, partition=N.PART_TILE)
        ctx.span_wait(0)
        assert np.array_equal(verdict & 0xff, exp["reason"].astype(np.uint16))
        ok = exp["reason"] == N.R_OK
        assert np.array_equal(hsh[ok], exp["hash"][ok])
    finally:
        for p in ptrs:
            lib.fcgpu_host_free(p)
        ctx.close()


def _counters(lib, h):
    v = (C.c_uint64 * N.NCOUNTERS)()
    assert lib.fcgpu_read_counters(h, v, N.NCOUNTERS) == N.OK
    return list(v)


@pytest.mark.gpu
@pytest.mark.parametrize("nsub", [4, 3, 9])
def test_gpu_auto_shared_queue_fuses_contexts(oracle, nsub):
    """FCGPU_SPAN_AUTO with >= 4 contexts: zero-copy block submissions go to the
    device's shared queue and are launched together (one k_rx launch carrying
    several contexts' batches; launched by the 4th pending submission, or by a
    wait on one still pending). Every batch gets the oracle's verdicts and
    hashes, and every context's counters count its own batches only."""
    lib = N.load()
    cfg = _cfg()
    nctx = 5
    ctxs, blks, exps = [], [], []
    try:
        for k in range(nctx):
            h = C.c_void_p()
            assert lib.fcgpu_open(0, 8192, C.byref(h)) == N.OK
            assert lib.fcgpu_configure(h, C.byref(cfg)) == N.OK
            assert lib.fcgpu_span_mode(h, N.SPAN_AUTO) == N.OK
            ctxs.append(h)
        for k in range(nsub):
            b = synth.c4(1000 + 300 * k, seed=700 + k)
            synth.inject_errors(b, 0.05, seed=800 + k)
            blks.append(Block(lib, ctxs[k % nctx], b, 8192))
            exps.append(oracle.process_batch(cfg, b))
        # submit everything (slot = round of the context), then wait in reverse
        subs = []
        for k in range(nsub):
            h, slot = ctxs[k % nctx], k // nctx
            blks[k].res[:] = 0xEE
            rc = lib.fcgpu_span_submit_block(h, slot, blks[k].pin, blks[k].in_bytes, 0, blks[k].frames_off,
                                             blks[k].n, blks[k].out, OUTS, N.PART_TILE)
            assert rc == N.OK, lib.fcgpu_last_error(h)
            subs.append((h, slot))
        for k in reversed(range(nsub)):
            h, slot = subs[k]
            assert lib.fcgpu_span_wait(h, slot) == N.OK, lib.fcgpu_last_error(h)
        valid = [0] * nctx
        for k in range(nsub):
            L, n, e = blks[k].L, blks[k].n, exps[k]
            v = blks[k].res[L.verdict:L.verdict + 2 * n].view(np.uint16)
            hs = blks[k].res[L.hash:L.hash + 4 * n].view(np.uint32)
            assert np.array_equal(v & 0xff, e["reason"].astype(np.uint16)), k
            ok = e["reason"] == N.R_OK
            assert np.array_equal(hs[ok], e["hash"][ok]), k
            valid[k % nctx] += int(ok.sum())
        for k in range(nctx):
            assert _counters(lib, ctxs[k])[N.CTR_COUNT] == valid[k], k
    finally:
        for blk in blks:
            blk.free()
        for h in ctxs:
            lib.fcgpu_close(h)


@pytest.mark.gpu
def test_gpu_auto_shared_queue_threads(oracle):
    """Eight threads, each with its own AUTO context and two slots, submitting
    and waiting concurrently through the shared queue (ctypes releases the
    GIL around the calls): every batch's results are the oracle's."""
    import threading
    lib = N.load()
    cfg = _cfg()
    nthr, rounds = 8, 12
    batches = []
    for k in range(4):
        b = synth.c4(2048 + 256 * k, seed=900 + k)
        synth.inject_errors(b, 0.05, seed=950 + k)
        batches.append((b, oracle.process_batch(cfg, b)))
    errors = []

    def worker(t):
        h = C.c_void_p()
        blk = []
        try:
            assert lib.fcgpu_open(0, 8192, C.byref(h)) == N.OK
            assert lib.fcgpu_configure(h, C.byref(cfg)) == N.OK
            assert lib.fcgpu_span_mode(h, N.SPAN_AUTO) == N.OK
            blk = [Block(lib, h, batches[(t + s) % 4][0], 8192) for s in range(2)]
            barrier.wait()
            for r in range(rounds):
                s = r % 2
                if r >= 2:
                    assert lib.fcgpu_span_wait(h, s) == N.OK, lib.fcgpu_last_error(h)
                    e = batches[(t + s) % 4][1]
                    L, n = blk[s].L, blk[s].n
                    v = blk[s].res[L.verdict:L.verdict + 2 * n].view(np.uint16)
                    assert np.array_equal(v & 0xff, e["reason"].astype(np.uint16))
                    blk[s].res[:] = 0xEE
                rc = lib.fcgpu_span_submit_block(h, s, blk[s].pin, blk[s].in_bytes, 0, blk[s].frames_off, blk[s].n,
                                                 blk[s].out, OUTS, N.PART_TILE)
                assert rc == N.OK, lib.fcgpu_last_error(h)
            for s in range(2):
                assert lib.fcgpu_span_wait(h, s) == N.OK
        except Exception as ex:  # noqa: BLE001 -- reported by the main thread
            errors.append(f"thread {t}: {ex!r}")
            barrier.abort()
        finally:
            for x in blk:
                x.free()
            if h:
                lib.fcgpu_close(h)

    barrier = threading.Barrier(nthr)
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(nthr)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=60)
    assert not any(th.is_alive() for th in ths), "a thread did not finish"
    assert not errors, errors


@pytest.mark.gpu
def test_gpu_auto_shared_queue_programs_and_flows(oracle):
    """The shared queue with configurations that carry per-context device state:
    decision programs (two contexts compiled to code, two interpreted -- each
    launch only fuses contexts with one configuration) and a context with a
    flow table among them (ordered: its batches keep their own launches).
    Verdicts and output ports as the oracle says for every batch."""
    from tests.test_program import random_program
    lib = N.load()
    rng = np.random.default_rng(641)
    b = synth.c4(6000 + 13, seed=642)
    synth.inject_errors(b, 0.02, seed=643)
    nout = 7
    prog = (N.PROG_IPFILTER, random_program(rng, b, N.PROG_IPFILTER, nout, 60), -1)
    pcfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_PROGRAM, nports=nout)
    pexp = oracle.process_batch(pcfg, b, program=prog)
    fcfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=4)
    ctxs, blks = [], []
    try:
        for k in range(4):
            c = N.Context(0, 8192, pcfg)
            c.set_program(*prog)
            c.program_jit(k < 2)
            assert lib.fcgpu_span_mode(c.h, N.SPAN_AUTO) == N.OK
            ctxs.append(c)
        fc = N.Context(0, 8192, fcfg)
        assert lib.fcgpu_flow_enable(fc.h, 1 << 15) == N.OK
        assert lib.fcgpu_span_mode(fc.h, N.SPAN_AUTO) == N.OK
        ctxs.append(fc)
        for c in ctxs:
            blks.append([Block(lib, c.h, b, 8192), Block(lib, c.h, b, 8192)])
        for s in range(2):
            for c, bl in zip(ctxs, blks):
                bl[s].res[:] = 0xEE
                rc = lib.fcgpu_span_submit_block(c.h, s, bl[s].pin, bl[s].in_bytes, 0, bl[s].frames_off, bl[s].n,
                                                 bl[s].out, OUTS, N.PART_TILE)
                assert rc == N.OK, lib.fcgpu_last_error(c.h)
        for s in range(2):
            for c in ctxs:
                assert lib.fcgpu_span_wait(c.h, s) == N.OK, lib.fcgpu_last_error(c.h)
        for k, (c, bl) in enumerate(zip(ctxs, blks)):
            for s in range(2):
                L, n = bl[s].L, bl[s].n
                v = bl[s].res[L.verdict:L.verdict + 2 * n].view(np.uint16)
                if k < 4:
                    assert np.array_equal(v & 0xff, pexp["reason"].astype(np.uint16)), (k, s)
                    assert np.array_equal(v >> 8, pexp["port"].astype(np.uint16)), (k, s)
                else:
                    fexp = oracle.process_batch(fcfg, b)
                    assert np.array_equal(v & 0xff, fexp["reason"].astype(np.uint16)), (k, s)
    finally:
        for bl in blks:
            for x in bl:
                x.free()
        for c in ctxs:
            c.close()


@pytest.mark.gpu
def test_gpu_auto_shared_queue_lb_tables(oracle):
    """The shared queue with LB_MODE cst_hash_agg contexts whose rings differ
    (two with the 1,200-bucket ring of 12 outputs, one with a 333-bucket ring,
    one with a 5,000-bucket ring read from global memory): a launch fuses only
    contexts with the same table, and every context's ports are the oracle's
    with its own ring."""
    lib = N.load()
    b = synth.c4(6000 + 13, seed=652)
    synth.inject_errors(b, 0.02, seed=653)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_TABLE, nports=12)
    rings = [N.lb_hash_ring(12, 1200), N.lb_hash_ring(12, 1200), N.lb_hash_ring(12, 333),
             N.lb_hash_ring(12, 5000)]
    ctxs, blks = [], []
    try:
        for r in rings:
            c = N.Context(0, 8192, cfg)
            c.set_lb_table(r)
            assert lib.fcgpu_span_mode(c.h, N.SPAN_AUTO) == N.OK
            ctxs.append(c)
            blks.append([Block(lib, c.h, b, 8192), Block(lib, c.h, b, 8192)])
        for s in range(2):
            for c, bl in zip(ctxs, blks):
                bl[s].res[:] = 0xEE
                rc = lib.fcgpu_span_submit_block(c.h, s, bl[s].pin, bl[s].in_bytes, 0, bl[s].frames_off, bl[s].n,
                                                 bl[s].out, OUTS, N.PART_TILE)
                assert rc == N.OK, lib.fcgpu_last_error(c.h)
        for s in range(2):
            for c in ctxs:
                assert lib.fcgpu_span_wait(c.h, s) == N.OK, lib.fcgpu_last_error(c.h)
        for k, (r, bl) in enumerate(zip(rings, blks)):
            exp = oracle.process_batch(cfg, b, lb_table=r)
            for s in range(2):
                L, n = bl[s].L, bl[s].n
                v = bl[s].res[L.verdict:L.verdict + 2 * n].view(np.uint16)
                assert np.array_equal(v & 0xff, exp["reason"].astype(np.uint16)), (k, s)
                assert np.array_equal(v >> 8, exp["port"].astype(np.uint16)), (k, s)
    finally:
        for bl in blks:
            for x in bl:
                x.free()
        for c in ctxs:
            c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [N.SPAN_COPY, N.SPAN_ZEROCOPY])
def test_gpu_block_anno8_matches_anno(oracle, mode):
    """FCGPU_OUT_ANNO8 (IPv4 check modes): the 8-B annotations decode to the
    fields of the 16-B ones (dst_ip, length, nh, th) for every packet, IP
    options and header errors included; refused for other check modes."""
    lib = N.load()
    b = synth.c4(5000, seed=660)
    synth.add_ip_options(b, 0.2, seed=661)
    synth.inject_errors(b, 0.03, seed=662)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=8)
    c = N.Context(0, 8192, cfg)
    try:
        assert lib.fcgpu_span_mode(c.h, mode) == N.OK
        blk = Block(lib, c.h, b, 8192)
        got = {}
        for name, outs in (("a16", OUTS | N.OUT_ANNO), ("a8", OUTS | N.OUT_ANNO8)):
            L = N.fcgpu_block_layout()
            assert lib.fcgpu_block_layout_for(c.h, b.n, outs, N.PART_TILE, C.byref(L)) == N.OK
            out = lib.fcgpu_host_alloc(L.bytes)
            res = np.ctypeslib.as_array(C.cast(out, C.POINTER(C.c_uint8)), shape=(L.bytes,))
            res[:] = 0xEE
            rc = lib.fcgpu_span_submit_block(c.h, 0, blk.pin, blk.in_bytes, 0, blk.frames_off, b.n, out, outs,
                                             N.PART_TILE)
            assert rc == N.OK, lib.fcgpu_last_error(c.h)
            assert lib.fcgpu_span_wait(c.h, 0) == N.OK
            width = 16 if name == "a16" else 8
            got[name] = res[L.anno:L.anno + width * b.n].copy()
            got[name + "_v"] = res[L.verdict:L.verdict + 2 * b.n].view(np.uint16).copy()
            lib.fcgpu_host_free(out)
        a16 = got["a16"].view(N.anno_dtype())
        a8 = got["a8"].view(np.dtype([("dst_ip", "<u4"), ("length", "<u2"), ("nh", "u1"), ("thl", "u1")]))
        ok = (got["a16_v"] & 0xFF) == N.R_OK
        assert ok.sum() > 0.8 * b.n and np.array_equal(got["a16_v"], got["a8_v"])
        assert np.array_equal(a8["dst_ip"][ok], a16["dst_ip"][ok])
        assert np.array_equal(a8["length"][ok], a16["length"][ok])
        assert np.array_equal(a8["nh"][ok].astype(np.uint16), a16["nh"][ok])
        assert np.array_equal(a8["nh"][ok].astype(np.uint16) + a8["thl"][ok], a16["th"][ok])
        exp = oracle.process_batch(cfg, b)
        assert np.array_equal(a8["dst_ip"][ok], exp["anno"]["dst_ip"][ok])
    finally:
        c.close()
    a = N.Context(0, 8192, N.make_cfg(check_mode=N.CHECK_AUTO, offset=0, classify=N.CLS_LB_HASH, nports=4))
    try:
        blk = Block(lib, a.h, b, 8192)
        rc = lib.fcgpu_span_submit_block(a.h, 0, blk.pin, blk.in_bytes, 0, blk.frames_off, b.n, blk.out,
                                         OUTS | N.OUT_ANNO8, N.PART_TILE)
        assert rc == N.EINVAL
    finally:
        a.close()
