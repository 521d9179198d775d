"""GPU parity: the HIP path through the C ABI vs the C oracle, bit-exact.

Every case runs fastclick_amd.device.process_batch (libfcgpu.so kernels) and
oracle.process_batch (fc_oracle.c) on the same seeded batch and compares the
reason code, output port, 32-bit flow hash, annotations, stable per-port
permutation and counters. The oracle itself is pinned to the compiled
reference by tests/test_golden.py.
"""
import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N
from tests.helpers import compare, repack, set_fragment

pytestmark = pytest.mark.gpu

BADSRC = [N.raw_addr("192.0.2.255"), N.raw_addr("255.255.255.255")]
GOODDST = [N.raw_addr("10.9.9.9")]


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from fastclick_amd import device
    N.load()
    return device


def _check(dev, oracle, batch, cfg, ctx, anno=True, perm=True):
    exp = oracle.process_batch(cfg, batch)
    for part in (N.PART_GLOBAL, N.PART_TILE):
        got = dev.process_batch(batch, cfg, anno=anno, perm=perm, partition=part)
        compare(got, exp, anno=anno, perm=perm, ctx=f"{ctx} part={part}")
        assert np.array_equal(got["counters"], exp["counters"]), \
            f"{ctx}: counters {got['counters'][:12]} vs {exp['counters'][:12]}"
    return got, exp


def test_c2_cksum_hash_classify16(dev, oracle):
    b = synth.c2(70_001)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    got, _ = _check(dev, oracle, b, cfg, "C2")
    assert (got["reason"] == N.R_OK).all()


@pytest.mark.parametrize("checksum", [True, False])
def test_c4_errors(dev, oracle, checksum):
    b = synth.c4(200_000, seed=40)
    kind = synth.inject_errors(b, 0.02, seed=41)
    cfg = N.make_cfg(offset=14, checksum=checksum, classify=N.CLS_LB_HASH, nports=16,
                     badsrc=BADSRC, gooddst=GOODDST)
    got, exp = _check(dev, oracle, b, cfg, f"C4 errors cksum={checksum}")
    # every injected error kind shows up as its reason (checksum only if enabled)
    for k in range(6):
        if k == synth.ERR_CKSUM and not checksum:
            continue
        assert (exp["reason"][kind == k] == k).mean() > 0.95


def test_c3_imix_flow5id(dev, oracle):
    b = synth.c3(150_000, nflows=10_000)
    cfg = N.make_cfg(offset=14, checksum=True, hash_mode=N.HASH_FLOW5ID,
                     classify=N.CLS_LB_HASH, nports=16)
    _check(dev, oracle, b, cfg, "C3")


def test_ip_options_and_fragments(dev, oracle):
    b = synth.c3(60_000, seed=31)
    synth.add_ip_options(b, 0.3)
    set_fragment(b, 0.1)
    synth.inject_errors(b, 0.01, seed=32)
    for ck in (True, False):
        cfg = N.make_cfg(offset=14, checksum=ck, classify=N.CLS_LB_HASH, nports=7)
        _check(dev, oracle, b, cfg, f"options ck={ck}")


def test_misaligned_offsets(dev, oracle):
    b = synth.c3(20_000, seed=33)
    synth.add_ip_options(b, 0.5, seed=34)
    synth.inject_errors(b, 0.02, seed=35)
    b = repack(b, misalign_seed=36)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16,
                     badsrc=BADSRC)
    _check(dev, oracle, b, cfg, "misaligned")


def test_offset_zero_and_large(dev, oracle):
    # frames starting at the IP header (after Strip(14)) and a deep OFFSET
    b = synth.c4(10_000, seed=50)
    synth.inject_errors(b, 0.02, seed=51)
    frames = [f[14:] for f in b.frames()]
    lens = np.array([len(f) for f in frames])
    hdr = np.zeros((b.n, 64), np.uint8)
    for i, f in enumerate(frames):
        hdr[i, :len(f)] = np.frombuffer(f, np.uint8)
    b0 = synth.pack(hdr, lens)
    cfg = N.make_cfg(offset=0, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    _check(dev, oracle, b0, cfg, "offset0")
    pad = 100
    hdr2 = np.zeros((b.n, 256), np.uint8)
    for i, f in enumerate(b.frames()):
        hdr2[i, pad:pad + len(f)] = np.frombuffer(f, np.uint8)
    b2 = synth.pack(hdr2, b.desc[:, 1].astype(np.int64) + pad)
    cfg = N.make_cfg(offset=pad + 14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    _check(dev, oracle, b2, cfg, "offset114")


@pytest.mark.parametrize("native", [0, 5, -1])
def test_c5_vlan_ip6(dev, oracle, native):
    b = synth.c5(80_000)
    cfg = N.make_cfg(check_mode=N.CHECK_AUTO, offset=0, checksum=True, classify=N.CLS_LB_HASH,
                     nports=16, native_vlan=native)
    got, exp = _check(dev, oracle, b, cfg, f"C5 native={native}")
    assert (exp["anno"]["ipver"] == 6).any()


def test_c5_ip6_bad_and_trim(dev, oracle):
    b = synth.c5(30_000, seed=55)
    rng = np.random.default_rng(56)
    A = b.arena
    for i in range(b.n):
        off, ln = (int(x) for x in b.desc[i])
        o = off + (18 if A[off + 12] == 0x81 else 14)
        if A[o] >> 4 != 6:
            continue
        r = rng.random()
        if r < 0.05:
            A[o + 8:o + 24] = 0xFF                       # bad source ff..ff
        elif r < 0.10:
            A[o + 4], A[o + 5] = 0x40, 0                 # payload length too large
        elif r < 0.20:
            A[o + 4], A[o + 5] = 0, int(rng.integers(0, 8))   # trimmed
        elif r < 0.25:
            b.desc[i, 1] = o - off + int(rng.integers(0, 40))  # shorter than 40 B
    cfg = N.make_cfg(check_mode=N.CHECK_AUTO, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    _check(dev, oracle, b, cfg, "C5 bad/trim")


def test_mark_mode(dev, oracle):
    b = synth.c4(20_000, seed=60)
    synth.inject_errors(b, 0.02, seed=61)
    cfg = N.make_cfg(check_mode=N.MARK_IP4, offset=14, hash_mode=N.HASH_FLOW5ID,
                     classify=N.CLS_LB_HASH, nports=5)
    _check(dev, oracle, b, cfg, "mark")


@pytest.mark.parametrize("n", [2, 4, 5, 8, 16])
def test_hash_ip_and_hashswitch(dev, oracle, n):
    b = synth.c3(20_000, seed=70 + n)
    synth.inject_errors(b, 0.01, seed=80 + n)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_HASH_IP, nports=n)
    _check(dev, oracle, b, cfg, f"hash_ip n={n}")
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_HASHSWITCH, nports=n,
                     hs_offset=26, hs_length=12)
    _check(dev, oracle, b, cfg, f"hashswitch n={n}")
    cfg = N.make_cfg(offset=14, classify=N.CLS_HASHSWITCH, nports=n, hs_offset=60, hs_length=70)
    _check(dev, oracle, b, cfg, f"hashswitch long n={n}")


def _shifted(b, seed):
    """The same frames at offsets 64*i + (0..15): windows at every shift."""
    rng = np.random.default_rng(seed)
    sh = rng.integers(0, 16, b.n)
    slot = int(max(int(b.desc[:, 1].max()) + 16, 64) + 63) & ~63
    arena = np.zeros(slot * b.n + 4096, np.uint8)
    desc = np.zeros((b.n, 2), np.uint32)
    for i, (o, ln) in enumerate(b.desc.tolist()):
        at = slot * i + int(sh[i])
        arena[at:at + ln] = b.arena[o:o + ln]
        desc[i] = (at, ln)
    return synth.Batch(arena=arena, desc=desc)


@pytest.mark.parametrize("n", [4, 8, 11])
def test_auto_bytesum_classifiers(dev, oracle, n):
    """hash_ip / HashSwitch on the CHECK_AUTO straight line (VLAN, IPv4 and
    IPv6 in one wave), their bytes inside the window at every shift, and
    HashSwitch ranges past it (general path)."""
    b = _shifted(synth.c5(12_000, seed=90 + n), 91 + n)
    for cls, o, ln in [(N.CLS_HASH_IP, 0, 1), (N.CLS_HASHSWITCH, 26, 12), (N.CLS_HASHSWITCH, 3, 40),
                       (N.CLS_HASHSWITCH, 40, 30), (N.CLS_HASHSWITCH, 70, 4)]:
        cfg = N.make_cfg(check_mode=N.CHECK_AUTO, checksum=True, classify=cls, nports=n, hs_offset=o, hs_length=ln)
        _check(dev, oracle, b, cfg, f"auto bytesum cls={cls} o={o} l={ln} n={n}")


@pytest.mark.parametrize("n", [3, 8, 16])
def test_ip4_bytesum_classifiers_shifted(dev, oracle, n):
    """The IPv4 straight line's byte sums at every window shift."""
    b = synth.c3(12_000, seed=95 + n)
    synth.inject_errors(b, 0.02, seed=96 + n)
    b = _shifted(b, 97 + n)
    for cls, o, ln in [(N.CLS_HASH_IP, 0, 1), (N.CLS_HASHSWITCH, 0, 64), (N.CLS_HASHSWITCH, 13, 35),
                       (N.CLS_HASHSWITCH, 50, 1)]:
        cfg = N.make_cfg(offset=14, checksum=True, classify=cls, nports=n, hs_offset=o, hs_length=ln)
        _check(dev, oracle, b, cfg, f"ip4 bytesum cls={cls} o={o} l={ln} n={n}")


@pytest.mark.parametrize("n", [1, 63, 64, 65, 255, 256, 257])
def test_ragged_sizes(dev, oracle, n):
    b = synth.c4(n, seed=90 + n)
    synth.inject_errors(b, 0.1, seed=91)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=64)
    _check(dev, oracle, b, cfg, f"n={n}")


def test_empty_batch(dev):
    ctx = N.Context(0, 16, N.make_cfg(offset=14))
    ctx.process(0, 0, 0)
    assert ctx.counters()[:2] == [0, 0]
    ctx.close()


def test_counters_accumulate_and_host_path(dev, oracle):
    import ctypes as C
    b = synth.c4(5000, seed=95)
    synth.inject_errors(b, 0.03, seed=96)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16, badsrc=BADSRC)
    exp = oracle.process_batch(cfg, b)
    ctx = N.Context(0, b.n, cfg)
    frames = b.frames()
    bufs = [C.create_string_buffer(f, len(f)) for f in frames]
    ptrs = (C.c_void_p * b.n)(*[C.addressof(x) for x in bufs])
    lens = np.ascontiguousarray(b.desc[:, 1], dtype=np.uint32)
    verdict = np.zeros(b.n, np.uint16)
    hsh = np.zeros(b.n, np.uint32)
    anno = np.zeros(b.n, N.anno_dtype())
    perm = np.zeros(b.n, np.uint32)
    start = np.zeros(cfg.nports + 2, np.uint32)
    tc = np.zeros(((b.n + 255) // 256) * 17, np.uint16)
    ptile = np.zeros(b.n, np.uint32)
    ctx.process_host(ptrs, lens.ctypes.data, b.n, verdict=verdict.ctypes.data, perm=ptile.ctypes.data,
                     tile_count=tc.ctypes.data, partition=N.PART_TILE)
    assert np.array_equal(ptile, exp["perm_tile"]) and np.array_equal(tc, exp["tile_count"])
    for _ in range(2):
        ctx.process_host(ptrs, lens.ctypes.data, b.n, verdict=verdict.ctypes.data,
                         hash=hsh.ctypes.data, anno=anno.ctypes.data, perm=perm.ctypes.data,
                         port_start=start.ctypes.data)
        got = dict(reason=(verdict & 0xFF).astype(np.uint8), port=(verdict >> 8).astype(np.uint8),
                   hash=hsh, anno=anno, perm=perm, port_start=start)
        compare(got, exp, ctx="host path")
    ctr = np.array(ctx.counters(), np.uint64)
    assert np.array_equal(ctr, 3 * exp["counters"])
    ctx.close()


@pytest.mark.parametrize("threads,pinned", [(1, False), (4, False), (3, True)])
def test_host_pipeline_chunks(dev, oracle, threads, pinned):
    """fcgpu_process_host over > 3 pipeline chunks (65,536 packets each, three
    streams): tile outputs, global-index perm, annotations and counters equal
    one oracle pass over the whole batch, for pageable and pinned outputs."""
    import ctypes as C
    n = 3 * 65536 + 4 * 65536 // 3 + 77      # 5 chunks, ragged last chunk and tile
    b = synth.c3(n, seed=97)
    synth.inject_errors(b, 0.02, seed=98)
    synth.add_ip_options(b, 0.05, seed=99)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16, badsrc=BADSRC)
    exp = oracle.process_batch(cfg, b)
    ctx = N.Context(0, n, cfg)
    ctx.set_host_threads(threads)
    base = b.arena.ctypes.data
    ptrs = (C.c_void_p * n)(*[base + int(o) for o in b.desc[:, 0]])
    lens = np.ascontiguousarray(b.desc[:, 1], dtype=np.uint32)
    ntiles = (n + 255) // 256
    keep = []

    def arr(count, dtype):
        dtype = np.dtype(dtype)
        if not pinned:
            return np.zeros(count, dtype)
        p = ctx.lib.fcgpu_host_alloc(count * dtype.itemsize)
        assert p
        keep.append(p)
        a = np.ctypeslib.as_array((C.c_uint8 * (count * dtype.itemsize)).from_address(p)).view(dtype)
        a[:] = 0
        return a
    verdict, hsh, anno = arr(n, np.uint16), arr(n, np.uint32), arr(n, N.anno_dtype())
    perm, tperm, tc = arr(n, np.uint32), arr(n, np.uint8), arr(ntiles * 17, np.uint16)
    for rep in range(2):
        ctx.process_host(ptrs, lens.ctypes.data, n, verdict=verdict.ctypes.data, hash=hsh.ctypes.data,
                         anno=anno.ctypes.data, perm=perm.ctypes.data, tile_perm=tperm.ctypes.data,
                         tile_count=tc.ctypes.data, partition=N.PART_TILE)
        got = dict(reason=(verdict & 0xFF).astype(np.uint8), port=(verdict >> 8).astype(np.uint8),
                   hash=hsh.copy(), anno=anno.copy(), perm_tile=perm.copy(), tile_count=tc.copy(),
                   tile_perm=tperm.copy())
        compare(got, exp, ctx=f"host pipeline threads={threads} pinned={pinned} rep={rep}")
    assert np.array_equal(np.array(ctx.counters(), np.uint64), 2 * exp["counters"])
    ctx.close()
    for p in keep:
        N.load().fcgpu_host_free(p)


def test_large_batch_properties(dev, oracle):
    """4M packets: full oracle comparison of hash/port plus partition
    properties (sorted runs, permutation, counts)."""
    n = 1 << 22
    b = synth.c4(n, seed=99)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    got = dev.process_batch(b, cfg, anno=False, perm=True)
    exp = oracle.process_batch(cfg, b)
    compare(got, exp, anno=False, ctx="4M")
    perm, start = got["perm"], got["port_start"]
    assert np.array_equal(np.sort(perm), np.arange(n, dtype=np.uint32))
    for p in range(17):
        run = perm[start[p]:start[p + 1]]
        assert (np.diff(run.astype(np.int64)) > 0).all()
        assert (got["port"][run] == p).all()
    gt = dev.process_batch(b, cfg, anno=False, perm=True, partition=N.PART_TILE)
    assert np.array_equal(gt["perm_tile"], exp["perm_tile"]) and np.array_equal(gt["tile_count"], exp["tile_count"])


@pytest.mark.parametrize("mode", [N.L4_UDP, N.L4_TCP])
def test_l4_checks_misaligned_and_host(dev, oracle, mode):
    """L4 checks on the reference-pinned L4 set replicated 40x at misaligned
    frame offsets (odd segment starts, partial 16-B chunks), device-resident
    and through the host path (whole frames staged), vs the oracle."""
    import ctypes as C
    from tests.test_golden import load, batch_of
    g = load("l4")
    base = batch_of(g)
    frames = base.frames() * 40
    b = repack(synth.from_frames(frames), misalign_seed=31)
    cfg = N.make_cfg(offset=14, checksum=True, l4_mode=mode, classify=N.CLS_LB_HASH, nports=16,
                     hash_mode=N.HASH_FLOWID)
    got, exp = _check(dev, oracle, b, cfg, f"l4 mode={mode}")
    assert (exp["reason"] == N.R_L4_CKSUM).sum() > 1000
    ctx = N.Context(0, b.n, cfg)
    ctx.set_host_threads(4)
    ptrs = (C.c_void_p * b.n)(*[b.arena.ctypes.data + int(o) for o in b.desc[:, 0]])
    lens = np.ascontiguousarray(b.desc[:, 1], dtype=np.uint32)
    verdict = np.zeros(b.n, np.uint16)
    hsh = np.zeros(b.n, np.uint32)
    ctx.process_host(ptrs, lens.ctypes.data, b.n, verdict=verdict.ctypes.data, hash=hsh.ctypes.data)
    assert np.array_equal(verdict & 0xFF, exp["reason"]) and np.array_equal(verdict >> 8, exp["port"])
    assert np.array_equal(hsh, exp["hash"])
    ctx.close()


def test_process_jobs_two_streams(dev, oracle):
    """fcgpu_process_jobs: six batches (three C4 shapes with errors) on two
    streams in one call give each batch the oracle's verdicts, hashes and
    tile partition; the counters sum over the jobs; a bad job in the list
    launches nothing (FCGPU_EINVAL before the first launch)."""
    import torch
    from fastclick_amd.device import DeviceBatch, DeviceOutputs
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16, badsrc=BADSRC)
    batches = []
    for s in range(3):
        b = synth.c4(30_000 + 1_001 * s, seed=60 + s)
        synth.inject_errors(b, 0.02, seed=70 + s)
        batches.append(b)
    exps = [oracle.process_batch(cfg, b) for b in batches]
    ctx = N.Context(0, 40_000, cfg)
    try:
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        dbs = [DeviceBatch.upload(b, device="cuda:0") for b in batches]
        outs, specs = [], []
        for k in range(6):
            b = dbs[k % 3]
            o = DeviceOutputs(b.n, 16, device="cuda:0", perm=True, partition=N.PART_TILE, anno=False)
            outs.append(o)
            specs.append((b.arena.data_ptr(), b.desc.data_ptr(), b.n, streams[k % 2].cuda_stream, o.ptrs()))
        ctx.run_jobs(ctx.jobs(specs))
        torch.cuda.synchronize()
        for k in range(6):
            got = outs[k].numpy()
            exp = exps[k % 3]
            assert np.array_equal(got["reason"], exp["reason"]), k
            assert np.array_equal(got["port"], exp["port"]), k
            ok = exp["reason"] == N.R_OK
            assert np.array_equal(got["hash"][ok], exp["hash"][ok]), k
            assert np.array_equal(got["tile_count"], exp["tile_count"]), k
            assert np.array_equal(got["perm_tile"], exp["perm_tile"]), k
        want = sum(2 * e["counters"].astype(np.int64) for e in exps)
        assert np.array_equal(np.array(ctx.counters(), np.int64), want)
        # one bad job (n > max_batch) -> error, and no job of the list ran
        before = np.array(ctx.counters(), np.int64)
        bad = list(specs[:2]) + [(specs[0][0], specs[0][1], 50_000, None, outs[0].ptrs())]
        with pytest.raises(RuntimeError):
            ctx.run_jobs(ctx.jobs(bad))
        torch.cuda.synchronize()
        assert np.array_equal(np.array(ctx.counters(), np.int64), before)
    finally:
        ctx.close()


def test_process_jobs_fused_global_large(dev, oracle):
    """Fused whole-batch partitions large enough that each scatter workgroup
    takes several tiles (5 ragged batches, 4.5M packets: 8 tiles per
    workgroup), against the oracle's permutation and port starts."""
    import torch
    from fastclick_amd.device import DeviceBatch, DeviceOutputs
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16, badsrc=BADSRC)
    sizes = [900_000, 899_937, 900_001, 913_131, 887_777]
    ctx = N.Context(0, max(sizes), cfg)
    try:
        specs, keep = [], []
        for k, n in enumerate(sizes):
            b = synth.c4(n, seed=700 + k)
            synth.inject_errors(b, 0.01, seed=710 + k)
            db = DeviceBatch.upload(b, device="cuda:0")
            o = DeviceOutputs(n, 16, device="cuda:0", perm=True, anno=False, partition=N.PART_GLOBAL,
                              port_start=True)
            keep.append((b, db, o))
            specs.append((db.arena.data_ptr(), db.desc.data_ptr(), n, None, o.ptrs()))
        ctx.run_jobs(ctx.jobs(specs))
        torch.cuda.synchronize()
        for k, (b, db, o) in enumerate(keep):
            exp = oracle.process_batch(cfg, b)
            got = o.numpy()
            assert np.array_equal(got["port"][:b.n], exp["port"]), k
            assert np.array_equal(got["port_start"], exp["port_start"]), k
            assert np.array_equal(got["perm"][:b.n], exp["perm"]), k
    finally:
        ctx.close()


@pytest.mark.parametrize("partition", [N.PART_TILE, N.PART_GLOBAL, None])
def test_process_jobs_fused(dev, oracle, partition):
    """fcgpu_process_jobs fuses a stream's consecutive jobs with disjoint
    outputs into one k_rx launch (up to 24 batches, the grid their tiles end
    to end): 30 ragged batches (1 .. 30,001 packets, one empty) on one stream
    -> two fused launches; every batch gets the oracle's results, the counters
    sum over the batches. Two jobs sharing an output set are not fused: the
    later one's results are what the set holds, as with one call per job.
    PART_GLOBAL: the whole-batch partitions of a fused launch (one scan and
    one scatter launch for all its batches); odd batches ask for port_start
    only (one scatter workgroup each)."""
    import torch
    from fastclick_amd.device import DeviceBatch, DeviceOutputs
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16, badsrc=BADSRC)
    sizes = [1, 255, 256, 257, 0, 30_001] + [1_000 + 997 * k for k in range(24)]
    batches = []
    for k, n in enumerate(sizes):
        b = synth.c4(max(n, 1), seed=200 + k)
        synth.inject_errors(b, 0.02, seed=300 + k)
        if n == 0:
            b = synth.Batch(arena=b.arena, desc=b.desc[:0].copy())
        batches.append(b)
    exps = [oracle.process_batch(cfg, b) for b in batches]
    tile = partition == N.PART_TILE
    glob = partition == N.PART_GLOBAL
    ctx = N.Context(0, 40_000, cfg)
    try:
        dbs = [DeviceBatch.upload(b, device="cuda:0") for b in batches]
        outs, specs = [], []
        for k, b in enumerate(dbs):
            o = DeviceOutputs(max(b.n, 1), 16, device="cuda:0", perm=tile or (glob and k % 2 == 0), anno=False,
                              partition=N.PART_TILE if tile else N.PART_GLOBAL, port_start=glob)
            outs.append(o)
            specs.append((b.arena.data_ptr(), b.desc.data_ptr(), b.n, None, o.ptrs()))
        ctx.set_timing(1)
        ctx.run_jobs(ctx.jobs(specs))
        torch.cuda.synchronize()
        ms, cnt = ctx.read_timing()
        assert cnt[0] == sum(1 for n in sizes if n)          # timing counts batches
        ctx.set_timing(0)
        for k, (b, o) in enumerate(zip(batches, outs)):
            if b.n == 0:
                continue
            got, exp = o.numpy(), exps[k]
            assert np.array_equal(got["reason"][:b.n], exp["reason"]), k
            assert np.array_equal(got["port"][:b.n], exp["port"]), k
            ok = exp["reason"] == N.R_OK
            assert np.array_equal(got["hash"][:b.n][ok], exp["hash"][ok]), k
            if tile:
                nt = (b.n + N.TILE - 1) // N.TILE
                assert np.array_equal(got["tile_count"][:nt * 17], exp["tile_count"]), k
                assert np.array_equal(got["perm_tile"][:b.n], exp["perm_tile"]), k
            if glob:
                assert np.array_equal(got["port_start"], exp["port_start"]), k
                if k % 2 == 0:
                    assert np.array_equal(got["perm"][:b.n], exp["perm"]), k
        want = sum(e["counters"].astype(np.int64) for e, b in zip(exps, batches) if b.n)
        assert np.array_equal(np.array(ctx.counters(), np.int64), want)
        # two jobs on one output set: sequential semantics (the second wins)
        shared = DeviceOutputs(40_000, 16, device="cuda:0", perm=tile, anno=False,
                               partition=N.PART_TILE if tile else N.PART_GLOBAL, port_start=False)
        pair = [(dbs[5].arena.data_ptr(), dbs[5].desc.data_ptr(), dbs[5].n, None, shared.ptrs()),
                (dbs[29].arena.data_ptr(), dbs[29].desc.data_ptr(), dbs[29].n, None, shared.ptrs())]
        ctx.run_jobs(ctx.jobs(pair))
        torch.cuda.synchronize()
        got = shared.numpy()
        n29 = batches[29].n
        assert np.array_equal(got["reason"][:n29], exps[29]["reason"])
        assert np.array_equal(got["reason"][n29:batches[5].n], exps[5]["reason"][n29:])
    finally:
        ctx.close()


@pytest.mark.parametrize("mode", ["c5_auto", "mark_crc", "ipclass", "lbtable_lds", "lbtable_global"])
def test_process_jobs_fused_equal_batches(dev, oracle, mode):
    """One fused k_rx launch over 24 equal batches (the equal-tile division of
    the grid) plus a ragged tail batch in another launch: C5's
    StripEtherVLANHeader + IPv4/IPv6 dispatch, MarkIPHeader + LB_MODE
    hash_crc (LDS tables), an IPClassifier program, LB_MODE cst_hash_agg with
    its ring in LDS (1,600 buckets) or read from global memory (70,000) --
    every batch's results are the oracle's."""
    import torch
    from fastclick_amd import click
    from fastclick_amd.device import DeviceBatch, DeviceOutputs
    program = None
    ring = None
    if mode.startswith("lbtable"):
        cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_TABLE, nports=16)
        ring = N.lb_hash_ring(16, 1600 if mode == "lbtable_lds" else 70_000)
        mk = lambda k, n: synth.c4(n, seed=650 + k)  # noqa: E731
    elif mode == "c5_auto":
        cfg = N.make_cfg(check_mode=N.CHECK_AUTO, offset=0, checksum=True, classify=N.CLS_LB_HASH, nports=16)
        mk = lambda k, n: synth.c5(n, seed=500 + k)  # noqa: E731
    elif mode == "mark_crc":
        cfg = N.make_cfg(check_mode=N.MARK_IP4, offset=14, classify=N.CLS_LB_CRC, nports=16)
        mk = lambda k, n: synth.c4(n, seed=600 + k)  # noqa: E731
    else:
        import bench
        cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_PROGRAM, nports=16)
        steps, oe = click.parse_program(bench.ipclass16_program())
        program = (N.PROG_IPFILTER, steps, oe)
        mk = lambda k, n: synth.c4(n, seed=700 + k)  # noqa: E731
    sizes = [4096] * 24 + [777]
    batches = [mk(k, n) for k, n in enumerate(sizes)]
    ctx = N.Context(0, 4096, cfg)
    try:
        if program is not None:
            ctx.set_program(*program)
        if ring is not None:
            ctx.set_lb_table(ring)
        dbs = [DeviceBatch.upload(b, device="cuda:0") for b in batches]
        outs = [DeviceOutputs(b.n, 16, device="cuda:0", perm=True, anno=False, partition=N.PART_TILE)
                for b in dbs]
        specs = [(b.arena.data_ptr(), b.desc.data_ptr(), b.n, None, o.ptrs()) for b, o in zip(dbs, outs)]
        ctx.run_jobs(ctx.jobs(specs))
        torch.cuda.synchronize()
        for k, (b, o) in enumerate(zip(batches, outs)):
            got = o.numpy()
            exp = oracle.process_batch(cfg, b, program=program, lb_table=ring)
            for key in ("reason", "port", "perm_tile"):
                assert np.array_equal(got[key][:b.n], exp[key]), (mode, k, key)
            ok = exp["reason"] == N.R_OK
            assert np.array_equal(got["hash"][:b.n][ok], exp["hash"][ok]), (mode, k)
    finally:
        ctx.close()
