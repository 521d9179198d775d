"""Header rewrites after the classifier: DecIPTTL and
SetIPChecksum on the device.

Pin: tests/golden/rw.npz holds, per packet, IP header bytes 8..11 (ttl,
protocol, checksum) as the reference itself dumps them after
`CheckIPHeader -> DecIPTTL[(MULTICAST false)] [-> SetIPChecksum]` and
`MarkIPHeader(14) -> SetIPChecksum`, plus which packets DecIPTTL sent to its
output 1 (tests/golden/gen_golden.py run_rw). The set covers TTL 0/1/2/255,
multicast destinations, IP options, bad checksums and headers SetIPChecksum
rejects (hl < 20). The oracle is checked against it on CPU; the device path
against the golden and against the oracle on seeded batches, including the
in-place arena write (FCGPU_RW_INPLACE).
"""
import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N
from tests.test_golden import load, batch_of

GONE = 0xFFFFFFFF
UNPINNED = 0xFFFFFFFE


def orig_bytes(b, nh_off=14):
    A = b.arena
    o = b.desc[:, 0].astype(np.int64) + nh_off
    w = np.zeros(b.n, np.uint32)
    for k in range(4):
        w |= A[np.minimum(o + 8 + k, len(A) - 1)].astype(np.uint32) << np.uint32(8 * k)
    return w


def effective(r, b):
    """Bytes 8..11 after the element: ip_rw for a packet that leaves with R_OK
    (rewritten or not), else the input's."""
    return np.where(r["reason"] == N.R_OK, r["ip_rw"], orig_bytes(b))


def check_rw(run, g):
    b = batch_of(g)
    cases = [("dec", N.RW_DECTTL, True), ("decnm", N.RW_DECTTL, False),
             ("decset", N.RW_DECTTL | N.RW_SETCKSUM, True)]
    for name, rw, mcast in cases:
        cfg = N.make_cfg(offset=14, checksum=True, rewrite=rw, ttl_multicast=mcast)
        r = run(cfg, b)
        exp = g[name]
        out = r["reason"] == N.R_OK
        if name != "decset":
            assert np.array_equal(r["reason"] == N.R_TTL_EXPIRED, g[name + "_expired"]), f"{name}: expired set"
            assert np.array_equal(out, exp != GONE), f"{name}: survivors"
        else:
            assert np.array_equal(out, exp != GONE), f"{name}: survivors"
        got = effective(r, b)
        assert np.array_equal(got[out], exp[out]), f"{name}: rewritten header bytes"
    cfg = N.make_cfg(check_mode=N.MARK_IP4, offset=14, rewrite=N.RW_SETCKSUM)
    r = run(cfg, b)
    exp = g["set"]
    pin = exp != UNPINNED
    assert np.array_equal((r["reason"] == N.R_OK)[pin], (exp != GONE)[pin]), "SetIPChecksum survivors"
    assert np.array_equal((r["reason"] == N.R_SETCKSUM_BAD)[pin], (exp == GONE)[pin])
    ok = pin & (exp != GONE)
    assert np.array_equal(effective(r, b)[ok], exp[ok]), "SetIPChecksum bytes"


def test_oracle_rewrite_golden(oracle):
    check_rw(lambda cfg, b: oracle.process_batch(cfg, b), load("rw"))


def test_oracle_rewrite_counters(oracle):
    g = load("rw")
    b = batch_of(g)
    r = oracle.process_batch(N.make_cfg(offset=14, checksum=True, rewrite=N.RW_DECTTL), b)
    c = r["counters"]
    exp = int(g["dec_expired"].sum())
    assert c[N.CTR_REASON + N.reason_slot(N.R_TTL_EXPIRED)] == exp
    # DecIPTTL's drops are not CheckIPHeader drops
    assert c[N.CTR_COUNT] == (r["reason"] == N.R_OK).sum() + exp


def _dev(cfg, b, **kw):
    from fastclick_amd import device
    return device.process_batch(b, cfg, anno=True, perm=True, **kw)


@pytest.mark.gpu
def test_gpu_rewrite_golden():
    check_rw(_dev, load("rw"))


@pytest.mark.gpu
@pytest.mark.parametrize("rw", [N.RW_DECTTL, N.RW_SETCKSUM, N.RW_DECTTL | N.RW_SETCKSUM])
@pytest.mark.parametrize("mode", [N.CHECK_IP4, N.MARK_IP4])
def test_gpu_rewrite_vs_oracle(oracle, rw, mode):
    g = load("rw")
    parts = [batch_of(g), synth.c4(50_000, seed=61)]
    synth.add_ip_options(parts[1], 0.1, seed=62)
    A = parts[1].arena
    rng = np.random.default_rng(63)
    for i in np.nonzero(rng.random(parts[1].n) < 0.2)[0]:
        o = int(parts[1].desc[i, 0]) + 14
        A[o + 8] = int(rng.integers(0, 3))
        synth._refresh_cksum(A, o)
    for b in parts:
        cfg = N.make_cfg(check_mode=mode, offset=14, checksum=mode == N.CHECK_IP4, rewrite=rw,
                         classify=N.CLS_LB_HASH, nports=8)
        got, exp = _dev(cfg, b), oracle.process_batch(cfg, b)
        for k in ("reason", "port", "hash", "ip_rw"):
            assert np.array_equal(got[k], exp[k]), f"{k} (rw={rw}, mode={mode})"
        assert np.array_equal(got["counters"], exp["counters"])


@pytest.mark.gpu
def test_gpu_rewrite_inplace():
    """FCGPU_RW_INPLACE: the device arena holds the rewritten header bytes."""
    import torch
    from fastclick_amd.device import DeviceBatch, DeviceOutputs, run_device
    g = load("rw")
    b = batch_of(g)
    cfg = N.make_cfg(offset=14, checksum=True, rewrite=N.RW_DECTTL | N.RW_SETCKSUM | N.RW_INPLACE)
    ctx = N.Context(0, b.n, cfg)
    try:
        db = DeviceBatch.upload(b)
        outs = DeviceOutputs(b.n, 1, ip_rw=True)
        run_device(ctx, db, outs)
        torch.cuda.synchronize()
        res = outs.numpy()
        arena = db.arena.cpu().numpy()
    finally:
        ctx.close()
    after = orig_bytes(synth.Batch(arena=arena, desc=b.desc))
    ok = res["reason"] == N.R_OK
    assert np.array_equal(res["ip_rw"][~ok], np.zeros((~ok).sum(), np.uint32))
    changed = ok & (res["ip_rw"] != orig_bytes(b))
    assert changed.sum() > 2000
    assert np.array_equal(after[ok], res["ip_rw"][ok])
    assert np.array_equal(after[changed], g["decset"][changed])
    assert np.array_equal(after[~changed], orig_bytes(b)[~changed])


@pytest.mark.gpu
def test_gpu_rewrite_fused_jobs(oracle):
    """Rewrites reported through ip_rw (not in place) fuse across queued
    batches (fcgpu_process_jobs): each batch's ip_rw, verdicts and tile
    partition match the oracle; batches with TTL 0/1/2 packets and IP options."""
    import torch
    from fastclick_amd.device import DeviceBatch, DeviceOutputs
    cfg = N.make_cfg(offset=14, checksum=True, rewrite=N.RW_DECTTL | N.RW_SETCKSUM, classify=N.CLS_LB_HASH,
                     nports=8)
    rng = np.random.default_rng(64)
    batches = []
    for k, n in enumerate([3000, 257, 40_000, 12_345, 1]):
        b = synth.c4(n, seed=640 + k)
        synth.add_ip_options(b, 0.1, seed=650 + k)
        for i in np.nonzero(rng.random(b.n) < 0.2)[0]:
            o = int(b.desc[i, 0]) + 14
            b.arena[o + 8] = int(rng.integers(0, 3))
            synth._refresh_cksum(b.arena, o)
        batches.append(b)
    ctx = N.Context(0, 40_000, cfg)
    try:
        dbs = [DeviceBatch.upload(b, device="cuda:0") for b in batches]
        outs = [DeviceOutputs(b.n, 8, device="cuda:0", perm=True, anno=False, partition=N.PART_TILE,
                              ip_rw=True) for b in batches]
        ctx.set_timing(1)
        ctx.run_jobs(ctx.jobs([(db.arena.data_ptr(), db.desc.data_ptr(), db.n, None, o.ptrs())
                               for db, o in zip(dbs, outs)]))
        torch.cuda.synchronize()
        _, cnt = ctx.read_timing()
        assert cnt[0] == len(batches)
        for k, (b, o) in enumerate(zip(batches, outs)):
            got, exp = o.numpy(), oracle.process_batch(cfg, b)
            for key in ("reason", "port", "ip_rw"):
                assert np.array_equal(got[key][:b.n], exp[key]), (k, key)
            nt = (b.n + N.TILE - 1) // N.TILE
            assert np.array_equal(got["perm_tile"][:b.n], exp["perm_tile"]), k
            assert np.array_equal(got["tile_count"][:nt * 9], exp["tile_count"]), k
    finally:
        ctx.close()
