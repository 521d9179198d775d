"""LoadBalancer's other per-packet hash modes: constant_hash_agg
(LB_MODE cst_hash_agg, CST_BUCKETS; include/click/loadbalancer.hh:585-589 over
the ring of build_hash_ring, :170-189) and direct_chash (LB_MODE chash,
hash_4tuple, :138-152 and :666-668).

Parity unpinned by reference vectors: no reference test configures these
modes. The ring and the ports are checked against the oracle's restatement
(oracle/fc_oracle.c fco_lb_hash_ring, fco_lb_table_port), which is checked
here against a hand-worked ring and a second, independent restatement.
"""
import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N


def _ring_py(nsel, size):
    """build_hash_ring restated again, in Python with 32-bit unsigned wrap
    (cantor is `unsigned`, include/click/algorithm.hh:136-138)."""
    ring = [None] * size
    fac = (size - 1) // nsel + 1
    for j in range(fac):
        for i in range(nsel):
            c = ((((i + j) * (i + j + 1)) & 0xFFFFFFFF) // 2 + j) & 0xFFFFFFFF
            ring[c % size] = i
    cur, out = 0, []
    for v in ring:
        if v is not None:
            cur = v
        out.append(cur)
    return np.array(out, np.uint32)


def test_hash_ring_hand_worked(oracle):
    # nsel 2, size 4: fac 2; j=0 places 0 at 0, 1 at 1; j=1 places 0 at
    # cantor(0,1)=2 and 1 at cantor(1,1)=4 % 4 = 0; bucket 3 takes 0 (bucket 2's)
    assert oracle.lb_hash_ring(2, 4).tolist() == [1, 1, 0, 0]
    # one bucket: the last server placed
    assert oracle.lb_hash_ring(5, 1).tolist() == [4]


@pytest.mark.parametrize("nsel,size", [(1, 100), (2, 200), (3, 7), (16, 1600), (16, 5000), (40, 4000),
                                       (64, 6400), (7, 100_000), (1, 200_000)])
def test_hash_ring_matches_second_restatement(oracle, nsel, size):
    r = oracle.lb_hash_ring(nsel, size)
    assert np.array_equal(r, _ring_py(nsel, size))
    assert int(r.max()) < nsel
    if size >= 100 * nsel:
        assert set(np.unique(r).tolist()) == set(range(nsel))


@pytest.mark.parametrize("nsel,size", [(2, 4), (16, 1600), (12, 333), (64, 6400), (7, 100_000), (1, 200_000)])
def test_product_ring_matches_oracle(oracle, nsel, size):
    """The library's ring (fcgpu_lb_hash_ring, host code: the element and the
    bench take their tables from it) against the oracle's restatement."""
    assert np.array_equal(N.lb_hash_ring(nsel, size), oracle.lb_hash_ring(nsel, size).astype(np.uint8))
    with pytest.raises(ValueError):
        N.lb_hash_ring(65, 100)


def test_config_lb_modes():
    from fastclick_amd import click as K
    c = K.element_cfg("GPUIPCheckClassify(OFFSET 14, N 8, LB_MODE chash)")
    assert (c.classify, c.hs_offset, c.hs_length, c.nports) == (N.CLS_HASHSWITCH, 26, 12, 8)
    c = K.element_cfg("GPUIPCheckClassify(OFFSET 14, N 8, LB_MODE cst_hash_agg, CST_BUCKETS 333)")
    assert c.classify == N.CLS_LB_TABLE
    c = K.element_cfg("GPUIPCheckClassify(OFFSET 14, N 8, LB_MODE hash_agg, HASH FLOW5ID)")
    assert c.classify == N.CLS_LB_HASH and c.hash_mode == N.HASH_FLOW5ID
    # byte sums behind Strip(OFFSET) count from the stripped data
    c = K.element_cfg("GPUIPCheckClassify(OFFSET 14, STRIP true, N 5, LB_MODE hash_ip)")
    assert (c.classify, c.hs_offset, c.hs_length) == (N.CLS_HASHSWITCH, 40, 8)
    c = K.element_cfg("GPUIPCheckClassify(OFFSET 14, STRIP true, N 5, LB_MODE chash)")
    assert (c.classify, c.hs_offset, c.hs_length) == (N.CLS_HASHSWITCH, 40, 12)
    c = K.element_cfg("GPUIPCheckClassify(OFFSET 14, STRIP true, N 5, HASHSWITCH 6 8)")
    assert (c.classify, c.hs_offset, c.hs_length) == (N.CLS_HASHSWITCH, 20, 8)
    c = K.element_cfg("GPUIPCheckClassify(MODE AUTO, STRIP false, N 5, LB_MODE hash_ip)")
    assert c.classify == N.CLS_HASH_IP
    for bad, msg in [("GPUIPCheckClassify(MODE AUTO, N 5, LB_MODE hash_ip)", "STRIP false"),
                     ("GPUIPCheckClassify(N 8, LB_MODE cst_hash_agg, CST_BUCKETS 0)", "CST_BUCKETS"),
                     ("GPUIPCheckClassify(N 8, LB_MODE rr)", "unsupported LB_MODE"),
                     ("GPUIPCheckClassify(N 8, LB_MODE hash, HASH FLOW5ID)", "hash_agg")]:
        with pytest.raises(K.ConfigError, match=msg):
            K.check_config(bad)


def _hash_4tuple(frame, length, n):
    """LoadBalancer::hash_4tuple (loadbalancer.hh:138-152)."""
    if length < 38:
        return 0
    d = int(frame[26:38].astype(np.int64).sum())
    return (d ^ (d >> 4)) & (n - 1) if n in (2, 4, 8) else d % n


@pytest.mark.parametrize("n", [4, 8, 11])
def test_oracle_chash_is_hash_4tuple(oracle, n):
    b = synth.c4(3000, seed=70 + n)
    b.desc[::97, 1] = 30            # short frames: port 0
    cfg = N.make_cfg(offset=14, classify=N.CLS_HASHSWITCH, hs_offset=26, hs_length=12, nports=n)
    e = oracle.process_batch(cfg, b)
    ok = e["reason"] == N.R_OK
    exp = [_hash_4tuple(b.arena[o:o + ln], int(e["anno"]["length"][i]), n)
           for i, (o, ln) in enumerate(b.desc.tolist())]
    assert np.array_equal(e["port"][ok], np.array(exp, np.uint8)[ok])


def _fold(h):
    h = h.astype(np.uint32)
    return (h >> 16) ^ (h & 0xFFFF)


@pytest.mark.parametrize("size", [1600, 5000, 70_000])
def test_oracle_table_port(oracle, size):
    b = synth.c4(5000, seed=80)
    ring = oracle.lb_hash_ring(16, size).astype(np.uint8)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_TABLE, nports=16)
    e = oracle.process_batch(cfg, b, lb_table=ring)
    ok = e["reason"] == N.R_OK
    assert np.array_equal(e["port"][ok], ring[_fold(e["hash"]) % size][ok])


# ---- the device path ------------------------------------------------------


def _table_cases():
    return [("c4", N.CHECK_IP4, 16, None), ("c4", N.CHECK_IP4, 16, 5000), ("c4", N.CHECK_IP4, 7, 70_000),
            ("c4", N.CHECK_IP4, 3, 1), ("c5", N.CHECK_AUTO, 16, None), ("c5", N.CHECK_AUTO, 40, 4096),
            ("c5", N.CHECK_AUTO, 5, 4097)]


@pytest.mark.gpu
@pytest.mark.parametrize("wl,mode,nports,size", _table_cases())
@pytest.mark.parametrize("part", [N.PART_TILE, N.PART_GLOBAL])
def test_gpu_lb_table_matches_oracle(oracle, wl, mode, nports, size, part):
    """k_rx with CLS_LB_TABLE: the table from LDS (<= 4096 buckets) or from
    global memory, longer tables truncated to the 65536 buckets the folded
    hash reaches, IPv4 and (CHECK_AUTO) IPv6 hashes, both partitions."""
    from fastclick_amd import device as D
    if wl == "c4":
        b = synth.c4(40_000, seed=90)
        synth.inject_errors(b, 0.01, seed=92)      # untagged IPv4 frames only
    else:
        b = synth.c5(40_000, seed=91)
    size = 100 * nports if size is None else size
    ring = oracle.lb_hash_ring(nports, size).astype(np.uint8)
    off = 14 if mode == N.CHECK_IP4 else 0
    cfg = N.make_cfg(check_mode=mode, offset=off, checksum=True, classify=N.CLS_LB_TABLE, nports=nports)
    e = oracle.process_batch(cfg, b, lb_table=ring)
    r = D.process_batch(b, cfg, partition=part, lb_table=ring)
    assert np.array_equal(r["verdict"], e["verdict"])
    assert np.array_equal(r["hash"], e["hash"])
    if part == N.PART_GLOBAL:
        assert np.array_equal(r["perm"], e["perm"])
    assert np.array_equal(r["counters"], e["counters"])


@pytest.mark.gpu
def test_gpu_lb_table_errors():
    ctx = N.Context(0, 1024, N.make_cfg(classify=N.CLS_LB_TABLE, nports=4))
    try:
        with pytest.raises(RuntimeError, match="nports"):
            ctx.set_lb_table(np.array([0, 1, 4], np.uint8))
        with pytest.raises(RuntimeError, match="size"):
            ctx.set_lb_table(np.zeros(0, np.uint8))
        ctx.set_lb_table(np.array([3, 2, 1, 0], np.uint8))
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("conf_mode,buckets", [("cst_hash_agg", None), ("cst_hash_agg", 333),
                                               ("cst_hash_agg", 100_000), ("chash", None)])
def test_element_lb_modes(oracle, conf_mode, buckets):
    """The element builds the ring itself (product code) at initialize: its
    ports equal the oracle's with the oracle's ring."""
    from fastclick_amd import click as K
    b = synth.c4(20_000, seed=95)
    synth.inject_errors(b, 0.02, seed=96)
    extra = f", CST_BUCKETS {buckets}" if buckets else ""
    conf = f"GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 12, LB_MODE {conf_mode}{extra})"
    r = K.run_element(conf, b, nsinks=13)
    if conf_mode == "chash":
        cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_HASHSWITCH, hs_offset=26, hs_length=12,
                         nports=12)
        e = oracle.process_batch(cfg, b)
    else:
        ring = oracle.lb_hash_ring(12, buckets or 1200).astype(np.uint8)
        cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_TABLE, nports=12)
        e = oracle.process_batch(cfg, b, lb_table=ring)
    assert np.array_equal(r["port"], e["port"].astype(np.uint32))


@pytest.mark.gpu
def test_element_bytesum_behind_strip(oracle):
    """STRIP true: the chain is Strip(14) -> CheckIPHeader -> FlowSwitch(hash_ip),
    whose byte sum reads the IP packet's bytes 26..33 = frame bytes 40..47."""
    from fastclick_amd import click as K
    b = synth.c4(20_000, seed=97)
    rng = np.random.default_rng(98)
    for off in b.desc[:, 0].tolist():                # random UDP payload (bytes 42..59)
        b.arena[off + 42:off + 60] = rng.integers(0, 256, 18, dtype=np.uint8)
    r = K.run_element("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, STRIP true, N 5, LB_MODE hash_ip)", b,
                      nsinks=6)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_HASHSWITCH, hs_offset=40, hs_length=8, nports=5)
    e = oracle.process_batch(cfg, b)
    assert np.array_equal(r["port"], e["port"].astype(np.uint32))
    assert len(np.unique(r["port"])) > 1
