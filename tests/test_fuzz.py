"""Fuzz parity: arbitrary frames through every mode, GPU vs oracle, bit-exact.

Frames are mutated from valid IPv4/IPv6/802.1Q frames (random bytes in the
headers, random lengths 0..200 including frames cut inside the header,
option lengths, fragment fields, version nibbles, L4 lengths) at random,
misaligned arena offsets, so the straight-line fast path, the general path and
the bytes-past-the-window loads all see hostile input. Each configuration
compares reason, port, hash, annotations, partition, counters -- and flow IDs
and rewritten header bytes where enabled -- with the C oracle (itself pinned
to the reference by tests/test_golden.py).

The CPU part only checks that the generator is deterministic and the oracle
runs on it (no GPU).
"""
import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N
from tests.helpers import compare, repack


def fuzz_batch(n, seed):
    rng = np.random.default_rng(seed)
    base = [synth.c4(n, seed=seed), synth.c5(n, seed=seed + 1)]
    synth.add_ip_options(base[0], 0.2, seed=seed + 2)
    frames = []
    for i in range(n):
        src = base[int(rng.integers(0, 2))]
        fr = bytearray(src.frame(int(rng.integers(0, src.n))))
        r = rng.random()
        if r < 0.5:                                  # flip random header bytes
            for _ in range(int(rng.integers(1, 6))):
                j = int(rng.integers(0, min(len(fr), 80)))
                fr[j] = int(rng.integers(0, 256))
        elif r < 0.6:                                # header fields that steer the parse
            o = 14 if fr[12:14] != b"\x81\x00" else 18
            if len(fr) > o + 10:
                fr[o] = int(rng.choice([0x45, 0x46, 0x4F, 0x44, 0x60, 0x35, 0x40]))
                fr[o + 6] = int(rng.integers(0, 256))
                fr[o + 2:o + 4] = int(rng.integers(0, 300)).to_bytes(2, "big")
        r = rng.random()
        if r < 0.15:                                 # cut anywhere, including inside the header
            fr = fr[:int(rng.integers(0, len(fr) + 1))]
        elif r < 0.25:                               # trailing bytes (take() trims them)
            fr += bytes(rng.integers(0, 256, int(rng.integers(1, 120)), dtype=np.uint8))
        frames.append(bytes(fr))
    return repack(synth.from_frames(frames), misalign_seed=seed + 3)


def test_fuzz_generator_and_oracle(oracle):
    a, b = fuzz_batch(2000, 7), fuzz_batch(2000, 7)
    assert np.array_equal(a.arena, b.arena) and np.array_equal(a.desc, b.desc)
    r = oracle.process_batch(N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=8), a)
    # the mutations reach every CheckIPHeader reason
    assert set(np.unique(r["reason"])) >= {0, 1, 2, 3, 4, 6}


BADSRC = [N.raw_addr("192.0.2.255"), N.raw_addr("255.255.255.255")]

CONFIGS = {
    "check-lb16": dict(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16, badsrc=BADSRC),
    "check-nocksum-flow5": dict(offset=14, checksum=False, hash_mode=N.HASH_FLOW5ID, classify=N.CLS_LB_HASH,
                                nports=7),
    "mark-haship": dict(check_mode=N.MARK_IP4, offset=14, classify=N.CLS_HASH_IP, nports=4),
    "check-hashswitch": dict(offset=14, checksum=True, classify=N.CLS_HASHSWITCH, nports=5, hs_offset=20,
                             hs_length=50),
    "auto": dict(check_mode=N.CHECK_AUTO, offset=0, checksum=True, classify=N.CLS_LB_HASH, nports=16),
    "auto-eh-reject-untagged": dict(check_mode=N.CHECK_AUTO, offset=0, checksum=True, classify=N.CLS_LB_HASH,
                                    nports=3, native_vlan=-1, process_eh=True),
    "check-udp": dict(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=4, l4_mode=N.L4_UDP),
    "mark-tcp-nocksum": dict(check_mode=N.MARK_IP4, offset=14, classify=N.CLS_LB_HASH, nports=4,
                             l4_mode=N.L4_TCP, l4_checksum=False),
    "check-rewrite": dict(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=4,
                          rewrite=N.RW_DECTTL | N.RW_SETCKSUM),
    "mark-setcksum": dict(check_mode=N.MARK_IP4, offset=14, classify=N.CLS_LB_HASH, nports=4,
                          rewrite=N.RW_SETCKSUM),
    "auto-qinq": dict(check_mode=N.CHECK_AUTO, offset=0, checksum=True, classify=N.CLS_LB_HASH, nports=5,
                      vlan_ethertype=0x88A8),
    "mark6": dict(check_mode=N.MARK_IP6, offset=14, classify=N.CLS_LB_HASH, nports=8),
    # round 5's per-packet classifiers on the fuzzed frames (the straight-line
    # paths and their declines): hash_crc, the cst_hash_agg ring (LDS and
    # global), hash_ip / chash byte sums; the ring and hash_ip behind CHECK_AUTO
    # (hash_crc hashes IPFlow5ID: IPv4 check modes only)
    "check-lbcrc": dict(offset=14, checksum=True, classify=N.CLS_LB_CRC, nports=16),
    "check-lbtable": dict(offset=14, checksum=True, classify=N.CLS_LB_TABLE, nports=16, lb_ring=1600),
    "check-lbtable-global": dict(offset=14, checksum=True, classify=N.CLS_LB_TABLE, nports=9, lb_ring=70_000),
    "check-haship": dict(offset=14, checksum=True, classify=N.CLS_HASH_IP, nports=8),
    "check-chash": dict(offset=14, checksum=True, classify=N.CLS_HASHSWITCH, nports=11, hs_offset=26, hs_length=12),
    "mark-lbcrc": dict(check_mode=N.MARK_IP4, offset=14, classify=N.CLS_LB_CRC, nports=6),
    "auto-lbtable": dict(check_mode=N.CHECK_AUTO, offset=0, checksum=True, classify=N.CLS_LB_TABLE, nports=12,
                         lb_ring=333),
    "auto-haship": dict(check_mode=N.CHECK_AUTO, offset=0, checksum=True, classify=N.CLS_HASH_IP, nports=4),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CONFIGS))
@pytest.mark.parametrize("seed", [101, 202])
def test_gpu_fuzz_vs_oracle(oracle, name, seed):
    from fastclick_amd import device
    b = fuzz_batch(20_000, seed)
    conf = dict(CONFIGS[name])
    ring = conf.pop("lb_ring", None)
    cfg = N.make_cfg(**conf)
    ring = None if ring is None else N.lb_hash_ring(cfg.nports, ring)
    exp = oracle.process_batch(cfg, b, lb_table=ring)
    for part in (N.PART_GLOBAL, N.PART_TILE):
        got = device.process_batch(b, cfg, anno=True, perm=True, partition=part, lb_table=ring)
        compare(got, exp, ctx=f"fuzz {name} seed={seed} part={part}")
        assert np.array_equal(got["counters"], exp["counters"]), f"fuzz {name}: counters"
        if cfg.rewrite:
            ok = exp["reason"] == N.R_OK
            assert np.array_equal(got["ip_rw"][ok], exp["ip_rw"][ok]), f"fuzz {name}: ip_rw"


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [N.CHECK_IP4, N.MARK_IP4])
def test_gpu_fuzz_flows_vs_oracle(oracle, mode):
    from fastclick_amd import device
    bs = [fuzz_batch(15_000, s) for s in (301, 302, 301)]
    cfg = N.make_cfg(check_mode=mode, offset=14, checksum=mode == N.CHECK_IP4, classify=N.CLS_LB_HASH,
                     nports=4, l4_mode=N.L4_UDP if mode == N.CHECK_IP4 else N.L4_NONE)
    res = device.process_batches(bs, cfg, max_flows=1 << 16, anno=True, perm=False)
    t = oracle.FlowTable(1 << 16)
    for b, r in zip(bs, res):
        e = oracle.process_batch(cfg, b)
        assert np.array_equal(r["reason"], e["reason"])
        assert np.array_equal(r["flowid"], t.batch(b, e))
    assert res[-1]["flow_count"] == t.count()


ELEMENT_CONFS = [
    "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash, BADSRC 192.0.2.255)",
    "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4, LB_MODE hash_ip, L4 UDP)",
    "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 8, DEC_TTL true, SET_CHECKSUM true, HASH FLOW5ID)",
    "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 12, LB_MODE cst_hash_agg, CST_BUCKETS 777)",
    "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE chash)",
]


@pytest.mark.gpu
@pytest.mark.parametrize("conf", ELEMENT_CONFS)
def test_gpu_fuzz_element_compact_vs_full(oracle, conf):
    """The fuzzed frames through the drop-in element: compact staging (the
    default, zero-copy through the shared path) against whole-capture
    staging, and the verdict-derived outputs against the oracle."""
    from fastclick_amd import click as K
    b = fuzz_batch(12_000, 404)
    base = conf[:-1] + ", BATCH 4096, ZEROCOPY true"
    full = K.run_element(base + ", COMPACT false)", b, burst=32, nsinks=17)
    comp = K.run_element(base + ")", b, burst=32, nsinks=17)
    for k in ("port", "seq", "agg", "dst", "len", "nh", "ip8", "batch"):
        assert np.array_equal(full[k], comp[k]), k
    assert full["handlers"] == comp["handlers"]
    cfg = K.element_cfg(conf)
    ring = oracle.lb_hash_ring(cfg.nports, 777).astype(np.uint8) if cfg.classify == N.CLS_LB_TABLE else None
    e = oracle.process_batch(cfg, b, lb_table=ring)
    ok = e["reason"] == N.R_OK
    assert int(comp["handlers"]["drops"]) == int((e["reason"] < N.R_OK).sum())
    assert np.array_equal(comp["agg"][ok], e["hash"][ok])
    assert np.array_equal(comp["port"], e["port"].astype(np.uint32))
