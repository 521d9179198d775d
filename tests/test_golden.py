"""Pin the oracle (and, with -m gpu, the HIP path) to the compiled reference.

Golden vectors in tests/golden/*.npz were produced by the FastClick reference
itself (tests/golden/gen_golden.py; provenance in PROVENANCE.json): CheckIPHeader
verdicts + drop reasons, AggregateHash values, trimmed lengths, FlowSwitch
LB_MODE hash ports (and their per-port order), HashSwitch ports, the
StripEtherVLANHeader/CheckIP6Header/CheckIPHeader mix, and known-answer tests
of click_in_cksum / IPFlowID / IP6FlowID::hashcode compiled from the reference
sources.

Documented exclusion: for non-first IPv4 fragments IPFlowID(const Packet*)
returns before assigning its fields (lib/ipflowid.cc:34-38), so the
reference's AGGREGATE value is uninitialised stack memory; those packets are
excluded from the hash comparison (our definition: the zero flow).
"""
import os

import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NP = 255
BADSRC = [N.raw_addr("192.0.2.255"), N.raw_addr("255.255.255.255")]
GOODDST = [N.raw_addr("10.9.9.9")]


def load(name):
    z = np.load(os.path.join(HERE, f"{name}.npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def batch_of(g):
    return synth.Batch(arena=g["arena"], desc=g["desc"])


def first_fragment_mask(g):
    b = batch_of(g)
    off = b.desc[:, 0].astype(np.int64) + 14
    fo = ((b.arena[off + 6].astype(np.int64) << 8) | b.arena[off + 7]) & 0x1FFF
    return fo == 0


def ip4_cfg(**kw):
    base = dict(offset=14, checksum=True, badsrc=BADSRC, gooddst=GOODDST)
    base.update(kw)
    return N.make_cfg(**base)


def check_ip4(run, g):
    """run(cfg, batch) -> result dict (oracle or device)."""
    b = batch_of(g)
    r = run(ip4_cfg(classify=N.CLS_LB_HASH, nports=16), b)
    assert np.array_equal(r["reason"], g["reason"]), "CheckIPHeader reason"
    ok = g["reason"] == 6
    ff = first_fragment_mask(g)
    assert np.array_equal(r["hash"][ok & ff], g["hash"][ok & ff]), "AggregateHash"
    if "anno" in r:
        assert np.array_equal(r["anno"]["length"][ok], g["length"][ok]), "take() length"
    # non-first fragments: the reference hashes an uninitialised IPFlowID (excluded)
    pinned = (g["lb16"] != NP) & ff
    assert pinned.sum() > 1000
    assert np.array_equal(r["port"][pinned], g["lb16"][pinned]), "FlowSwitch LB_MODE hash port"
    # per-port order of the reference's FlowSwitch outputs == our stable partition order
    start = np.concatenate([[0], np.cumsum(g["lb16_count"].astype(np.int64))])
    for k in range(16):
        ref_order = g["lb16_order"][start[k]:start[k + 1]]
        ref_order = ref_order[ff[ref_order]]
        ours = np.nonzero(pinned & (r["port"] == k))[0]
        assert np.array_equal(ours, np.sort(ref_order)) and np.array_equal(ref_order, np.sort(ref_order))
    # CheckIPHeader() default: CHECKSUM off (elements/ip/checkipheader.cc:110)
    rd = run(N.make_cfg(offset=14), b)
    assert np.array_equal((rd["reason"] == 6).astype(np.uint8), g["valid_default"])
    for m in (4, 7):
        rh = run(ip4_cfg(classify=N.CLS_HASHSWITCH, nports=m, hs_offset=26, hs_length=8), b)
        pin = g[f"hs{m}"] != NP
        assert np.array_equal(rh["port"][pin], g[f"hs{m}"][pin]), f"HashSwitch(26, 8) x{m}"
        # hash_ip (LoadBalancer) is the same byte sum over bytes 26..33
        ri = run(ip4_cfg(classify=N.CLS_HASH_IP, nports=m), b)
        assert np.array_equal(ri["port"][pin], g[f"hs{m}"][pin]), f"LB hash_ip x{m}"


def check_mix(run, g):
    b = batch_of(g)
    r = run(N.make_cfg(check_mode=N.CHECK_AUTO, checksum=True, classify=N.CLS_LB_HASH, nports=16), b)
    assert np.array_equal(r["reason"], g["reason"]), "StripEtherVLANHeader/CheckIP6Header/CheckIPHeader"
    ok = g["reason"] == 6
    if "anno" in r:
        assert np.array_equal(r["anno"]["length"][ok], g["length"][ok])
        assert np.array_equal(r["anno"]["ipver"][g["ipver"] > 0], g["ipver"][g["ipver"] > 0])
    v4 = ok & (g["ipver"] == 4)
    assert np.array_equal(r["hash"][v4], g["hash"][v4]), "AggregateHash (v4 in mix)"
    if bool(g["h6_pinned"]):
        v6 = ok & (g["ipver"] == 6)
        assert np.array_equal(r["hash"][v6], g["hash"][v6]), "IP6FlowID::hashcode"


def check_qinq(run, g):
    """VLANDecap(ETHERTYPE 0x88a8) + Strip(14) ahead of the version dispatch:
    only 802.1ad tags are removed (0x8100-tagged frames fail the checks),
    untagged frames get TCI 0 (NATIVE_VLAN 0 equivalent)."""
    b = batch_of(g)
    r = run(N.make_cfg(check_mode=N.CHECK_AUTO, checksum=True, classify=N.CLS_LB_HASH, nports=16,
                       native_vlan=0, vlan_ethertype=0x88A8), b)
    ok = g["qinq_valid"] == 1
    assert np.array_equal(r["reason"] == N.R_OK, ok), "VLANDecap(ETHERTYPE 0x88a8) verdicts"
    if "anno" in r:
        a = r["anno"]
        assert np.array_equal(a["ipver"][ok], g["qinq_ipver"][ok])
        assert np.array_equal((a["length"].astype(np.int64) - a["nh"])[ok], g["qinq_iplen"][ok])
    v4 = ok & (g["qinq_ipver"] == 4)
    assert np.array_equal(r["hash"][v4], g["qinq_hash"][v4])


def check_mark6(run, g):
    """MarkIP6Header(18 or 14): no validation, th = nh + 40; the IP6FlowID hash
    of the mix set's valid IPv6 packets equals the reference harness's."""
    b = batch_of(g)
    v6 = (g["reason"] == 6) & (g["ipver"] == 6)
    off = b.desc[:, 0].astype(np.int64)
    tagged = b.arena[off + 12] == 0x81
    for o, sel in ((18, v6 & tagged), (14, v6 & ~tagged)):
        r = run(N.make_cfg(check_mode=N.MARK_IP6, offset=o, classify=N.CLS_LB_HASH, nports=16), b)
        assert (r["reason"] == N.R_OK).all()
        if "anno" in r:
            assert (r["anno"]["th"].astype(np.int64) == o + 40).all() and (r["anno"]["ipver"] == 6).all()
        if bool(g["h6_pinned"]):
            assert np.array_equal(r["hash"][sel], g["hash"][sel])


def check_eh(run, g):
    """CheckIP6Header(BADADDRS 2001:db8::bad, PROCESS_EH true|false): verdict,
    IP6_NXT annotation, transport-header offset and trimmed length."""
    import ipaddress
    b = batch_of(g)
    bad6 = [b"\xff" * 16, ipaddress.IPv6Address("2001:db8::bad").packed]
    for tag, eh in (("eh", True), ("noeh", False)):
        cfg = N.make_cfg(check_mode=N.CHECK_AUTO, classify=N.CLS_LB_HASH, nports=4, bad6=bad6, process_eh=eh)
        r = run(cfg, b)
        ok = g[f"{tag}_valid"] == 1
        assert np.array_equal(r["reason"] == N.R_OK, ok), f"{tag}: verdicts"
        assert (r["reason"][~ok] == N.R_BAD_IP6).all()
        if "anno" in r:
            a = r["anno"]
            assert np.array_equal(a["ip6_nxt"][ok], g[f"{tag}_nxt"][ok]), f"{tag}: IP6_NXT"
            assert np.array_equal((a["th"] - a["nh"])[ok], g[f"{tag}_th"][ok]), f"{tag}: transport offset"
            assert np.array_equal(a["length"][ok], g[f"{tag}_length"][ok]), f"{tag}: take() length"
    assert (g["eh_th"][g["eh_valid"] == 1] > 40).sum() > 200


def test_oracle_eh_golden(oracle):
    check_eh(oracle.process_batch, load("eh"))


def test_oracle_ip4_golden(oracle):
    check_ip4(oracle.process_batch, load("ip4"))


def test_oracle_qinq_golden(oracle):
    check_qinq(oracle.process_batch, load("qinq"))


def test_oracle_mark6_mix(oracle):
    check_mark6(oracle.process_batch, load("mix"))


def test_oracle_mix_golden(oracle):
    check_mix(oracle.process_batch, load("mix"))


def test_oracle_known_answers(oracle):
    import ctypes as C
    k = load("kat")
    lib = oracle.load()
    pos = 0
    for ln, exp in zip(k["ck_lens"], k["ck"]):
        data = k["ck_blob"][pos:pos + ln].tobytes()
        pos += int(ln)
        assert oracle.in_cksum(data) == int(exp)
    for t, exp in zip(k["t4"], k["h4"]):
        s, sp, d, dp = (int.from_bytes(t[0:4].tobytes(), "little"), int.from_bytes(t[4:6].tobytes(), "little"),
                        int.from_bytes(t[6:10].tobytes(), "little"), int.from_bytes(t[10:12].tobytes(), "little"))
        assert lib.fco_ipflowid_hash(s, sp, d, dp) == int(exp)
    for t, exp in zip(k["t6"], k["h6"]):
        src = C.create_string_buffer(t[0:16].tobytes(), 16)
        dst = C.create_string_buffer(t[18:34].tobytes(), 16)
        sp = int.from_bytes(t[16:18].tobytes(), "little")
        dp = int.from_bytes(t[34:36].tobytes(), "little")
        assert lib.fco_ip6flowid_hash(src, sp, dst, dp) == int(exp)


def test_reference_harness_kat():
    """kat.npz re-derived from the reference's own lib/in_cksum.c and hash
    headers (oracle/ref/check_kat.py). That build needs the config.h the
    reference's configure writes; without it the KAT is frozen (derived in
    round 1) and this test SKIPS, visibly. The reference-held vectors of
    tests/test_refvectors.py pin A1/A2/A5/A13 independently of it."""
    import subprocess
    import sys
    script = os.path.join(os.path.dirname(HERE), "..", "oracle", "ref", "check_kat.py")
    p = subprocess.run([sys.executable, script], capture_output=True, text=True, timeout=600)
    if p.returncode == 3:
        pytest.skip(p.stdout.strip())
    assert p.returncode == 0, p.stdout + p.stderr


def test_survey_aggregates(oracle):
    """AggregateHash values the survey read from the reference binary."""
    lib = oracle.load()
    cases = [("1.0.0.1", 1234, "2.0.0.2", 5678, 506069210),
             ("10.1.2.3", 53, "192.168.7.9", 40000, 1480824533),
             ("255.255.255.255", 65535, "0.0.0.0", 0, 4294901760)]
    for s, sp, d, dp, h in cases:
        net = lambda p: ((p & 0xFF) << 8) | (p >> 8)  # noqa: E731
        assert lib.fco_ipflowid_hash(N.raw_addr(s), net(sp), N.raw_addr(d), net(dp)) == h


@pytest.mark.gpu
def test_gpu_ip4_golden():
    from fastclick_amd import device
    check_ip4(lambda cfg, b: device.process_batch(b, cfg), load("ip4"))


@pytest.mark.gpu
def test_gpu_eh_golden():
    from fastclick_amd import device
    for part in (N.PART_GLOBAL, N.PART_TILE):
        check_eh(lambda cfg, b: device.process_batch(b, cfg, partition=part), load("eh"))


@pytest.mark.gpu
def test_gpu_qinq_golden():
    from fastclick_amd import device
    check_qinq(lambda cfg, b: device.process_batch(b, cfg), load("qinq"))


@pytest.mark.gpu
def test_gpu_mark6_mix():
    from fastclick_amd import device
    check_mark6(lambda cfg, b: device.process_batch(b, cfg), load("mix"))


@pytest.mark.gpu
def test_gpu_mix_golden():
    from fastclick_amd import device
    check_mix(lambda cfg, b: device.process_batch(b, cfg), load("mix"))


def check_l4(run, g, partitions=(None,)):
    """CheckIPHeader(CHECKSUM true) -> CheckUDPHeader / CheckTCPHeader
    (CHECKSUM true and false): per-packet verdicts of the reference."""
    b = batch_of(g)
    for key, mode in (("udp", N.L4_UDP), ("tcp", N.L4_TCP)):
        for ck in (True, False):
            cfg = N.make_cfg(offset=14, checksum=True, l4_mode=mode, l4_checksum=ck,
                             classify=N.CLS_LB_HASH, nports=4)
            r = run(cfg, b)
            got = np.where(r["reason"] < 6, 255, r["reason"]).astype(np.uint8)
            exp = g[key].copy()
            if not ck:
                exp[exp == N.R_L4_CKSUM] = N.R_OK
            bad = np.nonzero(got != exp)[0]
            assert len(bad) == 0, f"{key} cksum={ck}: {len(bad)} differ, first {bad[:8]} {got[bad[:8]]} {exp[bad[:8]]}"
            ok = exp == N.R_OK
            assert (r["port"][~ok] == 4).all()
    assert (g["udp"] == N.R_L4_CKSUM).sum() > 50 and (g["tcp"] == N.R_L4_CKSUM).sum() > 50


def test_oracle_l4_golden(oracle):
    check_l4(oracle.process_batch, load("l4"))


@pytest.mark.gpu
def test_gpu_l4_golden():
    from fastclick_amd import device
    for part in (N.PART_GLOBAL, N.PART_TILE):
        check_l4(lambda cfg, b: device.process_batch(b, cfg, partition=part), load("l4"))
