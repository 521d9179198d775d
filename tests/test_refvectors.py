"""Parity against vectors the reference's own tests hold (tests/golden/
refvectors.json, written by tests/golden/gen_refvectors.py from the packets
and %expect sections of test/**/*.clicktest; provenance per set).

These pin the SURVEY 8(a) rows with reference-held data, not with fixtures a
locally built `click` produced:
  A1  click_in_cksum   -- every IP header the reference's own elements wrote a
                          checksum into verifies to 0 (oracle), and the HIP path
                          accepts them with CHECKSUM true;
  A2  CheckIPHeader    -- the packets the tests push through CheckIPHeader
                          (options, INTERFACES, OFFSET 0, fragments) are valid;
                          take() trims to ip_len; DST_IP_ANNO;
  A4  MarkIPHeader / IPInputCombo (iprouter's click-xform variant);
  A5  IPFlowID         -- the 5-tuples %expect lists, read after the options
                          (th = nh + hl), hashed by the survey-pinned formula;
  A12 Strip / OFFSET;  A13 StripEtherVLANHeader / VLANDecap(ETHERTYPE): IP
                          offset, VLAN_TCI_ANNO and what is left after the strip;
  L4  CheckTCPHeader   -- the IP-option packets pass with CHECKSUM true.
-m gpu runs the HIP path (and the element, for A13/A4) on the same vectors.
"""
import json
import os

import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def vectors():
    with open(os.path.join(HERE, "refvectors.json")) as f:
        return json.load(f)


def net16(p):
    return ((p & 0xFF) << 8) | (p >> 8)


def flow_hash(oracle, src, sport, dst, dport):
    """IPFlowID::hashcode low 32 (include/click/ipflowid.hh:153-164) through the
    oracle, pinned by SURVEY 0.2's binary values (tests/test_golden.py)."""
    return oracle.load().fco_ipflowid_hash(N.raw_addr(src), net16(sport), N.raw_addr(dst), net16(dport))


def all_headers(v):
    """Every IPv4 header in the set whose checksum the reference wrote (or that
    passes the reference's CheckIPHeader), with its source."""
    out = []
    f = bytes.fromhex(v["iprouter"]["frames"][0])
    out.append((f[14:14 + 20], v["iprouter"]["source"]))
    for c in v["ipfrag"]["cases"]:
        p = bytes.fromhex(c["packet"])
        out.append((p[:(p[0] & 15) * 4], c["src"]))
        for fr in c["fragments"]:
            fb = bytes.fromhex(fr)
            out.append((fb[:(fb[0] & 15) * 4], c["fragments_src"]))
    for h in v["tcpfull"]["headers"]:
        out.append((bytes.fromhex(h), v["tcpfull"]["source"]))
    for h in v["markipce"]["before"] + v["markipce"]["after"]:
        out.append((bytes.fromhex(h), v["markipce"]["source"]))
    for p in v["flow"]["packets"]:      # the flow tests' Print lines (tests/test_flow_reftest.py)
        out.append((bytes.fromhex(p["frame"])[:20], v["flow"]["source"]))
    return out


def test_refvectors_fixture():
    v = vectors()
    assert v["reference_tests_only"] and v["generator"] == "tests/golden/gen_refvectors.py"
    for k in ("iprouter", "ipopt", "vlan", "ipfrag", "tcpfull", "markipce", "flow"):
        assert v[k]["source"].startswith("test/"), k
    assert len(v["ipopt"]["frames"]) == 13 and len(v["vlan"]["cases"]) == 8
    for fr, e in zip(v["ipopt"]["frames"], v["ipopt"]["expect"]):
        b = bytes.fromhex(fr)
        assert len(b) == e["ip_len"] and (b[0] & 15) * 4 == e["hl"]


def test_oracle_reference_checksums(oracle):
    """A1: click_in_cksum over each reference-written header is 0."""
    hs = all_headers(vectors())
    assert len(hs) >= 14
    for h, src in hs:
        assert oracle.in_cksum(h) == 0, src
    # and a corrupted one is not (the check is not vacuous)
    h = bytearray(hs[0][0])
    h[8] ^= 1
    assert oracle.in_cksum(bytes(h)) != 0


# ---- per-set checks: run(cfg, batch) -> result dict (oracle or HIP path) ----

def e_valid(s):
    return s["expect"]["valid"]


def check_iprouter(run, oracle, n=None):
    from fastclick_amd import click as K
    s = vectors()["iprouter"]
    frame = bytes.fromhex(s["frames"][0])
    n = n or s["repeat"]
    assert n <= e_valid(s)
    b = synth.from_frames([frame] * n)
    e = s["expect"]
    h = flow_hash(oracle, e["flow"][0], e["flow"][1], e["flow"][2], e["flow"][3])
    for ck in ("false", "true"):    # CheckIPHeader's default is CHECKSUM false (checkipheader.cc:110)
        cfg = K.element_cfg(f"GPUIPCheckClassify(OFFSET 14, CHECKSUM {ck}, "
                            "INTERFACES 18.26.4.1/24 18.26.7.1/24, N 16, LB_MODE hash)")
        r = run(cfg, b)
        assert (r["reason"] == N.R_OK).all()
        assert int(r["counters"][N.CTR_COUNT]) == n       # %expect: all LIMIT packets counted
        a = r["anno"]
        assert (a["length"] == e["trimmed_len"]).all()
        assert (a["nh"] == 14).all() and (a["th"] == 34).all()
        assert (a["dst_ip"] == N.raw_addr("2.0.0.2")).all()
        assert (r["hash"] == h).all()
        assert (r["port"] == ((h >> 16) ^ (h & 0xFFFF)) % 16).all()


def check_ipopt(run, oracle):
    s = vectors()["ipopt"]
    frames = [bytes.fromhex(f) for f in s["frames"]]
    b = synth.from_frames(frames)
    for ck in (False, True):
        cfg = N.make_cfg(offset=0, checksum=ck, l4_mode=N.L4_TCP, l4_checksum=True,
                         classify=N.CLS_LB_HASH, nports=16)
        r = run(cfg, b)
        assert (r["reason"] == N.R_OK).all(), r["reason"]
        a = r["anno"]
        for i, e in enumerate(s["expect"]):
            assert int(a["th"][i]) == e["hl"] and int(a["nh"][i]) == 0, i
            assert int(a["length"][i]) == e["ip_len"], i
            src, sport, dst, dport, _ = e["flow"]
            assert int(a["dst_ip"][i]) == N.raw_addr(dst)
            assert int(r["hash"][i]) == flow_hash(oracle, src, sport, dst, dport), i
    # a corrupted option byte: the IPv4 checksum (over the options) now fails
    bad = [bytearray(f) for f in frames]
    for f in bad:
        if (f[0] & 15) > 5:
            f[21] ^= 0x40
    r = run(N.make_cfg(offset=0, checksum=True, classify=N.CLS_LB_HASH, nports=16),
            synth.from_frames([bytes(f) for f in bad]))
    hl = np.array([e["hl"] for e in s["expect"]])
    assert np.array_equal(r["reason"] == N.R_BAD_CKSUM, hl > 20)


def vlan_cases():
    return vectors()["vlan"]["cases"]


def check_vlan(run):
    """StripEtherVLANHeader / VLANDecap(ETHERTYPE) + Strip(14) ahead of the
    version dispatch (MODE AUTO): IP offset and TCI as the reference's frames
    say; the 4-byte 'IP packet' left is then too short (a drop)."""
    for c in vlan_cases():
        frame = bytes.fromhex(c["frame"])
        b = synth.from_frames([frame] * 3)
        cfg = N.make_cfg(check_mode=N.CHECK_AUTO, checksum=True, native_vlan=0,
                         vlan_ethertype=c["vlan_ethertype"], classify=N.CLS_LB_HASH, nports=4)
        r = run(cfg, b)
        assert (r["reason"] != N.R_OK).all(), c["src"]
        a = r["anno"]
        assert (a["nh"] == c["ip_off"]).all(), c["src"]
        assert frame[c["ip_off"]:] == bytes.fromhex(c["after"]), c["src"]
        if c["tci"] is not None:
            raw = bytes.fromhex(c["tci"])
            assert (a["vlan_tci"] == raw[0] | raw[1] << 8).all(), c["src"]


def check_ipfrag(run):
    for c in vectors()["ipfrag"]["cases"]:
        p = bytes.fromhex(c["packet"])
        mode = N.MARK_IP4 if c["mode"] == "MarkIPHeader" else N.CHECK_IP4
        r = run(N.make_cfg(offset=0, check_mode=mode, checksum=False, classify=N.CLS_LB_HASH, nports=4),
                synth.from_frames([p]))
        assert r["reason"][0] == N.R_OK, c["src"]
        assert r["anno"]["th"][0] == 24 and r["anno"]["length"][0] == len(p) == 44
        frags = [bytes.fromhex(f) for f in c["fragments"]]
        r = run(N.make_cfg(offset=0, checksum=True, classify=N.CLS_LB_HASH, nports=4), synth.from_frames(frags))
        assert (r["reason"] == N.R_OK).all(), c["fragments_src"]
        assert list(r["anno"]["length"]) == [len(f) for f in frags]
        assert list(r["anno"]["th"]) == [24, 20]


def check_headers_valid(run):
    """tcpfull / markipce headers as packets (header + zero payload up to
    ip_len): CheckIPHeader(OFFSET 0, CHECKSUM true) passes every one."""
    v = vectors()
    pkts = []
    for h in v["tcpfull"]["headers"] + v["markipce"]["before"] + v["markipce"]["after"]:
        hb = bytes.fromhex(h)
        L = int.from_bytes(hb[2:4], "big")
        pkts.append(hb + bytes(L - len(hb)))
    r = run(N.make_cfg(offset=0, checksum=True, classify=N.CLS_LB_HASH, nports=4), synth.from_frames(pkts))
    assert (r["reason"] == N.R_OK).all()


def test_oracle_iprouter(oracle):
    check_iprouter(oracle.process_batch, oracle)


def test_oracle_ipopt(oracle):
    check_ipopt(oracle.process_batch, oracle)


def test_oracle_vlan(oracle):
    check_vlan(oracle.process_batch)


def test_oracle_ipfrag(oracle):
    check_ipfrag(oracle.process_batch)


def test_oracle_headers_valid(oracle):
    check_headers_valid(oracle.process_batch)


def _dev(cfg, b):
    from fastclick_amd import device
    return device.process_batch(b, cfg)


@pytest.mark.gpu
def test_gpu_iprouter(oracle):
    check_iprouter(_dev, oracle)


@pytest.mark.gpu
def test_gpu_ipopt(oracle):
    check_ipopt(_dev, oracle)


@pytest.mark.gpu
def test_gpu_vlan():
    check_vlan(_dev)


@pytest.mark.gpu
def test_gpu_ipfrag():
    check_ipfrag(_dev)


@pytest.mark.gpu
def test_gpu_headers_valid():
    check_headers_valid(_dev)


@pytest.mark.gpu
def test_gpu_element_vlan():
    """The element in MODE AUTO (StripEtherVLANHeader / VLANDecap(ETHERTYPE) +
    Strip ahead of the checks): each reference frame leaves on the drop
    output with the bytes the reference's Print shows after the strip and
    VLAN_TCI_ANNO set from the tag."""
    from fastclick_amd import click as K
    for c in vlan_cases():
        frame = bytes.fromhex(c["frame"])
        b = synth.from_frames([frame] * 5)
        conf = (f"GPUIPCheckClassify(MODE AUTO, CHECKSUM true, N 2, LB_MODE hash, "
                f"VLAN_ETHERTYPE {c['vlan_ethertype']})")
        r = K.run_element(conf, b, nsinks=3)
        assert (r["port"] == 2).all(), c["src"]
        assert (r["len"] == len(bytes.fromhex(c["after"]))).all(), c["src"]
        tci = r["agg"] & 0xFFFF                 # VLAN_TCI_ANNO shares offset 20 with AGGREGATE_ANNO
        want = bytes.fromhex(c["tci"]) if c["tci"] is not None else b"\0\0"
        assert (tci == want[0] | want[1] << 8).all(), c["src"]


@pytest.mark.gpu
def test_gpu_element_iprouter_combo():
    """iprouter-01's chain as the element: Strip(14) -> CheckIPHeader(INTERFACES
    ...) and, for its click-xform variant, IPInputCombo(2) (PAINT 2, CHECKSUM
    true): every packet of the reference's frame leaves on output 0, trimmed
    to 14 + ip_len, painted, and `count` counts them all."""
    from fastclick_amd import click as K
    s = vectors()["iprouter"]
    frame = bytes.fromhex(s["frames"][0])
    n = 60000
    b = synth.from_frames([frame] * n)
    for conf in ("GPUIPCheckClassify(OFFSET 14, INTERFACES 18.26.4.1/24 18.26.7.1/24, STRIP true)",
                 "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, COLOR 2, STRIP true, "
                 "INTERFACES 18.26.4.1/24 18.26.7.1/24)"):
        r = K.run_element(conf, b, nsinks=2)
        assert (r["port"] == 0).all(), conf
        assert (r["len"] == s["expect"]["ip_len"]).all()     # stripped, then take() to ip_len
        assert r["handlers"]["count"] == str(n)
        if "COLOR" in conf:
            assert (r["paint"] == 2).all()
