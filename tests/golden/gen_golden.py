#!/usr/bin/env python3
"""Generate golden vectors from the compiled FastClick reference.

Run here (not on the GPU box): needs a userlevel FastClick build of the
reference tree (configure + make into /tmp/fcbuild, and a
--enable-ctx --enable-flow-dynamic build in /tmp/fcbuild3 for FlowSwitch) and
the reference harness oracle/_ref/fcref (oracle/ref/Makefile). Inputs are
synthetic, deterministic (fastclick_amd.synth, fixed seeds) and written as
pcaps with timestamp = 1000 + packet index, so every reference output line can
be mapped back to its input packet.

Outputs (committed): tests/golden/<set>.npz (inputs + expected outputs, only
data) and tests/golden/PROVENANCE.json (graphs, binary hashes, tool versions).

Per field, the reference mechanism that produced it:
  reason    CheckIPHeader(CHECKSUM true, BADSRC .., GOODDST ..): valid vs port-1
            split from one graph; per-packet reason of every dropped packet from
            a single-packet run of the same element with DETAILS true
            (drop_details handler, elements/ip/checkipheader.cc:241-266)
  hash      AggregateHash -> ToIPSummaryDump(FIELDS timestamp aggregate)
  length    ToDump(ENCAP IP) of the valid packets after Strip(14) (caplen)
  lb16      FlowSwitch(LB_MODE hash) behind CTXManager/CTXDispatcher (fcbuild3)
  hs4/hs7   HashSwitch(26, 8) with 4/7 outputs behind CheckIPHeader(OFFSET 14)
  v6        StripEtherVLANHeader -> Classifier(0/60%f0, -) -> CheckIP6Header /
            CheckIPHeader: verdicts and lengths; IP6FlowID hash from fcref
  reftests  the reference's own classifier tests (test/ip/IPFilter-0[1-7],
            test/standard/Classifier-01): printed programs (asserted equal to
            the text those tests expect), outputs on the prog set, and the
            short-packet cases with their transcribed expectations
  prog      IPClassifier (IPFILTER kind) and Classifier (CLASSIFIER kind)
            behind CheckIPHeader: each element's compiled program as its
            `program` handler prints it, and the output every packet left on
            (none = no rule matched -> NOMATCH)
  cksum/h6  click_in_cksum and IPFlowID/IP6FlowID::hashcode compiled from the
            reference sources by oracle/ref/Makefile (fcref)
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import json
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from fastclick_amd import synth  # noqa: E402

CLICK = os.environ.get("FC_CLICK", "/tmp/fcbuild/userlevel/click")
REFERENCE = os.environ.get("FC_REFERENCE", "/root/reference")
CLICK3 = os.environ.get("FC_CLICK3", "/tmp/fcbuild3/userlevel/click")
# --enable-research --enable-flow --enable-flow-dynamic --enable-ctx build
# (FlowIPManagerHMP lives in elements/research)
CLICK4 = os.environ.get("FC_CLICK4", "/tmp/fcbuild4/userlevel/click")
FCREF = os.path.join(ROOT, "oracle", "_ref", "fcref")
T0 = 1000
BADSRC = "192.0.2.255 255.255.255.255"
GOODDST = "10.9.9.9"
NOT_PINNED = 255


def write_pcap(path, frames):
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        for i, fr in enumerate(frames):
            f.write(struct.pack("<IIII", T0 + i, 0, len(fr), len(fr)))
            f.write(fr)


def read_pcap(path):
    out = {}
    with open(path, "rb") as f:
        data = f.read()
    pos = 24
    while pos + 16 <= len(data):
        ts, _, incl, orig = struct.unpack_from("<IIII", data, pos)
        pos += 16
        out[ts - T0] = (incl, data[pos:pos + incl])
        pos += incl
    return out


def read_ipsum(path, fields):
    rows = {}
    if not os.path.exists(path):
        return rows
    for line in open(path):
        if line.startswith("!") or not line.strip():
            continue
        parts = line.split()
        idx = int(float(parts[0])) - T0
        rows[idx] = parts[1:]
    return rows


def click(binary, cfg, cwd):
    r = subprocess.run([binary, "-e", cfg], cwd=cwd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        raise RuntimeError(f"click failed: {r.stderr[-2000:]}")
    return r.stdout, r.stderr


def reason_of_single(args):
    idx, pcap, chain_prefix, ck_args = args
    with tempfile.TemporaryDirectory() as d:
        frames = read_pcap_frames(pcap)
        write_pcap(os.path.join(d, "one.pcap"), [frames[idx]])
        out, err = click(CLICK, f"FromDump(one.pcap, STOP true, TIMING false) -> {chain_prefix}"
                         f"ck :: CheckIPHeader({ck_args}, DETAILS true) -> Discard; ck[1] -> Discard;"
                         " DriverManager(wait, print ck.drop_details)", d)
    counts = [int(line.split()[0]) for line in out.strip().splitlines()]
    assert len(counts) == 6, out
    if sum(counts) == 0:
        return idx, 6
    assert sum(counts) == 1, (idx, counts)
    return idx, counts.index(1)


_frames_cache = {}


def read_pcap_frames(pcap):
    if pcap not in _frames_cache:
        d = read_pcap(pcap)
        _frames_cache[pcap] = [d[i][1] for i in range(len(d))]
    return _frames_cache[pcap]


def make_ip4_set(n=2400, seed=2024):
    """Untagged IPv4 frames (60..252 B), ~2% of each error kind, IP options on
    15%, non-first fragments on 5%, a few TCP/ICMP protocol numbers."""
    rng = np.random.default_rng(seed)
    fl = synth._rand_flows(rng, n)
    flen = rng.choice([60, 60, 60, 74, 98, 128, 190, 252], n)
    proto = rng.choice([17, 17, 17, 6, 1], n)
    hdr = synth.build_headers(n, **fl, proto=proto, frame_len=flen)
    # a few GOODDST destinations so BADSRC/GOODDST interplay is exercised
    b = synth.pack(hdr, flen, meta=dict(set="ip4", seed=seed))
    synth.add_ip_options(b, 0.15, seed=seed + 1)
    A = b.arena
    frag = rng.random(n) < 0.05
    for i in np.nonzero(frag)[0]:
        o = int(b.desc[i, 0]) + 14
        fo = int(rng.integers(1, 0x1FFF))
        A[o + 6], A[o + 7] = (fo >> 8) & 0x1F, fo & 0xFF
        synth._refresh_cksum(A, o)
    kind = synth.inject_errors(b, 0.02, seed=seed + 2)
    good = rng.random(n) < 0.3
    for i in np.nonzero((kind == synth.ERR_BADSRC) & good)[0]:
        o = int(b.desc[i, 0]) + 14
        A[o + 16:o + 20] = [10, 9, 9, 9]
        synth._refresh_cksum(A, o)
    return b, kind


def make_mix_set(n=1600, seed=2025):
    """C5-style: 50% 802.1Q, 30% IPv6 (some bad/trimmed), IPv4 with errors."""
    b = synth.c5(n, seed=seed)
    rng = np.random.default_rng(seed + 1)
    A = b.arena
    for i in range(b.n):
        off = int(b.desc[i, 0])
        o = off + (18 if A[off + 12] == 0x81 else 14)
        r = rng.random()
        if A[o] >> 4 == 6:
            if r < 0.05:
                A[o + 8:o + 24] = 0xFF
            elif r < 0.10:
                A[o + 4], A[o + 5] = 0x40, 0
            elif r < 0.2:
                A[o + 4], A[o + 5] = 0, int(rng.integers(8, 20))
        else:
            if r < 0.05:
                A[o + 10] ^= 0x10
            elif r < 0.08:
                A[o] = 0x55
    return b


def run_ip4(b, tmp):
    pcap = os.path.join(tmp, "ip4.pcap")
    frames = b.frames()
    write_pcap(pcap, frames)
    n = b.n
    ck_args = f"CHECKSUM true, BADSRC {BADSRC}, GOODDST {GOODDST}"
    cfg = (f"FromDump(ip4.pcap, STOP true, TIMING false) -> Strip(14) -> ck :: CheckIPHeader({ck_args})"
           " -> AggregateHash -> t :: Tee(2); t[0] -> ToIPSummaryDump(good.ipsum, FIELDS timestamp aggregate);"
           " t[1] -> ToDump(good.pcap, ENCAP IP); ck[1] -> ToIPSummaryDump(bad.ipsum, FIELDS timestamp);")
    click(CLICK, cfg, tmp)
    good = read_ipsum(os.path.join(tmp, "good.ipsum"), 1)
    bad = read_ipsum(os.path.join(tmp, "bad.ipsum"), 0)
    dump = read_pcap(os.path.join(tmp, "good.pcap"))
    assert len(good) + len(bad) == n, (len(good), len(bad), n)
    reason = np.full(n, NOT_PINNED, np.uint8)
    hsh = np.zeros(n, np.uint32)
    length = np.zeros(n, np.uint16)
    for i, row in good.items():
        reason[i] = 6
        hsh[i] = int(row[0])
        length[i] = 14 + dump[i][0]
    with cf.ThreadPoolExecutor(8) as ex:
        for i, r in ex.map(reason_of_single, [(i, pcap, "Strip(14) -> ", ck_args) for i in sorted(bad)]):
            reason[i] = r
    # default CheckIPHeader (no CHECKSUM keyword) -> checksum NOT verified
    cfgd = ("FromDump(ip4.pcap, STOP true, TIMING false) -> Strip(14) -> ck :: CheckIPHeader()"
            " -> ToIPSummaryDump(gd.ipsum, FIELDS timestamp); ck[1] -> ToIPSummaryDump(bd.ipsum, FIELDS timestamp);")
    click(CLICK, cfgd, tmp)
    valid_default = np.zeros(n, np.uint8)
    for i in read_ipsum(os.path.join(tmp, "gd.ipsum"), 0):
        valid_default[i] = 1
    # FlowSwitch LB_MODE hash, 16 outputs (fcbuild3: ctx + flow-dynamic). UDP only
    # reaches the switch (CTXDispatcher rule 9/11); others: not pinned.
    lb16 = np.full(n, NOT_PINNED, np.uint8)
    lb16_order = []
    if os.path.exists(CLICK3):
        outs = " ".join(f"fs[{k}] -> ToIPSummaryDump(lb{k}.ipsum, FIELDS timestamp);" for k in range(16))
        cfg3 = (f"FromDump(ip4.pcap, STOP true, TIMING false) -> Strip(14) -> CheckIPHeader({ck_args})"
                " -> CTXManager(BUILDER 1, AGGCACHE false) -> CTXDispatcher(9/11 12/0/ffffffff:HASH-3"
                " 16/0/ffffffff:HASH-3 20/0/ffffffff:HASH-3 0, - drop) -> fs :: FlowSwitch(LB_MODE hash); " + outs)
        click(CLICK3, cfg3, tmp)
        for k in range(16):
            rows = read_ipsum(os.path.join(tmp, f"lb{k}.ipsum"), 0)
            for i in rows:
                lb16[i] = k
            lb16_order.append(list(rows.keys()))
    # HashSwitch(26, 8) on the unstripped frame behind CheckIPHeader(OFFSET 14)
    hs = {}
    for m in (4, 7):
        outs = " ".join(f"hs[{k}] -> ToIPSummaryDump(hs{m}_{k}.ipsum, FIELDS timestamp);" for k in range(m))
        cfgh = (f"FromDump(ip4.pcap, STOP true, TIMING false) -> CheckIPHeader(OFFSET 14, {ck_args})"
                f" -> hs :: HashSwitch(26, 8); " + outs)
        click(CLICK, cfgh, tmp)
        arr = np.full(n, NOT_PINNED, np.uint8)
        for k in range(m):
            for i in read_ipsum(os.path.join(tmp, f"hs{m}_{k}.ipsum"), 0):
                arr[i] = k
        hs[m] = arr
    return dict(reason=reason, hash=hsh, length=length, valid_default=valid_default, lb16=lb16,
                hs4=hs[4], hs7=hs[7],
                lb16_order=np.array([j for k in range(len(lb16_order)) for j in lb16_order[k]], np.uint32),
                lb16_count=np.array([len(x) for x in lb16_order], np.uint32))


def run_mix(b, tmp):
    pcap = os.path.join(tmp, "mix.pcap")
    write_pcap(pcap, b.frames())
    n = b.n
    cfg = ("FromDump(mix.pcap, STOP true, TIMING false) -> StripEtherVLANHeader(0) -> c :: Classifier(0/60%f0, -);"
           " c[0] -> ck6 :: CheckIP6Header -> ToDump(good6.pcap, ENCAP IP); ck6[1] -> ToDump(bad6.pcap, ENCAP IP);"
           " c[1] -> ck4 :: CheckIPHeader(CHECKSUM true) -> AggregateHash -> t :: Tee(2);"
           " t[0] -> ToIPSummaryDump(good4.ipsum, FIELDS timestamp aggregate); t[1] -> ToDump(good4.pcap, ENCAP IP);"
           " ck4[1] -> ToDump(bad4.pcap, ENCAP IP);")
    click(CLICK, cfg, tmp)
    good6 = read_pcap(os.path.join(tmp, "good6.pcap"))
    bad6 = read_pcap(os.path.join(tmp, "bad6.pcap"))
    good4 = read_ipsum(os.path.join(tmp, "good4.ipsum"), 1)
    g4d = read_pcap(os.path.join(tmp, "good4.pcap"))
    bad4 = read_pcap(os.path.join(tmp, "bad4.pcap"))
    assert len(good6) + len(bad6) + len(good4) + len(bad4) == n
    A = b.arena
    off = b.desc[:, 0].astype(np.int64)
    o = np.where(A[off + 12] == 0x81, 18, 14)
    reason = np.full(n, NOT_PINNED, np.uint8)
    length = np.zeros(n, np.uint16)
    hsh = np.zeros(n, np.uint32)
    ipver = np.zeros(n, np.uint8)
    for i, (incl, _) in good6.items():
        reason[i], ipver[i], length[i] = 6, 6, o[i] + incl
    for i in bad6:
        reason[i], ipver[i] = 7, 6
    for i, row in good4.items():
        reason[i], ipver[i], hsh[i], length[i] = 6, 4, int(row[0]), o[i] + g4d[i][0]
    for i in bad4:
        ipver[i] = 4       # reason: single-packet runs below
    todo = sorted(bad4)
    with tempfile.TemporaryDirectory() as d2:
        # re-run each bad IPv4 packet alone for its reason (after the VLAN strip)
        args = [(i, pcap, "StripEtherVLANHeader(0) -> ", "CHECKSUM true") for i in todo]
        with cf.ThreadPoolExecutor(8) as ex:
            for i, r in ex.map(reason_of_single, args):
                reason[i] = r
    # IP6FlowID hashes of valid IPv6 packets: reference harness (header-inline code)
    h6idx = [i for i in good6]
    if h6idx and os.path.exists(FCREF):
        recs = b"".join(_h6_record(A, int(off[i]) + int(o[i])) for i in h6idx)
        out = subprocess.run([FCREF, "flow6"], input=recs, capture_output=True, check=True).stdout
        vals = np.frombuffer(out, np.uint32)
        for i, v in zip(h6idx, vals):
            hsh[i] = v
    return dict(reason=reason, length=length, hash=hsh, ipver=ipver,
                h6_pinned=np.array(bool(h6idx) and os.path.exists(FCREF)))


def _h6_record(A, o):
    th = o + 40
    return (bytes(A[o + 8:o + 24]) + bytes(A[th:th + 2]) + bytes(A[o + 24:o + 40]) + bytes(A[th + 2:th + 4]))


IPC_RULES = ["udp && dst port 53", "tcp && (dst port 80 or dst port 443)", "src net 128.0.0.0/1 && udp",
             "dst port >= 1024 && dst port < 4096", "icmp", "ip frag", "src port > 60000",
             "ip ttl < 10", "ip tos 4"]
CLS_RULES = ["23/11 36/0035", "23/06 !36/0050", "12/0800 23/01", "26/80%c0", "14/46%4f", "30/0a"]
NOMATCH = 254


def make_prog_set(n=3000, seed=2026):
    """IPv4 frames shaped for the classifier rules: popular ports, TCP/UDP/ICMP,
    fragments (first and later), low TTLs, TOS 4, IP options, L4-truncated
    datagrams (short->yes paths) and ~2% invalid headers."""
    rng = np.random.default_rng(seed)
    fl = synth._rand_flows(rng, n)
    fl["dport"] = np.where(rng.random(n) < 0.6,
                           rng.choice([53, 80, 443, 1500, 3000, 4095, 4096, 8080, 7777, 8888, 7000, 137, 5353], n),
                           fl["dport"]).astype(np.uint32)
    r = rng.random(n)
    fl["sport"] = np.where(r < 0.2, rng.integers(59990, 65536, n),
                           np.where(r < 0.25, 68, np.where(r < 0.35, 0x0800, fl["sport"]))).astype(np.uint32)
    r = rng.random(n)
    fl["src"] = np.where(r < 0.05, (128 << 24) | (230 << 16) | (206 << 8) | rng.integers(0, 256, n),
                         np.where(r < 0.08, (2 << 24), fl["src"])).astype(np.uint64)
    fl["dst"] = np.where(rng.random(n) < 0.05, (128 << 24) | (230 << 16) | (206 << 8) | 7,
                         np.where(rng.random(n) < 0.05, 10 << 24, fl["dst"])).astype(np.uint64)
    flen = rng.choice([60, 60, 74, 98, 128, 190], n)
    proto = rng.choice([17, 17, 6, 6, 1, 47], n)
    hdr = synth.build_headers(n, **fl, proto=proto, frame_len=flen)
    b = synth.pack(hdr, flen, meta=dict(set="prog", seed=seed))
    synth.add_ip_options(b, 0.1, seed=seed + 1)
    A = b.arena
    macs = [bytes([0, 1, 2, 3, 4, 5]), bytes([0x10, 0x20, 0x30, 0x40, 0x50, 0x60]), bytes([9, 10, 11, 12, 13, 14]),
            bytes([0, 1, 0, 0, 0, 0])]
    for i in range(n):
        f0 = int(b.desc[i, 0])
        if rng.random() < 0.2:                 # Ethernet addresses for the MAC-offset rules
            A[f0 + 6 * int(rng.integers(0, 2)):][:6] = list(macs[int(rng.integers(0, len(macs)))])
        o = f0 + 14
        hl = int(A[o] & 15) * 4
        if A[o + 9] == 6:                      # TCP flags byte (SYN/ACK rules)
            A[o + hl + 13] = int(rng.choice([0x02, 0x12, 0x10, 0x18, 0x00]))
        r = rng.random()
        if r < 0.05:                       # non-first fragment
            fo = int(rng.integers(1, 0x1FFF))
            A[o + 6], A[o + 7] = (fo >> 8) & 0x1F, fo & 0xFF
        elif r < 0.08:                     # first fragment (MF)
            A[o + 6] |= 0x20
        if rng.random() < 0.1:
            A[o + 8] = int(rng.integers(1, 12))
        if rng.random() < 0.1:
            A[o + 1] = 4
        if rng.random() < 0.04:            # truncate the datagram inside the L4 header
            hl = int(A[o] & 15) * 4
            L = hl + int(rng.integers(0, 4))
            A[o + 2], A[o + 3] = L >> 8, L & 0xFF
        synth._refresh_cksum(A, o)
    kind = synth.inject_errors(b, 0.02, seed=seed + 2)
    return b, kind


def _program_of(out):
    lines = out.splitlines()
    k = max(i for i, l in enumerate(lines) if l.startswith("alignment offset"))
    j = k
    while j > 0 and (lines[j - 1].startswith(" ") or lines[j - 1][:1].isdigit()
                     or lines[j - 1].startswith("safe length") or lines[j - 1].startswith("all->")):
        j -= 1
    return "\n".join(lines[j:k + 1]) + "\n"


def run_prog(b, tmp):
    pcap = os.path.join(tmp, "prog.pcap")
    write_pcap(pcap, b.frames())
    n = b.n
    res = {}
    for name, elem, rules, pre in (("ipc", "IPClassifier", IPC_RULES, "Strip(14) -> CheckIPHeader(CHECKSUM true)"),
                                   ("cls", "Classifier", CLS_RULES, "CheckIPHeader(OFFSET 14, CHECKSUM true)")):
        m = len(rules)
        outs = " ".join(f"c[{k}] -> ToIPSummaryDump({name}{k}.ipsum, FIELDS timestamp);" for k in range(m))
        cfg = (f"FromDump(prog.pcap, STOP true, TIMING false) -> {pre} -> c :: {elem}({', '.join(rules)}); "
               f"{outs} DriverManager(wait, print c.program)")
        # invalid headers leave the checker on its port 1
        cfg = cfg.replace("CheckIPHeader(", "chk :: CheckIPHeader(", 1) + "; chk[1] -> ToIPSummaryDump(" \
            + f"{name}bad.ipsum, FIELDS timestamp);"
        out, _ = click(CLICK, cfg, tmp)
        prog = _program_of(out)
        got = np.full(n, NOMATCH, np.uint8)
        for k in range(m):
            for i in read_ipsum(os.path.join(tmp, f"{name}{k}.ipsum"), 0):
                got[i] = k
        for i in read_ipsum(os.path.join(tmp, f"{name}bad.ipsum"), 0):
            got[i] = 255
        res[f"{name}_out"] = got
        res[f"{name}_prog"] = np.frombuffer(prog.encode(), np.uint8)
        res[f"{name}_nout"] = np.array(m)
    return res


# Programs the reference's own tests pin (test/ip/IPFilter-0[4-7].clicktest,
# test/standard/Classifier-01.clicktest): (case, test file, element config,
# kind, number of outputs, path in front of the element). The printed program
# must equal the text the test expects; the outputs on the prog set come from
# the same compiled reference.
REFTEST_PROGRAMS = [
    ("IPFilter-04.c", "test/ip/IPFilter-04.clicktest",
     "IPClassifier(dst port 7777, dst port 8888, dst port 7000, icmp type echo, icmp, -)", "ipf", 6),
    ("IPFilter-04.d", "test/ip/IPFilter-04.clicktest",
     "IPFilter(0 udp dst port netbios-ns, 1 udp dst port 5353, 2 udp src port bootpc, 3 128.230.206.0/24, 4 -)",
     "ipf", 5),
    ("IPFilter-04.e", "test/ip/IPFilter-04.clicktest",
     "IPClassifier(proto icmp, dst port 53, (proto tcp and !(syn and !ack)) or (tcpudp port >= 1024), -)", "ipf", 4),
    ("IPFilter-05", "test/ip/IPFilter-05.clicktest",
     "IPFilter(allow tcp && dst 10.0.0.0/32 && src 2.0.0.0/32, allow tcp && dst 10.0.0.0/32 && dst port 80 "
     "&& src 2.0.0.0/32, allow all)", "ipf", 1),
    ("IPFilter-06", "test/ip/IPFilter-06.clicktest",
     "IPFilter(allow src 0:1:2:3:4:5, allow src 10.0.0.0 & 8.0.0.0 = 8.0.0.0, allow dst 10:20:30:40:50:60, "
     "allow host 9:A:B:C:D:E, deny all)", "ipf", 1),
    ("IPFilter-07.1", "test/ip/IPFilter-07.clicktest", "IPFilter(allow false)", "ipf", 1),
    ("IPFilter-07.2", "test/ip/IPFilter-07.clicktest", "IPFilter(allow false, allow false, allow false, allow true)",
     "ipf", 1),
    ("IPFilter-07.3", "test/ip/IPFilter-07.clicktest", "IPFilter(allow false, allow false, allow src 10.0.0.1)",
     "ipf", 1),
    ("IPFilter-07.5", "test/ip/IPFilter-07.clicktest", "IPFilter()", "ipf", 1),
    ("Classifier-01", "test/standard/Classifier-01.clicktest", "Classifier(1/01, -)", "cls", 2),
    # test/standard/Classifier-02.clicktest: the empty program (every packet to
    # output 0); that test holds no program text to compare with
    ("Classifier-02", None, "Classifier(-)", "cls", 1),
]
# The survey's CPU classifier benchmark ("+ IPClassifier with 16
# dst-port-range rules -> 16 ports"): 15 UDP dst-port ranges of 4096 + "-".
IPCLASS16 = ("IPClassifier(" + ", ".join(f"dst udp port >= {i * 4096} and dst udp port < {(i + 1) * 4096}"
                                         for i in range(15)) + ", -)")
BENCH_PROGRAMS = [("ipclass16", None, IPCLASS16, "ipf", 16)]

# Short-packet behaviour the reference's tests pin (IPFilter-01/02/03/08):
# FromIPSummaryDump(IN) -> PaintSwitch; branch k goes through `chain` into
# filter `f`. Expected outputs transcribed from each test's %expect section
# (X = dropped). Every packet is captured from the reference as it enters the
# filter (ToDump), with its network-header offset.
SHORT_IN_1 = "!data link timestamp sport\n" + "".join(f"{k} {2 * k + 1} 0\n" for k in range(8))
SHORT_IN_2 = "!data link timestamp sport\n" + "".join(f"{k // 2} {k + 1} {128 * (k % 2)}\n" for k in range(8))
SHORT_IN_3 = "!data link timestamp sport\n" + "".join(f"{k // 2} {k + 1} {128 * (k % 2)}\n" for k in range(4))
ETH = "EtherEncap(0x0800, 1:1:1:1:1:1, 2:2:2:2:2:2)"
SHORT_CASES = [
    ("IPFilter-01", "test/ip/IPFilter-01.clicktest:9-35", SHORT_IN_1,
     {"f0": "IPFilter(0 ip[19]&128==0)", "f1": "IPFilter(0 transp[1]&128==0)"},
     [("", "f0"), ("", "f1"), (ETH, "f0"), (ETH, "f1"), ("Truncate(19)", "f0"), ("Truncate(21)", "f1"),
      (f"Truncate(19) -> {ETH}", "f0"), (f"Truncate(21) -> {ETH}", "f1")],
     # A: 1, B: 3, A: 5, B: 7 pass; the truncated 9..15 are dropped
     {"f0": {1: 0, 5: 0, 9: "X", 13: "X"}, "f1": {3: 0, 7: 0, 11: "X", 15: "X"}}),
    ("IPFilter-02", "test/ip/IPFilter-02.clicktest:9-39", SHORT_IN_2,
     {"f0": "IPFilter(0 transp[1]&128==0, 1 -)", "f1": "IPFilter(0 transp[1]&128!=0, 1 -)",
      "fx": "IPFilter(0 transp[1]&128==0 || transp[1]&128==128)"},
     [("", "f0"), ("", "f1"), ("Truncate(21)", "f0"), ("Truncate(21)", "f1")],
     # A: 1 / B: 4 / C: 1 2 3 4; f0[1], f1[1] feed fx, which drops 5..8
     {"f0": {1: 0, 2: 1, 5: 1, 6: 1}, "f1": {3: 1, 4: 0, 7: 1, 8: 1},
      "fx": {1: 0, 2: 0, 3: 0, 4: 0, 5: "X", 6: "X", 7: "X", 8: "X"}}),
    ("IPFilter-03", "test/ip/IPFilter-03.clicktest:9-30", SHORT_IN_3,
     {"f0": "IPFilter(0 transp[1]&128!=0, 1 -)", "f1": "IPFilter(0 not (transp[1]&128==0))"},
     [("", "f0"), ("Truncate(21)", "f0")],
     # A: 2 / B: 2 3 4 (f0's output 1 feeds f1)
     {"f0": {1: 1, 2: 0, 3: 1, 4: 1}, "f1": {1: "X", 2: 0, 3: 0, 4: 0}}),
]


def _clicktest_text(rel):
    path = os.path.join(REFERENCE, rel)
    return open(path).read() if os.path.exists(path) else None


def _print_program(conf, nout):
    outs = " ".join(f"c[{k}] -> Idle;" for k in range(nout))
    r = subprocess.run([CLICK, "-e", f"Idle -> c :: {conf}; {outs}", "-qh", "c.program"],
                       capture_output=True, text=True, timeout=60)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    return r.stdout


def run_reftests(b, tmp):
    """Reference-test programs on the prog set + the short-packet cases."""
    pcap = os.path.join(tmp, "prog.pcap")
    write_pcap(pcap, b.frames())
    n = b.n
    out = {"programs": [], "short": []}
    for case, rel, conf, kind, nout in REFTEST_PROGRAMS + BENCH_PROGRAMS:
        prog = _print_program(conf, nout)
        text = _clicktest_text(rel) if rel else None
        if text is not None:
            want = prog.replace("[2147483647]", "[{{2147483647|X}}]")
            assert want in text, f"{case}: printed program differs from {rel}:\n{prog}"
        pre = ("Strip(14) -> chk :: CheckIPHeader(CHECKSUM true)" if kind == "ipf" and case != "IPFilter-06"
               else "chk :: CheckIPHeader(OFFSET 14, CHECKSUM true)")
        outs = " ".join(f"c[{k}] -> ToIPSummaryDump(rt{k}.ipsum, FIELDS timestamp);" for k in range(nout))
        for k in [*range(nout), "bad"]:
            if os.path.exists(os.path.join(tmp, f"rt{k}.ipsum")):
                os.remove(os.path.join(tmp, f"rt{k}.ipsum"))
        click(CLICK, f"FromDump(prog.pcap, STOP true, TIMING false) -> {pre} -> c :: {conf}; {outs} "
                     "chk[1] -> ToIPSummaryDump(rtbad.ipsum, FIELDS timestamp);", tmp)
        got = np.full(n, NOMATCH, np.int64)
        for k in range(nout):
            for i in read_ipsum(os.path.join(tmp, f"rt{k}.ipsum"), 0):
                got[i] = k
        for i in read_ipsum(os.path.join(tmp, "rtbad.ipsum"), 0):
            got[i] = 255
        out["programs"].append(dict(case=case, test=rel, config=conf, kind=kind, nout=nout,
                                    program=prog, outputs=got.tolist()))
    for case, rel, infile, filters, routes, expect in SHORT_CASES:
        d = os.path.join(tmp, case)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "IN"), "w") as f:
            f.write(infile)
        graph = ["FromIPSummaryDump(IN, STOP true) -> ps :: PaintSwitch;"]
        for k, (chain, _) in enumerate(routes):
            enc = "ETHER" if "EtherEncap" in chain else "IP"
            graph.append(f"ps[{k}] -> {chain + ' -> ' if chain else ''}ToDump(p{k}.pcap, ENCAP {enc});")
        click(CLICK, " ".join(graph), d)
        pkts = []
        for k, (chain, fname) in enumerate(routes):
            for ts_idx, (incl, data) in sorted(read_pcap(os.path.join(d, f"p{k}.pcap")).items()):
                ts = ts_idx + T0
                pkts.append(dict(ts=ts, filter=fname, nh=14 if "EtherEncap" in chain else 0,
                                 bytes=data.hex()))
        # fx in IPFilter-02 and f1 in IPFilter-03 also see the other filters' outputs
        feeds = {"IPFilter-02": {"fx": ["f0", "f1"]}, "IPFilter-03": {"f1": ["f0"]}}.get(case, {})
        for tgt, srcs in feeds.items():
            for p in list(pkts):
                if p["filter"] in srcs:
                    pkts.append(dict(p, filter=tgt))
        progs = {fn: _print_program(conf, 2 if ", 1 -" in conf else 1) for fn, conf in filters.items()}
        # the reference itself on each captured packet (must equal the test's expectation)
        for p in pkts:
            exp = expect[p["filter"]].get(p["ts"])
            if exp is None:
                continue
            p["expect"] = exp
        out["short"].append(dict(case=case, test=rel, filters=filters, programs=progs,
                                 packets=[p for p in pkts if "expect" in p]))
    return out


def run_combo(tmp):
    """IPInputCombo(COLOR 7, BADSRC .., GOODDST ..) on the ip4 set: which
    packets survive (it kills the rest) with their length, paint and dst anno
    (ipinputcombo.cc:65-141)."""
    g = np.load(os.path.join(HERE, "ip4.npz"))
    b = synth.Batch(arena=g["arena"], desc=g["desc"])
    pcap = os.path.join(tmp, "combo.pcap")
    write_pcap(pcap, b.frames())
    click(CLICK, f"FromDump(combo.pcap, STOP true, TIMING false) -> IPInputCombo(7, BADSRC {BADSRC}, "
                 f"GOODDST {GOODDST}) -> ToIPSummaryDump(combo.ipsum, FIELDS timestamp ip_len ip_dst)"
                 " -> Discard;", tmp)
    rows = read_ipsum(os.path.join(tmp, "combo.ipsum"), 2)
    n = b.n
    valid = np.zeros(n, np.uint8)
    iplen = np.zeros(n, np.uint16)
    for i, r in rows.items():
        valid[i] = 1
        iplen[i] = int(r[0])
    return dict(valid=valid, ip_len=iplen)


BAD6_EXTRA = "2001:db8::bad"


def make_eh_set(n=1200, seed=2027):
    """Untagged IPv6 frames with chains of 0-3 extension headers (hop-by-hop,
    routing, fragment, AH, destination options, no-next-header), UDP/TCP after
    them; payload lengths exact, short (take) or too long (bad); frames cut
    inside the chain; bad sources (ff..ff and BADSRC6)."""
    import ipaddress
    rng = np.random.default_rng(seed)
    frames = []
    bad_extra = ipaddress.IPv6Address(BAD6_EXTRA).packed
    for i in range(n):
        chain = b""
        k = int(rng.integers(0, 4))
        types = [int(rng.choice([0, 43, 44, 51, 60, 59])) for _ in range(k)]
        last = int(rng.choice([17, 6]))
        nxts = types + [last]
        for j, t in enumerate(types):
            nx = nxts[j + 1]
            if t in (0, 43, 60):
                ln = int(rng.integers(0, 3))
                body = bytes([nx, ln]) + bytes(rng.integers(0, 256, ln * 8 + 6, dtype=np.uint8))
            elif t == 51:
                ln = int(rng.integers(1, 7))
                size = ((ln + 2) * 4 + 7) // 8 * 8
                body = bytes([nx, ln]) + bytes(rng.integers(0, 256, size - 2, dtype=np.uint8))
            elif t == 44:
                body = bytes([nx, 0]) + bytes(rng.integers(0, 256, 6, dtype=np.uint8))
            else:   # 59: no next header; whatever follows is payload
                body = bytes(rng.integers(0, 256, 8, dtype=np.uint8))
            chain += body
        l4 = bytes(rng.integers(0, 256, 8 + int(rng.integers(0, 24)), dtype=np.uint8))
        payload = chain + l4
        pl6 = len(payload)
        r = rng.random()
        if r < 0.1:
            pl6 -= int(rng.integers(1, min(pl6, 16) + 1))      # take() trims
        elif r < 0.15:
            pl6 += int(rng.integers(1, 9))                      # longer than the packet: bad
        src = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
        r = rng.random()
        if r < 0.03:
            src = b"\xff" * 16
        elif r < 0.06:
            src = bad_extra
        hdr = bytes([0x60, 0, 0, 0]) + pl6.to_bytes(2, "big") + bytes([nxts[0], 64]) + src + \
            bytes(rng.integers(0, 256, 16, dtype=np.uint8))
        eth = bytes([2, 0, 0, 0, 0, 2, 2, 0, 0, 0, 0, 1, 0x86, 0xDD])
        fr = eth + hdr + payload
        if rng.random() < 0.12:                                  # cut inside the chain
            fr = bytearray(fr[:14 + 40 + int(rng.integers(0, max(len(chain), 1) + 1))])
            if rng.random() < 0.8:                               # ... with a payload length that fits
                rem = len(fr) - 54
                fr[18:20] = int(rng.integers(0, rem + 1)).to_bytes(2, "big")
            fr = bytes(fr)
        frames.append(fr)
    return synth.from_frames(frames, meta=dict(set="eh", seed=seed))


def run_eh(b, tmp):
    pcap = os.path.join(tmp, "eh.pcap")
    write_pcap(pcap, b.frames())
    n = b.n
    res = {}
    for eh in (True, False):
        tag = "eh" if eh else "noeh"
        outs = " ".join(f"ps[{k}] -> ToIPSummaryDump({tag}_nxt{k}.ipsum, FIELDS timestamp);" for k in range(61))
        cfg = (f"FromDump(eh.pcap, STOP true, TIMING false) -> Strip(14) -> c6 :: CheckIP6Header("
               f"BADADDRS {BAD6_EXTRA}, PROCESS_EH {str(eh).lower()}) -> t :: Tee(3); "
               f"t[0] -> ToDump({tag}_full.pcap, ENCAP IP); t[1] -> StripIPHeader -> ToDump({tag}_tp.pcap, ENCAP IP); "
               f"t[2] -> ps :: PaintSwitch(ANNO 16); {outs} c6[1] -> ToIPSummaryDump({tag}_bad.ipsum, FIELDS timestamp);")
        click(CLICK, cfg, tmp)
        full = read_pcap(os.path.join(tmp, f"{tag}_full.pcap"))
        tp = read_pcap(os.path.join(tmp, f"{tag}_tp.pcap"))
        bad = read_ipsum(os.path.join(tmp, f"{tag}_bad.ipsum"), 0)
        valid = np.zeros(n, np.uint8)
        length = np.zeros(n, np.uint16)
        thoff = np.zeros(n, np.uint16)
        nxt = np.full(n, 255, np.uint8)
        for i, (incl, _) in full.items():
            valid[i] = 1
            length[i] = 14 + incl
            thoff[i] = incl - tp[i][0]
        for k in range(61):
            for i in read_ipsum(os.path.join(tmp, f"{tag}_nxt{k}.ipsum"), 0):
                nxt[i] = k
        assert len(full) + len(bad) == n
        res.update({f"{tag}_valid": valid, f"{tag}_length": length, f"{tag}_th": thoff, f"{tag}_nxt": nxt})
    return res


def _csum16(data: bytes) -> int:
    if len(data) % 2:
        data += b"\0"
    s = int(np.frombuffer(data, ">u2").astype(np.uint64).sum()) if data else 0
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def make_l4_set(n=3000, seed=2028):
    """IPv4 frames for CheckUDPHeader / CheckTCPHeader: UDP/TCP/ICMP/GRE,
    payloads 0..1460 B (odd lengths included), IP options incl. LSRR/SSRR (the
    pseudo-header then uses the route's final destination), correct L4
    checksums, then: corrupted payload bytes, UDP checksum 0, bad uh_ulen,
    UDP shorter than the IP payload, bad TCP data offsets, trailing padding,
    and frames cut short (IP check fails first)."""
    rng = np.random.default_rng(seed)
    frames = []
    for i in range(n):
        proto = int(rng.choice([17, 17, 17, 6, 6, 6, 1, 47]))
        plen = int(rng.choice([0, 1, 7, 18, 33, 100, 257, 512, 999, 1400, 1460]))
        payload = bytes(rng.integers(0, 256, plen, dtype=np.uint8))
        src = bytes(rng.integers(0, 256, 4, dtype=np.uint8))
        dst = bytes(rng.integers(0, 256, 4, dtype=np.uint8))
        opts = b""
        final = dst
        r = rng.random()
        if r < 0.06:                         # LSRR / SSRR with 1-2 hops
            hops = int(rng.integers(1, 3))
            route = bytes(rng.integers(0, 256, 4 * hops, dtype=np.uint8))
            kind = int(rng.choice([131, 137]))
            opts = bytes([1, kind, 3 + 4 * hops, 4]) + route
            final = route[-4:]
        elif r < 0.12:                       # record route / NOPs (dst unchanged)
            opts = bytes([1, 1, 7, 7, 4]) + bytes(4) + bytes([0])
        elif r < 0.14:                       # malformed option length: scan stops
            opts = bytes([131, 1, 0, 0])
        while len(opts) % 4:
            opts += b"\0"
        hl = 20 + len(opts)
        if proto == 17:
            ulen = 8 + plen
            l4 = bytearray(rng.integers(0, 256, 2, dtype=np.uint8).tobytes() +
                           rng.integers(0, 256, 2, dtype=np.uint8).tobytes() + ulen.to_bytes(2, "big") + b"\0\0") + payload
        elif proto == 6:
            l4 = bytearray(rng.integers(0, 256, 12, dtype=np.uint8).tobytes()) + bytearray(8) + payload
            l4[12] = 5 << 4
            l4[13] = int(rng.choice([0x02, 0x10, 0x18]))
        else:
            l4 = bytearray(8) + payload
        L = hl + len(l4)
        ph = src + final + bytes([0, proto]) + len(l4).to_bytes(2, "big")
        if proto in (17, 6):
            ck = (~_csum16(ph + bytes(l4))) & 0xFFFF
            if proto == 17 and ck == 0:
                ck = 0xFFFF
            pos = 6 if proto == 17 else 16
            l4[pos:pos + 2] = ck.to_bytes(2, "big")
        ip = bytearray([0x40 | (hl // 4), 0]) + L.to_bytes(2, "big") + bytes(rng.integers(0, 256, 2, dtype=np.uint8)) + \
            bytes([0, 0, 64, proto, 0, 0]) + src + dst + opts
        r = rng.random()
        tail = b""
        if r < 0.08 and len(l4) > 8:         # corrupt one L4 byte (checksum now bad)
            j = int(rng.integers(0, len(l4)))
            l4[j] ^= 1 << int(rng.integers(0, 8))
        elif r < 0.13 and proto == 17:       # checksum 0: not verified
            l4[6:8] = b"\0\0"
            if len(l4) > 8:
                l4[int(rng.integers(8, len(l4)))] ^= 0xFF
        elif r < 0.16 and proto == 17:       # bad uh_ulen
            l4[4:6] = int(rng.choice([0, 7, len(l4) + 1, len(l4) + 100])).to_bytes(2, "big")
        elif r < 0.19 and proto == 17 and plen > 4:   # UDP shorter than the IP payload (valid checksum)
            short = 8 + plen - int(rng.integers(1, 5))
            l4[4:6] = short.to_bytes(2, "big")
            l4[6:8] = b"\0\0"
            ph2 = src + final + bytes([0, 17]) + short.to_bytes(2, "big")
            ck = (~_csum16(ph2 + bytes(l4[:short]))) & 0xFFFF
            l4[6:8] = (ck or 0xFFFF).to_bytes(2, "big")
        elif r < 0.22 and proto == 6:        # bad TCP data offset
            l4[12] = int(rng.choice([0, 4, 15])) << 4
        elif r < 0.26:                       # trailing padding (trimmed by CheckIPHeader)
            tail = bytes(rng.integers(0, 256, int(rng.integers(1, 20)), dtype=np.uint8))
        ip[10:12] = b"\0\0"
        ip[10:12] = ((~_csum16(bytes(ip))) & 0xFFFF).to_bytes(2, "big")
        eth = bytes([2, 0, 0, 0, 0, 2, 2, 0, 0, 0, 0, 1, 8, 0])
        fr = eth + bytes(ip) + bytes(l4) + tail
        if rng.random() < 0.02:              # cut: the IP check drops it
            fr = fr[:len(fr) - int(rng.integers(1, 8))]
        frames.append(fr)
    return synth.from_frames(frames, meta=dict(set="l4", seed=seed))


def run_l4(b, tmp):
    """Per packet and element (UDP, TCP): 255 = CheckIPHeader dropped it, 6 =
    passed, 10 NOT_UDP/NOT_TCP, 11 BAD_LENGTH, 12 BAD_CHECKSUM (a second run
    with CHECKSUM false separates length from checksum failures)."""
    pcap = os.path.join(tmp, "l4.pcap")
    write_pcap(pcap, b.frames())
    n = b.n
    A = b.arena
    proto = np.array([A[int(o) + 14 + 9] for o in b.desc[:, 0]])
    res = {}
    for el, want in (("CheckUDPHeader", 17), ("CheckTCPHeader", 6)):
        verdict = {}
        for ck in (True, False):
            tag = f"{el}_{int(ck)}"
            click(CLICK, f"FromDump(l4.pcap, STOP true, TIMING false) -> Strip(14) -> ip :: CheckIPHeader(CHECKSUM true) "
                         f"-> c :: {el}(CHECKSUM {str(ck).lower()}) -> ToIPSummaryDump({tag}_ok.ipsum, FIELDS timestamp); "
                         f"c[1] -> ToIPSummaryDump({tag}_bad.ipsum, FIELDS timestamp); "
                         f"ip[1] -> ToIPSummaryDump({tag}_ipbad.ipsum, FIELDS timestamp);", tmp)
            v = np.zeros(n, np.uint8)
            for i in read_ipsum(os.path.join(tmp, f"{tag}_ok.ipsum"), 0):
                v[i] = 1
            for i in read_ipsum(os.path.join(tmp, f"{tag}_bad.ipsum"), 0):
                v[i] = 2
            for i in read_ipsum(os.path.join(tmp, f"{tag}_ipbad.ipsum"), 0):
                v[i] = 3
            assert (v > 0).all()
            verdict[ck] = v
        out = np.full(n, 255, np.uint8)
        v1, v0 = verdict[True], verdict[False]
        out[v1 == 1] = 6
        bad = v1 == 2
        out[bad & (proto != want)] = 10
        out[bad & (proto == want) & (v0 == 2)] = 11
        out[bad & (proto == want) & (v0 == 1)] = 12
        assert (out[v1 == 3] == 255).all()
        res["udp" if want == 17 else "tcp"] = out
    return res


def make_flow_set(n=4000, nflows=300, seed=2029):
    """IPv4 frames drawn from a pool of 5-tuples with a skewed popularity, so
    flows repeat within and across batches: UDP/TCP/ICMP, the same address and
    port pair under different protocols (distinct IPFlow5IDs), swapped
    directions (distinct too), IP options (ports after the options), first
    fragments (MF set, offset 0), and ~1.5% of each CheckIPHeader error kind
    (those never reach the flow manager). Non-first fragments are left out:
    the reference hashes their uninitialised ports (lib/ipflowid.cc:34-38)."""
    rng = np.random.default_rng(seed)
    pool = synth._rand_flows(rng, nflows)
    proto_pool = rng.choice([17, 17, 6, 6, 1], nflows)
    # tuples that differ only by protocol or by direction
    for j in range(0, nflows // 10):
        a, b = 2 * j, 2 * j + 1
        for k in ("src", "dst", "sport", "dport"):
            pool[k][b] = pool[k][a]
        proto_pool[b] = 6 if proto_pool[a] == 17 else 17
    for j in range(nflows // 10, nflows // 5):
        a, b = 2 * j, 2 * j + 1
        pool["src"][b], pool["dst"][b] = pool["dst"][a], pool["src"][a]
        pool["sport"][b], pool["dport"][b] = pool["dport"][a], pool["sport"][a]
        proto_pool[b] = proto_pool[a]
    w = 1.0 / (1 + np.arange(nflows)) ** 0.8
    pick = rng.choice(nflows, n, p=w / w.sum())
    fl = {k: v[pick] for k, v in pool.items()}
    flen = rng.choice([60, 60, 60, 74, 98, 128], n)
    hdr = synth.build_headers(n, **fl, proto=proto_pool[pick], frame_len=flen)
    b = synth.pack(hdr, flen, meta=dict(set="flow", seed=seed))
    synth.add_ip_options(b, 0.1, seed=seed + 1)
    A = b.arena
    for i in np.nonzero(rng.random(n) < 0.05)[0]:          # first fragments (MF, offset 0)
        o = int(b.desc[i, 0]) + 14
        A[o + 6] |= 0x20
        synth._refresh_cksum(A, o)
    kind = synth.inject_errors(b, 0.015, seed=seed + 2, kinds=range(5))
    return b, kind, pick


def run_flow(b, tmp):
    """FlowIPManagerHMP -> StoreFlowID(OFFSET 0) on the checked stream: the
    8-byte ID StoreFlowID writes is 1 + the HMP flow ID (both count new flows in
    arrival order on one thread, storeflowid.cc:60-67); packets CheckIPHeader
    drops get FCGPU_FLOW_NONE."""
    if not os.path.exists(CLICK4):
        return None
    pcap = os.path.join(tmp, "flow.pcap")
    write_pcap(pcap, b.frames())
    click(CLICK4, "FromDump(flow.pcap, STOP true, TIMING false) -> Strip(14) -> CheckIPHeader(CHECKSUM true) "
                  "-> FlowIPManagerHMP(CAPACITY 65536) -> StoreFlowID(OFFSET 0) -> ToDump(flow_out.pcap);", tmp)
    got = read_pcap(os.path.join(tmp, "flow_out.pcap"))
    fid = np.full(b.n, 0xFFFFFFFF, np.uint32)
    for i, (_, data) in got.items():
        fid[i] = int.from_bytes(data[0:8], "little") - 1
    return dict(flowid=fid)


def make_rw_set(n=3000, seed=2030):
    """IPv4 frames for DecIPTTL / SetIPChecksum: TTL 0, 1, 2, random, 255;
    multicast destinations (224.0.0.0/4) on ~10%; IP options on 10%; ~2% bad
    checksums (CheckIPHeader drops them); and, for the MarkIPHeader ->
    SetIPChecksum run, ~3% of headers that do not fit (hl < 5 words, hl past
    the frame, frames cut inside the header)."""
    rng = np.random.default_rng(seed)
    fl = synth._rand_flows(rng, n)
    mc = rng.random(n) < 0.1
    mdst = ((0xE0 + rng.integers(0, 16, n, dtype=np.uint64)) << np.uint64(24)) | (fl["dst"] & np.uint64(0xFFFFFF))
    fl["dst"] = np.where(mc, mdst, fl["dst"])
    flen = rng.choice([60, 60, 74, 98, 128], n)
    hdr = synth.build_headers(n, **fl, frame_len=flen)
    b = synth.pack(hdr, flen, meta=dict(set="rw", seed=seed))
    synth.add_ip_options(b, 0.1, seed=seed + 1)
    A = b.arena
    ttl = rng.choice([0, 1, 2, 3, 64, 128, 255], n, p=[0.05, 0.05, 0.05, 0.05, 0.4, 0.2, 0.2])
    ttl = np.where(rng.random(n) < 0.3, rng.integers(0, 256, n), ttl)
    for i in range(n):
        o = int(b.desc[i, 0]) + 14
        A[o + 8] = ttl[i]
        synth._refresh_cksum(A, o)
    kind = synth.inject_errors(b, 0.02, seed=seed + 2, kinds=[synth.ERR_CKSUM])
    bad = np.full(n, -1, np.int8)
    r = rng.random(n)
    frames = b.frames()
    for i in range(n):
        if r[i] < 0.01:                      # hl < 5 words
            fr = bytearray(frames[i]); fr[14] = 0x40 | int(rng.integers(0, 5)); frames[i] = bytes(fr); bad[i] = 0
        elif r[i] < 0.02:                    # hl past the frame
            fr = bytearray(frames[i]); fr[14] = 0x4F; frames[i] = bytes(fr[:14 + 40]); bad[i] = 1
        elif r[i] < 0.03:                    # frame cut inside the header
            frames[i] = frames[i][:14 + int(rng.integers(0, 20))]; bad[i] = 2
    return synth.from_frames(frames, meta=dict(set="rw", seed=seed)), kind, bad


def run_rw(b, tmp, bad):
    """Per packet: IP header bytes 8..11 after the rewrite as the reference
    dumps them (little-endian u32), 0xFFFFFFFF when the element sent the packet
    elsewhere: DecIPTTL output 1 (ttl <= 1) or CheckIPHeader / SetIPChecksum
    drops (a separate mask says which)."""
    pcap = os.path.join(tmp, "rw.pcap")
    write_pcap(pcap, b.frames())
    res = {}

    def grab(name, off):
        out = np.full(b.n, 0xFFFFFFFF, np.uint32)
        for i, (_, data) in read_pcap(os.path.join(tmp, name)).items():
            out[i] = int.from_bytes(data[off + 8:off + 12], "little")
        return out

    def present(name):
        m = np.zeros(b.n, bool)
        for i in read_pcap(os.path.join(tmp, name)):
            m[i] = True
        return m

    for tag, dec in (("dec", "DecIPTTL"), ("decnm", "DecIPTTL(MULTICAST false)")):
        click(CLICK, f"FromDump(rw.pcap, STOP true, TIMING false) -> Strip(14) -> CheckIPHeader(CHECKSUM true) "
                     f"-> d :: {dec} -> ToDump({tag}_ok.pcap); d[1] -> ToDump({tag}_exp.pcap);", tmp)
        res[tag] = grab(f"{tag}_ok.pcap", 0)
        res[tag + "_expired"] = present(f"{tag}_exp.pcap")
    click(CLICK, "FromDump(rw.pcap, STOP true, TIMING false) -> Strip(14) -> CheckIPHeader(CHECKSUM true) "
                 "-> d :: DecIPTTL -> SetIPChecksum -> ToDump(decset_ok.pcap); d[1] -> Discard;", tmp)
    res["decset"] = grab("decset_ok.pcap", 0)
    # MarkIPHeader asserts that the header fits the buffer (packet.hh:2450):
    # frames whose header runs past their end are left out of this run
    # (0xFFFFFFFE: not pinned); hl < 20 is SetIPChecksum's own drop
    fr = b.frames()
    keep = [i for i in range(b.n) if bad[i] not in (1, 2)]
    with open(os.path.join(tmp, "rw_mark.pcap"), "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        for i in keep:
            f.write(struct.pack("<IIII", T0 + i, 0, len(fr[i]), len(fr[i])))
            f.write(fr[i])
    click(CLICK, "FromDump(rw_mark.pcap, STOP true, TIMING false) -> MarkIPHeader(14) -> SetIPChecksum "
                 "-> ToDump(set_ok.pcap);", tmp)
    res["set"] = grab("set_ok.pcap", 14)
    res["set"][(bad == 1) | (bad == 2)] = 0xFFFFFFFE
    return res


def make_qinq_set(n=1600, seed=2031):
    """The mix set with a third of its 802.1Q tags turned into 802.1ad
    (0x88a8) tags: under VLANDecap(ETHERTYPE 0x88a8) only those are decapped;
    0x8100-tagged frames keep their tag and fail the IP checks."""
    b = make_mix_set(n, seed)
    rng = np.random.default_rng(seed + 7)
    A = b.arena
    for i in range(b.n):
        off = int(b.desc[i, 0])
        if A[off + 12] == 0x81 and rng.random() < 0.34:
            A[off + 12], A[off + 13] = 0x88, 0xA8
    return b


def run_qinq(b, tmp):
    """VLANDecap(ETHERTYPE 0x88a8) -> Strip(14) -> Classifier(0/60%f0, -) =>
    CheckIP6Header | CheckIPHeader(CHECKSUM true) -> AggregateHash: per packet
    valid (1) / invalid (0), IP version of valid ones, v4 AGGREGATE, and the
    length after the check."""
    pcap = os.path.join(tmp, "qinq.pcap")
    write_pcap(pcap, b.frames())
    click(CLICK, "FromDump(qinq.pcap, STOP true, TIMING false) -> VLANDecap(ETHERTYPE 0x88a8) -> Strip(14) "
                 "-> c :: Classifier(0/60%f0, -);"
                 " c[0] -> ck6 :: CheckIP6Header -> ToDump(q_good6.pcap, ENCAP IP); ck6[1] -> Discard;"
                 " c[1] -> ck4 :: CheckIPHeader(CHECKSUM true) -> AggregateHash -> t :: Tee(2);"
                 " t[0] -> ToIPSummaryDump(q_good4.ipsum, FIELDS timestamp aggregate);"
                 " t[1] -> ToDump(q_good4.pcap, ENCAP IP); ck4[1] -> Discard;", tmp)
    n = b.n
    valid = np.zeros(n, np.uint8)
    ipver = np.zeros(n, np.uint8)
    hsh = np.zeros(n, np.uint32)
    iplen = np.zeros(n, np.uint16)
    for i, (incl, _) in read_pcap(os.path.join(tmp, "q_good6.pcap")).items():
        valid[i], ipver[i], iplen[i] = 1, 6, incl
    g4 = read_pcap(os.path.join(tmp, "q_good4.pcap"))
    for i, row in read_ipsum(os.path.join(tmp, "q_good4.ipsum"), 1).items():
        valid[i], ipver[i], hsh[i], iplen[i] = 1, 4, int(row[0]), g4[i][0]
    return dict(qinq_valid=valid, qinq_ipver=ipver, qinq_hash=hsh, qinq_iplen=iplen)


def run_kat(tmp):
    """click_in_cksum on random buffers (odd lengths included) and IPFlowID /
    IP6FlowID hashcodes on random tuples, from the reference harness."""
    if not os.path.exists(FCREF):
        return None
    rng = np.random.default_rng(77)
    lens = rng.integers(0, 80, 400)
    bufs = [rng.integers(0, 256, int(k), dtype=np.uint8).tobytes() for k in lens]
    rec = b"".join(struct.pack("<H", len(x)) + x for x in bufs)
    ck = np.frombuffer(subprocess.run([FCREF, "cksum"], input=rec, capture_output=True, check=True).stdout,
                       np.uint16)
    t4 = rng.integers(0, 256, (2000, 12), dtype=np.uint8)
    h4 = np.frombuffer(subprocess.run([FCREF, "flow4"], input=t4.tobytes(), capture_output=True,
                                      check=True).stdout, np.uint32)
    t6 = rng.integers(0, 256, (2000, 36), dtype=np.uint8)
    t6[:64, 32:34] = 0   # sport % 16 == 0 cases (the ROT(v,0) corner)
    t6[:64, 16:18] = rng.integers(0, 16, (64, 2)) * 16
    h6 = np.frombuffer(subprocess.run([FCREF, "flow6"], input=t6.tobytes(), capture_output=True,
                                      check=True).stdout, np.uint32)
    blob = np.frombuffer(b"".join(bufs), np.uint8)
    return dict(ck_lens=lens.astype(np.uint32), ck_blob=blob, ck=ck, t4=t4, h4=h4, t6=t6, h6=h6)


def sha(path):
    if not os.path.exists(path):
        return None
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def main(sets=("ip4", "mix", "prog", "reftests", "combo", "eh", "l4", "flow", "rw", "qinq", "kat")):
    prov_path = os.path.join(HERE, "PROVENANCE.json")
    prov = json.load(open(prov_path)) if os.path.exists(prov_path) else {}
    prov.update(generator="tests/golden/gen_golden.py", click=CLICK, click_sha256=sha(CLICK),
                click3=CLICK3, click3_sha256=sha(CLICK3), click4=CLICK4, click4_sha256=sha(CLICK4), fcref=FCREF, fcref_sha256=sha(FCREF),
                t0=T0, badsrc=BADSRC, gooddst=GOODDST, not_pinned=NOT_PINNED, nomatch=NOMATCH)
    with tempfile.TemporaryDirectory() as tmp:
        if "ip4" in sets:
            b, kind = make_ip4_set()
            r = run_ip4(b, tmp)
            np.savez_compressed(os.path.join(HERE, "ip4.npz"), arena=b.arena, desc=b.desc, kind=kind, **r)
            print("ip4:", np.bincount(r["reason"], minlength=7), "lb16 pinned", int((r["lb16"] != 255).sum()))
        if "mix" in sets:
            m = make_mix_set()
            rm = run_mix(m, tmp)
            np.savez_compressed(os.path.join(HERE, "mix.npz"), arena=m.arena, desc=m.desc, **rm)
            print("mix:", np.bincount(rm["reason"], minlength=8))
        if "prog" in sets:
            pb, pkind = make_prog_set()
            rp = run_prog(pb, tmp)
            np.savez_compressed(os.path.join(HERE, "prog.npz"), arena=pb.arena, desc=pb.desc, kind=pkind, **rp)
            print("prog: ipc", np.bincount(rp["ipc_out"], minlength=256)[[*range(9), 254, 255]],
                  "cls", np.bincount(rp["cls_out"], minlength=256)[[*range(6), 254, 255]])
        if "reftests" in sets:
            pb, _ = make_prog_set()
            rt = run_reftests(pb, tmp)
            with open(os.path.join(HERE, "reftests.json"), "w") as f:
                json.dump(rt, f, indent=0)
            for p in rt["programs"]:
                o = np.array(p["outputs"])
                print("reftests:", p["case"], np.bincount(o[o < 254]).tolist(), "nomatch", int((o == 254).sum()),
                      "invalid", int((o == 255).sum()))
        if "eh" in sets:
            eb = make_eh_set()
            re_ = run_eh(eb, tmp)
            np.savez_compressed(os.path.join(HERE, "eh.npz"), arena=eb.arena, desc=eb.desc, **re_)
            print("eh: valid", int(re_["eh_valid"].sum()), "th>40", int((re_["eh_th"] > 40).sum()),
                  "nxt", np.unique(re_["eh_nxt"]).tolist())
        if "l4" in sets:
            lb = make_l4_set()
            rl = run_l4(lb, tmp)
            np.savez_compressed(os.path.join(HERE, "l4.npz"), arena=lb.arena, desc=lb.desc, **rl)
            for k in ("udp", "tcp"):
                print("l4", k, {int(v): int(c) for v, c in zip(*np.unique(rl[k], return_counts=True))})
        if "flow" in sets:
            fb, fkind, fpick = make_flow_set()
            rf = run_flow(fb, tmp)
            if rf is not None:
                np.savez_compressed(os.path.join(HERE, "flow.npz"), arena=fb.arena, desc=fb.desc, kind=fkind,
                                    pick=fpick, **rf)
                v = rf["flowid"][rf["flowid"] != 0xFFFFFFFF]
                print("flow: classified", len(v), "flows", int(v.max()) + 1, "dropped",
                      int((rf["flowid"] == 0xFFFFFFFF).sum()))
        if "rw" in sets:
            rb, rkind, rbad = make_rw_set()
            rr = run_rw(rb, tmp, rbad)
            np.savez_compressed(os.path.join(HERE, "rw.npz"), arena=rb.arena, desc=rb.desc, kind=rkind, bad=rbad,
                                **rr)
            print("rw: dec ok", int((rr["dec"] != 0xFFFFFFFF).sum()), "expired", int(rr["dec_expired"].sum()),
                  "nm expired", int(rr["decnm_expired"].sum()), "set ok", int((rr["set"] != 0xFFFFFFFF).sum()))
        if "qinq" in sets:
            qb = make_qinq_set()
            rq = run_qinq(qb, tmp)
            np.savez_compressed(os.path.join(HERE, "qinq.npz"), arena=qb.arena, desc=qb.desc, **rq)
            print("qinq: valid", int(rq["qinq_valid"].sum()), "v6", int((rq["qinq_ipver"] == 6).sum()))
        if "combo" in sets:
            rc = run_combo(tmp)
            np.savez_compressed(os.path.join(HERE, "combo.npz"), **rc)
            print("combo: survivors", int(rc["valid"].sum()))
        if "kat" in sets:
            kat = run_kat(tmp)
            if kat is not None:
                np.savez_compressed(os.path.join(HERE, "kat.npz"), **kat)
                print("kat: cksum", len(kat["ck"]), "h4", len(kat["h4"]), "h6", len(kat["h6"]))
    prov.setdefault("sets", {}).update({
        "ip4": "CheckIPHeader(CHECKSUM true, BADSRC, GOODDST)/AggregateHash/FlowSwitch hash 16/HashSwitch(26,8)x{4,7}",
        "mix": "StripEtherVLANHeader(0) -> Classifier(0/60%f0,-) -> CheckIP6Header | CheckIPHeader(CHECKSUM true) -> AggregateHash",
        "prog": "Strip(14) -> CheckIPHeader(CHECKSUM true) -> IPClassifier(IPC_RULES) | CheckIPHeader(OFFSET 14, CHECKSUM true) -> Classifier(CLS_RULES): program text + per-packet output",
        "reftests": "programs printed by the reference for the configs of test/ip/IPFilter-0[4-7] and "
                    "test/standard/Classifier-01 (checked equal to those tests' expected text) + their outputs on "
                    "the prog set; IPFilter-01/02/03 short-packet cases (packets captured from the reference, "
                    "expected outputs from the tests' %expect sections)",
        "eh": "Strip(14) -> CheckIP6Header(BADADDRS 2001:db8::bad, PROCESS_EH true|false) -> Tee: ToDump (length), "
              "StripIPHeader -> ToDump (transport offset), PaintSwitch(ANNO 16) (IP6_NXT)",
        "l4": "Strip(14) -> CheckIPHeader(CHECKSUM true) -> CheckUDPHeader|CheckTCPHeader(CHECKSUM true|false): "
              "per-packet verdicts (reason split by the CHECKSUM false run)",
        "combo": "IPInputCombo(7, BADSRC, GOODDST) on the ip4 set: survivors and their ip_len",
        "flow": "Strip(14) -> CheckIPHeader(CHECKSUM true) -> FlowIPManagerHMP -> StoreFlowID(OFFSET 0) (click4: "
                "--enable-research --enable-flow-dynamic --enable-ctx): per-packet flow ID = stored ID - 1",
        "rw": "Strip(14) -> CheckIPHeader(CHECKSUM true) -> DecIPTTL[(MULTICAST false)] [-> SetIPChecksum] -> ToDump, "
              "DecIPTTL[1] -> ToDump; MarkIPHeader(14) -> SetIPChecksum -> ToDump: IP header bytes 8..11 per packet",
        "qinq": "VLANDecap(ETHERTYPE 0x88a8) -> Strip(14) -> Classifier(0/60%f0,-) -> CheckIP6Header | "
                "CheckIPHeader(CHECKSUM true) -> AggregateHash: validity, version, v4 hash, ip length",
        "kat": "fcref: click_in_cksum (lib/in_cksum.c), IPFlowID/IP6FlowID::hashcode (headers)",
    })
    prov["ipc_rules"] = IPC_RULES
    prov["cls_rules"] = CLS_RULES
    with open(prov_path, "w") as f:
        json.dump(prov, f, indent=1)


if __name__ == "__main__":
    main(tuple(sys.argv[1:]) or ("ip4", "mix", "prog", "reftests", "combo", "eh", "l4", "flow", "rw", "qinq",
                                 "kat"))
