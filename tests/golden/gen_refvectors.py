"""TEST INFRASTRUCTURE: golden vectors from the reference's own tests.

Reads the text of /root/reference/test/**/*.clicktest (study only: nothing of
the reference is compiled or run) and writes tests/golden/refvectors.json --
DATA, never the tests' text: the packets those tests feed their graphs
(built from their %file / DATA bytes) and the outcomes their %expect
sections state. Each set names its source file:line.

Sets (the SURVEY 8(a) rows they pin):
  iprouter  userlevel/iprouter-01.clicktest:45-57,105-107,242-243 -- the UDP
            frame InfiniteSource sends 600000 times through Strip(14) ->
            CheckIPHeader(INTERFACES 18.26.4.1/24 18.26.7.1/24) (and, in the
            click-xform variant OUTB, IPInputCombo); %expect: all 600000 reach
            the counter, i.e. every one is valid.                  [A2 A4 A12]
  ipopt     analysis/FromIPSummaryDump-ipopt-01.clicktest:37-51,68-83,93-106 --
            13 TCP packets with IP options (SSRR, RR, TS, NOP/EOL) that pass
            SetIPChecksum -> SetTCPChecksum -> CheckIPHeader -> CheckTCPHeader;
            %expect gives each one's total length and option length (OUT2) and
            5-tuple (OUT3).                                       [A1 A2 A5 L4]
  vlan      ethernet/VLANEncap-01.clicktest:26-33, VLANEncap-02.clicktest:20-24,
            EtherVLANEncap-01.clicktest:28-35 -- the exact frames the Print
            elements show, and what StripEtherVLANHeader / VLANDecap(ETHERTYPE)
            (+ Strip(14)) leave: 4 bytes "aaabacad" after an 802.1Q / 802.1ad
            tag or plain Ethernet, the frame unchanged when the tag protocol
            is not the one configured.                                  [A13]
  ipfrag    ip/IPFragmenter-01.clicktest:8,16-17, IPFragmenter-02.clicktest:8,16-17
            -- a 24-B-header packet CheckIPHeader(OFFSET 0) / MarkIPHeader(OFFSET
            0) passes, and the two fragments the reference emits, whose
            header checksums its own click_in_cksum wrote.        [A1 A2 A4 A5]
  tcpfull   tcpudp/StripTCPHeader-01.clicktest:34-39 -- IP headers (with
            checksums) of packets that pass CheckIPHeader(VERBOSE true).  [A1]
  markipce  ip/MarkIPCE-01.clicktest:19-24,36-43 -- packets FromIPSummaryDump
            (CHECKSUM true) builds that pass CheckIPHeader before and after
            MarkIPCE sets ECN CE with an incremental checksum update.    [A2]
  flow      flow/flow-no-dynamic.clicktest:9-17,25-31,36-63 and
            flow/flow-dynamic.clicktest:9-17,25-31,36-61 -- five UDP packets
            FromIPSummaryDump(CHECKSUM true, TIMING true [, BURST 2]) sends at
            t = 1, 3, 3, 3.1, 5 s through FlowIPManager_CuckooPP(RESERVE 2,
            TIMEOUT 5) (the IMP manager, CAPACITY 65536): each packet's first
            24 bytes as the test's Print lines show them (their IP checksums
            the reference wrote), the flow ID FlowPrint reports for each run,
            the PacketBatch runs (BURST 2), and the count / count_fids reads
            DriverManager makes at t = 0, 2 and 12 s.          [A1 (f)#1 IMP]

Restated here (cited): FromIPSummaryDump's ip_opt text -> option bytes
(elements/analysis/ipsumdump_ip.cc:628-851, placed and EOL-padded as :173-191),
the default IPv4 header (ipsumdumpinfo.cc:422-445: ttl 100), the TCP header
(:475-515: th_off 5, ports from the flow), SetIPChecksum / SetTCPChecksum
(fromipsumdump.cc:389, set_checksums; the TCP pseudo-header takes a source
route's final hop, lib/in_cksum.c:84-111), click_update_in_cksum
(include/clicknet/ip.h:181) for MarkIPCE.

Run:  python tests/golden/gen_refvectors.py   (needs /root/reference)
"""
import json
import os
import re
import struct

REF = os.environ.get("FC_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "refvectors.json")


def read(rel):
    with open(os.path.join(REF, "test", rel)) as f:
        return f.read()


def section(text, header):
    """Lines of the clicktest section that starts with `header`, and the
    1-based line number of its first line."""
    lines = text.split("\n")
    for i, ln in enumerate(lines):
        if ln.strip() == header:
            body = []
            for ln2 in lines[i + 1:]:
                if ln2.startswith("%"):
                    break
                body.append(ln2)
            while body and not body[-1].strip():
                body.pop()
            return body, i + 2
    raise KeyError(header)


def cksum(b):
    """RFC 1071 / click_in_cksum (lib/in_cksum.c:20-51): one's complement of
    the folded 16-bit sum (big-endian words here; the caller only checks the
    stored result, which is byte-order independent)."""
    if len(b) % 2:
        b = b + b"\0"
    s = sum(struct.unpack(f"!{len(b) // 2}H", b))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return ~s & 0xFFFF


def ip4(a):
    return bytes(int(x) for x in a.split("."))


# ---- FromIPSummaryDump ip_opt (ipsumdump_ip.cc:628-851) ---------------------
def _int(s, i, base=10):
    m = re.match(r"0[xX][0-9a-fA-F]+|[0-9]+", s[i:]) if base == 0 else re.match(r"[0-9]+", s[i:])
    if not m:
        return None, i
    t = m.group(0)
    v = int(t, 16) if t[:2].lower() == "0x" else (int(t, 8) if base == 0 and len(t) > 1 and t[0] == "0"
                                                   else int(t))
    return v, i + len(t)


def _ip(s, i, out):
    for k in range(4):
        v, i = _int(s, i)
        assert v is not None and v <= 255, s
        out.append(v)
        if k < 3:
            assert s[i] == "."
            i += 1
    return i


def ip_opt_bytes(s):
    out = bytearray()
    i, end = 0, len(s)
    if s in ("", "."):
        return bytes(out)
    while True:
        if s.startswith("rr{", i) or s.startswith("ssrr{", i) or s.startswith("lsrr{", i):
            kind = {"r": 7, "s": 137, "l": 131}[s[i]]
            i += 3 if s[i] == "r" else 5
            pos = len(out)
            out += bytes([kind, 0, 0])
            pointer = -1
            while True:
                if i < end and s[i] == "^" and pointer < 0:
                    pointer = len(out) - pos + 1
                    i += 1
                if i >= end or not s[i].isdigit():
                    break
                i = _ip(s, i, out)
                if i < end and s[i] == ",":
                    i += 1
            assert s[i] == "}"
            out[pos + 2] = pointer if pointer >= 0 else len(out) - pos + 1
            if i + 2 < end and s[i + 1] == "+" and s[i + 2].isdigit():
                v, i = _int(s, i + 2)
                out += bytes(4 * v)
            else:
                i += 1
            out[pos + 1] = len(out) - pos
        elif s.startswith("ts{", i) or s.startswith("ts.", i):
            pos = len(out)
            out += bytes([68, 0, 0, 0])
            flag = -1
            if s[i + 2] == ".":
                if s.startswith("ip{", i + 3):
                    flag, i = 1, i + 6
                elif s.startswith("preip{", i + 3):
                    flag, i = 3, i + 9
                else:
                    flag, j = _int(s, i + 3, 0)
                    assert s[j] == "{"
                    i = j + 1
            else:
                i += 3
            pointer = -1
            while True:
                if i < end and s[i] == "^" and pointer < 0:
                    pointer = len(out) - pos + 1
                    i += 1
                if i >= end or not (s[i].isdigit() or s[i] == "!"):
                    break
                entry = i
                while True:                      # retry_entry
                    if flag in (1, 3, -2):
                        i = _ip(s, i, out)
                        if pointer >= 0 and flag == -2:
                            flag = 3
                        if i + 1 < end and s[i] == "=":
                            if s[i + 1].isdigit() or s[i + 1] == "!":
                                i += 1
                            elif s[i + 1] == "?" and pointer >= 0:
                                out += bytes(4)
                                i += 2
                                break
                            else:
                                raise ValueError(s)
                        elif pointer >= 0:
                            out += bytes(4)
                            break
                        else:
                            raise ValueError(s)
                    top = 0
                    if s[i] == "!":
                        top, i = 0x80000000, i + 1
                    v, i = _int(s, i, 0)
                    if i < end and s[i] == "." and flag == -1:
                        flag, i = -2, entry
                        continue
                    if flag == -1:
                        flag = 0
                    out += struct.pack("!I", v | top)
                    break
                if i < end and s[i] == ",":
                    i += 1
            if i < end:
                assert s[i] == "}"
                i += 1
            if flag == -2:
                flag = 1
            out[pos + 2] = pointer if pointer >= 0 else len(out) - pos + 1
            if i + 1 < end and s[i] == "+" and s[i + 1].isdigit():
                v, i = _int(s, i + 1, 0)
                out += bytes(v * (8 if flag in (1, 3) else 4))
            overflow = 0
            if i + 2 < end and s[i] == "+" and s[i + 1] == "+" and s[i + 2].isdigit():
                overflow, i = _int(s, i + 2, 0)
            out[pos + 3] = (overflow << 4) | (flag & 0xF)
            out[pos + 1] = len(out) - pos
        elif s.startswith("nop", i):
            out.append(1)
            i += 3
        elif s.startswith("eol", i) and (i + 3 == end or s[i + 3] != ","):
            out.append(0)
            i += 3
        else:
            raise ValueError(f"ip_opt {s!r} at {i}")
        if i >= end:
            while len(out) > 40 and out[0] == 1:
                del out[0]
            assert len(out) <= 40
            return bytes(out)
        assert s[i] in ",;"
        i += 1


def pseudo_dst(iph):
    """The pseudo-header destination click_in_cksum_pseudohdr uses: the final
    hop of a source route option, else ip_dst (lib/in_cksum.c:84-111)."""
    i, end = 20, (iph[0] & 15) * 4
    while i < end:
        if iph[i] == 1:
            i += 1
            continue
        if iph[i] == 0 or i + 1 >= end or iph[i + 1] < 2 or i + iph[i + 1] > end:
            break
        if iph[i] in (137, 131) and iph[i + 1] >= 7:
            return iph[i + iph[i + 1] - 4:i + iph[i + 1]]
        i += iph[i + 1]
    return iph[16:20]


def ipv4_tcp(src, sport, dst, dport, opts=b"", ttl=100):
    """FromIPSummaryDump(ZERO true) -> SetIPChecksum -> SetTCPChecksum: an IPv4
    header (+ options, EOL-padded) and a 20-B TCP header, no payload."""
    hl = (20 + len(opts) + 3) & ~3
    total = hl + 20
    iph = bytearray(struct.pack("!BBHHHBBH4s4s", 0x40 | (hl >> 2), 0, total, 0, 0, ttl, 6, 0, ip4(src), ip4(dst)))
    iph += opts + bytes(hl - 20 - len(opts))
    iph[10:12] = struct.pack("!H", cksum(bytes(iph)))
    tcp = bytearray(struct.pack("!HHIIBBHHH", sport, dport, 0, 0, 5 << 4, 0, 0, 0, 0))
    pseudo = ip4(src) + pseudo_dst(bytes(iph)) + struct.pack("!BBH", 0, 6, 20)
    tcp[16:18] = struct.pack("!H", cksum(pseudo + bytes(tcp)))
    return bytes(iph + tcp)


def hexbytes(words):
    return bytes.fromhex("".join(words))


def gen_iprouter():
    rel = "userlevel/iprouter-01.clicktest"
    text = read(rel)
    m = re.search(r"InfiniteSource\(DATA \\<(.*?)>, LIMIT (\d+)", text, re.S)
    data = re.sub(r"//[^\n]*", "", m.group(1))
    frame = bytes.fromhex("".join(data.split()))
    limit = int(m.group(2))
    assert "CheckIPHeader(INTERFACES 18.26.4.1/24 18.26.7.1/24)" in text
    expect, line = section(text, "%expect OUTA OUTB")
    assert expect == [str(limit)]
    L = struct.unpack("!H", frame[16:18])[0]
    return dict(source=f"test/{rel}:45-57,105-107,242-243 (%expect at :{line})",
                frames=[frame.hex()], repeat=limit,
                conf="Strip(14) -> CheckIPHeader(INTERFACES 18.26.4.1/24 18.26.7.1/24)",
                expect=dict(valid=limit, ip_len=L, trimmed_len=14 + L,
                            flow=["1.0.0.1", 0x1369, "2.0.0.2", 0x1369, 17]))


def gen_ipopt():
    rel = "analysis/FromIPSummaryDump-ipopt-01.clicktest"
    text = read(rel)
    rows, l_in = section(text, "%file IN1")
    assert rows[0].split() == ["!data", "src", "sport", "dst", "dport", "proto", "ip_opt"]
    out2, l_o2 = section(text, "%cut %expect -a OUT2")
    out3, l_o3 = section(text, "%expect OUT3 OUT5")
    frames, exp = [], []
    for row, o2, o3 in zip(rows[1:], out2, out3):
        src, sport, dst, dport, proto, opt = row.split()
        assert proto == "T"
        opts = ip_opt_bytes(opt)
        f = ipv4_tcp(src, int(sport), dst, int(dport), opts)
        m = re.search(r"\(id 0, len (\d+)(?:, optlen=(\d+))?", o2)
        total, optlen = int(m.group(1)), int(m.group(2) or 0)
        hl = (f[0] & 15) * 4
        assert (len(f), hl - 20) == (total, optlen), (row, len(f), hl, o2)
        s3 = o3.split()
        assert s3[:5] == [src, sport, dst, dport, "T"]
        frames.append(f.hex())
        exp.append(dict(ip_len=total, hl=hl, flow=[s3[0], int(s3[1]), s3[2], int(s3[3]), 6]))
    return dict(source=f"test/{rel}:37-51 (%file IN1 at :{l_in}), %expect OUT2 lengths at :{l_o2}, "
                       f"OUT3 5-tuples at :{l_o3}",
                frames=frames, offset=0,
                conf="SetIPChecksum -> SetTCPChecksum -> CheckIPHeader -> CheckTCPHeader (all pass)",
                expect=exp)


def _print_frames(text):
    """name -> frame bytes from `%expect stderr` Print lines ("a:   22 | 0202...")."""
    body, line = section(text, "%expect stderr")
    out = {}
    for ln in body:
        m = re.match(r"(\w+):\s+(\d+) \| (.*)$", ln)
        b = hexbytes(m.group(3).split())
        assert len(b) == int(m.group(2))
        out[m.group(1)] = b
    return out, line


def gen_vlan():
    cases = []
    rel = "ethernet/EtherVLANEncap-01.clicktest"
    pf, line = _print_frames(read(rel))
    payload = pf["x"]
    # a, c, f: tagged frames; StripEtherVLANHeader (NATIVE_VLAN 0) -> b / d (payload)
    for k in ("a", "c", "f"):
        cases.append(dict(src=f"test/{rel}:{line} ({k})", frame=pf[k].hex(), vlan_ethertype=0x8100,
                          decap=True, ip_off=18, tci=pf[k][14:16].hex(), after=payload.hex()))
    cases.append(dict(src=f"test/{rel}:{line} (e)", frame=pf["e"].hex(), vlan_ethertype=0x8100,
                      decap=True, ip_off=14, tci="0000", after=payload.hex()))
    rel = "ethernet/VLANEncap-01.clicktest"
    pf, line = _print_frames(read(rel))
    # VLANDecap() -> Strip(14) -> b (payload)
    cases.append(dict(src=f"test/{rel}:{line} (a -> b)", frame=pf["a"].hex(), vlan_ethertype=0x8100,
                      decap=True, ip_off=18, tci=pf["a"][14:16].hex(), after=pf["b"].hex()))
    cases.append(dict(src=f"test/{rel}:{line} (f)", frame=pf["f"].hex(), vlan_ethertype=0x8100,
                      decap=True, ip_off=18, tci=pf["f"][14:16].hex(), after=payload.hex()))
    rel = "ethernet/VLANEncap-02.clicktest"
    pf, line = _print_frames(read(rel))
    # VLANDecap() leaves the 802.1ad frame unchanged (b == a); VLANDecap(ETHERTYPE 0x88a8) -> c
    assert pf["a"] == pf["b"] and pf["c"][12:] == pf["a"][16:]
    cases.append(dict(src=f"test/{rel}:{line} (a -> b, VLANDecap())", frame=pf["a"].hex(), vlan_ethertype=0x8100,
                      decap=False, ip_off=14, tci=None, after=pf["b"][14:].hex()))
    cases.append(dict(src=f"test/{rel}:{line} (a -> c, VLANDecap(ETHERTYPE 0x88a8))", frame=pf["a"].hex(),
                      vlan_ethertype=0x88A8, decap=True, ip_off=18, tci=pf["a"][14:16].hex(),
                      after=pf["c"][14:].hex()))
    return dict(source="test/ethernet/{EtherVLANEncap-01,VLANEncap-01,VLANEncap-02}.clicktest %expect stderr",
                cases=cases)


def gen_ipfrag():
    cases = []
    for rel, elem in (("ip/IPFragmenter-01.clicktest", "MarkIPHeader(OFFSET 0)"),
                      ("ip/IPFragmenter-02.clicktest", "CheckIPHeader(OFFSET 0)")):
        text = read(rel)
        m = re.search(r'InfiniteSource\(DATA "\\<(.*?)>"', text)
        pkt = hexbytes(m.group(1).split())
        assert elem in text
        body, line = section(text, "%expect stderr")
        frags = [hexbytes(ln.split("|")[1].split()) for ln in body if "|" in ln]
        cases.append(dict(src=f"test/{rel}:8 ({elem})", packet=pkt.hex(), mode=elem.split("(")[0],
                          fragments=[f.hex() for f in frags], fragments_src=f"test/{rel}:{line}"))
    return dict(source="test/ip/IPFragmenter-0{1,2}.clicktest", cases=cases)


def gen_tcpfull():
    rel = "tcpudp/StripTCPHeader-01.clicktest"
    body, line = section(read(rel), "%expect stderr")
    hdrs = []
    for ln in body:
        if ln.startswith("FULLTCP:"):
            h = hexbytes(ln.split("|")[1].split())[:20]
            if h.hex() not in hdrs:
                hdrs.append(h.hex())
    return dict(source=f"test/{rel}:{line} (FULLTCP lines: the IP header FromIPSummaryDump CHECKSUM true "
                       "wrote, which CheckIPHeader(VERBOSE true) passed)", headers=hdrs)


def gen_markipce():
    rel = "ip/MarkIPCE-01.clicktest"
    text = read(rel)
    rows, line = section(text, "%file IN")
    ecn = {"no": 0, "ect1": 1, "ect2": 2, "ce": 3}
    proto = int(rows[1].split()[1])
    before, after = [], []
    for r in rows[2:]:
        _, src, dst, e = r.split()
        h = bytearray(struct.pack("!BBHHHBBH4s4s", 0x45, ecn[e], 20, 0, 0, 100, proto, 0, ip4(src), ip4(dst)))
        h[10:12] = struct.pack("!H", cksum(bytes(h)))
        before.append(bytes(h).hex())
        # MarkIPCE (FORCE true): tos |= 3, checksum updated incrementally
        # (click_update_in_cksum, include/clicknet/ip.h:181: RFC 1624 eq. 3)
        old_w = (h[0] << 8) | h[1]
        h[1] |= 3
        new_w = (h[0] << 8) | h[1]
        s = (~struct.unpack("!H", h[10:12])[0] & 0xFFFF) + (~old_w & 0xFFFF) + new_w
        while s >> 16:
            s = (s & 0xFFFF) + (s >> 16)
        h[10:12] = struct.pack("!H", ~s & 0xFFFF)
        after.append(bytes(h).hex())
    exp, eline = section(text, "%expect OUT2")
    assert len(exp) == len(after) and all(x.endswith(" ce") for x in exp)
    return dict(source=f"test/{rel}:{line} (%file IN), %expect OUT2 at :{eline}", before=before, after=after)


def ipv4_udp(src, dst, payload, ttl=100):
    """FromIPSummaryDump(CHECKSUM true) for a "U" row with a payload: the
    default IPv4 header (ipsumdumpinfo.cc:422-445: ttl 100, id 0), a UDP
    header with ports 0 (no sport/dport field) and uh_ulen = ip_len - 20
    (fromipsumdump.cc:637-642), the payload bytes, then set_checksums
    (:384-402): the IP header checksum and the UDP checksum over the datagram
    with its pseudo-header."""
    total = 20 + 8 + len(payload)
    iph = bytearray(struct.pack("!BBHHHBBH4s4s", 0x45, 0, total, 0, 0, ttl, 17, 0, ip4(src), ip4(dst)))
    iph[10:12] = struct.pack("!H", cksum(bytes(iph)))
    udp = bytearray(struct.pack("!HHHH", 0, 0, 8 + len(payload), 0)) + payload
    pseudo = ip4(src) + ip4(dst) + struct.pack("!BBH", 0, 17, len(udp))
    udp[6:8] = struct.pack("!H", cksum(pseudo + bytes(udp)))
    return bytes(iph + udp)


def _flow_section(body, header):
    """The lines of one flow manager's run in a flow test's %expect stderr
    (from the line `header` to the next manager's)."""
    beg = body.index(header)
    first = next(k for k in range(beg, len(body)) if body[k].startswith("Placing "))
    end = len(body)
    for k in range(first + 1, len(body)):
        if body[k].startswith("Placing ") or body[k] in ("FlowIPManager_DPDK", "FlowIPManagerMP", "FlowIPManager"):
            end = k
            break
    return body[beg:end]


def _flow_trace(lines):
    """Print / FlowPrint / handler lines of one run -> the packets' first
    bytes (BEFORE order), the source's PacketBatches (Print(BEFORE) prints a
    whole batch before the manager sees it, so BEFORE lines with no AFTER line
    between them are one batch), the runs FlowPrint reports (packet indices,
    flow ID) and the handler reads in order (name, value, packets seen before
    it)."""
    before, runs, reads, bursts = [], [], [], []
    after_seen = 0
    last = None
    k = 0
    while k < len(lines):
        ln = lines[k]
        m = re.match(r"BEFORE:\s+(\d+) \| (.*)$", ln)
        if m:
            if last == "BEFORE":
                bursts[-1] += 1
            else:
                bursts.append(1)
            before.append((int(m.group(1)), hexbytes(m.group(2).split())))
            last = "BEFORE"
        m = re.match(r"AFTER:\s+\d+ \|", ln)
        if m:
            after_seen += 1
            last = "AFTER"
        m = re.match(r"fprint :: FlowPrint: (\d+) packets from flow (\d+)\.", ln)
        if m:
            cnt = int(m.group(1))
            runs.append(dict(packets=list(range(after_seen - cnt, after_seen)), flow=int(m.group(2))))
        m = re.match(r"fm\.(count|count_fids):$", ln)
        if m:
            reads.append(dict(handler=m.group(1), value=lines[k + 1], after_packets=len(before)))
            k += 1
        k += 1
    return before, runs, reads, bursts


def gen_flow():
    rel_nd, rel_d = "flow/flow-no-dynamic.clicktest", "flow/flow-dynamic.clicktest"
    text_nd, text_d = read(rel_nd), read(rel_d)
    assert "FlowIPManager_CuckooPP" in text_nd and "RESERVE 2, VERBOSE 1, TIMEOUT 5" in text_nd
    assert "FromIPSummaryDump(IN1, STOP false, CHECKSUM true, TIMING true)" in text_nd
    assert "FromIPSummaryDump(IN1, STOP false, CHECKSUM true, TIMING true, BURST 2)" in text_d
    rows, l_in = section(text_nd, "%file IN1")
    rows_d, _ = section(text_d, "%file IN1")
    assert rows == rows_d and rows[0].split() == ["!data", "timestamp", "src", "dst", "proto", "payload"]
    pkts = []
    for r in rows[1:]:
        t, src, dst, proto, payload = r.split()
        assert proto == "U"
        pkts.append(dict(t=float(t), frame=ipv4_udp(src, dst, payload.encode())))
    out = dict(source=f"test/{rel_nd}:9-17 (graph), :25-31 (%file IN1 at :{l_in}), %expect stderr; "
                      f"test/{rel_d}:9-17 (BURST 2), %expect stderr",
               manager=dict(kind="FlowIPManager_CuckooPP", capacity=65536, timeout_s=5, recycle_ms=1000),
               packets=[dict(t=p["t"], frame=p["frame"].hex()) for p in pkts])
    for key, text, header in (("single", text_nd, "Placing  ftest :: TestFlowSpace at [30-33]"),
                              ("burst2", text_d, "FlowIPManager_CuckooPP")):
        body, line = section(text, "%expect stderr")
        sec = _flow_section(body, header)
        assert "Real capacity for each table will be 65536" in sec
        before, runs, reads, bursts = _flow_trace(sec)
        # the Print lines are the packets' first 24 bytes, byte for byte
        assert len(before) == len(pkts)
        for (length, head), p in zip(before, pkts):
            assert length == len(p["frame"]) and head == p["frame"][:24], (key, head.hex(), p["frame"][:24].hex())
        ids = [None] * len(pkts)
        for run in runs:
            for i in run["packets"]:
                ids[i] = run["flow"]
        assert None not in ids
        out[key] = dict(expect_line=line, bursts=bursts, runs=runs, ids=ids, reads=reads)
    # the reads' times: DriverManager(read.., wait 2s, read.., wait 10s, read..)
    # on the FromIPSummaryDump TIMING clock (the first packet at t = 0)
    out["read_times_s"] = [0.0, 2.0, 12.0]
    return out


def main():
    out = dict(generator="tests/golden/gen_refvectors.py", reference_tests_only=True,
               iprouter=gen_iprouter(), ipopt=gen_ipopt(), vlan=gen_vlan(), ipfrag=gen_ipfrag(),
               tcpfull=gen_tcpfull(), markipce=gen_markipce(), flow=gen_flow())
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=False)
        f.write("\n")
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
