"""pcap ingress (include/fcpcap.h, fastclick_amd/pcap.py): FromDump's record
parsing (elements/userlevel/fromdump.cc:278-316, 418-500) into pinned chunks,
then fcgpu_span_submit (one H2D copy per chunk, no per-packet gather).

CPU: the reader against hand-built files in every header variant FromDump
accepts (both byte orders, nanosecond and modified-pcap magics, pre-2.3
caplen/len order, caplen > len, a truncated last record, records straddling
chunk boundaries). GPU: the golden sets written as pcaps and run through the
ingress give the reference's verdicts, hashes and flow IDs.
"""
import struct

import numpy as np
import pytest

from fastclick_amd import synth
from tests.test_golden import load, batch_of


def write_pcap(path, frames, *, magic=0xA1B2C3D4, swapped=False, minor=4, wire=None, swap_lens=False,
               linktype=1, cut_last=0):
    e = ">" if swapped else "<"
    with open(path, "wb") as f:
        f.write(struct.pack(e + "IHHiIII", magic, 2, minor, 0, 0, 65535, linktype))
        for i, fr in enumerate(frames):
            caplen, ln = len(fr), (wire[i] if wire is not None else len(fr))
            a, b = (ln, caplen) if swap_lens else (caplen, ln)
            f.write(struct.pack(e + "IIII", 1000 + i, 7 * i, a, b))
            if magic == 0xA1B2CD34:
                f.write(b"\xAA" * 8)
            f.write(fr)
    if cut_last:
        with open(path, "r+b") as f:
            f.seek(0, 2)
            f.truncate(f.tell() - cut_last)


def read_all(path, cap=1 << 16, max_pkts=1 << 16, threads=1):
    from fastclick_amd.pcap import PcapReader
    rd = PcapReader(path, threads)
    frames, wires, ts = [], [], []
    buf = np.zeros(cap, np.uint8)
    desc = np.zeros(2 * max_pkts, np.uint32)
    wire = np.zeros(max_pkts, np.uint32)
    tsn = np.zeros(max_pkts, np.uint64)
    while True:
        n, used = rd.read(buf.ctypes.data, cap, desc.ctypes.data, max_pkts, wire.ctypes.data, tsn.ctypes.data)
        if n == 0:
            break
        for i in range(n):
            o, ln = int(desc[2 * i]), int(desc[2 * i + 1])
            assert o + ln <= used
            frames.append(bytes(buf[o:o + ln]))
            wires.append(int(wire[i]))
            ts.append(int(tsn[i]))
    lt = rd.linktype
    rd.close()
    return frames, wires, ts, lt


def _frames(n=300, seed=5):
    rng = np.random.default_rng(seed)
    return [bytes(rng.integers(0, 256, int(k), dtype=np.uint8)) for k in rng.integers(1, 1600, n)]


@pytest.mark.parametrize("magic,swapped", [(0xA1B2C3D4, False), (0xA1B2C3D4, True), (0xA1B23C4D, False),
                                           (0xA1B23C4D, True), (0xA1B2CD34, False)])
def test_reader_header_variants(tmp_path, magic, swapped):
    fr = _frames()
    p = str(tmp_path / "x.pcap")
    write_pcap(p, fr, magic=magic, swapped=swapped, linktype=101)
    got, wire, ts, lt = read_all(p)
    assert got == fr and wire == [len(f) for f in fr] and lt == 101
    mult = 1 if magic == 0xA1B23C4D else 1000
    assert ts == [(1000 + i) * 10**9 + 7 * i * mult for i in range(len(fr))]


def test_reader_lengths_and_old_versions(tmp_path):
    fr = _frames(200, seed=6)
    p = str(tmp_path / "x.pcap")
    # snaplen-truncated records: caplen < len
    wire = [len(f) + 50 for f in fr]
    write_pcap(p, fr, wire=wire)
    got, w, _, _ = read_all(p)
    assert got == fr and w == wire
    # minor version 2: caplen and len are stored the other way round
    write_pcap(p, fr, wire=wire, minor=2, swap_lens=True)
    got, w, _, _ = read_all(p)
    assert got == fr and w == wire
    # caplen > len: FromDump keeps len bytes and skips the rest
    write_pcap(p, fr, wire=[max(1, len(f) - 3) for f in fr])
    got, _, _, _ = read_all(p)
    assert got == [f[:max(1, len(f) - 3)] for f in fr]


def test_reader_chunk_boundaries_and_truncation(tmp_path):
    fr = _frames(500, seed=7)
    p = str(tmp_path / "x.pcap")
    write_pcap(p, fr, cut_last=5)
    for cap, mx, th in ((2048, 1 << 16, 1), (1 << 16, 3, 1), (4096, 7, 1), (3 << 20, 1 << 16, 4)):
        got, _, _, _ = read_all(p, cap=cap, max_pkts=mx, threads=th)
        assert got == fr[:-1], (cap, mx, th)
    big = _frames(6000, seed=8)      # ~4.8 MB: several 1-MiB pieces per fill
    write_pcap(p, big, cut_last=3)
    for cap, th in ((3 << 20, 3), (5 << 20, 8), (1 << 20, 2)):
        got, _, _, _ = read_all(p, cap=cap, threads=th)
        assert got == big[:-1], (cap, th)


def test_reader_mapped_index_matches_read(tmp_path):
    """Zero-copy mode (fcpcap_map + fcpcap_index) yields the same records."""
    from fastclick_amd.pcap import PcapReader
    fr = _frames(3000, seed=9)
    p = str(tmp_path / "x.pcap")
    for kw in (dict(), dict(swapped=True, magic=0xA1B2CD34), dict(minor=2, swap_lens=True)):
        write_pcap(p, fr, cut_last=4, **kw)
        rd = PcapReader(p)
        base, size = rd.map()
        mem = (np.ctypeslib.as_array((__import__("ctypes").c_uint8 * size).from_address(base)))
        desc = np.zeros(2 * 700, np.uint32)
        got = []
        while True:
            n, off, nb = rd.index(700, 100_000, desc.ctypes.data)
            if n == 0:
                break
            assert nb <= 100_000 or n == 1
            for i in range(n):
                o, ln = off + int(desc[2 * i]), int(desc[2 * i + 1])
                got.append(bytes(mem[o:o + ln]))
        rd.close()
        assert got == fr[:-1], kw


def test_reader_rejects_bad_files(tmp_path):
    from fastclick_amd.pcap import PcapReader
    p = tmp_path / "bad.pcap"
    p.write_bytes(b"\x00" * 24)
    with pytest.raises(OSError, match="bad magic"):
        PcapReader(str(p))
    p.write_bytes(b"\xd4\xc3\xb2\xa1")
    with pytest.raises(OSError, match="too short"):
        PcapReader(str(p))
    write_pcap(str(p), [b"x" * 70000])
    with pytest.raises(OSError, match="bad packet header"):
        read_all(str(p), cap=1 << 17)


@pytest.mark.gpu
def test_gpu_pcap_ingress_golden(tmp_path):
    """ip4 golden set as a pcap: reasons and AggregateHash equal the reference's,
    chunked small enough that records straddle chunks."""
    from fastclick_amd import _native as N
    from fastclick_amd.pcap import process_pcap
    from tests.test_golden import ip4_cfg, first_fragment_mask
    g = load("ip4")
    b = batch_of(g)
    p = str(tmp_path / "ip4.pcap")
    write_pcap(p, b.frames())
    for chunk_pkts, chunk_bytes, mapped in ((1 << 16, 1 << 24, False), (256, 1 << 14, False),
                                            (1000, 1 << 16, False), (1 << 16, 1 << 24, True), (700, 1 << 16, True)):
        out, n, _ = process_pcap(p, ip4_cfg(classify=N.CLS_LB_HASH, nports=16), chunk_pkts=chunk_pkts,
                                 chunk_bytes=chunk_bytes, mapped=mapped)
        assert n == b.n
        reason = (out["verdict"] & 0xFF).astype(np.uint8)
        assert np.array_equal(reason, g["reason"])
        ok = (g["reason"] == 6) & first_fragment_mask(g)
        assert np.array_equal(out["hash"][ok], g["hash"][ok])


@pytest.mark.gpu
def test_gpu_pcap_ingress_flows(tmp_path):
    from fastclick_amd import _native as N
    from fastclick_amd.pcap import process_pcap
    g = load("flow")
    b = batch_of(g)
    p = str(tmp_path / "flow.pcap")
    write_pcap(p, b.frames())
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=4)
    out, n, _ = process_pcap(p, cfg, chunk_pkts=512, chunk_bytes=1 << 16, outputs=("verdict", "flowid"),
                             max_flows=1 << 16)
    assert np.array_equal(out["flowid"], g["flowid"])
    assert out["flow_count"] == int(g["flowid"][g["flowid"] != N.FLOW_NONE].max()) + 1


def _fake_chain_frame(rng, nrec):
    """A frame whose payload is itself a run of nrec tiny, plausible pcap
    records: a parallel walk that starts inside it syncs on a false chain."""
    body = b"".join(struct.pack("<IIII", 5, int(rng.integers(0, 999_999)), 8, 8) + bytes(8) for _ in range(nrec))
    return bytes(14) + body


def _index_all(path, threads, max_pkts, max_bytes):
    from fastclick_amd.pcap import PcapReader
    rd = PcapReader(path, threads)
    rd.map()
    desc = np.zeros(2 * max_pkts, np.uint32)
    wire = np.zeros(max_pkts, np.uint32)
    tsn = np.zeros(max_pkts, np.uint64)
    calls = []
    try:
        while True:
            try:
                n, off, nb = rd.index(max_pkts, max_bytes, desc.ctypes.data, wire.ctypes.data, tsn.ctypes.data)
            except OSError as e:
                calls.append(("error", str(e)))
                break
            calls.append((n, off, nb, desc[:2 * n].tobytes(), wire[:n].tobytes(), tsn[:n].tobytes()))
            if n == 0:
                break
    finally:
        rd.close()
    return calls


@pytest.mark.parametrize("variant", ["plain", "fake_chains", "truncated", "bad_mid", "nano_swapped"])
def test_reader_parallel_index_is_the_sequential_walk(tmp_path, variant):
    """fcpcap_index with 2-8 threads (chunks of >= 8 MiB walked in pieces,
    speculative piece starts, stitched) gives exactly the one-thread walk's
    calls: counts, chunk offsets and sizes, descriptors, wire lengths and
    time stamps -- also when frame payloads hold false record chains, the last
    record is cut, or a bad header (caplen > 65535) sits mid-file."""
    rng = np.random.default_rng(41)
    frames, total = [], 0
    noise = rng.integers(0, 256, 1 << 21, dtype=np.uint8).tobytes()
    while total < (26 << 20):
        if variant == "fake_chains" and rng.random() < 0.4:
            fr = _fake_chain_frame(rng, int(rng.integers(18, 60)))
        else:
            a = int(rng.integers(0, len(noise) - 1600))
            fr = noise[a:a + int(rng.integers(40, 1600))]
        frames.append(fr)
        total += len(fr) + 16
    p = str(tmp_path / "big.pcap")
    kw = {}
    if variant == "nano_swapped":
        kw = dict(magic=0xA1B23C4D, swapped=True)
    write_pcap(p, frames, cut_last=7 if variant == "truncated" else 0, **kw)
    if variant == "bad_mid":
        # frame 20000's header: caplen 70000 (FromDump: "bad packet header")
        off = 24 + sum(len(f) + 16 for f in frames[:20000])
        with open(p, "r+b") as f:
            f.seek(off + 8)
            f.write(struct.pack("<II", 70000, 70000))
    for max_pkts, max_bytes in ((1 << 20, 24 << 20), (40_000, 16 << 20), (1 << 20, 9 << 20)):
        ref = _index_all(p, 1, max_pkts, max_bytes)
        assert sum(c[0] for c in ref if c[0] != "error") > 0
        if variant == "bad_mid":
            assert ref[-1][0] == "error"
        for t in (2, 4, 8):
            assert _index_all(p, t, max_pkts, max_bytes) == ref, (t, max_pkts, max_bytes)
