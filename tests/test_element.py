"""The drop-in BatchElement (GPUIPCheckClassify) driven like a Click graph.

Source(BURST packets per PacketBatch) -> GPUIPCheckClassify(...) => Sink per
output. Checks the element-level contract of the replaced chain:
  - each packet leaves exactly once, on the output CLASSIFY_EACH_PACKET picks
    (invalid ones on output N if it exists, else killed);
  - input order is preserved within every output;
  - AGGREGATE / DST_IP annotations, take() trimming, header marks, Strip;
  - handlers count / drops / drop_details in CheckIPHeader's format.
"""
import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N
from tests.helpers import set_fragment

CONF = "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash, DETAILS true, BADSRC 192.0.2.255)"


def test_config_errors():
    from fastclick_amd import click as K
    K.check_config(CONF)
    for bad, msg in [("GPUIPCheckClassify(14)", "too many arguments"),
                     ("GPUIPCheckClassify(CHECKSUM maybe)", "CHECKSUM"),
                     ("GPUIPCheckClassify(N 65)", "N out of range"),
                     ("GPUIPCheckClassify(HASHSWITCH 26 0)", "length must be > 0"),
                     ("GPUIPCheckClassify(NATIVE_VLAN 5000)", "NATIVE_VLAN"),
                     ("GPUIPCheckClassify(OFFSET x)", "OFFSET"),
                     ("NoSuchElement", "unknown element class")]:
        with pytest.raises(K.ConfigError, match=msg):
            K.check_config(bad)


def _addrs(words, n):
    return [N.raw_addr(a) for a in words][:n]


def test_interfaces_keyword():
    """INTERFACES (CheckIPHeader::InterfacesArg, checkipheader.cc:56-80): each
    prefix's broadcast address is a bad source and its address a good
    destination, then 0.0.0.0 and 255.255.255.255; BADSRC / GOODDST, read
    after it, replace those lists whatever the keyword order."""
    from fastclick_amd import click as K
    c = K.element_cfg("GPUIPCheckClassify(OFFSET 14, INTERFACES 18.26.4.9/24 1.0.0.1/255.0.0.0 10.0.0.5 "
                      "18.26.7/24)")
    bad = ["18.26.4.255", "1.255.255.255", "10.0.0.5", "18.26.7.255", "0.0.0.0", "255.255.255.255"]
    good = ["18.26.4.9", "1.0.0.1", "10.0.0.5", "18.26.7.0"]
    assert list(c.badsrc)[:c.nbadsrc] == _addrs(bad, 99)
    assert list(c.gooddst)[:c.ngooddst] == _addrs(good, 99)
    for conf in ("GPUIPCheckClassify(INTERFACES 18.26.4.9/24, BADSRC 192.0.2.1)",
                 "GPUIPCheckClassify(BADSRC 192.0.2.1, INTERFACES 18.26.4.9/24)"):
        c = K.element_cfg(conf)
        assert list(c.badsrc)[:c.nbadsrc] == _addrs(["192.0.2.1"], 9)
        assert list(c.gooddst)[:c.ngooddst] == _addrs(["18.26.4.9"], 9)
    c = K.element_cfg("GPUIPCheckClassify(GOODDST 10.1.1.1, INTERFACES 18.26.4.9/24)")
    assert list(c.badsrc)[:c.nbadsrc] == _addrs(["18.26.4.255", "0.0.0.0", "255.255.255.255"], 9)
    assert list(c.gooddst)[:c.ngooddst] == _addrs(["10.1.1.1"], 9)
    for bad_conf in ("GPUIPCheckClassify(INTERFACES 18.26/24)",       # mask past the bytes given
                     "GPUIPCheckClassify(INTERFACES 18.26.4.9/33)",
                     "GPUIPCheckClassify(INTERFACES 300.1.1.1/8)",
                     "GPUIPCheckClassify(INTERFACES host.example/24)"):
        with pytest.raises(K.ConfigError, match="INTERFACES"):
            K.element_cfg(bad_conf)


@pytest.mark.gpu
def test_element_interfaces(oracle):
    """INTERFACES end to end: sources on the interfaces' broadcast addresses
    are dropped unless sent to an interface address (BAD_SADDR rule)."""
    from fastclick_amd import click as K
    rng = np.random.default_rng(520)
    n = 6000
    src = rng.integers(0, 2**32, n, dtype=np.uint64)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64)
    cand_src = [synth.ip4(18, 26, 4, 255), synth.ip4(1, 255, 255, 255), synth.ip4(0, 0, 0, 0),
                synth.ip4(255, 255, 255, 255)]
    cand_dst = [synth.ip4(18, 26, 4, 9), synth.ip4(1, 0, 0, 1)]
    pick = rng.random(n)
    src = np.where(pick < 0.3, np.array(cand_src, np.uint64)[rng.integers(0, 4, n)], src)
    dst = np.where(rng.random(n) < 0.3, np.array(cand_dst, np.uint64)[rng.integers(0, 2, n)], dst)
    hdr = synth.build_headers(n, src=src, dst=dst, sport=rng.integers(0, 2**16, n, dtype=np.uint32),
                              dport=rng.integers(0, 2**16, n, dtype=np.uint32), frame_len=60, width=64)
    b = synth.pack(hdr, 60)
    conf = "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4, LB_MODE hash, INTERFACES 18.26.4.9/24 1.0.0.1/8)"
    cfg = K.element_cfg(conf)
    e = oracle.process_batch(cfg, b)
    assert 0 < int((e["reason"] == N.R_BAD_SADDR).sum()) < n
    r = K.run_element(conf, b, nsinks=5)
    assert np.array_equal(r["port"], e["port"].astype(np.uint32))
    assert int(r["handlers"]["drops"]) == int((e["reason"] != N.R_OK).sum())


def expected(batch, cfg, oracle):
    return oracle.process_batch(cfg, batch)


def _cfg_for_conf():
    return N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16,
                      badsrc=[N.raw_addr("192.0.2.255")])


@pytest.mark.gpu
@pytest.mark.parametrize("nsinks,batch,part", [(17, 0, "TILE"), (16, 0, "TILE"), (17, 4096, "TILE"),
                                               (17, 4096, "GLOBAL"), (16, 100000, "GLOBAL")])
def test_element_outputs_order_annotations(oracle, nsinks, batch, part):
    from fastclick_amd import click as K
    b = synth.c4(20_000, seed=500)
    synth.add_ip_options(b, 0.1, seed=501)
    synth.inject_errors(b, 0.02, seed=502)
    conf = CONF[:-1] + f", BATCH {batch}, PARTITION {part})"
    r = K.run_element(conf, b, burst=32, nsinks=nsinks)
    e = expected(b, _cfg_for_conf(), oracle)
    port = e["port"].astype(np.uint32)
    exp_port = np.where(port < nsinks, port, 0xFFFFFFFF)
    assert np.array_equal(r["port"], exp_port)
    ok = e["reason"] == N.R_OK
    assert np.array_equal(r["agg"][ok], e["hash"][ok])
    assert np.array_equal(r["dst"][ok], e["anno"]["dst_ip"][ok])
    assert np.array_equal(r["len"][ok], e["anno"]["length"][ok])
    assert np.array_equal(r["nh"][ok], e["anno"]["nh"][ok].astype(np.int32))
    # every output keeps input order
    for p in range(nsinks):
        idx = np.nonzero(r["port"] == p)[0]
        assert (np.diff(r["seq"][idx].astype(np.int64)) > 0).all()
    h = r["handlers"]
    assert int(h["count"]) == int(ok.sum()) and int(h["drops"]) == int((~ok).sum())
    lines = h["drop_details"].strip("\n").split("\n")
    assert len(lines) == 6
    for i, line in enumerate(lines):
        assert line.endswith(N.REASON_TEXTS[i]) and " packets due to: " in line
        assert int(line.split()[0]) == int((e["reason"] == i).sum())
    if batch and part == "GLOBAL":
        assert r["batches"] <= 2 * 17 * (b.n // batch + 1) + 40


@pytest.mark.gpu
def test_element_strip_and_auto(oracle):
    from fastclick_amd import click as K
    b = synth.c5(10_000, seed=510)
    r = K.run_element("GPUIPCheckClassify(MODE AUTO, CHECKSUM true, N 8, LB_MODE hash)", b, nsinks=9)
    e = oracle.process_batch(N.make_cfg(check_mode=N.CHECK_AUTO, checksum=True,
                                        classify=N.CLS_LB_HASH, nports=8), b)
    assert np.array_equal(r["port"], e["port"].astype(np.uint32))
    ok = e["reason"] == N.R_OK
    # MODE AUTO strips like StripEtherVLANHeader: data starts at the IP header
    assert (r["nh"][ok] == 0).all()
    assert np.array_equal(r["len"][ok], e["anno"]["length"][ok] - e["anno"]["nh"][ok])
    assert np.array_equal(r["agg"][ok], e["hash"][ok])


@pytest.mark.gpu
def test_element_golden_flowswitch():
    """Element-level parity with the reference FlowSwitch goldens."""
    from fastclick_amd import click as K
    from tests.test_golden import load, batch_of, first_fragment_mask
    g = load("ip4")
    b = batch_of(g)
    r = K.run_element("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash, "
                      "BADSRC 192.0.2.255 255.255.255.255, GOODDST 10.9.9.9)", b, nsinks=17)
    ff = first_fragment_mask(g)
    pin = (g["lb16"] != 255) & ff
    assert np.array_equal(r["port"][pin], g["lb16"][pin].astype(np.uint32))
    ok = (g["reason"] == 6) & ff
    assert np.array_equal(r["agg"][ok], g["hash"][ok])
    assert np.array_equal(r["len"][g["reason"] == 6], g["length"][g["reason"] == 6])
    assert np.array_equal(r["port"] == 16, g["reason"] != 6)


@pytest.mark.gpu
def test_element_fragments_and_burst_sizes(oracle):
    from fastclick_amd import click as K
    b = synth.c3(8_000, seed=520)
    set_fragment(b, 0.2)
    e = oracle.process_batch(N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=4), b)
    for burst in (1, 32, 256, 8000):
        r = K.run_element("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4)", b, burst=burst, nsinks=5)
        assert np.array_equal(r["port"], e["port"].astype(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [0, 1024])
def test_element_per_packet_push(oracle, batch):
    """A non-batch upstream (Element::push per packet, lib/element.cc:3141-3147):
    packets are staged like a batch's, so outputs, order and annotations equal
    the BURST-32 run's and the oracle's."""
    from fastclick_amd import click as K
    b = synth.c3(3_000, seed=521)
    set_fragment(b, 0.1)
    conf = f"GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4, BATCH {batch})"
    e = oracle.process_batch(N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=4), b)
    r1 = K.run_element(conf, b, burst=K.PER_PACKET, nsinks=5)
    r32 = K.run_element(conf, b, burst=32, nsinks=5)
    assert np.array_equal(r1["port"], e["port"].astype(np.uint32))
    # without BATCH every single push is its own launch, so arrival order at the
    # sinks is input order rather than per-burst port order
    for k in ("port", "agg", "len", "dst") + (("seq",) if batch else ()):
        assert np.array_equal(r1[k], r32[k]), k
    if not batch:
        reached = r1["seq"] != 0xFFFFFFFF
        assert reached.sum() > 0.9 * b.n
        assert np.all(np.diff(r1["seq"][reached].astype(np.int64)) > 0)
    assert r1["handlers"] == r32["handlers"]


def test_config_color_keyword():
    from fastclick_amd import click as K
    K.check_config("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, STRIP true, COLOR 7)")
    with pytest.raises(K.ConfigError, match="COLOR"):
        K.check_config("GPUIPCheckClassify(COLOR 300)")


@pytest.mark.gpu
def test_element_ipinputcombo_golden():
    """IPInputCombo(7, BADSRC .., GOODDST ..) (ipinputcombo.cc:65-141) as the
    element in COLOR/STRIP mode with one output: the reference's survivors
    (tests/golden/combo.npz) leave in order with PAINT 7, the IP header at
    data(), length = ip_len; every other packet is killed."""
    from fastclick_amd import click as K
    from tests.test_golden import load, batch_of
    g = load("ip4")
    c = load("combo")
    r = K.run_element("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, STRIP true, COLOR 7, "
                      "BADSRC 192.0.2.255 255.255.255.255, GOODDST 10.9.9.9)", batch_of(g), nsinks=1)
    ok = c["valid"] == 1
    assert np.array_equal(r["port"] == 0, ok)
    assert (r["port"][~ok] == 0xFFFFFFFF).all()
    assert (r["paint"][ok] == 7).all()
    assert np.array_equal(r["len"][ok], c["ip_len"][ok].astype(np.uint32))
    assert (r["nh"][ok] == 0).all()
    assert np.all(np.diff(r["seq"][ok].astype(np.int64)) > 0)


def test_config_ip6_keywords():
    from fastclick_amd import click as K
    K.check_config("GPUIPCheckClassify(MODE AUTO, BADADDRS 2001:db8::bad ffff:ffff:ffff:ffff:ffff:ffff:ffff:ffff, "
                   "PROCESS_EH true)")
    for bad, msg in [("GPUIPCheckClassify(MODE AUTO, BADADDRS 10.0.0.1)", "BADADDRS"),
                     ("GPUIPCheckClassify(MODE AUTO, PROCESS_EH sometimes)", "PROCESS_EH")]:
        with pytest.raises(K.ConfigError, match=msg):
            K.check_config(bad)


@pytest.mark.gpu
def test_element_ip6_extension_headers():
    """CheckIP6Header(BADADDRS .., PROCESS_EH true) through the element (MODE
    AUTO, STRIP): reference verdicts; valid packets leave with the transport
    header where the reference put it and the reference's trimmed length."""
    from fastclick_amd import click as K
    from tests.test_golden import load, batch_of
    g = load("eh")
    r = K.run_element("GPUIPCheckClassify(MODE AUTO, BADADDRS 2001:db8::bad, PROCESS_EH true, N 1, "
                      "LB_MODE hash)", batch_of(g), nsinks=2)
    ok = g["eh_valid"] == 1
    assert np.array_equal(r["port"] == 0, ok) and (r["port"][~ok] == 1).all()
    # STRIP (MODE AUTO default): data() at the IPv6 header, length trimmed
    assert np.array_equal(r["len"][ok], g["eh_length"][ok].astype(np.uint32) - 14)
    assert (r["nh"][ok] == 0).all()


@pytest.mark.gpu
def test_element_flow_golden():
    """GPUIPCheckClassify(FLOW_CAPACITY ..): the flow ID annotation of every
    surviving packet equals FlowIPManagerHMP's (tests/golden/flow.npz); with a
    small capacity the new flows beyond it are killed and counted."""
    from fastclick_amd import click as K
    from tests.test_golden import load, batch_of
    g = load("flow")
    b = batch_of(g)
    ref = g["flowid"]
    for burst, batch in ((32, 1024), (256, 0)):
        r = K.run_element(f"GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4, FLOW_CAPACITY 100000, BATCH {batch})",
                          b, burst=burst, nsinks=5)
        ok = ref != 0xFFFFFFFF
        assert np.array_equal(r["flow"][ok], ref[ok])
        assert r["handlers"]["flow_count"] == str(int(ref[ok].max()) + 1)
    r = K.run_element("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4, FLOW_CAPACITY 40, BATCH 512)", b,
                      nsinks=5)
    full = (ref >= 40) & (ref != 0xFFFFFFFF)
    assert (r["port"][full] == 0xFFFFFFFF).all()
    assert np.array_equal(r["flow"][ref < 40], ref[ref < 40])
    assert r["handlers"]["flow_drops"] == str(int(full.sum()))


@pytest.mark.gpu
@pytest.mark.parametrize("runs", [True, False])
def test_element_flow_runs(runs):
    """FLOW_RUNS (default true): behind the flow table the packets of each
    output leave as one PacketBatch per run of one flow, as the flow managers'
    BatchBuilder pushes them (flowipmanagerhmp.cc:101-117,
    virtualflowmanager.hh:304-326). Departures come per device batch (BATCH),
    per 256-packet tile, per output; a new batch starts exactly where the
    output, the tile or (with runs) the flow changes. Invalid packets (output
    N) have no flow and leave as one batch per tile."""
    from fastclick_amd import click as K
    b = synth.c3(20_000, nflows=20, seed=80)
    synth.inject_errors(b, 0.01, seed=81)
    batch, nports = 4096, 4
    conf = (f"GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N {nports}, FLOW_CAPACITY 1024, BATCH {batch}"
            + ("" if runs else ", FLOW_RUNS false") + ")")
    r = K.run_element(conf, b, nsinks=nports + 1)
    left = np.nonzero(r["port"] != 0xFFFFFFFF)[0]
    order = left[np.argsort(r["seq"][left])]
    port = r["port"][order].astype(np.int64)
    flow = np.where(port < nports, r["flow"][order].astype(np.int64), -1) if runs else np.zeros(len(order), np.int64)
    key = np.stack([port, order // batch, (order % batch) // 256, flow], axis=1)
    change = np.any(key[1:] != key[:-1], axis=1)
    assert r["batches"] == int(change.sum()) + 1
    bi = r["batch"][order]
    assert np.array_equal(bi[1:] != bi[:-1], change)
    if runs:   # every batch behind the table holds one flow
        valid = port < nports
        pairs = np.unique(np.stack([bi[valid], flow[valid]], axis=1), axis=0)
        assert len(pairs) == len(np.unique(bi[valid]))


def test_config_flow_keywords():
    from fastclick_amd import click as K
    K.check_config("GPUIPCheckClassify(OFFSET 14, FLOW_CAPACITY 65536, FLOWID_ANNO 32)")
    with pytest.raises(K.ConfigError, match="FLOW_CAPACITY needs"):
        K.check_config("GPUIPCheckClassify(MODE AUTO, FLOW_CAPACITY 10)")
    with pytest.raises(K.ConfigError, match="FLOWID_ANNO"):
        K.check_config("GPUIPCheckClassify(FLOWID_ANNO 46)")
    K.check_config("GPUIPCheckClassify(OFFSET 14, FLOW_CAPACITY 64, FLOW_RUNS false)")
    with pytest.raises(K.ConfigError, match="FLOW_RUNS"):
        K.check_config("GPUIPCheckClassify(FLOW_RUNS maybe)")


@pytest.mark.gpu
def test_element_dec_ttl_golden():
    """GPUIPCheckClassify(DEC_TTL true[, SET_CHECKSUM true]): survivors carry
    the reference's rewritten ttl/checksum bytes; TTL-expired packets leave on
    output N (DecIPTTL output 1) -- tests/golden/rw.npz."""
    from fastclick_amd import click as K
    from tests.test_golden import load, batch_of
    g = load("rw")
    b = batch_of(g)
    for conf, key in (("DEC_TTL true", "dec"), ("DEC_TTL true, TTL_MULTICAST false", "decnm"),
                      ("DEC_TTL true, SET_CHECKSUM true", "decset")):
        r = K.run_element(f"GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 2, {conf})", b, nsinks=3)
        ok = g[key] != 0xFFFFFFFF
        assert (r["port"][ok] < 2).all(), key
        assert np.array_equal(r["ip8"][ok], g[key][ok]), key
        if key != "decset":
            assert (r["port"][g[key + "_expired"]] == 2).all(), key


@pytest.mark.gpu
def test_element_timer_releases_tail(oracle):
    """A partial batch (fewer packets than BATCH) is released by the TIMER
    once the source goes quiet -- MinBatch's timer (minbatch.cc:35,57-76) --
    with the same outputs flush() gives; with TIMER -1 nothing releases it."""
    from fastclick_amd import click as K
    b = synth.c4(3_000, seed=510)
    synth.inject_errors(b, 0.03, seed=511)
    conf = CONF[:-1] + ", BATCH 100000, TIMER 200)"
    r = K.run_element(conf, b, burst=32, nsinks=17, timer_flush=True)
    assert r["parked"] == b.n                      # all parked when the source stopped
    ref = K.run_element(conf, b, burst=32, nsinks=17)
    for k in ("port", "seq", "agg", "len"):
        assert np.array_equal(r[k], ref[k]), k
    e = expected(b, _cfg_for_conf(), oracle)
    assert np.array_equal(r["port"], e["port"].astype(np.uint32))
    r2 = K.run_element(CONF[:-1] + ", BATCH 100000, TIMER -1)", b, burst=32, nsinks=17, timer_flush=True)
    assert r2["parked"] == b.n and (r2["port"] == 0xFFFFFFFF).all()


@pytest.mark.gpu
def test_element_drop_chatter_text(capfd):
    """The first drop prints CheckIPHeader's message with the reason text
    (checkipheader.cc:146: "%s: IP header check failed: %s")."""
    from fastclick_amd import click as K
    b = synth.c2(600)
    o = int(b.desc[5, 0]) + 14
    b.arena[o + 10] ^= 0x40                        # packet 5: bad checksum, the first drop
    K.run_element(CONF, b, burst=32, nsinks=17)
    err = capfd.readouterr().err
    assert "GPUIPCheckClassify: IP header check failed: bad IPv4 checksum" in err
    assert err.count("IP header check failed") == 1      # once, not VERBOSE


ZC_CONFS = [
    ("c4", CONF[:-1] + ", BATCH 4096)", 17),
    ("c4", CONF[:-1] + ", BATCH 1000, SLOTS 3)", 17),
    ("c4", CONF[:-1] + ", BATCH 4096, PARTITION GLOBAL)", 17),
    ("c5", "GPUIPCheckClassify(MODE AUTO, CHECKSUM true, N 8, LB_MODE hash, BATCH 2048)", 9),
    ("c3", "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4, L4 UDP, BATCH 3000)", 5),
    ("c4", "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 8, DEC_TTL true, SET_CHECKSUM true, BATCH 4096)", 9),
    ("c4", "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4, FLOW_CAPACITY 5000, BATCH 4096)", 5),
]


@pytest.mark.gpu
@pytest.mark.parametrize("wl,conf,nsinks", ZC_CONFS)
def test_element_zerocopy_matches_copy(oracle, wl, conf, nsinks):
    """ZEROCOPY true (fcgpu_span_mode FCGPU_SPAN_ZEROCOPY: the kernels read the
    pinned staging block and write the results over PCIe, no copy engine)
    gives the element's outputs, annotations, rewritten bytes, flow IDs and
    handlers exactly as the copy mode does, and the oracle's ports."""
    from fastclick_amd import click as K
    b = getattr(synth, wl)(12_345, seed=530)
    if wl != "c5":
        synth.inject_errors(b, 0.02, seed=531)
    a = K.run_element(conf, b, burst=32, nsinks=nsinks)
    z = K.run_element(conf[:-1] + ", ZEROCOPY true)", b, burst=32, nsinks=nsinks)
    for k in ("port", "seq", "agg", "dst", "len", "nh", "flow", "ip8"):
        assert np.array_equal(a[k], z[k]), k
    assert a["handlers"] == z["handlers"]
    if "FLOW" not in conf and "DEC_TTL" not in conf and "L4" not in conf:
        cfg = K.element_cfg(conf)
        e = oracle.process_batch(cfg, b)
        port = e["port"].astype(np.uint32)
        assert np.array_equal(z["port"], np.where(port < nsinks, port, 0xFFFFFFFF))


@pytest.mark.gpu
def test_element_default_with_many_contexts(oracle):
    """The element's defaults (ZEROCOPY auto, BATCH auto) when four more AUTO
    contexts share the GPU, as in a 5-thread configuration: its batches go
    zero-copy through the shared queue, 4096 packets each -- outputs, order,
    annotations and handlers as the oracle says."""
    import ctypes as C
    from fastclick_amd import click as K
    lib = N.load()
    others = []
    try:
        for _ in range(4):
            h = C.c_void_p()
            assert lib.fcgpu_open(0, 4096, C.byref(h)) == N.OK
            assert lib.fcgpu_span_mode(h, N.SPAN_AUTO) == N.OK
            others.append(h)
        b = synth.c4(30_000, seed=540)
        synth.inject_errors(b, 0.02, seed=541)
        r = K.run_element(CONF, b, burst=32, nsinks=17)
        e = expected(b, _cfg_for_conf(), oracle)
        assert np.array_equal(r["port"], e["port"].astype(np.uint32))
        ok = e["reason"] == N.R_OK
        assert np.array_equal(r["agg"][ok], e["hash"][ok])
        assert np.array_equal(r["dst"][ok], e["anno"]["dst_ip"][ok])
        for p in range(17):
            idx = np.nonzero(r["port"] == p)[0]
            assert (np.diff(r["seq"][idx].astype(np.int64)) > 0).all()
        assert int(r["handlers"]["count"]) == int(ok.sum())
    finally:
        for h in others:
            lib.fcgpu_close(h)


def test_config_span_keywords():
    """ZEROCOPY true|false|auto, BATCH <n>|auto, SLOTS 2|3 (host-side parsing;
    the GPU tests above run each mode)."""
    from fastclick_amd import click as K
    for ok in ("ZEROCOPY auto", "ZEROCOPY true", "ZEROCOPY false", "BATCH auto", "BATCH 0", "BATCH 4096",
               "SLOTS 2", "SLOTS 3", "ZEROCOPY AUTO, BATCH AUTO, SLOTS 3"):
        K.check_config(f"GPUIPCheckClassify(OFFSET 14, {ok})")
    for bad, msg in (("ZEROCOPY maybe", "ZEROCOPY"), ("SLOTS 1", "SLOTS"), ("SLOTS 4", "SLOTS"),
                     ("BATCH -1", "BATCH"), ("BATCH many", "BATCH")):
        with pytest.raises(K.ConfigError, match=msg):
            K.check_config(f"GPUIPCheckClassify(OFFSET 14, {bad})")


COMPACT_CONFS = [
    ("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash, DETAILS true)", 17),
    ("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 8, LB_MODE hash_crc)", 9),
    ("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 5, LB_MODE hash_ip)", 6),
    ("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, HASHSWITCH 6 8, N 7)", 8),
    ("GPUIPCheckClassify(OFFSET 14, MODE MARK, N 4, LB_MODE hash_agg, HASH FLOW5ID)", 5),
    ("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4, L4 TCP, L4_CHECKSUM false)", 5),
    ("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 8, DEC_TTL true, SET_CHECKSUM true)", 9),
    ("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4, FLOW_CAPACITY 5000)", 5),
    ("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4, LB_MODE hash, L4 UDP)", 5),
    ("GPUIPCheckClassify(OFFSET 14, MODE MARK, N 4, LB_MODE hash_agg, HASH FLOW5ID, L4 UDP)", 5),
]


@pytest.mark.gpu
@pytest.mark.parametrize("conf,nsinks", COMPACT_CONFS)
@pytest.mark.parametrize("zc", ["false", "true"])
def test_element_compact_records_match_full(oracle, conf, nsinks, zc):
    """COMPACT true (the default: each packet stages only the frame bytes the
    chain reads -- header, options, ports / L4 length words, hash_ip's and
    HashSwitch's ranges -- in 16-B records whose neighbours are other
    packets' bytes) against COMPACT false (whole 64-B-slot captures): the same
    outputs, order, annotations, rewritten bytes, flow IDs and handlers, on
    packets with IP options, every header error, non-first fragments, TCP
    frames and truncated ones, in copy and zero-copy mode."""
    from fastclick_amd import click as K
    b = _hostile_batch(560)
    base = conf[:-1] + f", BATCH 4096, ZEROCOPY {zc}"
    full = K.run_element(base + ", COMPACT false)", b, burst=32, nsinks=nsinks)
    comp = K.run_element(base + ")", b, burst=32, nsinks=nsinks)
    e = oracle.process_batch(K.element_cfg(conf), b)
    if "MARK" in conf:
        # MarkIPHeader checks nothing: ports past a truncated packet's end are
        # whatever follows it in memory, for the reference as for either
        # staging (undefined); compared where defined
        ln = b.desc[:, 1].astype(np.int64)
        defined = (e["anno"]["th"].astype(np.int64) + 4 <= ln) & (14 + 20 <= ln)
        assert defined.sum() > 0.9 * b.n
        for k in ("port", "agg", "dst", "len", "nh"):
            assert np.array_equal(full[k][defined], comp[k][defined]), k
    else:
        for k in ("port", "seq", "agg", "dst", "len", "nh", "flow", "ip8", "batch"):
            assert np.array_equal(full[k], comp[k]), k
        assert full["handlers"] == comp["handlers"]
    if "FLOW" not in conf and "DEC_TTL" not in conf and "L4" not in conf:
        port = e["port"].astype(np.uint32)
        inside = (e["anno"]["th"].astype(np.int64) + 4 <= b.desc[:, 1].astype(np.int64)) | ("MARK" not in conf)
        assert np.array_equal(comp["port"][inside], np.where(port < nsinks, port, 0xFFFFFFFF)[inside])


def _hostile_batch(seed):
    from tests.helpers import set_fragment
    b = synth.c4(6000 + 11, seed=seed)
    synth.set_udp_checksums(b)               # CheckUDPHeader verifies them (options added below break some)
    synth.add_ip_options(b, 0.2, seed=seed + 1)
    synth.inject_errors(b, 0.03, seed=seed + 2)
    set_fragment(b, 0.05, seed=seed + 3)
    rng = np.random.default_rng(seed + 4)
    off = b.desc[:, 0].astype(np.int64) + 14
    tcp = rng.random(b.n) < 0.2
    b.arena[off[tcp] + 9] = 6
    for i in np.nonzero(tcp)[0]:
        o = int(off[i])
        th = o + (int(b.arena[o]) & 15) * 4
        if th + 13 <= int(b.desc[i, 0]) + int(b.desc[i, 1]):
            b.arena[th + 12] = 0x50                    # th_off 5: a well-formed TCP header
        synth._refresh_cksum(b.arena, o)
    short = rng.random(b.n) < 0.02
    b.desc[short, 1] = rng.integers(0, 40, int(short.sum()))
    return b


@pytest.mark.parametrize("conf", [c for c, _ in COMPACT_CONFS] + [
    "GPUIPCheckClassify(OFFSET 30, CHECKSUM true, N 5, LB_MODE hash_ip)",
    "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, HASHSWITCH 40 30, N 3)",
    "GPUIPCheckClassify(OFFSET 0, CHECKSUM true, N 8, LB_MODE hash)"])
def test_compact_layout_decides_nothing_else(oracle, conf):
    """The compact staging rule (capture.hh stage_plan / stage_end, exported
    as fcclick_stage_compact) against the oracle on the CPU: the oracle run
    on the compact layout -- only the bytes the chain reads, every other
    arena byte random -- gives the verdicts, ports, hashes and annotations it
    gives on the frames themselves, on packets with IP options, header
    errors, fragments, TCP and truncated frames."""
    from fastclick_amd import click as K
    b = _hostile_batch(580)
    if "OFFSET 0" in conf:     # IP packets without an Ethernet header
        b = synth.from_frames([f[14:] for f in b.frames()])
    if "OFFSET 30" in conf:    # 16 more bytes ahead of the IP header
        b = synth.from_frames([bytes(16) + f for f in b.frames()])
    rng = np.random.default_rng(581)
    comp = K.stage_compact(conf, b, fill=rng.integers(0, 256, 256 + 128 * b.n + 4096, dtype=np.uint8))
    assert comp is not None
    cfg = K.element_cfg(conf)
    ref = oracle.process_batch(cfg, b)
    got = oracle.process_batch(cfg, comp)
    ok = ref["reason"] == N.R_OK
    defined = np.ones(b.n, bool)
    if "MARK" in conf:       # ports / addresses past a truncated packet's end: undefined
        ln = b.desc[:, 1].astype(np.int64)
        defined = (ref["anno"]["th"].astype(np.int64) + 4 <= ln) & (14 + 20 <= ln)
    assert ok.sum() > (200 if "L4" in conf else 1000)
    for k in ("reason", "port"):
        assert np.array_equal(got[k][defined], ref[k][defined]), k
    both = ok & defined
    assert np.array_equal(got["hash"][both], ref["hash"][both])
    for f in ("dst_ip", "length", "nh", "th"):
        assert np.array_equal(got["anno"][f][both], ref["anno"][f][both]), f
    if cfg.rewrite:
        assert np.array_equal(got["ip_rw"][ok], ref["ip_rw"][ok])
    # and the layout is compact: records packed 8 B apart, far below the 64-B slots
    steps = np.diff(np.sort(comp.desc[:, 0].astype(np.int64)))
    assert (steps % 8 == 0).all() and np.median(steps) <= 48


def test_compact_layout_not_for_whole_captures():
    from fastclick_amd import click as K
    b = synth.c4(100, seed=590)
    for conf in ("GPUIPCheckClassify(MODE AUTO, N 2, LB_MODE hash)",
                 "GPUIPCheckClassify(OFFSET 14, N 2, PROGRAM \" 0 265/11000000%ff000000  yes->[0]  no->[1]\")"):
        assert K.stage_compact(conf, b) is None


@pytest.mark.gpu
def test_element_bench_timed_runs_and_checks():
    """fcclick_bench_timed (the element pushed for a fixed time, as the CPU
    baseline's threads are): 2 threads for 0.3 s give a rate; the element's
    errors and a non-positive duration are reported, not timed."""
    from fastclick_amd import click as K
    b = synth.c2(1 << 14)
    conf = "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash)"
    pps = K.bench_element(conf, b, threads=2, seconds=0.3)
    assert pps > 1e6
    with pytest.raises(RuntimeError, match="seconds"):
        K.bench_element(conf, b, threads=1, seconds=0.0)
    with pytest.raises(RuntimeError):
        K.bench_element("GPUIPCheckClassify(OFFSET 14, N 0)", b, threads=1, seconds=0.1)


@pytest.mark.gpu
@pytest.mark.parametrize("zc", ["false", "true"])
def test_element_compact_rest_of_frame_imix(oracle, zc):
    """CheckUDPHeader's checksum over IMIX datagrams (64 / 570 / 1500-B
    frames, valid non-zero checksums, 3 % header errors): records holding the
    frame from OFFSET to its end (COMPACT true) against whole captures."""
    from fastclick_amd import click as K
    b = synth.c3(9000, nflows=500, seed=610)
    synth.set_udp_checksums(b)
    synth.inject_errors(b, 0.03, seed=611)
    conf = f"GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 8, LB_MODE hash, L4 UDP, BATCH 4096, ZEROCOPY {zc}"
    full = K.run_element(conf + ", COMPACT false)", b, burst=32, nsinks=9)
    comp = K.run_element(conf + ")", b, burst=32, nsinks=9)
    for k in ("port", "seq", "agg", "dst", "len", "nh", "batch"):
        assert np.array_equal(full[k], comp[k]), k
    assert full["handlers"] == comp["handlers"]
    e = oracle.process_batch(K.element_cfg(conf + ")"), b)
    ok = e["reason"] == N.R_OK
    assert ok.sum() > 0.75 * b.n
    assert np.array_equal(comp["agg"][ok], e["hash"][ok])


@pytest.mark.gpu
@pytest.mark.parametrize("zc", ["false", "true"])
def test_element_desc32_widens_for_giant_frames(oracle, zc):
    """Compact records go to the device with 4-B descriptors (16-bit
    lengths); a frame longer than 65535 B in the middle of a batch turns the
    slot's descriptors back into (offset, length) pairs: every output the
    same as whole-capture staging."""
    from fastclick_amd import click as K
    b = synth.c4(3000, seed=620)
    frames = [b.frame(i) for i in range(b.n)]
    giant = bytearray(frames[7]) + bytes(65_600 - len(frames[7]))    # ip_len 46: take() trims it
    frames[1500] = bytes(giant)
    g = synth.from_frames(frames)
    conf = f"GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 8, LB_MODE hash, BATCH 1024, ZEROCOPY {zc}"
    full = K.run_element(conf + ", COMPACT false)", g, burst=32, nsinks=9)
    comp = K.run_element(conf + ")", g, burst=32, nsinks=9)
    for k in ("port", "seq", "agg", "dst", "len", "nh", "batch"):
        assert np.array_equal(full[k], comp[k]), k
    assert full["handlers"] == comp["handlers"]
    e = oracle.process_batch(K.element_cfg(conf + ")"), g)
    assert e["reason"][1500] == N.R_OK and comp["len"][1500] == 60
