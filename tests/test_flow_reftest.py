"""The IMP flow manager pinned by the reference's own flow tests.

test/flow/flow-no-dynamic.clicktest and test/flow/flow-dynamic.clicktest
(tests/golden/refvectors.json "flow", written by tests/golden/gen_refvectors.py)
push five UDP packets -- FromIPSummaryDump(CHECKSUM true, TIMING true[, BURST
2]) at t = 1, 3, 3, 3.1, 5 s -- through FlowIPManager_CuckooPP(RESERVE 2,
TIMEOUT 5): the IMP manager (include/click/flow/virtualflowmanager.hh:52-327)
with CAPACITY 65536 (the default, :64) and RECYCLE_INTERVAL 1 s (:69). Their
%expect sections state:
  * the flow IDs FlowPrint reports: 65535, 65534, 65534, 65534, 65533 -- pops
    from the top of the free-ID stack (:36-38, 264), flow 2's three packets
    sharing one ID, and flow 1's ID still out when flow 3 arrives (it expires
    at the maintainer run 5 s after its last packet, :185-205, and goes back
    on the stack one run later, :155-161);
  * with BURST 2, packets 2 and 3 arrive in one PacketBatch and leave as one
    run of flow 65534 (BatchBuilder, :304-326);
  * DriverManager's reads: count 0 / 1 / 0 and count_fids 0 / 65535 / 65536 at
    t = 0, 2, 12 s (count_fids is flows_stack_i, :389-391; the table's
    count is what the maintainer has not removed).
Each packet's first 24 bytes equal the test's Print lines (asserted by the
generator), so their IP header checksums -- the reference's click_in_cksum
output -- are A1 vectors too.

One documented divergence: the reference's first count_fids read (t = 0,
before any packet) prints 0. flows_stack_i is per thread and DriverManager's
first step reads a thread whose table does not exist (per_thread::operator->
indexes the calling thread's slot, include/click/sync.hh:109-113; the tables
live only on the passing threads, virtualflowmanager.hh:87-88); after the
initial pushes of 0 .. cap-1 a table's index is cap (:113-115). Here the
table exists from initialize, so that read gives 65536; every later read
matches the reference's text.
"""
import json
import os

import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
T0 = 10_000          # ms: the first packet's time on the element's clock (any origin)


def flowvec():
    with open(os.path.join(HERE, "refvectors.json")) as f:
        return json.load(f)["flow"]


def frames():
    return [bytes.fromhex(p["frame"]) for p in flowvec()["packets"]]


def pkt_ms(v):
    """FromIPSummaryDump TIMING: the first packet goes at once, the others at
    their timestamp offsets from it (fromipsumdump.cc:759-768)."""
    t = [p["t"] for p in v["packets"]]
    return [T0 + round((x - t[0]) * 1000) for x in t]


def script(v, key, maint_first=True):
    """The run as events on one clock (ms): ('b', packet indices, t) for each
    source PacketBatch, ('m', t) for each maintainer run (every RECYCLE_INTERVAL
    from t0, virtualflowmanager.hh:118-124,134-144), ('r', t) for each
    DriverManager read time. maint_first: a maintainer run due at the same
    time as a batch runs before it (the element's order); the reference's
    timer order at equal times is not observable in these tests, and both
    orders give its output (test_reference_flow_model/_oracle)."""
    m = v["manager"]
    tms = pkt_ms(v)
    ev, i = [], 0
    for n in v[key]["bursts"]:
        ev.append(("b", list(range(i, i + n)), tms[i]))
        i += n
    reads = [T0 + int(s * 1000) for s in v["read_times_s"]]
    end = reads[-1]
    for k in range(1, (end - T0) // m["recycle_ms"] + 1):
        ev.append(("m", T0 + k * m["recycle_ms"]))
    for t in reads:
        ev.append(("r", t))
    # time order; at one time the reads come first (the reference's read at
    # 2 s shows flow 1 only: it comes before the packets sent at 2 s), then the
    # maintainer run and the batch in either order
    rank = {"r": 0, "m": 1 if maint_first else 3, "b": 2}
    ev.sort(key=lambda e: (e[-1], rank[e[0]]))
    return ev


def expected_reads(v, key):
    """(count, count_fids) the reference printed at each read time; None where
    it printed nothing. The t = 0 count_fids is the documented divergence."""
    out = []
    for k, t in enumerate(v["read_times_s"]):
        before = {0: 0, 1: 1, 2: 5}[k]
        vals = {r["handler"]: r["value"] for r in v[key]["reads"] if r["after_packets"] == before}
        out.append((vals.get("count"), vals.get("count_fids")))
    return out


def batch_of(idx):
    fs = frames()
    return synth.from_frames([fs[i] for i in idx])


def cfg():
    return N.make_cfg(offset=0, checksum=True, classify=N.CLS_LB_HASH, nports=1)


def test_flow_vectors_fixture():
    v = flowvec()
    assert v["manager"] == dict(kind="FlowIPManager_CuckooPP", capacity=65536, timeout_s=5, recycle_ms=1000)
    assert v["single"]["ids"] == v["burst2"]["ids"] == [65535, 65534, 65534, 65534, 65533]
    assert v["single"]["bursts"] == [1] * 5 and v["burst2"]["bursts"] == [1, 2, 1, 1]
    assert [r["packets"] for r in v["burst2"]["runs"]] == [[0], [1, 2], [3], [4]]
    assert expected_reads(v, "single") == [("0", "0"), ("1", "65535"), ("0", "65536")]
    assert expected_reads(v, "burst2") == [("0", None), ("1", "65535"), ("0", "65536")]


def test_flow_packets_checksums(oracle):
    """A1: the IP headers the reference wrote (Print lines) verify to 0; the
    packets pass CheckIPHeader(OFFSET 0, CHECKSUM true) and the restated UDP
    checksums pass CheckUDPHeader."""
    for f in frames():
        assert oracle.in_cksum(f[:20]) == 0
    b = synth.from_frames(frames())
    r = oracle.process_batch(cfg(), b)
    assert (r["reason"] == N.R_OK).all()
    r = oracle.process_batch(N.make_cfg(offset=0, checksum=True, classify=N.CLS_LB_HASH, nports=1,
                                        l4_mode=N.L4_UDP, l4_checksum=True), b)
    assert (r["reason"] == N.R_OK).all()


def keys(idx):
    fs = frames()
    return [(fs[i][12:16], fs[i][16:20], fs[i][20:24], fs[i][9]) for i in idx]


def run_model(v, key, maint_first=True):
    from test_flow_imp import ImpModel
    m = v["manager"]
    t = ImpModel(m["capacity"], m["timeout_s"], m["recycle_ms"])
    ids, reads = [], []
    for e in script(v, key, maint_first):
        if e[0] == "m":
            t.maintain(e[1])
        elif e[0] == "b":
            ids.extend(int(x) for x in t.batch(keys(e[1]), e[2]))
        else:
            st = t.stats()
            reads.append((str(st["count"]), str(st["free_ids"] + 1)))
    return ids, reads


def run_oracle(O, v, key, maint_first=True):
    m = v["manager"]
    t = O.ImpFlowTable(m["capacity"], m["timeout_s"], m["recycle_ms"])
    ids, reads = [], []
    for e in script(v, key, maint_first):
        if e[0] == "m":
            t.maintain(e[1])
        elif e[0] == "b":
            b = batch_of(e[1])
            ids.extend(int(x) for x in t.batch(b, O.process_batch(cfg(), b), e[2]))
        else:
            st = t.stats()
            reads.append((str(st["count"]), str(st["free_ids"] + 1)))
    return ids, reads


def check_reads(v, key, reads):
    exp = expected_reads(v, key)
    assert len(reads) == len(exp)
    for k, ((c, f), (ec, ef)) in enumerate(zip(reads, exp)):
        assert c == ec, f"read {k}: count {c}, the reference printed {ec}"
        if k == 0:
            # the documented divergence: the reference read a thread with no table
            assert f == str(v["manager"]["capacity"]) and ef in ("0", None)
        elif ef is not None:
            assert f == ef, f"read {k}: count_fids {f}, the reference printed {ef}"


@pytest.mark.parametrize("key", ["single", "burst2"])
@pytest.mark.parametrize("maint_first", [True, False])
def test_reference_flow_model(key, maint_first):
    """The pure-Python restatement (tests/test_flow_imp.py ImpModel) gives the
    reference's IDs and reads."""
    v = flowvec()
    ids, reads = run_model(v, key, maint_first)
    assert ids == v[key]["ids"]
    check_reads(v, key, reads)


@pytest.mark.parametrize("key", ["single", "burst2"])
@pytest.mark.parametrize("maint_first", [True, False])
def test_reference_flow_oracle(oracle, key, maint_first):
    """The C oracle (fco_imp_*) gives the reference's IDs and reads."""
    v = flowvec()
    ids, reads = run_oracle(oracle, v, key, maint_first)
    assert ids == v[key]["ids"]
    check_reads(v, key, reads)


def test_reference_flow_script_shape():
    """The script's maintainer runs and their place around the packets: flow
    1 (t0) is released by the run at t0 + 6 s and its ID is back by t0 + 7 s,
    after flow 3's packet at t0 + 4 s took 65533."""
    ev = script(flowvec(), "single")
    assert [e[-1] - T0 for e in ev if e[0] == "m"] == [1000 * k for k in range(1, 13)]
    assert [e[-1] - T0 for e in ev if e[0] == "b"] == [0, 2000, 2000, 2100, 4000]
    assert [e[-1] - T0 for e in ev if e[0] == "r"] == [0, 2000, 12000]


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["single", "burst2"])
def test_gpu_reference_flow(key):
    """The device IMP manager (k_rx lookups, the new-flow pass popping the
    free-ID stack, k_flow_maintain) on the reference's events: IDs and
    fcgpu_flow_stats at the read times."""
    import torch
    from fastclick_amd import device
    v = flowvec()
    m = v["manager"]
    c = cfg()
    ids, reads = [], []
    with torch.cuda.device(0):
        ctx = N.Context(0, 64, c)
        try:
            ctx.flow_configure(N.FLOW_MGR_IMP, m["capacity"], m["timeout_s"], m["recycle_ms"])
            s = torch.cuda.current_stream()
            for e in script(v, key):
                if e[0] == "m":
                    ctx.flow_maintain(e[1], stream=s.cuda_stream)
                elif e[0] == "b":
                    b = batch_of(e[1])
                    ctx.flow_set_time(e[2])
                    db = device.DeviceBatch.upload(b, device="cuda:0")
                    outs = device.DeviceOutputs(b.n, c.nports, device="cuda:0", anno=False, perm=False,
                                                port_start=False, flowid=True)
                    device.run_device(ctx, db, outs)
                    torch.cuda.synchronize()
                    ids.extend(int(x) for x in outs.numpy()["flowid"])
                else:
                    torch.cuda.synchronize()
                    st = ctx.flow_stats()
                    reads.append((str(st["count"]), str(st["free_ids"] + 1)))
        finally:
            ctx.close()
    assert ids == v[key]["ids"]
    check_reads(v, key, reads)


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["single", "burst2"])
def test_element_reference_flow(key):
    """GPUIPCheckClassify(FLOW_MANAGER IMP, FLOW_TIMEOUT 5) on the harness's
    virtual clock, driven by the reference's events (fcclick_run_events): the
    source's bursts at the packets' times, the handler reads at t = 0, 2, 12 s
    (the element's Timer runs the maintainer runs due, as the reference's
    maintain_timer does with no packets). The FLOWID annotation of every
    packet, the output PacketBatches (one per run of one flow: packets 2 and 3
    of the BURST 2 run leave together), flow_count and flow_count_fids."""
    from fastclick_amd import click as K
    v = flowvec()
    m = v["manager"]
    conf = (f"GPUIPCheckClassify(OFFSET 0, CHECKSUM true, N 1, FLOW_CAPACITY {m['capacity']}, "
            f"FLOW_MANAGER IMP, FLOW_TIMEOUT {m['timeout_s']}, FLOW_RECYCLE_INTERVAL {m['recycle_ms'] / 1000}, "
            "BATCH 0)")
    b = synth.from_frames(frames())
    ev = []
    for e in script(v, key):
        if e[0] == "b":
            ev.append(("burst", e[-1] * 1_000_000, len(e[1])))
        elif e[0] == "r":
            ev.append(("read", e[-1] * 1_000_000))
    r = K.run_element_events(conf, b, ev, nsinks=2)
    assert [int(x) for x in r["flow"]] == v[key]["ids"]
    assert (r["port"] == 0).all()
    # one output PacketBatch per run the reference's FlowPrint reports
    for run in v[key]["runs"]:
        assert len({int(r["batch"][i]) for i in run["packets"]}) == 1, run
    assert len(set(int(x) for x in r["batch"])) == len(v[key]["runs"])
    reads = [(rd["flow_count"], rd["flow_count_fids"]) for rd in r["reads"]]
    check_reads(v, key, reads)
