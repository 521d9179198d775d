"""Flow table: FlowIPManagerHMP flow IDs on the device.

Pin: tests/golden/flow.npz was produced by the reference itself
(`CheckIPHeader(CHECKSUM true) -> FlowIPManagerHMP -> StoreFlowID(OFFSET 0)`,
tests/golden/gen_golden.py run_flow): StoreFlowID writes 1 + the flow's
arrival rank, the ID FlowIPManagerHMP gives it
(elements/research/flowipmanagerhmp.cc:96-126, storeflowid.cc:60-67). The C
oracle (fco_flow_*) is checked against it on CPU; the device path is checked
against both, with the stream cut into batches of several sizes (the table
persists across batches), and against the oracle on seeded workloads: every
packet a new flow (C4), a 10k-flow pool (C3), one flow (C2), repeated batches,
a table that fills up (FCGPU_FLOW_FULL), IP options, fragments and invalid
packets in the mix.
"""
import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N
from tests.test_golden import load, batch_of
from tests.helpers import set_fragment

NONE = N.FLOW_NONE
FULL = N.FLOW_FULL


def flow_cfg(**kw):
    base = dict(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    base.update(kw)
    return N.make_cfg(**base)


def split(b, sizes):
    out, pos = [], 0
    for s in sizes:
        desc = b.desc[pos:pos + s]
        out.append(synth.Batch(arena=b.arena, desc=np.ascontiguousarray(desc)))
        pos += s
    assert pos == b.n
    return out


def oracle_flows(O, cfg, batches, max_flows):
    t = O.FlowTable(max_flows)
    ids = []
    for b in batches:
        r = O.process_batch(cfg, b)
        ids.append(t.batch(b, r))
    return np.concatenate(ids), t.count()


def test_oracle_flow_golden(oracle):
    g = load("flow")
    b = batch_of(g)
    for sizes in ([b.n], [1000, 1500, b.n - 2500], [1] * 7 + [b.n - 7]):
        ids, cnt = oracle_flows(oracle, flow_cfg(), split(b, sizes), 1 << 20)
        assert np.array_equal(ids, g["flowid"]), f"flow IDs vs reference, batches {sizes[:3]}"
        assert cnt == int(g["flowid"][g["flowid"] != NONE].max()) + 1


def test_oracle_flow_full(oracle):
    g = load("flow")
    b = batch_of(g)
    ids, cnt = oracle_flows(oracle, flow_cfg(), [b], 50)
    ref = g["flowid"]
    assert cnt == 50
    assert np.array_equal(ids[ref < 50], ref[ref < 50])
    assert (ids[(ref >= 50) & (ref != NONE)] == FULL).all()


def _dev_flows(cfg, batches, max_flows, **kw):
    from fastclick_amd import device
    res = device.process_batches(batches, cfg, max_flows=max_flows, anno=True, perm=False, **kw)
    return np.concatenate([r["flowid"] for r in res]), res[-1]["flow_count"], res


@pytest.mark.gpu
def test_gpu_flow_golden():
    g = load("flow")
    b = batch_of(g)
    for sizes in ([b.n], [1000, 1500, b.n - 2500], [1, 255, 257, b.n - 513]):
        ids, cnt, _ = _dev_flows(flow_cfg(), split(b, sizes), 1 << 20)
        assert np.array_equal(ids, g["flowid"]), f"flow IDs vs reference, batches {sizes}"
        assert cnt == int(g["flowid"][g["flowid"] != NONE].max()) + 1


@pytest.mark.gpu
def test_gpu_flow_golden_full():
    g = load("flow")
    b = batch_of(g)
    ids, cnt, _ = _dev_flows(flow_cfg(), split(b, [700, b.n - 700]), 50)
    ref = g["flowid"]
    assert cnt == 50
    assert np.array_equal(ids[ref < 50], ref[ref < 50])
    assert (ids[(ref >= 50) & (ref != NONE)] == FULL).all()


def _mixed(n, nflows, seed):
    b = synth.c3(n, nflows=nflows, seed=seed)
    synth.add_ip_options(b, 0.05, seed=seed + 1)
    set_fragment(b, 0.02, seed=seed + 2)
    synth.inject_errors(b, 0.01, seed=seed + 3)
    return b


@pytest.mark.gpu
@pytest.mark.parametrize("name,batches,max_flows", [
    ("c4-all-new", lambda: [synth.c4(1 << 18, seed=41), synth.c4(1 << 18, seed=41)], 1 << 20),
    ("c3-10k", lambda: [_mixed(100_000, 10_000, 42), _mixed(70_001, 10_000, 43)], 1 << 20),
    ("c2-one", lambda: [synth.c2(65_536, seed=44)] * 3, 1 << 10),
    ("fills-up", lambda: [_mixed(30_000, 5_000, 45), _mixed(30_000, 5_000, 46)], 3_000),
    ("udp-tcp-check", lambda: [_mixed(20_000, 2_000, 47)], 1 << 16),
])
def test_gpu_flow_vs_oracle(oracle, name, batches, max_flows):
    bs = batches()
    kw = {}
    cfg = flow_cfg()
    if name == "udp-tcp-check":
        cfg = flow_cfg(l4_mode=N.L4_UDP)
    got, cnt, _ = _dev_flows(cfg, bs, max_flows, **kw)
    exp, ecnt = oracle_flows(oracle, cfg, bs, max_flows)
    if not np.array_equal(got, exp):
        bad = np.nonzero(got != exp)[0]
        raise AssertionError(f"{name}: {len(bad)} flow IDs differ, first {bad[:6]}: got {got[bad[:6]]} "
                             f"expected {exp[bad[:6]]}")
    assert cnt == ecnt, name


@pytest.mark.gpu
def test_gpu_flow_mark_and_program_modes(oracle):
    """The flow stage sits between the checks and the classifier: MarkIPHeader
    mode, and packets a classifier program does not match still get IDs."""
    bs = [_mixed(20_000, 1_500, 50)]
    cfg = flow_cfg(check_mode=N.MARK_IP4, checksum=False)
    got, cnt, _ = _dev_flows(cfg, bs, 1 << 16)
    exp, ecnt = oracle_flows(oracle, cfg, bs, 1 << 16)
    assert np.array_equal(got, exp) and cnt == ecnt
    # IPClassifier(udp && dst port even, -> [X]): odd destination ports match no
    # rule (jump -2^31+1 = [X]); they still have flow IDs
    nomatch = -2147483647
    steps = [(256 + 8, 17 << 8, 0xff00, 1, nomatch, 0), (512, 0, 0x01000000, -1, nomatch, 0)]
    prog = (N.PROG_IPFILTER, steps, -1)
    cfg = flow_cfg(classify=N.CLS_PROGRAM, nports=2)
    got, cnt, res = _dev_flows(cfg, bs, 1 << 16, program=prog)
    oracle.set_program(*prog)
    exp, ecnt = oracle_flows(oracle, cfg, bs, 1 << 16)
    assert (res[0]["reason"] == N.R_NO_MATCH).any()
    assert np.array_equal(got, exp) and cnt == ecnt


@pytest.mark.gpu
def test_gpu_flow_max_batch():
    """The new-flow pass keeps one word per 64 packets in LDS: a context whose
    max_batch is above FCGPU_FLOW_MAX_BATCH cannot enable the table."""
    ctx = N.Context(0, N.FLOW_MAX_BATCH + 1, flow_cfg())
    try:
        with pytest.raises(RuntimeError, match="FLOW_MAX_BATCH"):
            ctx.flow_enable(1024)
    finally:
        ctx.close()
    ctx = N.Context(0, N.FLOW_MAX_BATCH, flow_cfg())
    try:
        ctx.flow_enable(1024)
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_flow_rejects_auto_mode():
    from fastclick_amd import device
    b = synth.c5(1024, seed=3)
    cfg = N.make_cfg(check_mode=N.CHECK_AUTO, offset=0, checksum=True, nports=4)
    with pytest.raises(RuntimeError, match="IPv4 check mode"):
        device.process_batches([b], cfg, max_flows=1024)


def _with_new(base, k, seed):
    """base's packets with k packets of fresh flows (about 4 packets each)
    inserted at random positions: a batch with about k misses."""
    rng = np.random.default_rng(seed)
    frames = [base.frame(i) for i in range(base.n)]
    if k:
        new = synth.c3(k, nflows=max(k // 4, 1), seed=seed + 1000)
        pos = np.sort(rng.integers(0, len(frames) + 1, k))
        for j, p in enumerate(pos[::-1]):
            frames.insert(int(p), new.frame(k - 1 - j))
    return synth.from_frames(frames)


@pytest.mark.gpu
@pytest.mark.parametrize("max_flows", [1 << 16, 2_600])
def test_gpu_flow_finish_paths(oracle, max_flows):
    """Every shape of the new-flow pass (fcgpu_flow.hh), chosen from the class
    of the previous batch's misses: a cold table -> the grid-wide kernels; a
    small batch (100 misses) after a large one -> grid-wide again; then
    k_flow_finish with one chunk (200); a large batch there (6,000, the hint
    was wrong) -> k_flow_finish in six 1024-miss chunks, later chunks taking
    the IDs of flows that began in earlier ones from their committed slots;
    grid-wide (5,000); no misses; one chunk (150); three chunks (3,000); one
    new flow on the last packet. With max_flows 2,600 the table fills inside
    these paths (FCGPU_FLOW_FULL)."""
    base = synth.c3(20_000, nflows=2_000, seed=60)
    plan = [(0, 0), (100, 1), (200, 2), (6_000, 3), (5_000, 4), (0, 5), (150, 6), (3_000, 7)]
    bs = [base if k == 0 and s == 0 else _with_new(base, k, 61 + s) for k, s in plan]
    last = [base.frame(i) for i in range(base.n)] + [synth.c4(1, seed=99).frame(0)]
    bs.append(synth.from_frames(last))
    cfg = flow_cfg()
    got, cnt, res = _dev_flows(cfg, bs, max_flows)
    exp, ecnt = oracle_flows(oracle, cfg, bs, max_flows)
    for j, (r, b) in enumerate(zip(res, bs)):
        o = exp[sum(x.n for x in bs[:j]):][:b.n]
        assert np.array_equal(r["flowid"], o), f"batch {j}: {np.count_nonzero(r['flowid'] != o)} IDs differ"
    assert cnt == ecnt


def test_oracle_nonfirst_fragments_key_on_proto(oracle):
    """IPFlow5ID(p) of a non-first fragment keeps only ip_p (lib/ipflowid.cc:
    34-38: IPFlowID returns before assign(), addresses stay 0): all non-first
    fragments of one protocol are one flow, whatever their addresses."""
    b = synth.c4(4_000, seed=61)
    frag = set_fragment(b, 0.2, seed=62)
    cfg = flow_cfg()
    ids, _ = oracle_flows(oracle, cfg, [b], 1 << 16)
    r = oracle.process_batch(cfg, b)
    nf = np.zeros(b.n, bool)
    nf[frag] = True
    nf &= r["reason"] == N.R_OK
    assert nf.sum() > 100 and len(np.unique(ids[nf])) == 1
    assert not np.isin(ids[~nf & (r["reason"] == N.R_OK)], ids[nf]).any()


@pytest.mark.gpu
def test_gpu_nonfirst_fragments_flow(oracle):
    from fastclick_amd import device
    b = synth.c4(30_000, seed=63)
    set_fragment(b, 0.15, seed=64)
    synth.inject_errors(b, 0.01, seed=65)
    cfg = flow_cfg()
    batches = split(b, [10_000, 20_000])
    exp, cnt = oracle_flows(oracle, cfg, batches, 1 << 16)
    got = device.process_batches(batches, cfg, max_flows=1 << 16, anno=False, perm=False)
    assert np.array_equal(np.concatenate([g["flowid"] for g in got]), exp)
    assert got[-1]["flow_count"] == cnt


@pytest.mark.gpu
@pytest.mark.parametrize("manager", ["hmp", "imp"])
def test_gpu_flow_fused_jobs(oracle, manager):
    """fcgpu_process_jobs with a flow table fuses up to 8 batches per k_rx
    launch (lookups only read the table; each batch keeps its miss records)
    and runs the batches' new-flow passes after it in batch order: a stream
    cut into 13 batches -- flows recurring across batches, new ones in every
    batch, a table that fills -- gets the IDs of one batch at a time."""
    import torch
    from fastclick_amd.device import DeviceBatch, DeviceOutputs
    b = _mixed(130_000, 6_000, 81)
    bs = split(b, [10_000] * 13)
    cfg = flow_cfg()
    cap = 4_000
    if manager == "hmp":
        exp, ecnt = oracle_flows(oracle, cfg, bs, cap)
    else:
        t = oracle.ImpFlowTable(cap, 0, 1000)
        exp = np.concatenate([t.batch(x, oracle.process_batch(cfg, x), 5) for x in bs])
        ecnt = t.stats()["count"]
    ctx = N.Context(0, 10_000, cfg)
    try:
        if manager == "hmp":
            ctx.flow_enable(cap)
        else:
            ctx.flow_configure(N.FLOW_MGR_IMP, cap)
            ctx.flow_set_time(5)
        s = torch.cuda.current_stream()
        dbs = [DeviceBatch.upload(x, device="cuda:0") for x in bs]
        outs = [DeviceOutputs(x.n, cfg.nports, device="cuda:0", perm=True, partition=N.PART_TILE, flowid=True)
                for x in bs]
        specs = [(d.arena.data_ptr(), d.desc.data_ptr(), d.n, s.cuda_stream, o.ptrs()) for d, o in zip(dbs, outs)]
        ctx.run_jobs(ctx.jobs(specs))
        torch.cuda.synchronize()
        got = np.concatenate([o.numpy()["flowid"] for o in outs])
        if not np.array_equal(got, exp):
            bad = np.nonzero(got != exp)[0]
            raise AssertionError(f"{manager}: {len(bad)} IDs differ, first {bad[:6]}: {got[bad[:6]]} vs {exp[bad[:6]]}")
        assert (got == FULL).any()
        assert ctx.flow_count() == ecnt
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("max_flows", [1 << 16, 1_985])
def test_gpu_flow_elephants(oracle, max_flows):
    """Batches whose misses are mostly a few new flows, interleaved packet by
    packet: the lanes of a wave that share a flow follow one lane through the
    placement (flow_place_wave). 150k packets of 3 new flows (grid-wide pass);
    then 800 and 900 packets of 2 new flows each among 2,000 known flows (grid
    pass, then the single-block pass after a small batch). With max_flows 1,985
    (the 1,983 known flows + 2) the third elephant and every later new flow
    find the table full, so followers of a lane that found
    no ID take FCGPU_FLOW_FULL."""
    base = synth.c3(10_000, nflows=2_000, seed=70)
    eleph = synth.c3(150_000, nflows=3, seed=71)
    rng = np.random.default_rng(72)

    def few_new(k, seed):
        frames = [base.frame(i) for i in range(base.n)]
        new = synth.c3(k, nflows=2, seed=seed)
        pos = np.sort(rng.integers(0, len(frames) + 1, k))
        for j, p in enumerate(pos[::-1]):
            frames.insert(int(p), new.frame(k - 1 - j))
        return synth.from_frames(frames)

    bs = [base, eleph, few_new(800, 73), few_new(900, 74)]
    cfg = flow_cfg()
    got, cnt, res = _dev_flows(cfg, bs, max_flows)
    exp, ecnt = oracle_flows(oracle, cfg, bs, max_flows)
    for j, (r, b) in enumerate(zip(res, bs)):
        o = exp[sum(x.n for x in bs[:j]):][:b.n]
        assert np.array_equal(r["flowid"], o), f"batch {j}: {np.count_nonzero(r['flowid'] != o)} IDs differ"
    assert cnt == ecnt
    if max_flows == 1_985:
        assert (got == FULL).any()
