"""Flow managers with timeouts (the IMP half of the
VirtualFlowManager family): FCGPU_FLOW_MGR_IMP on the device.

Reference: VirtualFlowManagerIMP over FlowManagerIMPState
(include/click/flow/virtualflowmanager.hh:25-47, 52-327) with
TimerWheel (include/click/timerwheel.hh), the manager of FlowIPManager_CuckooPP
/ FlowIPManagerIMP (elements/flow/flowipmanager_cuckoopp.cc:57-121).

Parity unpinned: the reference's IMP managers need DPDK (rte_hash, the
cuckoo++ table), absent here, and its tests hold no flow-ID vectors for them.
The device is checked against the C restatement (oracle fco_imp_*, written
with the reference's linked lists), and that restatement against a second,
independent pure-Python one below (ImpModel, same structure as the reference:
a Python list as the stack, dict-linked wheel buckets and released list), on
seeded event sequences: batches stamped with a clock, maintainer runs every
RECYCLE_INTERVAL, flows drifting out of use so that they expire, a table that
fills up, IDs coming back one run after their release.
"""
import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N

NONE = N.FLOW_NONE
FULL = N.FLOW_FULL


def flow_cfg(**kw):
    base = dict(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    base.update(kw)
    return N.make_cfg(**base)


def next_pow2(x):
    p = 1
    while p < x:
        p <<= 1
    return p


class ImpModel:
    """Pure-Python restatement of VirtualFlowManagerIMP, FlowManagerIMPState
    and TimerWheel, on keys (any hashable). Mirrors the reference's structure
    line by line; times in ms."""

    def __init__(self, capacity, timeout_s, recycle_ms):
        self.cap = next_pow2(capacity)                            # :85
        self.stack = list(range(self.cap))                        # :113-115 (push 0 .. cap-1)
        self.table = {}                                           # key -> flow id
        self.key_of, self.lastseen, self.link = {}, {}, {}
        self.recycle_ms = recycle_ms                              # :71-74
        self.eps = max(1, 1000 // recycle_ms)
        self.timeout_ms = timeout_s * 1000
        self.te = timeout_s * self.eps
        size = next_pow2(self.te + 2)                             # TimerWheel::initialize
        self.mask = size - 1
        self.buckets = [None] * size
        self.index = 0
        self.qbsr = None

    def schedule_after(self, f, after):                           # TimerWheel::schedule_after
        b = (self.index + after) & self.mask
        self.link[f] = self.buckets[b]
        self.buckets[b] = f

    def batch(self, keys, now):
        out = []
        for k in keys:
            if k is None:
                out.append(NONE)
                continue
            f = self.table.get(k)
            if f is None:
                if len(self.stack) <= 1:       # only ID 0 left: "table is full" (:264-268)
                    out.append(FULL)
                    continue
                f = self.stack.pop()
                self.table[k] = f
                self.key_of[f] = k
                if self.te:
                    self.schedule_after(f, self.te)               # :293-296
            self.lastseen[f] = now                                # :236-239, 311-313
            out.append(f)
        return np.array(out, np.uint32)

    def maintain(self, now):
        if not self.te:
            return
        while self.qbsr is not None:                              # :155-161
            nxt = self.link[self.qbsr]
            self.stack.append(self.qbsr)
            self.qbsr = nxt
        cur = self.index & self.mask
        f = self.buckets[cur]
        while f is not None:                                      # run_timers
            nxt = self.link[f]
            old = ((now - self.lastseen[f] + 2**31) % 2**32) - 2**31
            if old <= 0:
                self.schedule_after(f, self.te)                   # :174-180
            elif old + self.recycle_ms >= self.timeout_ms:        # :185-205
                del self.table[self.key_of[f]]
                self.link[f] = self.qbsr
                self.qbsr = f
            else:
                # :209-211; r >= 1 (timerwheel.hh:25 asserts timeout > 0)
                self.schedule_after(f, max(1, ((self.timeout_ms - old) * self.eps) // 1000))
            f = nxt
        self.buckets[cur] = None
        self.index += 1

    def stats(self):
        q, f = 0, self.qbsr
        while f is not None:
            q, f = q + 1, self.link[f]
        return dict(count=len(self.table), free_ids=len(self.stack) - 1, pending=q)


def make_batch(pool, idx):
    hdr = synth.build_headers(len(idx), **{k: v[idx] for k, v in pool.items()}, frame_len=60, width=64)
    return synth.pack(hdr, 60)


def batch_keys(pool, idx):
    return [(int(pool["src"][i]), int(pool["dst"][i]), int(pool["sport"][i]), int(pool["dport"][i]))
            for i in idx]


def scenario(seed, *, npool, nsteps, sizes, window, drift, dt_ms, recycle_ms, t0=10_000_000):
    """Events ('m', t) / ('b', pool indices, t): batches whose flows come from a
    window of the pool that drifts forward (older flows go idle and expire),
    with the maintainer runs that are due before each batch, every
    recycle_ms from the first batch (the element's catch-up,
    gpu_core.hh flow_clock)."""
    rng = np.random.default_rng(seed)
    pool = synth._rand_flows(rng, npool)
    ev, t, nxt, base = [], t0, t0 + recycle_ms, 0
    for s in range(nsteps):
        t += int(rng.integers(dt_ms[0], dt_ms[1] + 1))
        while t - nxt >= 0:
            ev.append(("m", nxt))
            nxt += recycle_ms
        n = int(sizes[s % len(sizes)])
        lo = base % npool
        idx = (lo + rng.integers(0, window, n)) % npool
        ev.append(("b", idx, t))
        base += int(rng.integers(drift[0], drift[1] + 1))
    return pool, ev


SCENARIOS = {
    # a 2 s timeout swept by a 250 ms maintainer (TE 8 epochs, 16 buckets)
    "churn": dict(cap=8192, timeout_s=2, recycle_ms=250,
                  sc=dict(seed=5, npool=40_000, nsteps=80, sizes=[300, 2500, 40, 1200], window=1500,
                          drift=(100, 600), dt_ms=(20, 400), recycle_ms=250)),
    # a table that fills: new flows FULL until the maintainer hands IDs back
    "fills": dict(cap=512, timeout_s=1, recycle_ms=100,
                  sc=dict(seed=6, npool=5_000, nsteps=30, sizes=[700, 90, 1500], window=900,
                          drift=(50, 400), dt_ms=(30, 300), recycle_ms=100)),
    # a RECYCLE_INTERVAL that does not divide 1000 ms (eps = 3 floored): flows
    # idle 667-699 ms of a 1 s timeout have under one epoch left and are
    # rescheduled one epoch ahead, not released early
    "recycle300": dict(cap=8192, timeout_s=1, recycle_ms=300,
                       sc=dict(seed=8, npool=20_000, nsteps=60, sizes=[500, 1800, 60], window=1200,
                               drift=(50, 400), dt_ms=(10, 120), recycle_ms=300)),
    # no timeout: IDs cap-1, cap-2, ... and the table fills for good
    "no-timeout": dict(cap=1000, timeout_s=0, recycle_ms=1000,
                       sc=dict(seed=7, npool=3_000, nsteps=6, sizes=[400], window=3_000,
                               drift=(0, 0), dt_ms=(10, 20), recycle_ms=1000)),
}


def run_model(spec):
    pool, ev = scenario(**spec["sc"])
    m = ImpModel(spec["cap"], spec["timeout_s"], spec["recycle_ms"])
    out = []
    for e in ev:
        if e[0] == "m":
            m.maintain(e[1])
        else:
            out.append(m.batch(batch_keys(pool, e[1]), e[2]))
    return pool, ev, out, m.stats()


def run_oracle(O, spec, pool, ev):
    cfg = flow_cfg()
    t = O.ImpFlowTable(spec["cap"], spec["timeout_s"], spec["recycle_ms"])
    out = []
    for e in ev:
        if e[0] == "m":
            t.maintain(e[1])
        else:
            b = make_batch(pool, e[1])
            out.append(t.batch(b, O.process_batch(cfg, b), e[2]))
    return out, t.stats()


def test_model_semantics():
    """Hand-checked IMP behaviour: IDs cap-1, cap-2, ...; ID 0 never given; an
    idle flow released by one run is reused only after the next run, LIFO."""
    m = ImpModel(4, 1, 500)                  # cap 4, TE 2 epochs, 4 buckets
    assert list(m.batch(["a", "b", "c", "d"], 0)) == [3, 2, 1, FULL]
    m.maintain(500)                          # bucket 0: nothing
    assert list(m.batch(["a"], 600)) == [3]
    m.maintain(1000)                         # bucket 1: nothing
    m.maintain(1500)                         # bucket 2: a (seen 900 ms ago: 900+500 >= 1000) expires;
    #                                          b, c (idle 1500 ms) expire too
    assert m.stats() == dict(count=0, free_ids=0, pending=3)
    assert list(m.batch(["d"], 1600)) == [FULL]     # released IDs not back yet
    m.maintain(2000)
    # walked c, b, a (LIFO bucket); pushed back from the released list's head
    # (a, the last released) first, so c is on top
    assert m.stack == [0, 3, 2, 1]
    assert list(m.batch(["e", "f", "g"], 2100)) == [1, 2, 3]


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_oracle_vs_model(oracle, name):
    """The C restatement (linked lists in C) and the Python one agree on
    every flow ID and on the handler counts."""
    spec = SCENARIOS[name]
    pool, ev, exp, st = run_model(spec)
    got, ost = run_oracle(oracle, spec, pool, ev)
    for j, (g, e) in enumerate(zip(got, exp)):
        assert np.array_equal(g, e), f"{name} batch {j}: {np.count_nonzero(g != e)} IDs differ"
    assert ost == st
    allids = np.concatenate(exp)
    assert (allids != 0).all()
    if name == "fills":
        assert (allids == FULL).any() and (allids[allids != FULL] < 512).all()
    if name == "churn":
        assert (allids == FULL).sum() == 0
        # IDs were reused: more distinct flows than the capacity saw IDs
        assert len(set(k for e in ev if e[0] == "b" for k in map(int, e[1]))) > 8192


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_gpu_imp_vs_oracle(oracle, name):
    """Device IMP manager (k_rx lookups, new-flow pass popping the free-ID
    stack, k_flow_maintain + k_flow_rebuild) against the oracle, batch by
    batch, plus fcgpu_flow_stats against the oracle's counts."""
    import torch
    from fastclick_amd import device
    spec = SCENARIOS[name]
    pool, ev = scenario(**spec["sc"])
    exp, ost = run_oracle(oracle, spec, pool, ev)
    cfg = flow_cfg()
    nmax = max(len(e[1]) for e in ev if e[0] == "b")
    with torch.cuda.device(0):
        ctx = N.Context(0, nmax, cfg)
        try:
            ctx.flow_configure(N.FLOW_MGR_IMP, spec["cap"], spec["timeout_s"], spec["recycle_ms"])
            s = torch.cuda.current_stream()
            j = 0
            for e in ev:
                if e[0] == "m":
                    ctx.flow_maintain(e[1], stream=s.cuda_stream)
                    continue
                b = make_batch(pool, e[1])
                ctx.flow_set_time(e[2])
                db = device.DeviceBatch.upload(b, device="cuda:0")
                outs = device.DeviceOutputs(b.n, cfg.nports, device="cuda:0", anno=False, perm=False,
                                            port_start=False, flowid=True)
                device.run_device(ctx, db, outs)
                torch.cuda.synchronize()
                got = outs.numpy()["flowid"]
                if not np.array_equal(got, exp[j]):
                    bad = np.nonzero(got != exp[j])[0]
                    raise AssertionError(f"{name} batch {j}: {len(bad)} IDs differ, first at {bad[:5]}: "
                                         f"got {got[bad[:5]]} expected {exp[j][bad[:5]]}")
                j += 1
            st = ctx.flow_stats()
            assert (st["count"], st["free_ids"], st["pending"]) == (ost["count"], ost["free_ids"], ost["pending"])
            assert ctx.flow_count() == ost["count"]
        finally:
            ctx.close()


@pytest.mark.gpu
def test_gpu_imp_big_buckets(oracle):
    """Batches of 60k packets over 40k-flow windows: new flows take the
    grid-wide pass, and each maintainer run walks buckets of tens of thousands
    of flows (many 1024-entry chunks, several destinations per chunk)."""
    import torch
    from fastclick_amd import device
    spec = dict(cap=1 << 17, timeout_s=1, recycle_ms=125,
                sc=dict(seed=11, npool=400_000, nsteps=14, sizes=[60_000, 20_000], window=40_000,
                        drift=(10_000, 30_000), dt_ms=(60, 260), recycle_ms=125))
    pool, ev = scenario(**spec["sc"])
    exp, ost = run_oracle(oracle, spec, pool, ev)
    cfg = flow_cfg()
    with torch.cuda.device(0):
        ctx = N.Context(0, 60_000, cfg)
        try:
            ctx.flow_configure(N.FLOW_MGR_IMP, spec["cap"], spec["timeout_s"], spec["recycle_ms"])
            s = torch.cuda.current_stream()
            j = 0
            for e in ev:
                if e[0] == "m":
                    ctx.flow_maintain(e[1], stream=s.cuda_stream)
                    continue
                b = make_batch(pool, e[1])
                ctx.flow_set_time(e[2])
                db = device.DeviceBatch.upload(b, device="cuda:0")
                outs = device.DeviceOutputs(b.n, cfg.nports, device="cuda:0", anno=False, perm=False,
                                            port_start=False, flowid=True)
                device.run_device(ctx, db, outs)
                torch.cuda.synchronize()
                got = outs.numpy()["flowid"]
                assert np.array_equal(got, exp[j]), f"batch {j}: {np.count_nonzero(got != exp[j])} IDs differ"
                j += 1
            st = ctx.flow_stats()
            assert (st["count"], st["free_ids"], st["pending"]) == (ost["count"], ost["free_ids"], ost["pending"])
            assert st["epochs"] > 10 and ost["pending"] > 0
        finally:
            ctx.close()


@pytest.mark.gpu
def test_gpu_imp_config_errors():
    ctx = N.Context(0, 1024, flow_cfg())
    try:
        with pytest.raises(RuntimeError, match="IMP"):
            ctx.flow_configure(N.FLOW_MGR_HMP, 1024, timeout_s=5)
        with pytest.raises(RuntimeError, match="timer wheel"):
            ctx.flow_configure(N.FLOW_MGR_IMP, 1024, timeout_s=3600, recycle_ms=10)
        with pytest.raises(RuntimeError, match="recycle"):
            ctx.flow_configure(N.FLOW_MGR_IMP, 1024, timeout_s=5, recycle_ms=0)
        ctx.flow_configure(N.FLOW_MGR_IMP, 1000, timeout_s=0)
        st = ctx.flow_stats()
        assert st["capacity"] == 1024 and st["free_ids"] == 1023 and st["count"] == 0
        ctx.flow_maintain(0)          # no timeout: no-op
    finally:
        ctx.close()


def test_config_imp_keywords():
    from fastclick_amd import click as K
    K.check_config("GPUIPCheckClassify(OFFSET 14, FLOW_CAPACITY 65536, FLOW_MANAGER IMP, FLOW_TIMEOUT 30, "
                   "FLOW_RECYCLE_INTERVAL 0.5)")
    with pytest.raises(K.ConfigError, match="FLOW_TIMEOUT needs"):
        K.check_config("GPUIPCheckClassify(OFFSET 14, FLOW_CAPACITY 10, FLOW_TIMEOUT 5)")
    with pytest.raises(K.ConfigError, match="FLOW_MANAGER"):
        K.check_config("GPUIPCheckClassify(OFFSET 14, FLOW_CAPACITY 10, FLOW_MANAGER CUCKOO)")
    with pytest.raises(K.ConfigError, match="FLOW_RECYCLE_INTERVAL"):
        K.check_config("GPUIPCheckClassify(OFFSET 14, FLOW_MANAGER IMP, FLOW_RECYCLE_INTERVAL 0)")


@pytest.mark.gpu
def test_element_imp_ids(oracle):
    """GPUIPCheckClassify(FLOW_MANAGER IMP, FLOW_CAPACITY 1000): flow IDs are
    the free-ID stack's pops (1023, 1022, ...) in packet order, new flows past
    the capacity are killed, flow_count is the table's size."""
    from fastclick_amd import click as K
    rng = np.random.default_rng(21)
    pool = synth._rand_flows(rng, 3_000)
    idx = rng.integers(0, 3_000, 6_000)
    b = make_batch(pool, idx)
    t = oracle.ImpFlowTable(1000, 0, 1000)
    exp = t.batch(b, oracle.process_batch(flow_cfg(), b), 0)
    for burst, batch in ((64, 1024), (256, 0)):
        r = K.run_element(f"GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4, FLOW_CAPACITY 1000, "
                          f"FLOW_MANAGER IMP, BATCH {batch})", b, burst=burst, nsinks=5)
        ok = exp != FULL
        assert np.array_equal(r["flow"][ok], exp[ok])
        assert (r["port"][~ok] == 0xFFFFFFFF).all()
        assert r["handlers"]["flow_count"] == "1023"
        assert r["handlers"]["flow_drops"] == str(int((~ok).sum()))


@pytest.mark.gpu
def test_gpu_imp_reset_and_stats():
    """fcgpu_flow_reset on an IMP table: the stack is full again (IDs restart
    at cap-1), the table and the wheel empty; fcgpu_flow_stats follows."""
    import torch
    from fastclick_amd import device
    rng = np.random.default_rng(3)
    pool = synth._rand_flows(rng, 500)
    b = make_batch(pool, rng.integers(0, 500, 3000))
    cfg = flow_cfg()
    ctx = N.Context(0, b.n, cfg)
    try:
        ctx.flow_configure(N.FLOW_MGR_IMP, 1024, timeout_s=2, recycle_ms=500)
        db = device.DeviceBatch.upload(b, device="cuda:0")
        ids = []
        for _ in range(2):
            ctx.flow_set_time(100)
            outs = device.DeviceOutputs(b.n, cfg.nports, device="cuda:0", flowid=True)
            device.run_device(ctx, db, outs)
            torch.cuda.synchronize()
            ids.append(outs.numpy()["flowid"])
            st = ctx.flow_stats()
            nfl = len(np.unique(ids[-1]))
            assert (st["count"], st["free_ids"], st["pending"], st["epochs"]) == (nfl, 1023 - nfl, 0, 0)
            assert ids[-1].max() == 1023 and ids[-1].min() == 1024 - nfl
            ctx.flow_reset()
        assert np.array_equal(ids[0], ids[1])
    finally:
        ctx.close()


@pytest.mark.gpu
def test_element_imp_timeouts_virtual_clock(oracle):
    """The element's IMP glue end to end on the harness's virtual clock
    (fcclick_run_clocked): bursts 150 ms apart, BATCH 0 (a device batch per
    PacketBatch), FLOW_TIMEOUT 1 s, FLOW_RECYCLE_INTERVAL 0.1 s -- the
    maintainer runs due before each batch run first (every 100 ms from the
    first batch), flows drifting out of use expire and their IDs are reused,
    exactly as the oracle replaying the same events says."""
    from fastclick_amd import click as K
    rng = np.random.default_rng(17)
    pool = synth._rand_flows(rng, 3_000)
    nb, burst, t0 = 40, 64, 5_000_000_000           # ns
    idx = np.concatenate([(b * 40 + rng.integers(0, 300, burst)) % 3_000 for b in range(nb)])
    b = make_batch(pool, idx)
    clock = np.array([t0 + k * 150_000_000 for k in range(nb)], np.uint64)
    conf = ("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4, FLOW_CAPACITY 256, FLOW_MANAGER IMP, "
            "FLOW_TIMEOUT 1, FLOW_RECYCLE_INTERVAL 0.1, BATCH 0)")
    r = K.run_element(conf, b, burst=burst, nsinks=5, burst_ns=clock)
    # the oracle replays the element's events (gpu_core.hh flow_clock)
    cfg = flow_cfg()
    t = oracle.ImpFlowTable(256, 1, 100)
    nxt = None
    exp = []
    for k in range(nb):
        now = int(clock[k] // 1_000_000) & 0xFFFFFFFF
        if nxt is None:
            nxt = now + 100
        while now - nxt >= 0:
            t.maintain(nxt)
            nxt += 100
        part = synth.Batch(arena=b.arena, desc=np.ascontiguousarray(b.desc[k * burst:(k + 1) * burst]))
        exp.append(t.batch(part, oracle.process_batch(cfg, part), now))
    exp = np.concatenate(exp)
    ok = exp != FULL
    assert ok.sum() > 1000 and (~ok).sum() > 0          # some flows found the table full
    assert np.array_equal(r["flow"][ok], exp[ok])
    assert (r["port"][~ok] == 0xFFFFFFFF).all()
    assert len(np.unique(exp[ok])) < len(np.unique(idx))  # IDs were reused
    assert r["handlers"]["flow_drops"] == str(int((~ok).sum()))
