"""Flow re-shard across GPUs (fcgpu_exchange_plan / _pack / _unpack and the
one-pass fcgpu_exchange_build,
fastclick_amd/csrc/fcgpu_exchange.hh) against its numpy restatement
(oracle/exchange.py): records, segment sizes and send buffers bit-exact
(slot padding included), on ragged frames at unaligned offsets, empty
batches, all-invalid batches, 1 to 64 owners and a 1M-packet batch; the
receive side through a simulated all-to-all. The 2-rank gloo exchange itself
is tests/test_dist.py."""
import numpy as np
import pytest

from fastclick_amd import _native as N
from fastclick_amd import dist as D
from fastclick_amd import synth
from oracle import exchange as X

torch = pytest.importorskip("torch")


def _ragged(n, seed, max_len=1600):
    """n frames of 0..max_len bytes at random (unaligned) offsets of a random
    arena, with the ABI's slack after it."""
    rng = np.random.default_rng(seed)
    size = 1 << 21
    arena = rng.integers(0, 256, size + 256, dtype=np.uint8)
    ln = rng.integers(0, max_len + 1, n).astype(np.uint32)
    off = (rng.integers(0, size - max_len, n)).astype(np.uint32)
    return arena, np.stack([off, ln], 1) if n else np.zeros((0, 2), np.uint32)


def _dev(a, dt):
    return torch.from_numpy(np.ascontiguousarray(a).view(dt)).cuda()


def _pack_gpu(ctx, arena, desc, perm, ps, world, rank):
    from fastclick_amd import device
    send, meta, seg_n, seg_b = device.exchange_pack(ctx, _dev(arena, np.uint8), _dev(desc, np.int32),
                                                    _dev(perm.astype(np.uint32), np.int32),
                                                    _dev(ps.astype(np.uint32), np.int32), world, rank)
    torch.cuda.synchronize()
    return (send.cpu().numpy(), meta.cpu().numpy().view(np.uint32).reshape(-1, 4), seg_n,
            np.array(seg_b, dtype=np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("world,n,seed", [(1, 5000, 1), (3, 5000, 2), (8, 20000, 3), (64, 20000, 4),
                                          (5, 1, 5), (2, 1023, 6), (2, 1025, 7), (2, 2049, 8)])
def test_gpu_exchange_pack_matches_oracle(world, n, seed):
    arena, desc = _ragged(n, seed)
    rng = np.random.default_rng(seed + 100)
    owner = rng.integers(-1, world, n)
    perm, ps = X.partition(owner, world)
    ctx = N.Context(0, max(n, 1))
    try:
        send, meta, seg_n, seg_b = _pack_gpu(ctx, arena, desc, perm, ps, world, rank=7)
    finally:
        ctx.close()
    emeta, eseg = X.plan(desc, perm, ps, world, 7)
    esend = X.pack(arena, desc, emeta, ps, eseg, world)
    assert np.array_equal(seg_b, eseg)
    assert seg_n == [int(ps[d + 1] - ps[d]) for d in range(world)]
    assert np.array_equal(meta, emeta)
    total = int(eseg.sum())
    assert np.array_equal(send[:total], esend)
    assert len(send) == total + D.ARENA_PAD and not send[total:].any()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["empty", "all_invalid", "zero_lengths"])
def test_gpu_exchange_edges(case):
    world = 4
    n = {"empty": 0, "all_invalid": 3000, "zero_lengths": 3000}[case]
    arena, desc = _ragged(n, 11)
    owner = np.full(n, -1) if case == "all_invalid" else np.arange(n) % world
    if case == "zero_lengths":
        desc[::2, 1] = 0
    perm, ps = X.partition(owner, world)
    ctx = N.Context(0, max(n, 1))
    try:
        send, meta, seg_n, seg_b = _pack_gpu(ctx, arena, desc, perm, ps, world, rank=0)
    finally:
        ctx.close()
    emeta, eseg = X.plan(desc, perm, ps, world, 0)
    assert np.array_equal(seg_b, eseg) and np.array_equal(meta, emeta)
    assert np.array_equal(send[:int(eseg.sum())], X.pack(arena, desc, emeta, ps, eseg, world))
    if case != "zero_lengths":
        assert len(meta) == 0 and int(seg_b.sum()) == 0


@pytest.mark.gpu
def test_gpu_exchange_owner_pass_and_simulated_all_to_all(oracle):
    """Four ranks' shards of a C3 IMIX batch with errors: the owner pass
    (LB_MODE hash over 4 outputs, whole-batch partition) and the pack on the
    GPU, the segments moved as an all-to-all would, the descriptors unpacked
    on the GPU: every valid packet lands once, on the rank its flow hash
    names, with its bytes, in (source rank, source index) order."""
    from fastclick_amd import device
    from fastclick_amd.device import DeviceBatch, DeviceOutputs
    world = 4
    b = synth.c3(40_000, nflows=3000, seed=21)
    synth.inject_errors(b, 0.03, seed=22)
    cfg = N.make_cfg(offset=14, checksum=True, hash_mode=N.HASH_FLOWID, classify=N.CLS_LB_HASH, nports=world)
    full = oracle.process_batch(cfg, b)
    parts, shards = [], []
    ctx = N.Context(0, b.n, cfg)
    try:
        for rank in range(world):
            lo, hi = D.shard_range(b.n, world, rank)
            shard = synth.Batch(arena=b.arena, desc=np.ascontiguousarray(b.desc[lo:hi]))
            db = DeviceBatch.upload(shard, device="cuda:0")
            outs = DeviceOutputs(shard.n, world, device="cuda:0", perm=True, port_start=True,
                                 partition=N.PART_GLOBAL)
            device.run_device(ctx, db, outs)
            send, meta, seg_n, seg_b = device.exchange_pack(ctx, db.arena, db.desc, outs.perm, outs.port_start,
                                                            world, rank)
            torch.cuda.synchronize()
            ps = outs.port_start.cpu().numpy().view(np.uint32)
            exp_perm, exp_ps = X.partition(np.where(full["reason"][lo:hi] == N.R_OK,
                                                    full["port"][lo:hi].astype(np.int64), -1), world)
            assert np.array_equal(ps[:world + 1], exp_ps[:world + 1])
            emeta, eseg = X.plan(shard.desc, exp_perm, exp_ps, world, rank)
            assert np.array_equal(meta.cpu().numpy().view(np.uint32), emeta)
            assert seg_b == [int(x) for x in eseg]
            parts.append((send, meta, seg_n, seg_b))
            shards.append(lo)
        # the all-to-all, as RCCL would deliver it: receiver r gets source s's
        # segment r, sources in rank order
        for r in range(world):
            bufs, metas, displ, at = [], [], [], 0
            for send, meta, seg_n, seg_b in parts:
                b0 = sum(seg_b[:r])
                m0 = sum(seg_n[:r])
                bufs.append(send[b0:b0 + seg_b[r]])
                metas.append(meta[m0:m0 + seg_n[r]])
                displ.append(at)
                at += seg_b[r]
            buf = torch.cat(bufs + [torch.zeros(D.ARENA_PAD, dtype=torch.uint8, device="cuda:0")])
            rmeta = torch.cat(metas)
            rdesc = device.exchange_unpack(ctx, rmeta, displ)
            torch.cuda.synchronize()
            rm = rmeta.cpu().numpy().view(np.uint32)
            assert np.array_equal(rdesc.cpu().numpy().view(np.uint32), X.unpack(rm, displ))
            g = np.array([shards[s] + i for i, s in zip(rm[:, 2], rm[:, 3])], dtype=np.int64)
            want = np.nonzero((full["reason"] == N.R_OK) & (full["port"] == r))[0]
            assert np.array_equal(g, want)
            hb = buf.cpu().numpy()
            for k, (o, n_) in enumerate(rdesc.cpu().numpy().view(np.uint32).tolist()):
                assert bytes(hb[o:o + n_]) == b.frame(int(g[k]))
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_exchange_1m_batch():
    """The full-size batch: 1M C4 packets (uniform 5-tuples) to 8 owners,
    records and send buffer bit-exact against the restatement."""
    world, n = 8, 1 << 20
    b = synth.c4(n, seed=31)
    owner = np.random.default_rng(32).integers(-1, world, n)
    perm, ps = X.partition(owner, world)
    arena = np.concatenate([b.arena, np.zeros(256, np.uint8)])
    ctx = N.Context(0, n)
    try:
        send, meta, seg_n, seg_b = _pack_gpu(ctx, arena, b.desc, perm, ps, world, rank=3)
    finally:
        ctx.close()
    emeta, eseg = X.plan(b.desc, perm, ps, world, 3)
    assert np.array_equal(seg_b, eseg) and np.array_equal(meta, emeta)
    assert np.array_equal(send[:int(eseg.sum())], X.pack(arena, b.desc, emeta, ps, eseg, world))


def _build_gpu(ctx, arena, desc, owner, world, rank, send_cap=None):
    """fcgpu_exchange_build from verdicts whose port is the owner (world = stays)."""
    from fastclick_amd import device
    port = np.where((owner >= 0) & (owner < world), owner, world).astype(np.uint16)
    verdict = (port << 8) | np.where(port < world, N.R_OK, 1).astype(np.uint16)
    if send_cap is None:
        # these ragged frames overlap in their arena: the default bound (the
        # arena's bytes + 4 per packet) assumes they do not
        send_cap = int(((desc[:, 1].astype(np.int64) + 15) & ~15).sum()) if len(desc) else 0
    send, meta, seg_n, seg_b = device.exchange_build(ctx, _dev(arena, np.uint8), _dev(desc, np.int32),
                                                     _dev(verdict, np.int16), world, rank, send_cap=send_cap)
    torch.cuda.synchronize()
    sn = seg_n.cpu().numpy().astype(np.int64)
    m = int(sn.sum())
    return (send.cpu().numpy(), meta[:m].cpu().numpy().view(np.uint32).reshape(-1, 4), sn,
            seg_b.cpu().numpy().astype(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("world,n,seed", [(1, 5000, 1), (3, 5000, 2), (8, 20000, 3), (64, 20000, 4),
                                          (5, 1, 5), (2, 255, 6), (2, 257, 7), (7, 2049, 8), (16, 70000, 9)])
def test_gpu_exchange_build_matches_oracle(world, n, seed):
    """fcgpu_exchange_build (from verdicts, tile by tile) writes the records,
    segment sizes and send buffer the restatement gives for the stable
    partition of the same owners -- what plan + pack write -- on ragged frames
    at unaligned offsets, tiles cut anywhere, 1 to 64 owners."""
    arena, desc = _ragged(n, seed)
    owner = np.random.default_rng(seed + 100).integers(-1, world, n)
    perm, ps = X.partition(owner, world)
    ctx = N.Context(0, max(n, 1))
    try:
        send, meta, seg_n, seg_b = _build_gpu(ctx, arena, desc, owner, world, rank=5)
    finally:
        ctx.close()
    emeta, eseg = X.plan(desc, perm, ps, world, 5)
    assert np.array_equal(seg_b, eseg)
    assert seg_n.tolist() == [int(ps[d + 1] - ps[d]) for d in range(world)]
    assert np.array_equal(meta, emeta)
    total = int(eseg.sum())
    assert np.array_equal(send[:total], X.pack(arena, desc, emeta, ps, eseg, world))


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["empty", "all_invalid", "zero_lengths", "one_owner", "short_cap"])
def test_gpu_exchange_build_edges(case):
    """No packets, none leaving, zero-length frames, every packet to one owner
    (one match-any group per wave), and a send buffer smaller than the
    segments (nothing written past it)."""
    world = 4
    n = {"empty": 0}.get(case, 3000)
    arena, desc = _ragged(n, 12)
    owner = np.full(n, -1) if case == "all_invalid" else np.full(n, 2) if case == "one_owner" \
        else np.arange(n) % world
    if case == "zero_lengths":
        desc[::2, 1] = 0
    perm, ps = X.partition(owner, world)
    emeta, eseg = X.plan(desc, perm, ps, world, 0)
    cap = int(eseg.sum()) // 2 if case == "short_cap" else None
    ctx = N.Context(0, max(n, 1))
    try:
        send, meta, seg_n, seg_b = _build_gpu(ctx, arena, desc, owner, world, 0, send_cap=cap)
    finally:
        ctx.close()
    assert np.array_equal(seg_b, eseg) and np.array_equal(meta, emeta)
    esend = X.pack(arena, desc, emeta, ps, eseg, world)
    if case == "short_cap":
        # every frame whose slot ends within the buffer is there; nothing past it
        assert len(send) == cap + D.ARENA_PAD
        dst = np.concatenate([[0], np.cumsum(eseg)])[:-1]
        own = np.searchsorted(ps[:world + 1].astype(np.int64), np.arange(len(emeta)), side="right") - 1
        end = dst[own] + emeta[:, 0].astype(np.int64) + ((emeta[:, 1].astype(np.int64) + 15) & ~15)
        ok = end <= cap
        for k in np.nonzero(ok)[0][:200]:
            o = int(dst[own[k]] + emeta[k, 0])
            assert np.array_equal(send[o:o + int(emeta[k, 1])], esend[o:o + int(emeta[k, 1])])
    else:
        assert np.array_equal(send[:int(eseg.sum())], esend)
    if case in ("empty", "all_invalid"):
        assert len(meta) == 0 and int(seg_b.sum()) == 0


@pytest.mark.gpu
def test_gpu_exchange_build_1m_and_owner_pass(oracle):
    """1M C4 packets with errors: the owner pass (LB_MODE hash over 8 outputs,
    verdicts only) then fcgpu_exchange_build, against the restatement run on
    the oracle's owners; then each owner's segment as its receiver gets it
    from this one source, unpacked on the device: the descriptors point at
    every packet's bytes."""
    from fastclick_amd import device
    from fastclick_amd.device import DeviceBatch, DeviceOutputs
    world, n = 8, 1 << 20
    b = synth.c4(n, seed=33)
    synth.inject_errors(b, 0.01, seed=34)
    cfg = N.make_cfg(offset=14, checksum=True, hash_mode=N.HASH_FLOWID, classify=N.CLS_LB_HASH, nports=world)
    exp = oracle.process_batch(cfg, b)
    owner = np.where(exp["reason"] == N.R_OK, exp["port"].astype(np.int64), -1)
    perm, ps = X.partition(owner, world)
    emeta, eseg = X.plan(b.desc, perm, ps, world, 0)
    ctx = N.Context(0, n, cfg)
    try:
        db = DeviceBatch.upload(b, device="cuda:0")
        outs = DeviceOutputs(n, world, device="cuda:0", verdict=True, hash=False)
        device.run_device(ctx, db, outs)
        send, meta, seg_n, seg_b = device.exchange_build(ctx, db.arena, db.desc, outs.verdict, world, 0)
        torch.cuda.synchronize()
        assert np.array_equal(seg_b.cpu().numpy().astype(np.uint64), eseg)
        sn = seg_n.cpu().numpy().astype(np.int64)
        assert sn.tolist() == [int(ps[d + 1] - ps[d]) for d in range(world)]
        m = int(sn.sum())
        assert np.array_equal(meta[:m].cpu().numpy().view(np.uint32), emeta)
        total = int(eseg.sum())
        hs = send.cpu().numpy()
        assert np.array_equal(hs[:total], X.pack(b.arena, b.desc, emeta, ps, eseg, world))
        sb = np.concatenate([[0], np.cumsum(eseg)]).astype(np.int64)
        for d in (0, 5):
            seg = hs[sb[d]:sb[d + 1]]
            rmeta = meta[int(ps[d]):int(ps[d + 1])]
            rd = device.exchange_unpack(ctx, rmeta, [0]).cpu().numpy().view(np.uint32)
            assert np.array_equal(rd, X.unpack(emeta[ps[d]:ps[d + 1]], [0]))
            for k in range(0, len(rd), 997):
                o, ln = (int(x) for x in rd[k])
                assert bytes(seg[o:o + ln]) == b.frame(int(emeta[ps[d] + k, 2]))
    finally:
        ctx.close()


def _build_fixed_gpu(ctx, arena, desc, owner, world, rank, recs, segb):
    from fastclick_amd import device
    port = np.where((owner >= 0) & (owner < world), owner, world).astype(np.uint16)
    verdict = (port << 8) | np.where(port < world, N.R_OK, 1).astype(np.uint16)
    meta = torch.full((world * (recs + 1), 4), -1, dtype=torch.int32, device="cuda:0")
    send = torch.zeros(world * segb + D.ARENA_PAD, dtype=torch.uint8, device="cuda:0")
    device.exchange_build_fixed(ctx, _dev(arena, np.uint8), _dev(desc, np.int32), _dev(verdict, np.int16), world,
                                rank, recs, segb, meta, send)
    torch.cuda.synchronize()
    return meta, send


@pytest.mark.gpu
@pytest.mark.parametrize("world,n,seed,slack", [(1, 5000, 41, 1.0), (3, 5000, 42, 1.25), (8, 20000, 43, 1.25),
                                                (64, 20000, 44, 2.0), (2, 257, 45, 1.25), (16, 70000, 46, 1.1),
                                                (4, 3000, 47, 0.5), (8, 9000, 48, 0.9)])
def test_gpu_exchange_fixed_matches_oracle(world, n, seed, slack):
    """fcgpu_exchange_build_fixed writes every owner's header, records and
    frames at its fixed place as the restatement does (overflowing owners:
    the header alone, flag set), and after an equal-split all-to-all
    (simulated over copies of this one source's buffers, as every rank sent
    the same) fcgpu_exchange_unpack_fixed gives the restatement's descriptors
    and count -- or count 0 and the stall word set to the step when a segment
    overflowed. fcgpu_process_counted then checks exactly the first *count
    packets of the bound."""
    from fastclick_amd import device
    arena, desc = _ragged(n, seed)
    owner = np.random.default_rng(seed + 100).integers(-1, world, n)
    cap_bytes = int(((desc[:, 1].astype(np.int64) + 15) & ~15).sum())
    if slack >= 1:
        recs, segb = device.fixed_capacity(n, cap_bytes, world, slack)
    else:
        recs, segb = max(1, int(n / world * slack)), (int(cap_bytes / world * slack) + 15) // 16 * 16
    ctx = N.Context(0, max(n, 1))
    try:
        meta, send = _build_fixed_gpu(ctx, arena, desc, owner, world, 3, recs, segb)
        em, es, defined, dm = X.build_fixed(arena, desc, owner, world, 3, recs, segb)
        hm = meta.cpu().numpy().view(np.uint32)
        assert np.array_equal(hm[dm], em[dm])
        hs = send.cpu().numpy()
        assert np.array_equal(hs[:world * segb][defined], es[defined])
        over = em[::recs + 1][:world, 3].astype(bool)
        # receiver 0 of `world` sources that all sent these buffers
        parts = [(em, es)] * world
        rmeta_np, rbuf_np = X.all_to_all_fixed(parts, world, recs, segb)[0]
        rmeta = torch.from_numpy(rmeta_np.view(np.int32)).to("cuda:0")
        rbuf = torch.from_numpy(np.concatenate([rbuf_np, np.zeros(D.ARENA_PAD, np.uint8)])).to("cuda:0")
        rdesc = torch.zeros((world * recs, 2), dtype=torch.int32, device="cuda:0")
        count = torch.zeros(1, dtype=torch.int32, device="cuda:0")
        stall = torch.zeros(1, dtype=torch.int32, device="cuda:0")
        device.exchange_unpack_fixed(ctx, rmeta, world, recs, segb, rdesc, count, stall, 7)
        torch.cuda.synchronize()
        edesc, ecount, estall = X.unpack_fixed(rmeta_np, world, recs, segb, 0, 7)
        assert int(count.item()) == ecount and int(stall.item()) == estall
        assert bool(over[0]) == (estall == 7)
        if ecount:
            assert np.array_equal(rdesc[:ecount].cpu().numpy().view(np.uint32), edesc)
            # the received frames are this source's owner-0 frames, in order
            idx = np.nonzero(owner == 0)[0]
            for k in range(0, min(len(idx), ecount), 97):
                o, ln = (int(x) for x in edesc[k])
                assert bytes(rbuf_np[o:o + ln]) == bytes(arena[desc[idx[k], 0]:desc[idx[k], 0] + ln])
        # a later step while stalled stays stalled (count 0, the first step kept)
        device.exchange_unpack_fixed(ctx, rmeta, world, recs, segb, rdesc, count, stall, 8)
        torch.cuda.synchronize()
        assert int(stall.item()) == estall and (int(count.item()) == 0) == bool(estall)
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("flow", [False, True])
def test_gpu_process_counted_matches_prefix(oracle, flow):
    """fcgpu_process_counted over a bound of 9000 packets with the count on the
    device: its outputs and counters are fcgpu_process's over the first
    *count - base packets (2 chunks of a context whose max_batch is 5000),
    per-tile counts past them 0; with a flow table, the same flow IDs and
    table as fcgpu_process over exactly those packets."""
    from fastclick_amd.device import DeviceBatch, DeviceOutputs
    b = synth.c3(9000, nflows=800, seed=51)
    synth.inject_errors(b, 0.03, seed=52)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=8)
    live = 6203
    db = DeviceBatch.upload(b, device="cuda:0")
    res = []
    for counted in (False, True):
        ctx = N.Context(0, 5000, cfg)
        try:
            if flow:
                ctx.flow_enable(20000)
            ctr = torch.zeros(N.CTR_SHARDS, N.NCOUNTERS, dtype=torch.int64, device="cuda:0")
            ctx.use_counters(ctr.data_ptr())
            outs = [DeviceOutputs(5000, 8, device="cuda:0", verdict=True, hash=True, tile_perm=True,
                                  partition=N.PART_TILE, flowid=flow) for _ in range(2)]
            for o in outs:
                o.tile_count.fill_(-1)
            cnt = torch.tensor([live], dtype=torch.int32, device="cuda:0")
            for k, (c0, m) in enumerate(((0, 5000), (5000, 4000 if counted else live - 5000))):
                dptr = db.desc[c0:].data_ptr()
                if counted:
                    ctx.process_counted(db.arena.data_ptr(), dptr, m, cnt.data_ptr(), c0, **outs[k].ptrs())
                else:
                    ctx.process(db.arena.data_ptr(), dptr, m, **outs[k].ptrs())
            torch.cuda.synchronize()
            res.append(dict(ctr=N.derive_counters(ctr.sum(0).cpu().numpy()), outs=outs,
                            flows=ctx.flow_count() if flow else 0))
        finally:
            ctx.close()
    a, c = res
    assert np.array_equal(a["ctr"], c["ctr"])
    assert a["flows"] == c["flows"]
    m2 = live - 5000
    for k, m in ((0, 5000), (1, m2)):
        for key in ("verdict", "hash") + (("flowid",) if flow else ()):
            x = getattr(a["outs"][k], key)[:m].cpu().numpy()
            y = getattr(c["outs"][k], key)[:m].cpu().numpy()
            assert np.array_equal(x, y), (k, key)
    nb = 9
    t_live = -(-m2 // 256)
    tc = c["outs"][1].tile_count.cpu().numpy().reshape(-1, nb)
    assert np.array_equal(tc[:t_live], a["outs"][1].tile_count.cpu().numpy().reshape(-1, nb)[:t_live])
    assert (tc[t_live:-(-4000 // 256)] == 0).all()


def test_exchange_rejects_bad_arguments():
    """Argument checks need no device: a null context, world 0 or > 64."""
    lib = N.load()
    assert lib.fcgpu_exchange_plan(None, None, None, None, 0, 1, 0, None, None, None) == N.EINVAL
    assert lib.fcgpu_exchange_pack(None, None, None, None, None, 0, 1, None, 0, None) == N.EINVAL
    arr = (N.C.c_uint64 * 1)()
    assert lib.fcgpu_exchange_unpack(None, None, 0, arr, 1, None, None) == N.EINVAL
    assert lib.fcgpu_exchange_build(None, None, None, None, 0, 1, 0, None, None, None, None, 0, None) == N.EINVAL


@pytest.mark.gpu
def test_gpu_exchange_build_sequence_one_context():
    """Builds one after another on one context, worlds of 1 to 64 owners,
    empty to 1M-packet batches: every build equals the restatement -- no
    per-tile counts or scans carried over from the build before."""
    ctx = N.Context(0, 1 << 20)
    try:
        for k, (world, n) in enumerate([(4, 3000), (4, 3000), (32, 5000), (8, 70000), (4, 0), (16, 20000),
                                        (1, 257), (2, 1 << 20), (64, 4000), (3, 9999)]):
            arena, desc = _ragged(n, 300 + k, max_len=64 if n > 100_000 else 1600)
            owner = np.random.default_rng(400 + k).integers(-1, world, n)
            perm, ps = X.partition(owner, world)
            send, meta, seg_n, seg_b = _build_gpu(ctx, arena, desc, owner, world, rank=k % max(world, 1))
            emeta, eseg = X.plan(desc, perm, ps, world, k % max(world, 1))
            assert np.array_equal(seg_b, eseg), (k, world, n)
            assert seg_n.tolist() == [int(ps[d + 1] - ps[d]) for d in range(world)], (k, world, n)
            assert np.array_equal(meta, emeta), (k, world, n)
            total = int(eseg.sum())
            assert np.array_equal(send[:total], X.pack(arena, desc, emeta, ps, eseg, world)), (k, world, n)
    finally:
        ctx.close()
