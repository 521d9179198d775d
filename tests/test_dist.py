"""World-size-2 gloo tests of the multi-GPU split/reduce logic on CPU.

Each rank takes its contiguous shard of a seeded batch; the per-shard counters
(computed here by the oracle, standing in for the device since this host has no
GPU) are reduced with fastclick_amd.dist exactly as bench.py reduces the device
replicas, and must equal the single-process totals. Per-output offsets from
the all-gather must reproduce the global stable partition.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fastclick_amd import synth, dist as D
from fastclick_amd import _native as N


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        b = synth.c4(10_007, seed=77)
        synth.inject_errors(b, 0.03, seed=78)
        cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
        lo, hi = D.shard_range(b.n, world, rank)
        shard = synth.Batch(arena=b.arena, desc=np.ascontiguousarray(b.desc[lo:hi]))
        r = O.process_batch(cfg, shard)
        # replicas layout as on the device: [CTR_SHARDS, NCOUNTERS]; put the
        # shard's counts in replica (rank % shards), the rest zero
        rep = torch.zeros(N.CTR_SHARDS, N.NCOUNTERS, dtype=torch.int64)
        rep[rank % N.CTR_SHARDS] = torch.from_numpy(r["counters"].astype(np.int64))
        tot = D.reduce_counters(rep)
        counts = torch.from_numpy(np.diff(r["port_start"].astype(np.int64)))
        before, gtot = D.output_offsets(counts)
        # global positions of this shard's packets in the whole-batch partition
        pos = []
        for p in range(17):
            run = r["perm"][r["port_start"][p]:r["port_start"][p + 1]] + lo
            pos.append((p, int(before[p]), run.tolist()))
        q.put((rank, tot.numpy(), gtot.numpy(), pos))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_counter_allreduce_and_offsets(oracle):
    world = 2
    port = 29500 + (os.getpid() % 1000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    b = synth.c4(10_007, seed=77)
    synth.inject_errors(b, 0.03, seed=78)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    full = oracle.process_batch(cfg, b)
    for rank, tot, gtot, pos in res:
        assert np.array_equal(tot, full["counters"].astype(np.int64))
        assert np.array_equal(gtot, np.diff(full["port_start"].astype(np.int64)))
    # stitching shard runs at their all-gathered offsets == global partition
    perm = np.full(b.n, -1, np.int64)
    for rank, tot, gtot, pos in res:
        for p, before, run in pos:
            start = int(full["port_start"][p]) + before
            perm[start:start + len(run)] = run
    assert np.array_equal(perm, full["perm"].astype(np.int64))


def test_shard_range_covers():
    for n in (0, 1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [D.shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def _flow_batch():
    b = synth.c3(6_001, nflows=700, seed=91)
    synth.inject_errors(b, 0.03, seed=92)
    return b


def _owner_cfg(world):
    # FlowSwitch(LB_MODE hash) over the ranks on the IPFlowID hash: a function of the 5-tuple
    return N.make_cfg(offset=14, checksum=True, hash_mode=N.HASH_FLOWID, classify=N.CLS_LB_HASH, nports=world)


def _flow_worker(rank, world, port, q, built=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from oracle import exchange as X
        b = _flow_batch()
        lo, hi = D.shard_range(b.n, world, rank)
        shard = synth.Batch(arena=b.arena, desc=np.ascontiguousarray(b.desc[lo:hi]))
        r = O.process_batch(_owner_cfg(world), shard)      # stands in for the device pass
        perm, ps = X.partition(np.where(r["reason"] == N.R_OK, r["port"].astype(np.int64), -1), world)
        meta, seg = X.plan(shard.desc, perm, ps, world, rank)   # ... and for the HIP pack
        send = np.concatenate([X.pack(shard.arena, shard.desc, meta, ps, seg, world),
                               np.zeros(D.ARENA_PAD, np.uint8)])
        seg_n = [int(ps[d + 1]) - int(ps[d]) for d in range(world)]
        if built:    # the sizes as fcgpu_exchange_build leaves them: tensors, counts exchanged first
            buf, rmeta, displ = D.exchange_built(torch.from_numpy(send), torch.from_numpy(meta.view(np.int32)),
                                                 torch.tensor(seg_n, dtype=torch.int32),
                                                 torch.tensor([int(x) for x in seg], dtype=torch.int64))
        else:
            buf, rmeta, displ = D.exchange_segments(torch.from_numpy(send), torch.from_numpy(meta.view(np.int32)),
                                                    seg_n, [int(x) for x in seg], group=None)
        rmeta = rmeta.numpy().view(np.uint32)
        desc = X.unpack(rmeta, displ)
        src = rmeta[:, 2:4].copy().view(np.int64).ravel()
        # the global packet index of each received packet: its source shard's lo + index
        g = np.array([D.shard_range(b.n, world, int(s >> 32))[0] + int(s & 0xFFFFFFFF) for s in src],
                     dtype=np.int64)
        q.put((rank, buf.numpy(), desc, g))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("built", [False, True])
def test_two_rank_exchange_by_flow(oracle, built):
    """Packets of one 6k-packet batch, split over 2 ranks, are re-sharded by
    the flow hash: the records and send buffers the HIP kernels build (their
numpy restatement, oracle/exchange.py, stands in on the CPU) go through
fastclick_amd.dist.exchange_segments (gloo all-to-all) -- or, built, through
dist.exchange_built, which takes the segment sizes as tensors the way
fcgpu_exchange_build leaves them and exchanges the counts first:
    every valid packet lands exactly once, on the rank its flow hash names,
    with its frame bytes intact and in source order; each rank's flow table
    then sees whole flows (IDs from per-rank tables are in order of first
    appearance within that rank's packets)."""
    world = 2
    port = 29500 + ((os.getpid() + 500) % 1000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_flow_worker, args=(r, world, port + built, q, built)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    b = _flow_batch()
    full = oracle.process_batch(_owner_cfg(world), b)
    valid = np.nonzero(full["reason"] == N.R_OK)[0]
    seen = np.concatenate([g for _, _, _, g in res])
    assert np.array_equal(np.sort(seen), valid)                  # every valid packet once
    for rank, arena, desc, g in res:
        assert np.all(full["port"][g] == rank)                    # on its flow's rank
        assert np.all(np.diff(g) > 0)                             # source order kept
        for k in range(len(g)):
            o, n_ = int(desc[k, 0]), int(desc[k, 1])
            assert bytes(arena[o:o + n_]) == b.frame(int(g[k]))
        # the rank's table over its packets gives the IDs a table over the
        # whole batch restricted to this rank's flows would (relabelled 0..)
        rb = synth.Batch(arena=arena, desc=np.ascontiguousarray(desc))
        cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=4)
        ids = oracle.FlowTable(1 << 16).batch(rb, oracle.process_batch(cfg, rb))
        whole = oracle.FlowTable(1 << 16).batch(b, oracle.process_batch(cfg, b))[g]
        first_seen = {}
        for v in whole:
            first_seen.setdefault(int(v), len(first_seen))
        assert np.array_equal(ids, np.array([first_seen[int(v)] for v in whole], dtype=ids.dtype))


@pytest.mark.gpu
def test_gpu_exchange_pack_and_flow_table(oracle):
    """The device path of the flow re-sharding at world size 1: the owner pass
    (LB_MODE hash over 2 ranks on the IPFlowID hash, whole-batch partition)
    runs on the GPU and matches the oracle; exchange_by_flow packs the packets
    owned by rank 0 with the HIP kernels; the flow table over the received
    batch gives the oracle's IDs."""
    from fastclick_amd import device
    from fastclick_amd.device import DeviceBatch, DeviceOutputs
    b = _flow_batch()
    cfg = N.make_cfg(offset=14, checksum=True, hash_mode=N.HASH_FLOWID, classify=N.CLS_LB_HASH, nports=1)
    exp2 = oracle.process_batch(_owner_cfg(2), b)
    # world 1: the owner pass names output 0 for every valid packet
    ctx = N.Context(0, b.n, cfg)
    try:
        db = DeviceBatch.upload(b, device="cuda:0")
        outs = DeviceOutputs(b.n, 1, device="cuda:0", perm=True, port_start=True, partition=N.PART_GLOBAL)
        device.run_device(ctx, db, outs)
        arena, desc, src = D.exchange_by_flow(ctx, db.arena, db.desc, outs.perm, outs.port_start)
        torch.cuda.synchronize()
    finally:
        ctx.close()
    g = src.cpu().numpy()
    want = np.nonzero(exp2["reason"] == N.R_OK)[0]
    assert np.array_equal(g & 0xFFFFFFFF, want) and np.all(g >> 32 == 0)
    rb = synth.Batch(arena=arena.cpu().numpy(), desc=desc.cpu().numpy().view(np.uint32))
    assert np.all(rb.arena[-D.ARENA_PAD:] == 0)
    for k in range(len(g)):
        o, n_ = int(rb.desc[k, 0]), int(rb.desc[k, 1])
        assert o % 16 == 0 and bytes(rb.arena[o:o + n_]) == b.frame(int(g[k]))
    fcfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=4)
    res = device.process_batches([rb], fcfg, max_flows=1 << 16, anno=False, perm=False)
    ids = oracle.FlowTable(1 << 16).batch(rb, oracle.process_batch(fcfg, rb))
    assert np.array_equal(res[0]["flowid"], ids)


def test_exchange_format_round_trip():
    """The re-shard format (oracle/exchange.py, the HIP kernels' checker):
    three ranks' ragged frames at unaligned offsets, packed by owner, moved by
    a simulated all-to-all and unpacked, land on their owners exactly once
    with their bytes, in (source rank, source index) order, 16-B aligned, the
    slot padding zero."""
    from oracle import exchange as X
    rng = np.random.default_rng(5)
    world = 3
    arena = rng.integers(0, 256, 200_000, dtype=np.uint8)
    parts, srcs = [], []
    for rank in range(world):
        n = int(rng.integers(0, 400))
        ln = rng.integers(0, 300, n).astype(np.uint32)
        off = rng.integers(0, 190_000, n).astype(np.uint32)
        desc = np.stack([off, ln], 1)
        owner = rng.integers(-1, world, n)
        perm, ps = X.partition(owner, world)
        meta, seg = X.plan(desc, perm, ps, world, rank)
        assert np.all(np.diff(meta[:, 2].astype(np.int64)[ps[0]:ps[1]]) > 0)
        send = X.pack(arena, desc, meta, ps, seg, world)
        assert len(send) == int(sum(seg)) and len(send) == int(((ln[owner >= 0].astype(np.int64) + 15) // 16 * 16).sum())
        parts.append((send, meta, ps, seg))
        srcs.append((desc, owner))
    for r, (buf, meta, displ) in enumerate(X.all_to_all(parts, world)):
        d = X.unpack(meta, displ)
        want = [(s, i) for s, (desc, owner) in enumerate(srcs) for i in np.nonzero(owner == r)[0]]
        assert [(int(a), int(b)) for a, b in zip(meta[:, 3], meta[:, 2])] == want
        for (o, n_), (s, i) in zip(d.tolist(), want):
            so, sn = srcs[s][0][i].tolist()
            assert n_ == sn and o % 16 == 0
            assert np.array_equal(buf[o:o + n_], arena[so:so + sn])
            assert np.all(buf[o + n_:o + ((n_ + 3) & ~3)] == 0)


def _segments_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import exchange as X
        rng = np.random.default_rng(100 + rank)
        n = 0 if rank == 2 else 300                     # rank 2 sends nothing
        arena = rng.integers(0, 256, 50_000, dtype=np.uint8)
        desc = np.stack([rng.integers(0, 49_000, n), rng.integers(0, 200, n)], 1).astype(np.uint32) \
            if n else np.zeros((0, 2), np.uint32)
        owner = rng.choice([0, 2, -1], n)               # nobody sends to rank 1
        perm, ps = X.partition(owner, world)
        meta, seg = X.plan(desc, perm, ps, world, rank)
        send = np.concatenate([X.pack(arena, desc, meta, ps, seg, world), np.zeros(D.ARENA_PAD, np.uint8)])
        seg_n = [int(ps[d + 1]) - int(ps[d]) for d in range(world)]
        buf, rmeta, displ = D.exchange_segments(torch.from_numpy(send), torch.from_numpy(meta.view(np.int32)),
                                                seg_n, [int(x) for x in seg])
        q.put((rank, arena, desc, owner, buf.numpy(), rmeta.numpy().view(np.uint32), displ))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_three_rank_exchange_segments_with_empty_segments():
    """exchange_segments over gloo with 3 ranks where one rank sends nothing
    and one receives nothing: every rank gets exactly the frames addressed to
    it, in (source rank, source index) order, its buffer ending in the ABI's
    zero pad."""
    from oracle import exchange as X
    world = 3
    port = 29500 + ((os.getpid() + 700) % 1000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_segments_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r[0]: r[1:] for r in (q.get(timeout=240) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        _, _, _, buf, rmeta, displ = res[r]
        assert not buf[len(buf) - D.ARENA_PAD:].any()
        want = [(s, i) for s in range(world) for i in np.nonzero(res[s][2] == r)[0]]
        assert [(int(a), int(b)) for a, b in zip(rmeta[:, 3], rmeta[:, 2])] == want
        if r == 1:
            assert len(rmeta) == 0 and len(buf) == D.ARENA_PAD
        d = X.unpack(rmeta, displ)
        for (o, n_), (s, i) in zip(d.tolist(), want):
            so, sn = res[s][1][i].tolist()
            assert n_ == sn and np.array_equal(buf[o:o + n_], res[s][0][so:so + sn])


def _fixed_owner(src, n):
    # source 0 sends 90 % of its packets to rank 1, source 1 half to each
    i = np.arange(n)
    return np.where(i % 10 != 0, 1, 0) if src == 0 else i % 2


def _fixed_worker(rank, world, port, q):
    """Two steps of the fixed-capacity re-shard (the HIP build and unpack
    restated by oracle/exchange.py, the all-to-alls through
    dist.exchange_fixed over gloo): step 1 with room for everything, step 2
    with segments of 60 % of a batch -- source 0's 90 % for rank 1 does not
    fit, so rank 1 stalls and rank 0 does not. dist.first_stalled names step
    2 on both ranks, both replay it through the counted exchange
    (dist.exchange_segments), and only rank 1 takes the replayed packets."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import exchange as X
        b = _flow_batch()
        lo, hi = D.shard_range(b.n, world, rank)
        shard = synth.Batch(arena=b.arena, desc=np.ascontiguousarray(b.desc[lo:hi]))
        n = hi - lo
        owner = _fixed_owner(rank, n)
        cap = int(((shard.desc[:, 1].astype(np.int64) + 15) & ~15).sum())
        got, stall, replayed = [], 0, 0
        for step, frac in ((1, 1.0), (2, 0.6)):
            c = torch.tensor([int(n * frac), (int(cap * frac) + 15) // 16 * 16], dtype=torch.int64)
            dist.all_reduce(c, op=dist.ReduceOp.MIN)      # the ranks agree on one capacity
            recs, segb = int(c[0]), int(c[1])
            meta, send, _, _ = X.build_fixed(shard.arena, shard.desc, owner, world, rank, recs, segb)
            rmeta, rbuf = D.exchange_fixed(torch.from_numpy(meta.view(np.int32)),
                                           torch.from_numpy(np.concatenate([send, np.zeros(D.ARENA_PAD, np.uint8)])),
                                           recs, segb)
            rmeta = rmeta.numpy().view(np.uint32)
            rbuf = rbuf.numpy()
            assert len(rbuf) == world * segb + D.ARENA_PAD and not rbuf[world * segb:].any()
            desc, count, stall = X.unpack_fixed(rmeta, world, recs, segb, stall, step)
            if count:
                rows = recs + 1
                src = np.concatenate([rmeta[s * rows + 1:s * rows + 1 + int(rmeta[s * rows, 0])]
                                      for s in range(world)])
                got.append([(int(x[3]), int(x[2]), bytes(rbuf[d[0]:d[0] + d[1]])) for x, d in zip(src, desc)])
        first = D.first_stalled(stall)
        if first:       # the replay: every step from `first`, counted, collectively
            perm, ps = X.partition(owner, world)
            meta, seg = X.plan(shard.desc, perm, ps, world, rank)
            send = np.concatenate([X.pack(shard.arena, shard.desc, meta, ps, seg, world),
                                   np.zeros(D.ARENA_PAD, np.uint8)])
            seg_n = [int(ps[d + 1]) - int(ps[d]) for d in range(world)]
            buf, rm, displ = D.exchange_segments(torch.from_numpy(send), torch.from_numpy(meta.view(np.int32)),
                                                 seg_n, [int(x) for x in seg])
            rm = rm.numpy().view(np.uint32)
            desc = X.unpack(rm, displ)
            buf = buf.numpy()
            if stall and 2 >= stall:      # this rank's own stalled step on: its table takes them
                got.append([(int(x[3]), int(x[2]), bytes(buf[d[0]:d[0] + d[1]])) for x, d in zip(rm, desc)])
                replayed += 1
        q.put((rank, stall, first, replayed, got))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_fixed_exchange_and_overflow_replay():
    """The fixed-capacity re-shard over gloo, two ranks: with room, each rank
    receives exactly its packets (source rank, source order, frame bytes);
    when a step's segment overflows, its receiver stalls (count 0), every rank
    learns the first stalled step (dist.first_stalled), the step is replayed
    through the counted exchange, and only the stalled rank takes the
    replayed packets (the other already has them) -- the fallback the bench
    counts (config.flow_reshard.fallback_steps)."""
    world = 2
    port = 29500 + ((os.getpid() + 700) % 1000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fixed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    b = _flow_batch()
    for rank, stall, first, replayed, got in res:
        assert first == 2
        assert stall == (2 if rank == 1 else 0) and replayed == (1 if rank == 1 else 0)
        exp = []
        for src in range(world):
            lo, hi = D.shard_range(b.n, world, src)
            own = _fixed_owner(src, hi - lo)
            exp += [(src, i, b.frame(lo + i)) for i in range(hi - lo) if own[i] == rank]
        assert len(got) == 2
        for batch in got:
            assert batch == exp
