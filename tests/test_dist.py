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


def _flow_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        b = _flow_batch()
        lo, hi = D.shard_range(b.n, world, rank)
        shard = synth.Batch(arena=b.arena, desc=np.ascontiguousarray(b.desc[lo:hi]))
        r = O.process_batch(_owner_cfg(world), shard)      # stands in for the device pass
        owner = torch.from_numpy(np.where(r["reason"] == N.R_OK, r["port"].astype(np.int64), -1))
        arena, desc, src = D.exchange_by_flow(torch.from_numpy(shard.arena), torch.from_numpy(
            shard.desc.view(np.int32)), owner)
        # the global packet index of each received packet: its source shard's lo + index
        src = src.numpy()
        g = np.array([D.shard_range(b.n, world, int(s >> 32))[0] + int(s & 0xFFFFFFFF) for s in src],
                     dtype=np.int64)
        q.put((rank, arena.numpy(), desc.numpy().view(np.uint32), g))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_exchange_by_flow(oracle):
    """Packets of one 6k-packet batch, split over 2 ranks, are re-sharded by
    the flow hash with fastclick_amd.dist.exchange_by_flow (gloo all-to-all):
    every valid packet lands exactly once, on the rank its flow hash names,
    with its frame bytes intact and in source order; each rank's flow table
    then sees whole flows (IDs from per-rank tables are in order of first
    appearance within that rank's packets)."""
    world = 2
    port = 29500 + ((os.getpid() + 500) % 1000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_flow_worker, args=(r, world, port, q)) for r in range(world)]
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
    """The device half of the flow re-sharding at world size 1: the owner pass
    (LB_MODE hash over 2 ranks on the IPFlowID hash) runs on the GPU and
    matches the oracle; exchange_by_flow packs rank 0's packets from CUDA
    tensors (the all-to-all itself is covered by the 2-rank gloo test); the
    flow table over the packed batch gives the oracle's IDs."""
    from fastclick_amd import device
    from fastclick_amd.device import DeviceBatch
    b = _flow_batch()
    cfg = _owner_cfg(2)
    got = device.process_batch(b, cfg, anno=False, perm=False, partition=N.PART_TILE)
    exp = oracle.process_batch(cfg, b)
    assert np.array_equal(got["port"], exp["port"])
    db = DeviceBatch.upload(b, device="cuda:0")
    port = torch.from_numpy(got["port"].astype(np.int64)).cuda()
    ok = torch.from_numpy(got["reason"] == N.R_OK).cuda()
    owner = torch.where(ok & (port == 0), torch.zeros_like(port), torch.full_like(port, -1))
    arena, desc, src = D.exchange_by_flow(db.arena, db.desc, owner)
    g = src.cpu().numpy() & 0xFFFFFFFF
    want = np.nonzero((exp["reason"] == N.R_OK) & (exp["port"] == 0))[0]
    assert np.array_equal(g, want)
    rb = synth.Batch(arena=arena.cpu().numpy(), desc=desc.cpu().numpy().view(np.uint32))
    for k in range(0, len(g), 97):
        o, n_ = int(rb.desc[k, 0]), int(rb.desc[k, 1])
        assert bytes(rb.arena[o:o + n_]) == b.frame(int(g[k]))
    fcfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=4)
    res = device.process_batches([rb], fcfg, max_flows=1 << 16, anno=False, perm=False)
    ids = oracle.FlowTable(1 << 16).batch(rb, oracle.process_batch(fcfg, rb))
    assert np.array_equal(res[0]["flowid"], ids)


def test_gather_frames_chunked_matches_whole():
    """_gather_frames in small chunks equals a per-frame concatenation, and
    exchange_by_flow's received arena carries the ABI's zeroed tail."""
    rng = np.random.default_rng(5)
    arena = torch.from_numpy(rng.integers(0, 256, 50_000, dtype=np.uint8))
    ln = torch.from_numpy(rng.integers(0, 300, 200)).to(torch.int64)
    off = torch.from_numpy(rng.integers(0, 49_000 - 300, 200)).to(torch.int64)
    want = np.concatenate([arena.numpy()[o:o + n] for o, n in zip(off.tolist(), ln.tolist())])
    for chunk in (1, 97, 1000, 1 << 24):
        got = D._gather_frames(arena, off, ln, chunk_bytes=chunk)
        assert np.array_equal(got.numpy(), want)
    desc = torch.stack([off, ln], 1).to(torch.int32)
    ra, rd, _ = D.exchange_by_flow(arena, desc, torch.zeros(200, dtype=torch.int64))
    assert ra.numel() == int(ln.sum()) + D.ARENA_PAD and int(ra[-D.ARENA_PAD:].sum()) == 0
    assert np.array_equal(ra[:int(ln.sum())].numpy(), want)
