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
