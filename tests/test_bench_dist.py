"""bench.py's own rank function at world size 2 (gloo, CPU).

bench.rank_main is the code every bench rank runs: shard selection, warmup,
the barrier-bracketed timed region, max-over-ranks timing, the counter
all-reduce and the per-output offset all-gather, and the checks on them. Here
it runs with a CPU stand-in for the device processor whose counters come from
the C oracle on the rank's shard (this host has no GPU); the GPU case is
test_gpu_bench_two_ranks (two ranks sharing cuda:0 over gloo).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class OracleProcessor:
    """CPU stand-in with DeviceProcessor's interface: each step's counters
    are the oracle's counters of this rank's shard of the step's batch."""

    def __init__(self, args, lo, hi, gpu):
        import bench
        from fastclick_amd import synth, _native as N
        from oracle import oracle as O
        b, self.valid_per_batch = bench.make_host_batch(args)
        shard = synth.Batch(arena=b.arena, desc=np.ascontiguousarray(b.desc[lo:hi]))
        cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=args.nports,
                         badsrc=[N.raw_addr(a) for a in bench.ERROR_BADSRC] if args.errors else ())
        self.per_step = O.process_batch(cfg, shard)["counters"].astype(np.int64)
        self.steps = args.steps
        self.ctr = torch.zeros(N.CTR_SHARDS, N.NCOUNTERS, dtype=torch.int64)
        self.n = hi - lo

    def warmup(self, k):
        pass

    def run_timed(self):
        self.ctr[3] += torch.from_numpy(self.per_step * self.steps)

    def sync(self):
        pass

    def counters(self):
        return self.ctr

    def timing(self):
        return None

    def close(self):
        pass


def _rank(rank, world, port, argv, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        args = bench.parse(argv)
        line = bench.rank_main(args, OracleProcessor, world=world, rank=rank, gpu=0, backend="gloo",
                               dev_for_collectives="cpu")
        lo, hi = bench.shard_of(args, world, rank)
        q.put((rank, line, lo, hi))
    finally:
        dist.destroy_process_group()


def _run_two(argv):
    world = 2
    port = 29700 + (os.getpid() % 500)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, argv, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.timeout(300)
def test_bench_rank_main_strong_two_ranks(oracle):
    """--shard strong: one 20,000-packet C4 batch per step split in two; the
    all-reduced valid count is steps x the whole batch, n_gpus is 2, and the
    two shards tile the batch."""
    res = _run_two(["--gpus", "2", "--shard", "strong", "--packets", "20000", "--steps", "3",
                    "--warmup", "1", "--no-cpu", "--nbuf", "1"])
    line = res[0][1]
    assert res[1][1] is None
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["packets_per_step"] == 20000
    assert (res[0][2], res[0][3], res[1][2], res[1][3]) == (0, 10000, 10000, 20000)
    assert line["value"] > 0 and line["steps"] == 3


@pytest.mark.timeout(300)
def test_bench_rank_main_errors_two_ranks(oracle):
    """--errors: the with-errors mix; rank_main checks the
    all-reduced valid count against the packets the mix left valid."""
    res = _run_two(["--gpus", "2", "--shard", "strong", "--packets", "20000", "--steps", "2",
                    "--warmup", "1", "--no-cpu", "--nbuf", "1", "--errors", "0.01", "--workload", "c4"])
    line = res[0][1]
    assert line["config"]["errors_per_kind"] == 0.01
    assert 0.93 < line["config"]["valid_fraction"] < 0.97


@pytest.mark.timeout(300)
def test_bench_rank_main_weak_two_ranks(oracle):
    """--shard weak: every rank its own batch; total = world x steps x n."""
    res = _run_two(["--gpus", "2", "--packets", "5000", "--steps", "2", "--warmup", "1",
                    "--no-cpu", "--nbuf", "1"])
    line = res[0][1]
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["packets_per_step"] == 10000


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_gpu_bench_two_ranks():
    """`bench.py --gpus 2 --backend gloo` without WORLD_SIZE starts two local
    ranks (both on cuda:0 here), each running the device path; the line
    reports n_gpus 2 and the all-reduced valid count checks out inside."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    for shard in ("weak", "strong"):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                            "--shard", shard, "--packets", "65536", "--steps", "4", "--warmup", "2",
                            "--nbuf", "2", "--no-cpu"], env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        line = json.loads(r.stdout.strip().splitlines()[-1])
        assert line["n_gpus"] == 2 and line["scaling"] == shard
        assert line["config"]["packets_per_step"] == (131072 if shard == "weak" else 65536)


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("gpus,exchange,slack", [(1, "fixed", 1.25), (2, "fixed", 1.25), (1, "counted", 1.25),
                                                 (2, "counted", 1.25), (1, "fixed", 0.5), (2, "fixed", 0.4)])
def test_gpu_bench_flow_reshard(gpus, exchange, slack):
    """`bench.py --flow-reshard`: every step runs the owner pass, the exchange
    kernels, the all-to-alls (gloo on one GPU for 2 ranks) and the flow table
    over the received batch; inside the run the all-reduced valid count is
    every packet once, and the tables' flow counts add up to the distinct
    5-tuples of the ranks' batches (config.flow_reshard.checked). The fixed
    exchange (no host sync per step) with too small a capacity (slack < 1)
    stalls at its first step and replays every step through the counted
    exchange, with the same checked result."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["FCGPU_RESHARD_STAGES"] = "2"       # stage markers on every 2nd timed step: step 1 of 0..2
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--backend", "gloo",
                        "--flow-reshard", "--workload", "c4", "--packets", "65536", "--steps", "3", "--warmup", "1",
                        "--nbuf", "2", "--no-cpu", "--reshard-exchange", exchange, "--reshard-slack", str(slack)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    fr = line["config"]["flow_reshard"]
    assert fr["checked"] and fr["flow_table_flows"] == fr["distinct_5tuples"] == 65536 * gpus
    assert fr["packets_received"] == fr["packets_sent"] == 65536 * gpus * 3
    assert set(fr["stage_ms_per_step"]) == {"owner_pass", "build", "exchange", "unpack", "flow_pass"}
    assert fr["stage_sampled_steps"] == 1
    assert fr["exchange"] == exchange
    if exchange == "fixed":
        assert fr["fallback_steps"] == (3 if slack < 1 else 0)


def test_flow_reshard_options():
    import bench
    a = bench.parse(["--flow-reshard", "--workload", "c4"])
    assert a.flow_reshard and a.streams == 1
    for bad in (["--flow-reshard"], ["--flow-reshard", "--workload", "c4", "--shard", "strong"],
                ["--flow-reshard", "--workload", "c4", "--flow-manager", "imp"]):
        with pytest.raises(SystemExit):
            bench.parse(bad)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_strong_shards_rotate_beyond_the_infinity_cache(world):
    """--shard strong (C4, 1M packets): every rank uploads only its own
    frames (an arena of ~1/world of the batch, descriptors rebased onto it,
    the frames' bytes unchanged) and rotates over enough copies of them that
    the bytes its steps touch exceed 1.15 GB -- HBM, not the 256 MB Infinity
    Cache, at every point of the strong curve."""
    import bench
    from fastclick_amd import synth
    args = bench.parse(["--gpus", str(world), "--shard", "strong"])
    host, _ = bench.make_host_batch(args)
    assert host.n == 1 << 20
    for rank in range(world):
        lo, hi = bench.shard_of(args, world, rank)
        arena, desc = bench.shard_arrays(host, lo, hi)
        assert desc.shape == (hi - lo, 2)
        assert arena.nbytes <= host.arena.nbytes // world + 4096
        touched = arena.nbytes + desc.nbytes
        nbuf = bench.rotation_nbuf(touched)
        assert nbuf * touched >= 1.15e9 and (nbuf - 1) * touched < 1.15e9 or nbuf == 4
        for i in (0, (hi - lo) // 2, hi - lo - 1):   # the frames travel unchanged
            o, ln = (int(x) for x in desc[i])
            oo, lln = (int(x) for x in host.desc[lo + i])
            assert ln == lln and o % 256 == oo % 256
            assert bytes(arena[o:o + ln]) == bytes(host.arena[oo:oo + ln])
        shard = synth.Batch(arena=arena, desc=desc)
        assert shard.frame(hi - lo - 1) == host.frame(hi - 1)
    assert bench.rotation_nbuf(131072 * 64 + 256 + 131072 * 8) == 122   # 122 x 9.4 MB at N = 8
    # the default rotation reads HBM; --nbuf 1..3 of the C2 batch is labelled cache-resident
    touched = (1 << 20) * 72
    assert bench.residency(bench.rotation_nbuf(touched) * touched) == "hbm"
    for nbuf in (1, 2, 3):
        assert bench.residency(nbuf * touched).startswith("cache-resident")
    assert bench.residency(8 * touched).startswith("mixed")


def test_nccl_world_larger_than_devices_fails_at_startup():
    import bench
    with pytest.raises(SystemExit, match="one GPU per rank"):
        bench.check_devices(8, 1, "nccl")
    bench.check_devices(2, 1, "gloo")     # a rehearsal on one GPU
    bench.check_devices(8, 8, "nccl")
    with pytest.raises(SystemExit, match="no HIP device"):
        bench.check_devices(1, 0, "nccl")
