"""Headline benchmark: Mpps, device-resident, 64 B IPv4 cksum + classify.

Workload (BASELINE.json configs[1], C2): 1,048,576 packets of 60-B UDP/IPv4
frames (64 B on the wire) in 64-B slots, one 5-tuple, resident in HBM. One
step = one pass of the hot path over one batch:

    CheckIPHeader(OFFSET 14, CHECKSUM true) -> AggregateHash (IPFlowID low 32)
    -> FlowSwitch LB_MODE hash over 16 outputs -> stable per-port partition

i.e. k_rx + k_scan + k_part of libfcgpu.so. Steps rotate over --nbuf distinct
batches placed in different HBM regions (default 16 x 72 MB = 1.15 GB > the
256 MB Infinity Cache), so every step reads its packets from HBM.

Multi-GPU (torchrun, one process per GPU): each rank processes its own batch
per step (weak scaling, no data-path collective); the per-port / per-reason
counters are summed across ranks with one all-reduce over RCCL at the end of
the timed region (the reference sums per-thread counters on read).

rank 0 prints ONE JSON line (contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PKT_BYTES_READ = 72          # 64-B header window + 8-B descriptor
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--nbuf", type=int, default=16)
    ap.add_argument("--nports", type=int, default=16)
    ap.add_argument("--no-perm", action="store_true", help="skip the partition")
    ap.add_argument("--partition", choices=["tile", "global"], default="tile",
                    help="tile: each 256-packet tile is one classified PacketBatch (1 launch); "
                         "global: the whole batch is one (3 launches)")
    ap.add_argument("--no-timing", action="store_true", help="no per-kernel HIP events")
    ap.add_argument("--timing-every", type=int, default=8,
                    help="bracket every k-th step's kernels with HIP events (ext-launch "
                         "start/stop on the launch stream); sampling keeps the event cost "
                         "out of most steps")
    ap.add_argument("--streams", type=int, default=1,
                    help="HIP streams the consecutive steps alternate over (each with its own "
                         "context and output buffers), so one batch's tail overlaps the next "
                         "batch's head, as back-to-back NIC batches would")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process-group backend (nccl = RCCL over xGMI; gloo only to rehearse "
                         "several ranks on one GPU)")
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5"], default="c2",
                    help="c2: one 5-tuple (BASELINE configs[1], the headline); c3: IMIX "
                         "64/570/1500 B 7:4:1 over 10k 5-tuples (configs[2]); c4: independent "
                         "uniform random 5-tuples (configs[3]); c5: 50%% 802.1Q + 30%% IPv6 mix "
                         "through StripEtherVLANHeader + CheckIP6Header/CheckIPHeader (configs[4])")
    ap.add_argument("--flow-capacity", type=int, default=0,
                    help="> 0: the device flow table (FlowIPManagerHMP flow IDs, fcgpu_flow_enable) "
                         "behind the check, with this many IDs; its new-flow pass runs every step")
    ap.add_argument("--classify", choices=["lb", "ipclass16"], default="lb",
                    help="lb: FlowSwitch LB_MODE hash x16 (headline); ipclass16: the survey's "
                         "IPClassifier with 15 UDP dst-port ranges + '-' (program printed by the "
                         "reference compiler, tests/golden/reftests.json)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


WORKLOADS = {
    "c2": "C2: 64 B IPv4/UDP (60-B frames in 64-B slots), 1M-packet device-resident batch, single 5-tuple",
    "c3": "C3: IMIX 64/570/1500 B (7:4:1) IPv4/UDP, 10k uniform 5-tuples, 1M-packet device-resident batch "
          "(first 64 B of each frame read)",
    "c4": "C4: 64 B IPv4/UDP (60-B frames in 64-B slots), 1M-packet device-resident batch, independent "
          "uniform 5-tuples",
    "c5": "C5: 50% 802.1Q-tagged, 30% IPv6 (80-B frames) / 70% IPv4 (60-B), 1M-packet device-resident batch",
}


def ipclass16_program():
    """The survey's 16-output IPClassifier as compiled by the reference (text)."""
    with open(os.path.join(ROOT, "tests", "golden", "reftests.json")) as f:
        progs = {p["case"]: p for p in json.load(f)["programs"]}
    return progs["ipclass16"]["program"]


def cpu_baseline(seconds: float, flows: int = 1, program: str | None = None):
    """Reported CPU baseline: the scalar restatement of the reference elements
    (oracle/cpu_baseline.cc: 32-packet linked-list PacketBatch, CheckIPHeader ->
    AggregateHash -> FlowSwitch hash -> CLASSIFY_EACH_PACKET, atomic counters),
    one pipeline per core, on this host."""
    exe = os.path.join(ROOT, "oracle", "_build", "fc_cpu_baseline")
    if not os.path.exists(exe):
        try:
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "baseline"])
        except Exception:
            return None
    cores = len(os.sched_getaffinity(0))
    cores = max(1, min(cores, 16))
    cmd = [exe, "--seconds", str(seconds), "--threads", str(cores), "--flows", str(flows)]
    tmp = None
    if program is not None:
        import tempfile
        tmp = tempfile.NamedTemporaryFile("w", suffix=".prog", delete=False)
        tmp.write(program)
        tmp.close()
        cmd += ["--program", tmp.name]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=seconds * 4 + 60)
        res = json.loads(out.stdout.strip().splitlines()[-1])
    except Exception as e:  # reported baseline only
        print(f"cpu baseline failed: {e}", file=sys.stderr)
        return None
    finally:
        if tmp is not None:
            os.unlink(tmp.name)
    return dict(value=round(res["mpps"], 3), unit="Mpps", cores=res["threads"], kind="port",
                sample=res["sample"], mpps_1core=round(res.get("mpps_1core", 0.0), 3))


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    gpu = local % max(ndev, 1)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    local = gpu

    from fastclick_amd import synth, _native as N
    from fastclick_amd.device import DeviceBatch, DeviceOutputs

    n = args.packets
    host = dict(c2=synth.c2, c3=synth.c3, c4=synth.c4, c5=synth.c5)[args.workload](n)
    # nbuf distinct copies at distinct HBM addresses
    bufs = []
    for k in range(args.nbuf):
        bufs.append(DeviceBatch.upload(host, device=dev))
    del host
    program = None
    if args.classify == "ipclass16":
        from fastclick_amd import click
        text = ipclass16_program()
        steps, oe = click.parse_program(text)
        program = (N.PROG_IPFILTER, steps, oe)
        args.nports = 16
    auto = args.workload == "c5"
    cfg = N.make_cfg(check_mode=N.CHECK_AUTO if auto else N.CHECK_IP4, offset=0 if auto else 14,
                     checksum=True, hash_mode=N.HASH_FLOWID,
                     classify=N.CLS_LB_HASH if program is None else N.CLS_PROGRAM, nports=args.nports)
    part = N.PART_TILE if args.partition == "tile" else N.PART_GLOBAL
    tile = part == N.PART_TILE
    nstreams = max(1, args.streams)
    # per stream: its own context (workspace) and output buffers
    ctxs, streams, optrs, outs_keep = [], [], [], []
    for _ in range(nstreams):
        ctxs.append(N.Context(local, n, cfg))
        if program is not None:
            ctxs[-1].set_program(*program)
        if args.flow_capacity:
            ctxs[-1].flow_enable(args.flow_capacity)
        streams.append(torch.cuda.Stream(dev))
        o = DeviceOutputs(n, args.nports, device=dev, verdict=True, hash=True, anno=False,
                          perm=(not args.no_perm) and not tile, tile_perm=(not args.no_perm) and tile,
                          port_start=not args.no_perm, partition=part, flowid=args.flow_capacity > 0)
        outs_keep.append(o)
        optrs.append(o.ptrs())
    ctx = ctxs[0]
    # the first stream also carries the counter all-reduce; it waits for the others
    main_stream = streams[0]
    torch.cuda.set_stream(main_stream)

    def step(k):
        j = k % nstreams
        b = bufs[k % len(bufs)]
        ctxs[j].process(b.arena.data_ptr(), b.desc.data_ptr(), n, stream=streams[j].cuda_stream,
                        **optrs[j])

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize()
    # counters accumulate straight into a torch tensor so RCCL can reduce them
    ctr_t = torch.zeros(N.CTR_SHARDS, N.NCOUNTERS, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    for c in ctxs:
        c.use_counters(ctr_t.data_ptr())
    timing_on = not args.no_timing
    if timing_on:
        for c in ctxs:
            c.read_timing()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    every = max(1, args.timing_every)
    for k in range(args.steps):
        if timing_on and k % every == 0:
            c = ctxs[k % nstreams]
            c.set_timing(True)
            step(k)
            c.set_timing(False)
        else:
            step(k)
    for s_ in streams[1:]:
        main_stream.wait_stream(s_)
    if world > 1:
        # per-port / per-reason counters summed across GPUs: one RCCL all-reduce
        # of the device counter vector (xGMI), like PER_THREAD_SUM on read
        from fastclick_amd.dist import reduce_counters
        glob = reduce_counters(ctr_t if args.backend == "nccl" else ctr_t.cpu())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        total_valid = int(N.derive_counters(glob.cpu().numpy())[N.CTR_COUNT])
    else:
        total_valid = int(N.derive_counters(ctr_t.sum(0).cpu().numpy())[N.CTR_COUNT])

    timing = None
    if not args.no_timing:
        ms, cnt = [0.0] * 3, [0] * 3
        for c in ctxs:
            m_, c_ = c.read_timing()
            ms = [a + b for a, b in zip(ms, m_)]
            cnt = [a + b for a, b in zip(cnt, c_)]
        timing = dict(k_rx_ms=ms[0] / max(cnt[0], 1), k_scan_ms=ms[1] / max(cnt[1], 1),
                      k_part_ms=ms[2] / max(cnt[2], 1), launches=cnt)

    total_pkts = n * args.steps * world
    assert total_valid == total_pkts, f"valid count {total_valid} != {total_pkts}"
    mpps = total_pkts / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3

    if rank == 0:
        roof = None
        if timing:
            t_launch = timing["k_rx_ms"] * 1e-3
            achieved = PKT_BYTES_READ * n / t_launch / 1e9
            traffic = None
            try:
                with open(args.traffic_json) as f:
                    tj = json.load(f)
                if tj.get("packets") == n:
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                pass
            roof = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(achieved / HBM_PEAK_GBS, 4), traffic=traffic,
                        kernel="k_rx", kernel_ms=round(timing["k_rx_ms"], 5),
                        scan_ms=round(timing["k_scan_ms"], 5), part_ms=round(timing["k_part_ms"], 5))
        cpu = None
        if world == 1 and not args.no_cpu and not auto and not args.flow_capacity:
            cpu = cpu_baseline(args.cpu_seconds, flows=dict(c2=1, c3=10000).get(args.workload, 4096),
                               program=ipclass16_program() if program is not None else None)
        line = {
            "metric": "Mpps device-resident, 64 B IPv4 cksum+classify, 1/2/4/8 MI355X",
            "value": round(mpps, 1),
            "unit": "Mpps",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": (WORKLOADS[args.workload]
                             + ("; StripEtherVLANHeader + CheckIP6Header/CheckIPHeader(CHECKSUM true)"
                                if auto else "; CheckIPHeader(CHECKSUM true)")
                             + (f" + FlowIPManagerHMP flow table ({args.flow_capacity} IDs)"
                                if args.flow_capacity else "")
                             + " + AggregateHash + "
                             + ("FlowSwitch hash 16 outputs" if program is None else
                                "IPClassifier(15 UDP dst-port ranges, -) 16 outputs")
                             + ("" if args.no_perm else
                                " + stable per-port partition of every 256-packet PacketBatch"
                                if args.partition == "tile" else
                                " + stable per-port partition of the whole 1M-packet batch")),
                "classify": args.classify,
                "partition": "none" if args.no_perm else args.partition,
                "streams": nstreams,
                "packets_per_step_per_gpu": n,
                "hbm_batches": args.nbuf,
                "nports": args.nports,
                "parallelism": f"batch-sharded x{world}, counters all-reduced "
                               f"({'RCCL' if args.backend == 'nccl' else 'gloo'})",
            },
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    for c in ctxs:
        c.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
