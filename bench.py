"""Headline benchmark: Mpps, device-resident, 64 B IPv4 cksum + classify.

Workload (BASELINE.json configs[1], C2): 1,048,576 packets of 60-B UDP/IPv4
frames (64 B on the wire) in 64-B slots, one 5-tuple, resident in HBM. One
step = one pass of the hot path over one batch:

    CheckIPHeader(OFFSET 14, CHECKSUM true) -> AggregateHash (IPFlowID low 32)
    -> FlowSwitch LB_MODE hash over 16 outputs -> stable per-port partition

i.e. k_rx of libfcgpu.so (plus k_scan + k_part with --partition global).
Steps rotate over --nbuf distinct copies of the rank's batch placed in
different HBM regions (default: >= 1.15 GB of touched bytes per GPU, e.g.
16 x 72 MB at 1M 64-B packets, > 4x the 256 MB Infinity Cache), so every step
reads its packets from HBM. The timed steps are submitted by
one fcgpu_process_jobs call (no per-step Python on the launch path), each
with its own output buffers, on one stream (--streams: more streams, as rx
queues would); the library fuses a stream's queued batches into k_rx
launches of up to 24 batches (--fuse), so the launch ramp and tail are paid
once per launch, not once per batch.

Multi-GPU: one process per GPU (torchrun, or `--gpus N` without WORLD_SIZE,
which starts the N local rank processes itself). --shard weak (default):
every rank processes its own 1M-packet batches (scaling "weak", no data-path
collective). --shard strong (configs[3], C4): one 1M-packet batch per step is
split over the ranks with dist.shard_range (131,072 packets per GPU at N=8;
every shard is a whole number of 256-packet PacketBatches, so no per-step
exchange is needed either); each rank uploads only its shard's frames
(shard_arrays) and rotates over enough copies of them to stay beyond the
Infinity Cache (122 x 9.4 MB of frames + descriptors at N=8). After the timed region the per-port / per-reason
counters are all-reduced over RCCL (the reference sums per-thread counters on
read, include/click/sync.hh:384) and the per-output offsets all-gathered
(dist.output_offsets); both are checked.

rank 0 prints ONE JSON line (contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PKT_BYTES_READ = 72          # 64-B header window + 8-B descriptor
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "Mpps device-resident, 64 B IPv4 cksum+classify, 1/2/4/8 MI355X"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU). Under torchrun it must equal WORLD_SIZE; without "
                         "WORLD_SIZE, N > 1 starts the N local rank processes")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--packets", type=int, default=1 << 20,
                    help="packets per step per GPU (weak) or per step in total (strong)")
    ap.add_argument("--shard", choices=["weak", "strong"], default="weak")
    ap.add_argument("--nbuf", type=int, default=0,
                    help="distinct HBM copies of this rank's batch (its shard with --shard strong) the "
                         "steps rotate over; 0 (default): enough for >= 1.15 GB of touched bytes per GPU, "
                         "at least 4 (16 x 72 MB for 1M 64-B frames, 122 x 9.4 MB for a 1/8 strong shard, "
                         "4 x 420 MB for IMIX) -- beyond the 256 MB Infinity Cache at every N")
    ap.add_argument("--nports", type=int, default=16)
    ap.add_argument("--no-perm", action="store_true", help="skip the partition")
    ap.add_argument("--partition", choices=["tile", "global"], default="tile",
                    help="tile: each 256-packet tile is one classified PacketBatch (1 launch); "
                         "global: the whole batch is one (3 launches)")
    ap.add_argument("--fuse", type=int, default=24,
                    help="batches one k_rx launch may carry (fcgpu_process_jobs fuses consecutive jobs of "
                         "a stream whose outputs are disjoint, up to 24): each step gets its own output set "
                         "among fuse x streams; 1 = one launch per batch")
    ap.add_argument("--no-timing", action="store_true", help="no per-kernel HIP events")
    ap.add_argument("--timing-every", type=int, default=0,
                    help="bracket the k_rx launch covering every k-th timed batch with HIP events "
                         "(stream markers on the launch stream, hipEventRecord; created before the "
                         "timed region). Each event idles the queue ~4 us, so the default samples "
                         "sparsely: 8 (a fused launch of 20 batches is one bracketed launch)")
    ap.add_argument("--streams", type=int, default=1,
                    help="HIP streams the consecutive steps alternate over (each with its own output "
                         "buffers), as batches of several rx queues would. Default 1: the steps are "
                         "queued on one stream and fused into k_rx launches of up to --fuse batches")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process-group backend (nccl = RCCL over xGMI; gloo only to rehearse "
                         "several ranks on one GPU)")
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5"], default=None,
                    help="c2: one 5-tuple (BASELINE configs[1], the headline); c3: IMIX "
                         "64/570/1500 B 7:4:1 over 10k 5-tuples (configs[2]); c4: independent "
                         "uniform random 5-tuples (configs[3]); c5: 50%% 802.1Q + 30%% IPv6 mix "
                         "through StripEtherVLANHeader + CheckIP6Header/CheckIPHeader (configs[4]). "
                         "Default c2, or c4 with --shard strong")
    ap.add_argument("--layout", choices=["wire", "split"], default="wire",
                    help="wire (default): every frame whole in 64-B aligned slots, as received; split: "
                         "the first 64 B of every frame in a dense ring of 64-B slots (two per 128-B "
                         "line), as a NIC's header/data buffer split delivers them -- a labelled variant, "
                         "never the config number")
    ap.add_argument("--frame-bytes", type=int, default=64,
                    help="c2/c4 frame size on the wire (64..1518; captured = size - 4 FCS bytes, "
                         "ip_len = captured - 14, fastudpflows.cc:146-175); the kernel still reads "
                         "the 64-B header window of every frame")
    ap.add_argument("--flow-capacity", type=int, default=0,
                    help="> 0: the device flow table (FlowIPManagerHMP flow IDs, fcgpu_flow_enable) "
                         "behind the check, with this many IDs; its new-flow pass runs every step "
                         "(one stream: the table assigns IDs in batch order)")
    ap.add_argument("--errors", type=float, default=0.0,
                    help="c2/c4: corrupt this fraction of the packets per error kind (bad version, "
                         "header length, ip_len, checksum, BADSRC source; SURVEY 8(d) 'with-errors "
                         "mix', e.g. 0.01); the invalid ones leave on the drop output")
    ap.add_argument("--flow-manager", choices=["hmp", "imp"], default="hmp",
                    help="hmp: FlowIPManagerHMP IDs 0,1,2,...; imp: VirtualFlowManagerIMP (free-ID "
                         "stack; with --flow-timeout, every packet stamps its flow and the maintainer "
                         "run is timed outside the timed region: flow_maintain_ms)")
    ap.add_argument("--flow-timeout", type=int, default=0, help="imp: TIMEOUT in s (0: none)")
    ap.add_argument("--flow-recycle-ms", type=int, default=1000, help="imp: RECYCLE_INTERVAL in ms")
    ap.add_argument("--classify", choices=["lb", "lbcrc", "lbtable", "haship", "ipclass16"], default="lb",
                    help="lb: FlowSwitch LB_MODE hash x16 (headline); lbcrc: LB_MODE hash_crc x16 "
                         "(CRC32-C of the IPFlow5ID, DPDK builds); lbtable: LB_MODE cst_hash_agg x16 "
                         "(the 1600-bucket consistent-hash ring); haship: LB_MODE hash_ip x16 (byte sum of "
                         "frame bytes 26..33); ipclass16: the survey's "
                         "IPClassifier with 15 UDP dst-port ranges + '-' (program printed by the "
                         "reference compiler, tests/golden/reftests.json)")
    ap.add_argument("--l4", choices=["none", "udp", "tcp"], default="none",
                    help="CheckUDPHeader / CheckTCPHeader behind the IPv4 check (pseudo-header checksum "
                         "over the whole segment; the synthetic frames are UDP, so tcp sends them all to "
                         "the drop output)")
    ap.add_argument("--rewrite", action="store_true",
                    help="DecIPTTL + SetIPChecksum behind the classifier; the rewritten header bytes go "
                         "to an ip_rw output per batch (not in place: the rotating batches are reused)")
    ap.add_argument("--flow-reshard", action="store_true",
                    help="(f)#1 x (e): every step re-shards the rank's batch by flow before the flow table "
                         "(SURVEY 8(f) #1 on several GPUs): the device owner pass (LB_MODE hash over the "
                         "world's ranks, verdicts), fcgpu_exchange_build, the RCCL all-to-alls of counts, "
                         "records and frames (dist.exchange_built), fcgpu_exchange_unpack, "
                         "then the FlowIPManagerHMP pass over the received batch; C4 (uniform 5-tuples, a "
                         "different batch per rank). Per-stage times and checked flow counts in "
                         "config.flow_reshard; a labelled variant, never the headline")
    ap.add_argument("--reshard-exchange", choices=["fixed", "counted"], default="fixed",
                    help="--flow-reshard: fixed = equal-split all-to-alls of fixed-capacity owner segments "
                         "(fcgpu_exchange_build_fixed / _unpack_fixed, fcgpu_process_counted: no host sync "
                         "per step; a step whose segments overflow stalls and is replayed through the counted "
                         "exchange, config.flow_reshard.fallback_steps); counted = dist.exchange_built "
                         "(one host sync per step for the split sizes)")
    ap.add_argument("--reshard-slack", type=float, default=1.25,
                    help="--flow-reshard fixed: an owner segment holds a uniform share of the batch x this "
                         "(below 1, also at one rank: forces overflows, to exercise the replay)")
    ap.add_argument("--program-jit", type=int, default=1,
                    help="ipclass16: 1 = the program compiled to code (fcgpu_program_jit, hiprtc, before "
                         "the warmup); 0 = the step interpreter")
    ap.add_argument("--prefault", type=int, default=1,
                    help="1: read every rotating batch before the warmup, repeatedly for at least "
                         "--prefault-ms (page translations resident, GPU clocks up after the idle "
                         "process start); 0: off")
    ap.add_argument("--prefault-ms", type=float, default=250.0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    a = ap.parse_args(argv)
    if a.workload is None:
        a.workload = "c4" if a.shard == "strong" else "c2"
    if a.frame_bytes != 64 and a.workload not in ("c2", "c4"):
        ap.error("--frame-bytes applies to c2/c4")
    if a.errors and (a.workload not in ("c2", "c4") or a.frame_bytes != 64 or not 0 < a.errors <= 0.2):
        ap.error("--errors applies to 64-B c2/c4, with a rate in (0, 0.2]")
    if not 64 <= a.frame_bytes <= 1518:
        ap.error("--frame-bytes must be in [64, 1518]")
    if (a.l4 != "none" or a.rewrite) and a.workload == "c5":
        ap.error("--l4 / --rewrite need an IPv4 workload (c2, c3, c4)")
    if a.flow_capacity and a.streams > 1:
        # one table per context, IDs in batch order: a second stream would
        # either race on the table's scratch or need a second table
        a.streams = 1
    if a.partition == "global" and a.streams > 1 and not a.no_perm:
        a.streams = 1    # the whole-batch partition uses context scratch
    if a.flow_reshard:
        if a.workload != "c4" or a.shard != "weak" or a.frame_bytes != 64 or a.layout != "wire" or a.errors:
            ap.error("--flow-reshard runs 64-B C4 batches, weak sharding, wire layout")
        if a.flow_manager != "hmp":
            ap.error("--flow-reshard uses the HMP table")
        a.streams = 1
    return a


WORKLOADS = {
    "c2": "C2: {F} B IPv4/UDP ({C}-B frames in {S}-B slots), {N}-packet device-resident batch, single 5-tuple",
    "c3": "C3: IMIX 64/570/1500 B (7:4:1) IPv4/UDP, 10k uniform 5-tuples, {N}-packet device-resident batch "
          "(first 64 B of each frame read)",
    "c4": "C4: {F} B IPv4/UDP ({C}-B frames in {S}-B slots), {N}-packet device-resident batch, independent "
          "uniform 5-tuples",
    "c5": "C5: 50% 802.1Q-tagged, 30% IPv6 (80-B frames) / 70% IPv4 (60-B), {N}-packet device-resident batch",
}


# the device code k_rx is compiled from (host-side library changes do not move its traffic)
KERNEL_SOURCES = ("fastclick_amd/csrc/fcgpu_device.hh", "fastclick_amd/csrc/fcgpu_flow.hh")


def kernel_source_sha() -> str:
    """Hash of the k_rx sources: the stored PMC traffic (profiles/pmc_traffic.json)
    counts only while the kernel it was measured on is the one running."""
    import hashlib
    h = hashlib.sha256()
    for p in KERNEL_SOURCES:
        with open(os.path.join(ROOT, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def ipclass16_program():
    """The survey's 16-output IPClassifier as compiled by the reference (text)."""
    with open(os.path.join(ROOT, "tests", "golden", "reftests.json")) as f:
        progs = {p["case"]: p for p in json.load(f)["programs"]}
    return progs["ipclass16"]["program"]


# ---- host CPU description and the reported CPU baseline --------------------

def host_cpu_info():
    """nproc, the CPUs this process may run on, the cgroup CPU quota and the
    model. On the GPU box nproc shows the whole machine; the job's share is
    the quota (or 16 CPUs per GPU, the box's stated share)."""
    info = dict(nproc=os.cpu_count(), affinity=len(os.sched_getaffinity(0)), cgroup_quota=None, model=None)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            info["cgroup_quota"] = round(int(q) / int(per), 2)
    except Exception:
        pass
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except Exception:
        pass
    share = info["affinity"]
    if info["cgroup_quota"]:
        share = min(share, max(1, int(info["cgroup_quota"])))
    why = "affinity" if share == info["affinity"] else "cgroup quota"
    if os.environ.get("GRAFT_REPO_ROOT") and share > 16:
        share, why = 16, "the GPU box's CPU share per GPU"
    env = os.environ.get("FCGPU_CPU_THREADS")
    if env:
        share, why = max(1, int(env)), "FCGPU_CPU_THREADS"
    info["threads_used"] = share
    info["threads_basis"] = why
    return info


def _run_cpu(exe, seconds, threads, flows, stages, program):
    cmd = [exe, "--seconds", str(seconds), "--threads", str(threads), "--flows", str(flows),
           "--stages", str(stages)]
    tmp = None
    if program is not None:
        import tempfile
        tmp = tempfile.NamedTemporaryFile("w", suffix=".prog", delete=False)
        tmp.write(program)
        tmp.close()
        cmd += ["--program", tmp.name]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=seconds * 4 + 60)
        return json.loads(out.stdout.strip().splitlines()[-1])
    finally:
        if tmp is not None:
            os.unlink(tmp.name)


def cpu_baseline(seconds: float, flows: int = 1, program: str | None = None):
    """Reported CPU baseline: the scalar restatement of the reference elements
    (oracle/cpu_baseline.cc: 32-packet linked-list PacketBatch, atomic
    counters, one pipeline per core) on this host: the C2 chain
    Strip(14) -> CheckIPHeader(CHECKSUM true) -> AggregateHash -> FlowSwitch
    hash x16 (or the IPClassifier program) -> Discard, and beside it C1's
    Strip(14) -> CheckIPHeader(CHECKSUM true) -> Discard."""
    exe = os.path.join(ROOT, "oracle", "_build", "fc_cpu_baseline")
    if not os.path.exists(exe):
        try:
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "baseline"])
        except Exception:
            return None
    info = host_cpu_info()
    th = info["threads_used"]
    try:
        main = _run_cpu(exe, seconds * 2 / 3, th, flows, 3, program)
        c1 = _run_cpu(exe, seconds / 3, th, 4096, 1, None)
    except Exception as e:  # reported baseline only
        print(f"cpu baseline failed: {e}", file=sys.stderr)
        return None
    return dict(value=round(main["mpps"], 3), unit="Mpps", cores=main["threads"], kind="port",
                sample=main["sample"], mpps_1core=round(main.get("mpps_1core", 0.0), 3),
                c1_value=round(c1["mpps"], 3), c1_mpps_1core=round(c1.get("mpps_1core", 0.0), 3),
                c1_sample=c1["sample"], nproc=info["nproc"], affinity=info["affinity"],
                cgroup_quota=info["cgroup_quota"], cores_basis=info["threads_basis"], cpu_model=info["model"],
                calibration=CPU_CALIBRATION)


# The port against the reference binary (within +-20 % per stage,
# or the ratio stated). Measured once in the survey container, where the
# reference was built (it cannot run on the GPU box): 1 thread, the same trace.
CPU_CALIBRATION = {
    "source": "DESIGN.md section 5.5 (survey container, reference click binary vs oracle/cpu_baseline.cc, "
              "1 thread, same trace)",
    "ns_per_pkt": {"CheckIPHeader(CHECKSUM true)": {"port": 10.5, "reference": 12.7},
                   "AggregateHash": {"port": 3.8, "reference": 3.1}},
    "harness_floor_mpps": {"port": 121.0, "reference": 22.5},
    "end_to_end_port_over_reference": 2.0,
    "note": "the port's per-element costs are within -17 %/+23 % of the reference's, but its replay "
            "harness is ~5x lighter than Click's FromDump/ReplayUnqueue -> Discard, so the port's "
            "end-to-end Mpps is ~2x what the reference itself would reach on these cores: "
            "value is an upper bound for the reference, not the reference",
}


# ---- launching the local ranks ---------------------------------------------

def spawn_local_ranks(args) -> int:
    """`--gpus N` without WORLD_SIZE: start N rank processes of this script
    (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, 127.0.0.1), wait, return the
    worst exit code. Runs before anything touches the GPU, and starts the
    ranks as children (never exec)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        for p in procs:
            code = p.wait()
            rc = rc or code
            if code:
                for q in procs:          # one rank failed: the others would hang in a collective
                    if q.poll() is None:
                        q.kill()
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
                q.wait()
    return rc


# ---- the rank ----------------------------------------------------------------

def shard_of(args, world, rank):
    """(lo, hi) packet range of this rank within a step's batch."""
    from fastclick_amd.dist import shard_range
    if args.shard == "strong":
        return shard_range(args.packets, world, rank)
    return 0, args.packets


# CheckIPHeader(BADSRC ..) of the with-errors mix (the addresses synth's
# BADSRC errors use, plus the limited broadcast)
ERROR_BADSRC = ("192.0.2.255", "255.255.255.255")


def make_host_batch(args):
    """The workload's host batch; with --errors also the number of packets
    the mix leaves valid. --layout split: its header-split form."""
    from fastclick_amd import synth
    b = _make_host_batch(args)
    valid = b.n
    if args.errors:
        kind = synth.inject_errors(b, args.errors, seed=41,
                                   kinds=(synth.ERR_VERSION, synth.ERR_HLEN, synth.ERR_IPLEN, synth.ERR_CKSUM,
                                          synth.ERR_BADSRC))
        valid = int((kind < 0).sum())
    if getattr(args, "layout", "wire") == "split":
        b = synth.header_split(b, 64)
    return b, valid


def traffic_key(args, per_gpu):
    """The key of a workload's PMC traffic in profiles/pmc_traffic.json: every
    option that changes what k_rx reads or writes."""
    parts = [args.workload, f"fb{args.frame_bytes}", getattr(args, "layout", "wire"), f"n{per_gpu}"]
    if args.flow_capacity:
        parts.append(f"flow{args.flow_capacity}{args.flow_manager}")
    if args.classify != "lb":
        parts.append(args.classify)
    if args.l4 != "none":
        parts.append("l4" + args.l4)
    if args.rewrite:
        parts.append("rewrite")
    if args.no_perm or args.partition != "tile":
        parts.append("nopart" if args.no_perm else args.partition)
    if args.errors:
        parts.append(f"err{args.errors:g}")
    return "/".join(parts)


def _make_host_batch(args):
    from fastclick_amd import synth
    n = args.packets
    if args.workload in ("c2", "c4") and args.frame_bytes != 64:
        import numpy as np
        cap = args.frame_bytes - 4
        if args.workload == "c2":
            hdr = synth.build_headers(n, src=synth.ip4(10, 0, 0, 1), dst=synth.ip4(10, 0, 0, 2),
                                      sport=1234, dport=5678, frame_len=cap, width=64)
        else:
            rng = np.random.default_rng(4)
            hdr = synth.build_headers(n, **synth._rand_flows(rng, n), frame_len=cap, width=64)
        return synth.pack(hdr, cap, meta=dict(config=args.workload.upper(), frame_bytes=args.frame_bytes))
    return dict(c2=synth.c2, c3=synth.c3, c4=synth.c4, c5=synth.c5)[args.workload](n)


ROTATION_BYTES = 1_150_000_000   # > 4 x the 256 MB Infinity Cache of one MI355X
MALL_BYTES = 256 << 20           # the Infinity Cache (MALL) of one MI355X


def residency(rotation_bytes) -> str:
    """Where the timed steps' input comes from, by the rotation's size (SURVEY
    8(d): a cache-resident number is reported apart and labelled)."""
    if not rotation_bytes:
        return "n/a"
    if rotation_bytes >= ROTATION_BYTES:
        return "hbm"
    if rotation_bytes <= MALL_BYTES:
        return "cache-resident: the rotation fits the 256 MB Infinity Cache (not an HBM figure)"
    return "mixed: the rotation is under 4x the Infinity Cache (not an HBM figure)"


def shard_arrays(host, lo, hi, pad=256):
    """The frames of desc[lo:hi] alone: (arena, desc) with the descriptors
    rebased onto an arena that holds only this rank's bytes (plus `pad`
    zero bytes, the header-window over-read include/fastclick_gpu.h allows).

    The slice keeps every frame's offset modulo 256, so the shard's frames sit
    in 128-B lines exactly as they did in the whole batch (two 64-B slots per
    line for C2/C4). synth lays frames out in index order, so desc[lo:hi]'s
    bytes are one contiguous range; the whole batch is returned as is."""
    import numpy as np
    desc = np.ascontiguousarray(host.desc[lo:hi])
    if lo == 0 and hi == host.n:
        return host.arena, desc
    if hi <= lo:
        return np.zeros(pad, np.uint8), desc.reshape(0, 2)
    off = desc[:, 0].astype(np.int64)
    end = int((off + desc[:, 1].astype(np.int64)).max()) + pad
    base = int(off.min()) & ~255
    arena = np.zeros(end - base, np.uint8)
    src = host.arena[base:min(end, host.arena.size)]
    arena[:src.size] = src
    desc = desc.copy()
    desc[:, 0] -= np.uint32(base)
    return arena, desc


def rotation_nbuf(touched: int, nbuf: int = 0) -> int:
    """Distinct HBM copies of a rank's batch the steps rotate over: --nbuf, or
    enough that the rotation (copies x the bytes one step touches: arena +
    descriptors) is >= ROTATION_BYTES, and at least 4. Sized from the rank's
    own shard, so a strong shard of 1/N of the batch gets N times the copies
    (122 x 9.4 MB at N = 8) and every point of the curve reads HBM."""
    if nbuf:
        return nbuf
    return max(4, -(-ROTATION_BYTES // max(int(touched), 1)))


def check_devices(world: int, ndev: int, backend: str) -> None:
    """One process per GPU: RCCL cannot run two ranks of one communicator on
    one device, so an nccl world larger than the visible devices fails here,
    at startup, instead of hanging inside the first collective."""
    if ndev == 0:
        raise SystemExit("bench.py: no HIP device visible")
    if backend == "nccl" and world > ndev:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} ranks but {ndev} visible GPU(s): the nccl backend "
                         "needs one GPU per rank (--backend gloo only rehearses several ranks on one GPU)")


class DeviceProcessor:
    """The hot path on this rank's GPU: nbuf HBM-resident copies of this
    rank's shard of the batch (one allocation, rows 4 KB aligned), one
    context, --streams output sets; steps submitted through
    fcgpu_process_jobs."""

    def __init__(self, args, lo, hi, gpu):
        import numpy as np
        import torch
        from fastclick_amd import _native as N
        from fastclick_amd.device import DeviceOutputs
        self.N, self.torch, self.args = N, torch, args
        dev = torch.device("cuda", gpu)
        self.dev = dev
        host, self.valid_per_batch = make_host_batch(args)
        self.frame_meta = dict(slot=int(host.desc[1, 0] - host.desc[0, 0]) if host.n > 1 else 64,
                               captured=int(host.desc[0, 1]))
        n = hi - lo
        self.n = n
        arena_np, desc_np = shard_arrays(host, lo, hi)
        del host
        touched = arena_np.nbytes + desc_np.nbytes
        args.nbuf = rotation_nbuf(touched, args.nbuf)
        self.rotation_bytes = args.nbuf * touched
        # nbuf copies at distinct HBM addresses, filled by device-side copies
        stride = -(-arena_np.size // 4096) * 4096
        arena = torch.from_numpy(arena_np).to(dev)
        desc = torch.from_numpy(desc_np.view(np.int32)).to(dev)
        self.arena_all = torch.empty((args.nbuf, stride), dtype=torch.uint8, device=dev)
        self.desc_all = torch.empty((args.nbuf,) + tuple(desc.shape), dtype=torch.int32, device=dev)
        self.arena_all[:, :arena.numel()].copy_(arena.expand(args.nbuf, -1))
        self.desc_all.copy_(desc.expand(args.nbuf, *desc.shape))
        del arena, desc
        self.bufs = [(self.arena_all[k], self.desc_all[k]) for k in range(args.nbuf)]
        program = None
        if args.classify == "ipclass16":
            from fastclick_amd import click
            steps, oe = click.parse_program(ipclass16_program())
            program = (N.PROG_IPFILTER, steps, oe)
            args.nports = 16
        self.auto = args.workload == "c5"
        classify = (N.CLS_PROGRAM if program is not None else
                    N.CLS_LB_CRC if args.classify == "lbcrc" else
                    N.CLS_LB_TABLE if args.classify == "lbtable" else
                    N.CLS_HASH_IP if args.classify == "haship" else N.CLS_LB_HASH)
        cfg = N.make_cfg(check_mode=N.CHECK_AUTO if self.auto else N.CHECK_IP4, offset=0 if self.auto else 14,
                         checksum=True, hash_mode=N.HASH_FLOWID, classify=classify, nports=args.nports,
                         badsrc=[N.raw_addr(a) for a in ERROR_BADSRC] if args.errors else (),
                         l4_mode=dict(none=N.L4_NONE, udp=N.L4_UDP, tcp=N.L4_TCP)[args.l4],
                         rewrite=(N.RW_DECTTL | N.RW_SETCKSUM) if args.rewrite else 0)
        part = N.PART_TILE if args.partition == "tile" else N.PART_GLOBAL
        tile = part == N.PART_TILE
        self.ctx = N.Context(gpu, max(n, 1), cfg)
        if program is not None:
            self.ctx.set_program(*program)
            if args.program_jit:
                self.ctx.program_jit(True)
        if classify == N.CLS_LB_TABLE:
            self.ctx.set_lb_table(N.lb_hash_ring(args.nports))
        self.maintain_ms = None
        if args.flow_capacity:
            if args.flow_manager == "imp":
                self.ctx.flow_configure(N.FLOW_MGR_IMP, args.flow_capacity, args.flow_timeout,
                                        args.flow_recycle_ms)
                self.ctx.flow_set_time(1_000_000)
            else:
                self.ctx.flow_enable(args.flow_capacity)
        self.streams = [torch.cuda.Stream(dev) for _ in range(max(1, args.streams))]
        # one output set per step of a fused launch (fcgpu_process_jobs
        # fuses only jobs whose outputs do not overlap)
        nsets = len(self.streams) * max(1, min(args.fuse, 24))
        self.outs = [DeviceOutputs(max(n, 1), args.nports, device=dev, verdict=True, hash=True, anno=False,
                                   perm=(not args.no_perm) and not tile,
                                   tile_perm=(not args.no_perm) and tile, port_start=not args.no_perm,
                                   partition=part, flowid=args.flow_capacity > 0, ip_rw=args.rewrite)
                     for _ in range(nsets)]
        self.ctr = torch.zeros(N.CTR_SHARDS, N.NCOUNTERS, dtype=torch.int64, device=dev)
        self.timing_every = 0 if args.no_timing else (args.timing_every or min(8, max(1, args.steps)))

    def _jobs(self, first, count):
        """Steps first .. first+count-1 as one fcgpu_process_jobs submission."""
        specs = []
        ns = len(self.streams)
        for k in range(first, first + count):
            a, d = self.bufs[k % len(self.bufs)]
            j = k % ns
            specs.append((a.data_ptr(), d.data_ptr(), self.n, self.streams[j].cuda_stream,
                          self.outs[k % len(self.outs)].ptrs()))
        return self.ctx.jobs(specs)

    def _run(self, sub):
        self.ctx.run_jobs(sub)

    def warmup(self, steps):
        if self.args.prefault:
            # read every rotating batch (a read-only reduction), so the timed
            # steps meet resident page translations, as buffers a NIC keeps
            # filling would be, and keep doing so for --prefault-ms so the
            # GPU's clocks are up: after the idle process start (or a test
            # run) a single pass left the first timed region up to 8 % slower
            # in kernel time (profiles/r02_final/bench.log). The warmup steps
            # that follow stream 72 MB each, so none of this is left in the
            # Infinity Cache.
            t_end = time.perf_counter() + self.args.prefault_ms * 1e-3
            while True:
                self.arena_all.max()
                self.desc_all.max()
                self.torch.cuda.synchronize()
                if time.perf_counter() >= t_end:
                    break
        warm = self._jobs(0, steps)
        self.timed = self._jobs(steps, self.args.steps)   # built before the warmup
        # creates the event pool now, and times every warmup launch: the first
        # launch with timing events pays a one-time cost in HIP (~9 us of host
        # enqueue, profiles/r02_s9/diag*.log) that belongs in the warmup, not
        # in the timed region (the pool hands the same events out again)
        self.ctx.set_timing(1 if self.timing_every else 0)
        self._run(warm)
        self.torch.cuda.synchronize()
        self.ctx.read_timing()                      # drop warmup samples
        if self.args.flow_capacity and self.args.flow_manager == "imp" and self.args.flow_timeout:
            self._time_maintainer()
        self.ctx.set_timing(self.timing_every)      # sample count restarts at the timed region
        self.ctx.use_counters(self.ctr.data_ptr())  # timed steps count into the tensor

    def _time_maintainer(self):
        """Maintainer runs at the batches' own time stamp until one walks the
        wheel bucket holding the batch's flows (lastseen not in the past:
        every flow is rescheduled, virtualflowmanager.hh:174-180, so the table
        is unchanged); that run's device time, table rebuild included."""
        torch = self.torch
        s = self.streams[0]
        best = 0.0
        te = self.args.flow_timeout * max(1, 1000 // self.args.flow_recycle_ms)
        for _ in range(min(te + 2, 256)):             # run te + 1 walks the warmup's bucket
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            self.ctx.flow_maintain(1_000_000, stream=s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            best = max(best, e0.elapsed_time(e1))
        self.maintain_ms = best

    def run_timed(self):
        self._run(self.timed)

    def sync(self):
        self.torch.cuda.synchronize()

    def counters(self):
        return self.ctr

    def timing(self):
        if not self.timing_every:
            return None
        ms, cnt = self.ctx.read_timing()
        return dict(k_rx_ms=ms[0] / max(cnt[0], 1), k_scan_ms=ms[1] / max(cnt[1], 1),
                    k_part_ms=ms[2] / max(cnt[2], 1), launches=cnt)

    def close(self):
        self.ctx.close()


class ReshardProcessor:
    """--flow-reshard: the flow re-shard inside each step.
    Rank r's batch is its own C4 batch (seed 4 + r: independent uniform
    5-tuples, so every rank's flows are new to the others); per step:

      owner pass   k_rx: LB_MODE hash over `world` outputs (the FlowSwitch
                   formula on the IPFlowID hash), verdicts only -> each
                   packet's owner rank
      build        fcgpu_exchange_build (3 kernels): records and send buffer
                   straight from the verdicts, every load in input order
      exchange     dist.exchange_built: RCCL all-to-all of the per-owner
                   counts from the device, one host sync for the split sizes,
                   then the records and the frame bytes (world 1: the send
                   buffer is the received one, no collective)
      unpack       fcgpu_exchange_unpack: records -> descriptors
      flow pass    k_rx with the FlowIPManagerHMP table + the new-flow pass over
                   the received batch (tile partition, 16 outputs)

    The same --nbuf rotation as the headline keeps the owner pass reading
    HBM. The flow pass's counters are the step's counters (so the all-reduced
    valid count checks that every packet arrived exactly once), and after the
    timed region post_check() all-reduces the tables' flow counts against the
    distinct 5-tuples of all ranks' batches."""

    def __init__(self, args, lo, hi, gpu):
        import numpy as np
        import torch
        import torch.distributed as dist
        from fastclick_amd import _native as N, synth
        from fastclick_amd.device import DeviceOutputs
        self.N, self.torch, self.args, self.np = N, torch, args, np
        dev = torch.device("cuda", gpu)
        self.dev = dev
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank() if self.world > 1 else 0
        n = hi - lo
        self.n = n
        seed = 4 + self.rank
        host = synth.c4(n, seed=seed)
        fl = synth._rand_flows(np.random.default_rng(seed), n)
        keys = np.stack([fl["src"].astype(np.uint64) << 32 | fl["dst"].astype(np.uint64),
                         fl["sport"].astype(np.uint64) << 16 | fl["dport"].astype(np.uint64)], axis=1)
        self.distinct = int(np.unique(keys, axis=0).shape[0])      # this rank's distinct 5-tuples
        self.valid_per_batch = n
        touched = host.arena.nbytes + host.desc.nbytes
        args.nbuf = rotation_nbuf(touched, args.nbuf)
        self.rotation_bytes = args.nbuf * touched
        stride = -(-host.arena.size // 4096) * 4096
        arena = torch.from_numpy(host.arena).to(dev)
        desc = torch.from_numpy(host.desc.view(np.int32)).to(dev)
        self.arena_all = torch.empty((args.nbuf, stride), dtype=torch.uint8, device=dev)
        self.desc_all = torch.empty((args.nbuf,) + tuple(desc.shape), dtype=torch.int32, device=dev)
        self.arena_all[:, :arena.numel()].copy_(arena.expand(args.nbuf, -1))
        self.desc_all.copy_(desc.expand(args.nbuf, *desc.shape))
        del arena, desc, host
        self.bufs = [(self.arena_all[k], self.desc_all[k]) for k in range(args.nbuf)]
        own_cfg = N.make_cfg(offset=14, checksum=True, hash_mode=N.HASH_FLOWID, classify=N.CLS_LB_HASH,
                             nports=self.world)
        self.ctx_own = N.Context(gpu, max(n, 1), own_cfg)
        self.own_out = DeviceOutputs(max(n, 1), self.world, device=dev, verdict=True, hash=False)
        self.send_cap = stride + 16 * max(n, 1)     # every frame's 16-B slot (the arena's bytes + 16 per packet)
        # a rank receives ~n packets (uniform owners); the flow pass takes them
        # in batches of at most cap (the flow table's largest batch,
        # FCGPU_FLOW_MAX_BATCH), in order, so any count fits
        self.cap = min(N.FLOW_MAX_BATCH, 2 * max(n, 1))
        flow_cfg = N.make_cfg(offset=14, checksum=True, hash_mode=N.HASH_FLOWID, classify=N.CLS_LB_HASH,
                              nports=args.nports)
        self.ctx_flow = N.Context(gpu, self.cap, flow_cfg)
        self.ctx_flow.flow_enable(args.flow_capacity or 2 * max(n, 1))     # room for every flow a rank owns
        self.flow_out = DeviceOutputs(self.cap, args.nports, device=dev, verdict=True, hash=True,
                                      tile_perm=True, partition=N.PART_TILE, flowid=True)
        self.ctr = torch.zeros(N.CTR_SHARDS, N.NCOUNTERS, dtype=torch.int64, device=dev)
        self.received = 0
        self.stage_ms = [0.0] * 5
        self.ev = None
        self.timed_steps = 0
        # the fixed-capacity exchange: every buffer sized once, the step's
        # counts stay on the device (received packets summed there too)
        self.fixed = args.reshard_exchange == "fixed"
        # FCGPU_RESHARD_HOST=1: the host's own time per stage of the fixed
        # step (enqueue work), reported in config.flow_reshard
        self.host_t = [0.0] * 6 if os.environ.get("FCGPU_RESHARD_HOST") == "1" else None
        self.recv_dev = torch.zeros(1, dtype=torch.int64, device=dev)   # the unpack adds each timed step's count
        self.fallback_steps = 0
        self.step_id = 0
        self.step_k = {}
        if self.fixed:
            from fastclick_amd import device as DV
            from fastclick_amd.dist import ARENA_PAD
            if args.reshard_slack < 1:      # forced overflows (also at one rank)
                recs = max(1, int(n * args.reshard_slack))
                segb = (max(16, int(self.send_cap * args.reshard_slack)) + 15) // 16 * 16
            else:
                recs, segb = DV.fixed_capacity(n, self.send_cap, self.world, args.reshard_slack)
            self.recs, self.segb = recs, segb
            W = self.world
            self.fmeta = torch.empty((W * (recs + 1), 4), dtype=torch.int32, device=dev)
            self.fsend = torch.zeros(W * segb + ARENA_PAD, dtype=torch.uint8, device=dev)
            self.frmeta = torch.empty_like(self.fmeta) if W > 1 else None
            self.frbuf = torch.zeros(W * segb + ARENA_PAD, dtype=torch.uint8, device=dev) if W > 1 else None
            self.fdesc = torch.empty((W * recs, 2), dtype=torch.int32, device=dev)
            self.fcount = torch.zeros(1, dtype=torch.int32, device=dev)
            self.fstall = torch.zeros(1, dtype=torch.int32, device=dev)

    def _step(self, k, timed):
        if self.fixed:
            return self._step_fixed(k, timed)
        return self._step_counted(k, timed)

    def _step_fixed(self, k, timed):
        """One step, no host sync: owner pass, fixed-capacity build, equal-split
        all-to-alls, unpack (the received count stays on the device), the flow
        pass over the bound with that count (fcgpu_process_counted)."""
        import torch
        from fastclick_amd import device as DV
        from fastclick_amd.dist import exchange_fixed
        a, d = self.bufs[k % len(self.bufs)]
        s = torch.cuda.current_stream()
        ev = self.ev[k - self.first] if timed and self.ev else None
        ht = self.host_t
        if ht is not None:
            h0 = time.perf_counter()
        if ev:
            ev[0].record(s)
        o = self.own_out
        self.ctx_own.process(a.data_ptr(), d.data_ptr(), self.n, stream=s.cuda_stream, **o.ptrs())
        if ev:
            ev[1].record(s)
        if ht is not None:
            h1 = time.perf_counter()
        DV.exchange_build_fixed(self.ctx_own, a, d, o.verdict, self.world, self.rank, self.recs, self.segb,
                                self.fmeta, self.fsend, stream=s)
        if ev:
            ev[2].record(s)
        if ht is not None:
            h2 = time.perf_counter()
        out = (self.frmeta, self.frbuf) if self.world > 1 else None
        rmeta, rbuf = exchange_fixed(self.fmeta, self.fsend, self.recs, self.segb, out=out)
        if ev:
            ev[3].record(s)
        if ht is not None:
            h3 = time.perf_counter()
        self.step_id += 1
        self.step_k[self.step_id] = (k, timed)
        DV.exchange_unpack_fixed(self.ctx_own, rmeta, self.world, self.recs, self.segb, self.fdesc, self.fcount,
                                 self.fstall, self.step_id, total=self.recv_dev if timed else None, stream=s)
        if ev:
            ev[4].record(s)
        if ht is not None:
            h4 = time.perf_counter()
        f = self.flow_out
        bound = self.world * self.recs
        for c0 in range(0, bound, self.cap):
            self.ctx_flow.process_counted(rbuf.data_ptr(), self.fdesc[c0:].data_ptr(), min(self.cap, bound - c0),
                                          self.fcount.data_ptr(), c0, stream=s.cuda_stream, **f.ptrs())
        if ev:
            ev[5].record(s)
        if ht is not None:
            h5 = time.perf_counter()
            for j, (x, y) in enumerate(((h0, h1), (h1, h2), (h2, h3), (h3, h4), (h4, h5))):
                ht[j] += y - x
            ht[5] += 1

    def _repair(self):
        """The fixed exchange's stalled steps (a segment overflowed; every later
        step stalled too): replayed in order through the counted exchange --
        collective, so every rank replays from the earliest stalled step of any
        rank, and processes a step's packets only from its own stalled step on.
        One host read of the stall word (where the caller synchronises anyway)."""
        if not self.fixed:
            return
        from fastclick_amd.dist import first_stalled
        mine = int(self.fstall.item())
        first = first_stalled(mine)
        if first:
            for sid in range(first, self.step_id + 1):
                k, timed = self.step_k[sid]
                self._step_counted(k, timed, process=bool(mine) and sid >= mine, replay=True)
                self.fallback_steps += 1 if timed else 0      # timed steps replayed
            self.fstall.zero_()
        self.step_k.clear()

    def _step_counted(self, k, timed, process=True, replay=False):
        import torch
        from fastclick_amd import device as DV
        from fastclick_amd.dist import exchange_built
        N = self.N
        a, d = self.bufs[k % len(self.bufs)]
        s = torch.cuda.current_stream()
        ev = self.ev[k - self.first] if timed and self.ev and not replay else None
        if ev:
            ev[0].record(s)
        o = self.own_out
        self.ctx_own.process(a.data_ptr(), d.data_ptr(), self.n, stream=s.cuda_stream, **o.ptrs())
        if ev:
            ev[1].record(s)
        send, meta, seg_n, seg_bytes = DV.exchange_build(self.ctx_own, a, d, o.verdict, self.world, self.rank,
                                                         send_cap=self.send_cap)
        if ev:
            ev[2].record(s)
        buf, rmeta, displ = exchange_built(send, meta, seg_n, seg_bytes)
        if ev:
            ev[3].record(s)
        rdesc = DV.exchange_unpack(self.ctx_own, rmeta, displ)
        m = int(rdesc.shape[0])
        if ev:
            ev[4].record(s)
        f = self.flow_out
        if not process:          # a replayed step this rank's table already took
            m = 0
        for c0 in range(0, m, self.cap):
            k = min(self.cap, m - c0)
            self.ctx_flow.process(buf.data_ptr(), rdesc[c0:].data_ptr(), k, stream=s.cuda_stream, **f.ptrs())
        if ev:
            ev[5].record(s)      # read after the timed region: no sync per step
        if timed:
            self.received += m

    def warmup(self, steps):
        for k in range(max(steps, 1)):
            self._step(k, False)
        self._repair()
        self.torch.cuda.synchronize()
        self.ctx_flow.use_counters(self.ctr.data_ptr())      # timed steps count into the tensor
        # six markers on every STAGE_EVERY-th timed step (FCGPU_RESHARD_STAGES,
        # default 5; 0: none), created here and read after the timed region,
        # so the steps are not synchronised one by one. Markers cost the step
        # ~20 us when every step has them (113 -> 133 us at N = 1,
        # profiles/r06_reshard/stages), hence the sample
        every = int(os.environ.get("FCGPU_RESHARD_STAGES", "5") or 0)
        self.stage_every = every
        self.ev = [[self.torch.cuda.Event(enable_timing=True) for _ in range(6)] if k % every == every - 1 else None
                   for k in range(self.args.steps)] if every > 0 else None
        self.first = max(steps, 1)

    def run_timed(self):
        for k in range(self.args.steps):
            self._step(self.first + k, True)
        self._repair()           # inside the timed region: replays are work done
        self.timed_steps = self.args.steps

    def sync(self):
        self.torch.cuda.synchronize()

    def counters(self):
        return self.ctr

    def timing(self):
        return None

    def post_check(self, backend):
        """After the timed region: every rank's table holds exactly the flows
        it owns, so the tables' counts add up to the distinct 5-tuples of all
        ranks' batches (all-reduced; the batches' uniform 96-bit keys do not
        repeat across ranks), and every packet arrived once."""
        import torch
        import torch.distributed as dist
        dev = self.dev if backend == "nccl" else "cpu"
        received = self.received + int(self.recv_dev.item())
        v = torch.tensor([self.ctx_flow.flow_count(), self.distinct, received,
                          self.n * self.timed_steps], dtype=torch.int64, device=dev)
        if self.world > 1:
            dist.all_reduce(v, op=dist.ReduceOp.SUM)
        flows, distinct, received, sent = (int(x) for x in v.cpu().tolist())
        if flows != distinct:
            raise AssertionError(f"flow tables hold {flows} flows, the batches have {distinct} distinct 5-tuples")
        if received != sent:
            raise AssertionError(f"{received} packets received, {sent} sent")
        sampled = [ev for ev in self.ev[:self.timed_steps] if ev] if self.ev else []
        if sampled:
            torch.cuda.synchronize()
            for ev in sampled:
                for j in range(5):
                    self.stage_ms[j] += ev[j].elapsed_time(ev[j + 1])
        names = ("owner_pass", "build", "exchange", "unpack", "flow_pass")
        fx = ({"exchange": "fixed", "seg_recs": self.recs, "seg_bytes": self.segb,
               "slack": self.args.reshard_slack, "fallback_steps": self.fallback_steps}
              if self.fixed else {"exchange": "counted"})
        if self.host_t is not None and self.host_t[5]:
            fx["host_us_per_step"] = {k: round(1e6 * t / self.host_t[5], 1) for k, t in
                                      zip(("owner_pass", "build", "exchange", "unpack", "flow_pass"), self.host_t)}
        return {"flow_table_flows": flows, "distinct_5tuples": distinct, "packets_received": received,
                "packets_sent": sent, "checked": True, **fx,
                **({"stage_ms_per_step": {k: round(t / len(sampled), 4) for k, t in zip(names, self.stage_ms)},
                    "stage_sampled_steps": len(sampled),
                    "stage_basis": f"HIP events on the step's stream, every {self.stage_every}th timed step, "
                                   "read after the timed region (their "
                                   "sum is below ms_per_step by the host's own work"
                                   + (")" if self.fixed else " and the exchange's host sync for the "
                                      "split sizes)")}
                   if sampled else {})}

    def close(self):
        self.ctx_own.close()
        self.ctx_flow.close()


def _diag_regions(proc, elapsed, enq, timing, repeats=6):
    """FCGPU_BENCH_DIAG=1 (diagnostics, stderr only; the JSON line is the
    first region's): the timed region repeated in the same process on the
    same jobs and output sets, so a first-region-only cost shows up."""
    snap = proc.counters().clone()     # the repeats count too: restored below
    regs = []
    for _ in range(repeats):
        proc.sync()
        t0 = time.perf_counter()
        proc.run_timed()
        t1 = time.perf_counter()
        proc.sync()
        regs.append(((time.perf_counter() - t0) * 1e6, (t1 - t0) * 1e6))
    print(json.dumps({"diag": {"region_us": round(elapsed * 1e6, 1), "enqueue_us": round(enq * 1e6, 1),
                               "kernel_ms": timing and timing["k_rx_ms"],
                               "repeat_region_us": [round(r, 1) for r, _ in regs],
                               "repeat_enqueue_us": [round(e, 1) for _, e in regs]}}),
          file=sys.stderr, flush=True)
    proc.timing()   # drop the repeats' samples
    proc.counters().copy_(snap)


def rank_main(args, processor_factory, *, world, rank, gpu, backend, dev_for_collectives):
    """One rank of the benchmark: build, warm up, time exactly args.steps
    steps between barrier + device sync on both sides, take the max over
    ranks, reduce the counters and output offsets (after the timed region),
    check them, and return the JSON line (rank 0) or None.

    processor_factory(args, lo, hi, gpu) -> an object with warmup(k),
    run_timed(), sync(), counters() (int64 [CTR_SHARDS, NCOUNTERS] tensor),
    timing() and close(). Tests drive this with a CPU processor."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from fastclick_amd import _native as N
    from fastclick_amd.dist import output_offsets, reduce_counters

    lo, hi = shard_of(args, world, rank)
    proc = processor_factory(args, lo, hi, gpu)
    try:
        proc.warmup(args.warmup)
        if world > 1:
            dist.barrier()
        proc.sync()
        t0 = time.perf_counter()
        proc.run_timed()
        t_enq = time.perf_counter()
        proc.sync()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        timing = proc.timing()
        if os.environ.get("FCGPU_BENCH_DIAG"):
            _diag_regions(proc, elapsed, t_enq - t0, timing)
        maintain_ms = getattr(proc, "maintain_ms", None)
        post = proc.post_check(backend) if hasattr(proc, "post_check") else None

        # after the timed region: max time over ranks, counters summed over
        # ranks (RCCL all-reduce of the device vector), per-output offsets
        t_red = time.perf_counter()
        collective = world > 1 and dist.is_available() and dist.is_initialized()
        ctr = proc.counters()
        glob = reduce_counters(ctr if backend == "nccl" else ctr.cpu())
        if backend == "nccl":
            torch.cuda.synchronize()
        red_ms = (time.perf_counter() - t_red) * 1e3
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev_for_collectives)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        gv = N.derive_counters(glob.cpu().numpy())
        local = N.derive_counters(ctr.sum(0).cpu().numpy())
        nb = args.nports + 1
        lport = torch.from_numpy(local[N.CTR_PORT:N.CTR_PORT + nb].astype(np.int64)).to(dev_for_collectives)
        before, gtot = output_offsets(lport)
        gtot = gtot.cpu().numpy()
    finally:
        proc.close()

    total_pkts = (args.packets if args.shard == "strong" else args.packets * world) * args.steps
    valid = int(gv[N.CTR_COUNT])
    expect_valid = total_pkts if args.workload in ("c2", "c4") else None
    vpb = getattr(proc, "valid_per_batch", None)
    if args.errors and vpb is not None:
        # every rank builds the whole batch: the strong shards add up to it
        expect_valid = vpb * args.steps * (1 if args.shard == "strong" else world)
    if expect_valid is not None and valid != expect_valid:
        raise AssertionError(f"valid count {valid} != {expect_valid}")
    if not np.array_equal(gtot, gv[N.CTR_PORT:N.CTR_PORT + nb].astype(np.int64)):
        raise AssertionError("all-gathered per-output counts disagree with the all-reduced counters")
    if rank != 0:
        return None
    mpps = total_pkts / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3
    per_gpu = hi - lo
    roof = None
    if timing and timing["launches"][0] and timing["k_rx_ms"] > 0:
        kernel_s = timing["k_rx_ms"] * 1e-3
        step_s = ms_per_step * 1e-3
        nstreams = max(1, args.streams)
        # one stream: bytes per launch / the launch's own duration. Several
        # streams overlap launches, so a launch's duration includes its
        # neighbours' share of HBM: the step time is the per-launch figure
        basis = "kernel" if nstreams == 1 else "step"
        t_launch = kernel_s if basis == "kernel" else step_s
        achieved = PKT_BYTES_READ * per_gpu / t_launch / 1e9
        traffic, traffic_src = None, None
        key = traffic_key(args, per_gpu)
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f).get("entries", {})
            # the stored PMC figure (rocprofv3 cannot run inside the bench) counts
            # only for this workload and only while the kernel sources are the
            # ones it was measured on
            ent = tj.get(key)
            if ent is not None:
                if ent.get("source_sha16") == kernel_source_sha():
                    traffic = ent.get("hbm_bytes_per_launch")
                    traffic_src = ent.get("source")
                else:
                    traffic_src = "stale: profiles/pmc_traffic.json was measured on other kernel sources"
        except Exception:
            pass
        roof = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(achieved / HBM_PEAK_GBS, 4), traffic=traffic, traffic_source=traffic_src,
                    traffic_key=key,
                    kernel="k_rx", basis=basis,
                    bytes_per_launch=PKT_BYTES_READ * per_gpu,
                    per="batch (a k_rx launch carries up to config.batches_per_launch batches: "
                        "kernel_ms = the sampled launches' event time in the timed region / their batches)",
                    kernel_ms=round(timing["k_rx_ms"], 5),
                    kernel_frac=round(PKT_BYTES_READ * per_gpu / kernel_s / 1e9 / HBM_PEAK_GBS, 4),
                    scan_ms=round(timing["k_scan_ms"], 5), part_ms=round(timing["k_part_ms"], 5),
                    sampled_batches=timing["launches"][0])
    cpu = None
    if world == 1 and not args.no_cpu and args.workload in ("c2", "c3", "c4") and not args.flow_capacity \
            and not args.flow_reshard and args.classify in ("lb", "ipclass16"):   # the chains the port runs
        cpu = cpu_baseline(args.cpu_seconds, flows=dict(c2=1, c3=10000).get(args.workload, 4096),
                           program=ipclass16_program() if args.classify == "ipclass16" else None)
    fb = args.frame_bytes
    slot = max(64, (fb - 4 + 63) // 64 * 64)
    wl = WORKLOADS[args.workload].format(F=fb, C=fb - 4, S=slot, N=per_gpu)
    auto = args.workload == "c5"
    line = {
        "metric": METRIC,
        "value": round(mpps, 1),
        "unit": "Mpps",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": args.shard,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": (wl
                         + ("; StripEtherVLANHeader + CheckIP6Header/CheckIPHeader(CHECKSUM true)"
                            if auto else "; CheckIPHeader(CHECKSUM true)")
                         + ("; header-split arena: the first 64 B of every frame in a dense 64-B slot ring "
                            "(a NIC's header/data buffer split; labelled variant, not the config number)"
                            if args.layout == "split" else "")
                         + (f" (with-errors mix: {args.errors:g} each of bad version, header length, "
                            f"ip_len, checksum, BADSRC)" if args.errors else "")
                         + (f" + Check{args.l4.upper()}Header" if args.l4 != "none" else "")
                         + (f" + flow re-shard across the {world} rank(s) (owner pass, fcgpu_exchange_build, "
                            f"all-to-alls of counts, records and frames, fcgpu_exchange_unpack) + FlowIPManagerHMP "
                            f"flow table over the received batch" if args.flow_reshard else "")
                         + ((f" + FlowIPManagerHMP flow table ({args.flow_capacity} IDs)"
                             if args.flow_manager == "hmp" else
                             f" + VirtualFlowManagerIMP flow table (CAPACITY {args.flow_capacity}, "
                             f"TIMEOUT {args.flow_timeout}, RECYCLE_INTERVAL {args.flow_recycle_ms} ms)")
                            if args.flow_capacity else "")
                         + " + AggregateHash + "
                         + ({"lb": "FlowSwitch hash 16 outputs",
                             "lbcrc": "FlowSwitch LB_MODE hash_crc 16 outputs",
                             "lbtable": "FlowSwitch LB_MODE cst_hash_agg 16 outputs (1600-bucket ring)",
                             "haship": "FlowSwitch LB_MODE hash_ip 16 outputs"}.get(
                                args.classify, "IPClassifier(15 UDP dst-port ranges, -) 16 outputs"))
                         + ("" if args.no_perm else
                            " + stable per-port partition of every 256-packet PacketBatch"
                            if args.partition == "tile" else
                            " + stable per-port partition of the whole batch")
                         + (" + DecIPTTL + SetIPChecksum (rewritten bytes to ip_rw)" if args.rewrite else "")),
            "classify": args.classify + (" (compiled program)" if args.classify == "ipclass16" and args.program_jit
                                         else " (interpreted program)" if args.classify == "ipclass16" else ""),
            **({"errors_per_kind": args.errors,
                "valid_fraction": round(valid / total_pkts, 4)} if args.errors else {}),
            "partition": "none" if args.no_perm else args.partition,
            "streams": max(1, args.streams),
            "batches_per_launch": max(1, min(args.fuse, 8 if args.flow_capacity else 24,
                                             -(-args.steps // max(1, args.streams)))),
            "frame_bytes": fb,
            "layout": args.layout,
            "packets_per_step_per_gpu": per_gpu,
            "packets_per_step": args.packets if args.shard == "strong" else args.packets * world,
            "hbm_batches": args.nbuf,
            **({"rotation_bytes_per_gpu": int(proc.rotation_bytes),
                "residency": residency(proc.rotation_bytes)}
               if getattr(proc, "rotation_bytes", None) else {}),
            "nports": args.nports,
            **({"flow_maintain_ms": round(maintain_ms, 4)} if maintain_ms is not None else {}),
            **({"flow_reshard": post} if post is not None else {}),
            "parallelism": ((f"batch-sharded x{world}" if args.shard == "weak" else
                             f"one batch split x{world} (dist.shard_range)")
                            + f", counters all-reduced after the timed region "
                              f"({'RCCL' if backend == 'nccl' else 'gloo'}, {red_ms:.3f} ms)"
                            if collective else
                            f"one GPU: no collective (world 1); counter replicas summed on the device "
                            f"after the timed region ({red_ms:.3f} ms)"),
        },
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    return line


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(spawn_local_ranks(args))
    world = int(world_env or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one process per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    check_devices(world, ndev, args.backend)
    gpu = local % ndev
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(gpu)
    try:
        line = rank_main(args, ReshardProcessor if args.flow_reshard else DeviceProcessor, world=world, rank=rank,
                         gpu=gpu, backend=args.backend,
                         dev_for_collectives=torch.device("cuda", gpu) if args.backend == "nccl" else "cpu")
        if line is not None:
            print(json.dumps(line), flush=True)
    finally:
        if world > 1:
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
