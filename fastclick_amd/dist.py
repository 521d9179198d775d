"""Multi-GPU helpers: batch sharding and counter reduction.

The path is stateless per packet, so a batch splits into contiguous index
ranges, one per GPU, with no data-path collective. The only exchange is the
counter vector (per-output counts and per-reason counts; "count" and "drops"
follow from them, _native.derive_counters / fcgpu_counters_derive): each GPU
keeps FCGPU_CTR_SHARDS replicas that are summed locally and then all-reduced
across ranks -- the MI355X analogue of FastClick's per_thread<> counters summed
by PER_THREAD_SUM on read (include/click/sync.hh:56,384). When a globally
ordered per-output list is wanted, an all-gather of the per-rank per-output
counts gives every shard its output offsets (concatenating shard outputs in
rank order preserves CLASSIFY_EACH_PACKET order).

With a flow table (fcgpu_flow_enable) the path is stateful per flow. FastClick
keeps one flow table per core and relies on the NIC's RSS hash to send every
packet of a flow to the same core. The GPU analogue:
batches whose packets arrive on any GPU are re-sharded by flow first.
`exchange_by_flow` moves each packet to the rank its flow hash names: HIP
kernels pack the leaving frames by owner and write a 16-B record per packet
(fcgpu_exchange_plan / _pack), RCCL all-to-alls move the counts, the records
and the frame bytes over xGMI, and a HIP kernel turns the received records
into descriptors (fcgpu_exchange_unpack). Every flow then
lives in exactly one rank's table. The owner of a packet is the device
classifier's output with LB_MODE hash over `world` outputs: the
FlowSwitch/LoadBalancer formula on the IPFlowID hash, a function of the
5-tuple.

Backend-agnostic: "nccl" (RCCL over xGMI) on GPUs, "gloo" in CPU tests.
"""
from __future__ import annotations


ARENA_PAD = 256   # zeroed bytes after a received arena (include/fastclick_gpu.h over-read)


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [begin, end) packet range of `rank` among `world` shards."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return (n * rank) // world, (n * (rank + 1)) // world


def _collective(group, force):
    """Whether to issue the collective: a process group exists and has more
    than one rank, or `force` (a world-1 group still runs the RCCL call, so
    the N = 1 case exercises the same code as N = 8)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return force or dist.get_world_size(group) > 1


def reduce_counters(replicas, group=None, force=False):
    """Sum a [replicas, NCOUNTERS] int64 tensor over replicas, then over ranks.
    Returns the global NCOUNTERS vector (same device as the input)."""
    import torch.distributed as dist
    local = replicas.sum(0) if replicas.dim() == 2 else replicas.clone()
    if _collective(group, force):
        dist.all_reduce(local, op=dist.ReduceOp.SUM, group=group)
    return local


def output_offsets(local_counts, group=None, force=False):
    """All-gather every rank's per-output counts [nout] and return this rank's
    start offset within each output's global list, plus the global totals."""
    import torch
    import torch.distributed as dist
    if not _collective(group, force):
        return torch.zeros_like(local_counts), local_counts.clone()
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    parts = [torch.empty_like(local_counts) for _ in range(world)]
    dist.all_gather(parts, local_counts, group=group)
    stacked = torch.stack(parts)                  # [world, nout]
    before = stacked[:rank].sum(0) if rank else torch.zeros_like(local_counts)
    return before, stacked.sum(0)


def exchange_segments(send, meta, seg_n, seg_bytes, group=None):
    """The all-to-all of the flow re-shard: every rank sends owner d's records
    (meta rows) and frame bytes (its segment of `send`) to rank d. send ends
    with ARENA_PAD zero bytes; meta is an int32 [m, 4] tensor of fcgpu_xmeta
    records; seg_n / seg_bytes are host lists of per-owner packet and byte
    counts. Returns (buffer, meta, src_displ): the received segments
    concatenated in source-rank order and followed by ARENA_PAD zero bytes
    (the ABI's header-window over-read), their records, and where each
    source's segment starts. Plumbing only (torch.distributed: RCCL over xGMI
    on GPUs, gloo in CPU tests); the records and bytes are built and read by
    the HIP kernels (fastclick_amd.device.exchange_pack / exchange_unpack)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if len(seg_n) != world or len(seg_bytes) != world:
        raise ValueError(f"{len(seg_n)} segments for a world of {world}")
    if world == 1:
        return send, meta, [0]
    if send.is_cuda and dist.get_backend(group) == "gloo":
        # a rehearsal of several ranks on one GPU (bench.py --backend gloo):
        # gloo's all-to-all takes host tensors
        buf, rmeta, displ = exchange_segments(send.cpu(), meta.cpu(), seg_n, seg_bytes, group=group)
        return buf.to(send.device), rmeta.to(send.device), displ
    dev = send.device
    cnt = torch.tensor([[int(a), int(b)] for a, b in zip(seg_n, seg_bytes)], dtype=torch.int64, device=dev)
    rcnt = torch.empty_like(cnt)
    dist.all_to_all_single(rcnt, cnt, group=group)           # [world, 2] from every rank
    # the one host sync of the exchange: the receive sizes of the next two
    # all-to-alls are host split lists (RCCL needs them at enqueue). Its cost
    # is the round trip of this 16*world-byte all-to-all, measured with the
    # rest of the exchange by bench.py --flow-reshard (config.flow_reshard)
    rc = rcnt.cpu().tolist()
    rn, rb = [r[0] for r in rc], [r[1] for r in rc]
    total = int(sum(rb))
    if total + ARENA_PAD >= 1 << 32:
        raise ValueError("received frames exceed the 4 GiB a uint32 descriptor offset addresses")
    rmeta = torch.empty((int(sum(rn)), 4), dtype=torch.int32, device=dev)
    dist.all_to_all_single(rmeta, meta.contiguous(), rn, [int(x) for x in seg_n], group=group)
    buf = torch.empty(total + ARENA_PAD, dtype=torch.uint8, device=dev)
    buf[total:].zero_()
    sent = int(sum(seg_bytes))
    dist.all_to_all_single(buf[:total], send[:sent], rb, [int(x) for x in seg_bytes], group=group)
    displ, at = [], 0
    for b in rb:
        displ.append(at)
        at += b
    return buf, rmeta, displ


def exchange_built(send, meta, seg_n, seg_bytes, group=None):
    """The all-to-all of a send side built by device.exchange_build (segment
    sizes still on the device): the per-owner counts go to their owners
    straight from the device tensors, and one host sync reads this rank's
    sizes and the sizes it receives together -- the all-to-alls of records
    and frames need them as host split lists. Returns exchange_segments'
    (buffer, meta, src_displ)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if seg_n.numel() != world or seg_bytes.numel() != world:
        raise ValueError(f"{seg_n.numel()} owner segments for a world of {world}")
    cnt = torch.stack([seg_n.to(torch.int64), seg_bytes], dim=1)      # [world, 2]
    if world > 1 and not (send.is_cuda and dist.get_backend(group) == "gloo"):
        rcnt = torch.empty_like(cnt)
        dist.all_to_all_single(rcnt, cnt, group=group)
        both = torch.cat([cnt, rcnt]).cpu().tolist()                  # the one host sync
        mine, theirs = both[:world], both[world:]
    else:
        mine, theirs = cnt.cpu().tolist(), None
    sn, sb = [int(r[0]) for r in mine], [int(r[1]) for r in mine]
    total = sum(sb)
    if total + ARENA_PAD > send.numel() or max(sb, default=0) > 0xFFFFFFFF:
        raise ValueError(f"exchange_built: {total} B of segments for a {send.numel() - ARENA_PAD}-B send "
                         "buffer (aliasing descriptors?) or an owner's segment past 4 GiB")
    m = sum(sn)
    if world == 1:
        # the send buffer is the received one: zero its pad after the frames
        send[total:total + ARENA_PAD].zero_()
        return send, meta[:m], [0]
    if theirs is None:                                                # gloo rehearsal: host all-to-alls
        return exchange_segments(send[:total + ARENA_PAD], meta[:m], sn, sb, group=group)
    dev = send.device
    rn, rb = [int(r[0]) for r in theirs], [int(r[1]) for r in theirs]
    rtotal = sum(rb)
    if rtotal + ARENA_PAD >= 1 << 32:
        raise ValueError("received frames exceed the 4 GiB a uint32 descriptor offset addresses")
    rmeta = torch.empty((sum(rn), 4), dtype=torch.int32, device=dev)
    dist.all_to_all_single(rmeta, meta[:m].contiguous(), rn, sn, group=group)
    buf = torch.empty(rtotal + ARENA_PAD, dtype=torch.uint8, device=dev)
    buf[rtotal:].zero_()
    dist.all_to_all_single(buf[:rtotal], send[:total], rb, sb, group=group)
    displ, at = [], 0
    for b in rb:
        displ.append(at)
        at += b
    return buf, rmeta, displ


def exchange_fixed(meta, send, seg_recs, seg_bytes, group=None, out=None):
    """The all-to-alls of the fixed-capacity re-shard (fcgpu_exchange_build_fixed):
    meta int32 [world * (seg_recs + 1), 4] and send uint8 [world * seg_bytes
    (+ pad)] go out with equal splits -- owner d's segment to rank d -- so no
    split size is read on the host and the step never waits for the device.
    Returns (rmeta, rbuf): source s's segment at s, rbuf followed by ARENA_PAD
    zero bytes (out: preallocated (rmeta, rbuf) to receive into). World 1: the
    send side is the received one (no collective; send's pad must be zero)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    rows, nb = world * (seg_recs + 1), world * seg_bytes
    if meta.shape[0] < rows or send.numel() < nb:
        raise ValueError(f"exchange_fixed: {meta.shape[0]} rows / {send.numel()} B for a world of {world}")
    if world == 1:
        return meta, send
    if send.is_cuda and dist.get_backend(group) == "gloo":
        # a rehearsal of several ranks on one GPU: gloo's all-to-all takes host tensors
        rm, rb = exchange_fixed(meta[:rows].cpu(), send[:nb].cpu(), seg_recs, seg_bytes, group=group)
        return rm.to(meta.device), rb.to(send.device)
    if out is None:
        rmeta = torch.empty((rows, 4), dtype=meta.dtype, device=meta.device)
        rbuf = torch.empty(nb + ARENA_PAD, dtype=torch.uint8, device=send.device)
        rbuf[nb:].zero_()
    else:
        rmeta, rbuf = out
    dist.all_to_all_single(rmeta[:rows], meta[:rows].contiguous(), group=group)
    dist.all_to_all_single(rbuf[:nb], send[:nb], group=group)
    return rmeta, rbuf


def first_stalled(step, group=None):
    """The fixed-capacity re-shard's replay point: `step` is this rank's stall
    word (the first step whose received segments overflowed, 0: none). Returns
    the earliest stalled step over all ranks (0: none) -- every rank replays
    the steps from there through the counted exchange (its all-to-alls are
    collective), and a rank processes a replayed step's packets only from its
    own stalled step on (the ones before it already went through its flow
    table)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return int(step)
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    big = 1 << 62
    v = torch.tensor([int(step) if step else big], dtype=torch.int64, device=dev)
    dist.all_reduce(v, op=dist.ReduceOp.MIN, group=group)
    r = int(v.item())
    return 0 if r == big else r


def exchange_by_flow(ctx, arena, desc, perm, port_start, group=None):
    """Re-shard this rank's device batch by owner rank (one all-to-all).

    ctx: a fastclick_amd._native.Context on this rank's GPU; arena / desc: the
    batch (uint8 tensor; int32 [n, 2] uint32 bit patterns); perm / port_start:
    the whole-batch partition of the device pass that named every packet's
    owner (LB_MODE hash over `world` outputs; the invalid list, output
    `world`, stays here). Returns (arena_recv, desc_recv, src): the frames this
    rank now owns, in (source rank, source index) order, each at a 16-B aligned
    offset with its bytes and length exact, the buffer followed by ARENA_PAD
    zero bytes; their descriptors; src = source_rank << 32 | source_index.
    Pack and unpack are HIP kernels (fcgpu_exchange_*); there is no CPU path."""
    import torch
    import torch.distributed as dist
    from . import device as DV
    if not arena.is_cuda:
        raise RuntimeError("exchange_by_flow runs on device tensors (fcgpu_exchange_*)")
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    send, meta, seg_n, seg_bytes = DV.exchange_pack(ctx, arena, desc, perm, port_start, world, rank)
    buf, rmeta, displ = exchange_segments(send, meta, seg_n, seg_bytes, group=group)
    desc_recv = DV.exchange_unpack(ctx, rmeta, displ)
    src = rmeta[:, 2:4].contiguous().view(torch.int64).flatten()
    return buf, desc_recv, src
