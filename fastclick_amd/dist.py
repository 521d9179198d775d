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
`exchange_by_flow` moves each packet to the rank its flow hash names, with one
RCCL all-to-all of counts and one of frame bytes over xGMI. Every flow then
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


def exchange_by_flow(arena, desc, owner, group=None):
    """Re-shard one rank's packets by owner rank (an all-to-all over `group`).

    arena: uint8 tensor of frame bytes; desc: int32 [n, 2] (offset, length)
    into it; owner: int64 [n], the destination rank of each packet (-1 keeps
    nothing: the packet is dropped here, e.g. one that failed the checks).
    Returns (arena_recv, desc_recv, src): the frames this rank now owns,
    packed back to back in (source rank, source index) order and followed by
    ARENA_PAD zero bytes (the header-window over-read the ABI allows), their
    descriptors (uint32 offset/length bit patterns in int32), and
    src = source_rank << 32 | source_index per packet. The frames keep their
    bytes and lengths exactly.
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    dev = arena.device
    owner = owner.to(torch.int64)
    if owner.numel() and int(owner.max()) >= world:
        raise ValueError(f"owner rank {int(owner.max())} outside a world of {world}")
    keep = owner >= 0
    idx = torch.nonzero(keep).flatten()
    dst = owner[idx]
    order = idx[torch.argsort(dst, stable=True)]             # packets grouped by destination
    off = desc[order, 0].to(torch.int64) & 0xFFFFFFFF
    ln = desc[order, 1].to(torch.int64) & 0xFFFFFFFF
    send_n = torch.bincount(owner[order], minlength=world)
    payload = _gather_frames(arena, off, ln)
    send_b = torch.zeros(world, dtype=torch.int64, device=dev).index_add_(0, owner[order], ln)
    meta = torch.stack([ln, (rank << 32) | order], 1)        # [m, 2] length, source tag
    if world == 1:
        recv_n, recv_b, rmeta, rpay = send_n, send_b, meta, payload
    else:
        cnt = torch.stack([send_n, send_b], 1).contiguous()
        rcnt = torch.empty_like(cnt)
        dist.all_to_all_single(rcnt, cnt, group=group)       # [world, 2] from every rank
        recv_n, recv_b = rcnt[:, 0], rcnt[:, 1]
        sn, rn = send_n.tolist(), recv_n.tolist()
        rmeta = torch.empty(int(sum(rn)), 2, dtype=torch.int64, device=dev)
        dist.all_to_all_single(rmeta, meta.contiguous(), rn, sn, group=group)
        rpay = torch.empty(int(recv_b.sum()), dtype=torch.uint8, device=dev)
        dist.all_to_all_single(rpay, payload.contiguous(), recv_b.tolist(), send_b.tolist(), group=group)
    rlen = rmeta[:, 0]
    roff = torch.cumsum(rlen, 0) - rlen
    if rpay.numel() >= (1 << 32) - ARENA_PAD:
        raise ValueError("received frames exceed the 4 GiB a uint32 descriptor offset addresses")
    # the ABI's over-read contract (include/fastclick_gpu.h): the arena stays
    # readable 128 B past every frame start and 16 B past every frame end
    arena_recv = torch.zeros(rpay.numel() + ARENA_PAD, dtype=torch.uint8, device=dev)
    arena_recv[:rpay.numel()] = rpay
    # offsets/lengths are uint32 bit patterns in an int32 tensor (DeviceBatch layout)
    desc_recv = torch.stack([roff, rlen], 1).to(torch.int64)
    desc_recv = torch.where(desc_recv >= (1 << 31), desc_recv - (1 << 32), desc_recv).to(torch.int32)
    return arena_recv, desc_recv, rmeta[:, 1]


def _gather_frames(arena, off, ln, chunk_bytes=1 << 24):
    """Frames [off[k], off[k] + ln[k]) of arena, back to back. Gathers in
    chunks of whole frames of about chunk_bytes, so the int64 byte index
    never exceeds ~8 x chunk_bytes of temporary memory."""
    import torch
    total = int(ln.sum()) if ln.numel() else 0
    out = torch.empty(total, dtype=torch.uint8, device=arena.device)
    if total == 0:
        return out
    ends = torch.cumsum(ln, 0)
    starts = ends - ln
    bounds = [0]
    if total > chunk_bytes:
        cut = torch.searchsorted(ends, torch.arange(chunk_bytes, total, chunk_bytes, device=ln.device))
        bounds += sorted(set(int(c) + 1 for c in cut.tolist()))
    if bounds[-1] != ln.numel():
        bounds.append(ln.numel())
    for a, b in zip(bounds[:-1], bounds[1:]):
        if b <= a:
            continue
        o, l, s0 = off[a:b], ln[a:b], int(starts[a])
        m = int(l.sum())
        pos = torch.arange(m, device=arena.device) - torch.repeat_interleave(starts[a:b] - s0, l)
        out[s0:s0 + m] = arena[torch.repeat_interleave(o, l) + pos]
    return out
