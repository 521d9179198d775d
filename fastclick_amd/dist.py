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

Backend-agnostic: "nccl" (RCCL over xGMI) on GPUs, "gloo" in CPU tests.
"""
from __future__ import annotations


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [begin, end) packet range of `rank` among `world` shards."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return (n * rank) // world, (n * (rank + 1)) // world


def reduce_counters(replicas, group=None):
    """Sum a [replicas, NCOUNTERS] int64 tensor over replicas, then over ranks.
    Returns the global NCOUNTERS vector (same device as the input)."""
    import torch.distributed as dist
    local = replicas.sum(0) if replicas.dim() == 2 else replicas.clone()
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(local, op=dist.ReduceOp.SUM, group=group)
    return local


def output_offsets(local_counts, group=None):
    """All-gather every rank's per-output counts [nout] and return this rank's
    start offset within each output's global list, plus the global totals."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return torch.zeros_like(local_counts), local_counts.clone()
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    parts = [torch.empty_like(local_counts) for _ in range(world)]
    dist.all_gather(parts, local_counts, group=group)
    stacked = torch.stack(parts)                  # [world, nout]
    before = stacked[:rank].sum(0) if rank else torch.zeros_like(local_counts)
    return before, stacked.sum(0)
