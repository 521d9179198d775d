"""Device-resident batches and one-call helpers over the C ABI.

torch provides the device memory and the stream (plumbing only); every packet
byte is processed by the HIP kernels in libfcgpu.so.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _native as N


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("no HIP device visible to torch")
    return torch


@dataclass
class DeviceBatch:
    arena: "object"      # torch.uint8 cuda tensor
    desc: "object"       # torch.int32 cuda tensor [n, 2] (uint32 bit pattern)
    n: int

    @classmethod
    def upload(cls, batch, device="cuda"):
        torch = _torch()
        arena = torch.from_numpy(np.ascontiguousarray(batch.arena)).to(device)
        desc = torch.from_numpy(np.ascontiguousarray(batch.desc).view(np.int32)).to(device)
        return cls(arena=arena, desc=desc, n=batch.n)


class DeviceOutputs:
    def __init__(self, n, nports, device="cuda", *, verdict=True, hash=True, anno=False,
                 perm=False, port_start=False, partition=N.PART_GLOBAL, tile_perm=False, flowid=False,
                 ip_rw=False):
        torch = _torch()
        self.n = n
        self.nports = nports
        self.partition = partition
        mk = lambda k, dt: torch.empty(k, dtype=dt, device=device)  # noqa: E731
        self.verdict = mk(n, torch.int16) if verdict else None
        self.hash = mk(n, torch.int32) if hash else None
        self.flowid = mk(n, torch.int32) if flowid else None
        self.ip_rw = mk(n, torch.int32) if ip_rw else None
        self.anno = mk(n * 16, torch.uint8) if anno else None
        tile = partition == N.PART_TILE
        self.perm = mk(n, torch.int32) if perm else None
        self.tile_perm = mk(n, torch.uint8) if (tile and (tile_perm or perm)) else None
        self.port_start = mk(nports + 2, torch.int32) if port_start and not tile else None
        ntiles = (n + N.TILE - 1) // N.TILE
        self.tile_count = mk(ntiles * (nports + 1), torch.int16) if (perm or tile_perm) and tile else None

    def ptrs(self):
        p = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
        return dict(verdict=p(self.verdict), hash=p(self.hash), anno=p(self.anno),
                    perm=p(self.perm), port_start=p(self.port_start),
                    tile_count=p(self.tile_count), partition=self.partition,
                    tile_perm=p(self.tile_perm), flowid=p(self.flowid), ip_rw=p(self.ip_rw))

    def numpy(self):
        out = {}
        if self.verdict is not None:
            v = self.verdict.cpu().numpy().view(np.uint16)
            out["verdict"] = v
            out["reason"] = (v & 0xFF).astype(np.uint8)
            out["port"] = (v >> 8).astype(np.uint8)
        if self.hash is not None:
            out["hash"] = self.hash.cpu().numpy().view(np.uint32)
        if self.ip_rw is not None:
            out["ip_rw"] = self.ip_rw.cpu().numpy().view(np.uint32)
        if self.flowid is not None:
            out["flowid"] = self.flowid.cpu().numpy().view(np.uint32)
        if self.anno is not None:
            out["anno"] = self.anno.cpu().numpy().view(N.anno_dtype())
        if self.perm is not None:
            key = "perm_tile" if self.partition == N.PART_TILE else "perm"
            out[key] = self.perm.cpu().numpy().view(np.uint32)
        if self.tile_count is not None:
            out["tile_count"] = self.tile_count.cpu().numpy().view(np.uint16)
        if self.tile_perm is not None:
            out["tile_perm"] = self.tile_perm.cpu().numpy()
        if self.port_start is not None:
            out["port_start"] = self.port_start.cpu().numpy().view(np.uint32)
        return out


def run_device(ctx: N.Context, dbatch: DeviceBatch, outs: DeviceOutputs, stream=None):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    ctx.process(dbatch.arena.data_ptr(), dbatch.desc.data_ptr(), dbatch.n,
                stream=s.cuda_stream, **outs.ptrs())


def process_batch(batch, cfg, *, anno=True, perm=True, device_index=0, partition=N.PART_GLOBAL,
                  program=None, program_jit=False, lb_table=None):
    """One batch on a fresh context (see process_batches)."""
    return process_batches([batch], cfg, anno=anno, perm=perm, device_index=device_index,
                           partition=partition, program=program, program_jit=program_jit,
                           lb_table=lb_table)[0]


def process_batches(batches, cfg, *, anno=True, perm=True, device_index=0, partition=N.PART_GLOBAL,
                    program=None, max_flows=0, program_jit=False, lb_table=None):
    """Upload host Batches, run the device path over them in order on one
    context, return per-batch numpy results and the running counter vector.
    Convenience for tests and smoke(). program: optional (kind, steps,
    output_everything) for CLS_PROGRAM (fcgpu_set_program), compiled to code
    with program_jit (fcgpu_program_jit); max_flows > 0 enables the flow table
    (its state carries across the batches); lb_table: the CLS_LB_TABLE table
    (fcgpu_set_lb_table)."""
    torch = _torch()
    res = []
    with torch.cuda.device(device_index):
        ctx = N.Context(device_index, max(max(b.n for b in batches), 1), cfg)
        try:
            if program is not None:
                ctx.set_program(*program)
                if program_jit:
                    ctx.program_jit(True)
            if lb_table is not None:
                ctx.set_lb_table(lb_table)
            if max_flows:
                ctx.flow_enable(max_flows)
            for batch in batches:
                db = DeviceBatch.upload(batch, device=f"cuda:{device_index}")
                outs = DeviceOutputs(batch.n, cfg.nports, device=f"cuda:{device_index}",
                                     anno=anno, perm=perm, port_start=perm, partition=partition,
                                     flowid=max_flows > 0, ip_rw=cfg.rewrite != 0)
                run_device(ctx, db, outs)
                torch.cuda.synchronize()
                r = outs.numpy()
                r["counters"] = np.array(ctx.counters(), dtype=np.uint64)
                if max_flows:
                    r["flow_count"] = ctx.flow_count()
                res.append(r)
        finally:
            ctx.close()
    return res


def exchange_pack(ctx: N.Context, arena, desc, perm, port_start, world, rank, stream=None):
    """The send side of the flow re-shard (fcgpu_exchange_plan + _pack, HIP):
    perm / port_start from a device pass with LB_MODE hash over `world`
    outputs and the whole-batch partition. Returns (send, meta, seg_n,
    seg_bytes): the send buffer (followed by ARENA_PAD zero bytes, so at world
    1 it is the received arena as is), the int32 [m, 4] fcgpu_xmeta records of
    the m leaving packets in owner order, and per owner its packet and byte
    counts (host lists: the all-to-all's split sizes). One host sync, for
    those counts."""
    torch = _torch()
    from .dist import ARENA_PAD
    n = int(desc.shape[0])
    dev = desc.device
    s = stream if stream is not None else torch.cuda.current_stream()
    meta = torch.empty((max(n, 1), 4), dtype=torch.int32, device=dev)
    seg = torch.empty(world, dtype=torch.int64, device=dev)
    ctx.exchange_plan(desc.data_ptr(), perm.data_ptr(), port_start.data_ptr(), n, world, rank,
                      meta.data_ptr(), seg.data_ptr(), stream=s.cuda_stream)
    with torch.cuda.stream(s):
        host = torch.cat([port_start[:world + 1].to(torch.int64), seg]).cpu()
    ps = host[:world + 1].tolist()
    seg_bytes = host[world + 1:].tolist()
    m = min(ps[world], n)
    seg_n = [min(ps[d + 1], m) - min(ps[d], m) for d in range(world)]
    if max(seg_bytes, default=0) > 0xFFFFFFFF:
        # a record's offset within its owner's segment is 32 bits
        # (fcgpu_xmeta.off): the pack refuses such a segment
        raise ValueError(f"exchange_pack: an owner's segment of {max(seg_bytes)} B exceeds the 4 GiB "
                         "a record offset addresses; split the batch")
    total = int(sum(seg_bytes))
    send = torch.empty(total + ARENA_PAD, dtype=torch.uint8, device=dev)
    with torch.cuda.stream(s):
        send[total:].zero_()
    ctx.exchange_pack(arena.data_ptr(), port_start.data_ptr(), meta.data_ptr(), seg.data_ptr(),
                      n, world, send.data_ptr(), total, stream=s.cuda_stream)
    return send, meta[:m], seg_n, seg_bytes


def exchange_build(ctx: N.Context, arena, desc, verdict, world, rank, send_cap=None, stream=None):
    """The send side in one call (fcgpu_exchange_build, HIP) from the owner
    pass's verdicts (LB_MODE hash over `world` outputs, FCGPU_OUT_VERDICT
    only). Returns (send, meta, seg_n, seg_bytes) as device tensors: the send
    buffer (send_cap bytes + ARENA_PAD), the int32 [n, 4] record buffer (its
    first sum(seg_n) rows are the records, in owner order), per owner its
    packet count (int32) and byte count (int64). No host sync: send_cap
    defaults to the arena's bytes + 16 per packet, which holds every leaving
    frame's slot unless descriptors alias; the caller reads seg_bytes (one
    sync it needs anyway for the all-to-all) and dist.exchange_segments
    checks the total against the buffer."""
    torch = _torch()
    from .dist import ARENA_PAD
    n = int(desc.shape[0])
    dev = desc.device
    s = stream if stream is not None else torch.cuda.current_stream()
    if send_cap is None:
        send_cap = int(arena.numel()) + 16 * n
    meta = torch.empty((max(n, 1), 4), dtype=torch.int32, device=dev)
    seg_n = torch.empty(world, dtype=torch.int32, device=dev)
    seg_b = torch.empty(world, dtype=torch.int64, device=dev)
    send = torch.empty(int(send_cap) + ARENA_PAD, dtype=torch.uint8, device=dev)
    ctx.exchange_build(arena.data_ptr(), desc.data_ptr(), verdict.data_ptr(), n, world, rank, meta.data_ptr(),
                       seg_n.data_ptr(), seg_b.data_ptr(), send.data_ptr(), int(send_cap), stream=s.cuda_stream)
    return send, meta, seg_n, seg_b


def exchange_unpack(ctx: N.Context, meta, src_displ, stream=None):
    """The receive side (fcgpu_exchange_unpack, HIP): records -> int32 [k, 2]
    descriptors (uint32 bit patterns) into the received buffer, whose source r
    segment starts at src_displ[r]."""
    torch = _torch()
    k = int(meta.shape[0])
    s = stream if stream is not None else torch.cuda.current_stream()
    desc = torch.empty((max(k, 1), 2), dtype=torch.int32, device=meta.device)
    ctx.exchange_unpack(meta.data_ptr() if k else 0, k, src_displ, desc.data_ptr(), stream=s.cuda_stream)
    return desc[:k]


# ---- the fixed-capacity re-shard (no host sync per step) -------------------

def fixed_capacity(n: int, send_cap: int, world: int, slack: float = 1.25):
    """Per-owner capacities of the fixed-capacity exchange (fcgpu_exchange_build_fixed):
    a uniform owner's share of the batch's n packets and send_cap slot bytes
    (the arena's bytes + 16 per packet bound them) times `slack`, plus a floor
    (256 packets, 64 KiB), never more than the whole batch. World 1: the
    whole batch, so a segment cannot overflow. Returns (seg_recs, seg_bytes)."""
    if world <= 1:
        return max(n, 1), (max(send_cap, 16) + 15) // 16 * 16
    recs = min(max(n, 1), int(n / world * slack) + 256)
    nbytes = min(max(send_cap, 16), int(send_cap / world * slack) + (64 << 10))
    return recs, (nbytes + 15) // 16 * 16


def exchange_build_fixed(ctx: N.Context, arena, desc, verdict, world, rank, seg_recs, seg_bytes, meta, send,
                         stream=None):
    """fcgpu_exchange_build_fixed into preallocated device buffers: meta int32
    [world * (seg_recs + 1), 4] (each owner's header + records), send uint8
    [world * seg_bytes + ARENA_PAD]. No host sync."""
    torch = _torch()
    n = int(desc.shape[0])
    s = stream if stream is not None else torch.cuda.current_stream()
    ctx.exchange_build_fixed(arena.data_ptr(), desc.data_ptr(), verdict.data_ptr(), n, world, rank, seg_recs,
                             seg_bytes, meta.data_ptr(), send.data_ptr(), stream=s.cuda_stream)


def exchange_unpack_fixed(ctx: N.Context, rmeta, world, seg_recs, seg_bytes, desc, count, stall, step,
                          total=None, stream=None):
    """fcgpu_exchange_unpack_fixed: the received segments -> desc int32 [world *
    seg_recs, 2] (the first *count rows), count / stall int32 [1] device words;
    total (int64 [1], optional) += count."""
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    ctx.exchange_unpack_fixed(rmeta.data_ptr(), world, seg_recs, seg_bytes, desc.data_ptr(), count.data_ptr(),
                              stall.data_ptr(), step, total=total.data_ptr() if total is not None else 0,
                              stream=s.cuda_stream)
