"""TEST INFRASTRUCTURE ONLY: numpy restatement of the flow re-shard's send
buffer and records (fcgpu_exchange_plan / _pack / _unpack, include/fastclick_gpu.h),
the checker of fastclick_amd/csrc/fcgpu_exchange.hh.

FastClick has no cross-device exchange: each core owns the flows the NIC's
RSS hash sends it (VirtualFlowManagerIMP::process,
include/click/flow/virtualflowmanager.hh:249-330). The GPU path re-shards
packets by their owner rank instead, so the format here is this repository's
own specification; what ties it to the reference is the property the tests
check on top of it: every valid packet reaches the rank its flow hash names
exactly once, with its bytes and length, in source order -- the per-core
flow tables then see whole flows, as under RSS.

Only tests/ use this module.
"""
from __future__ import annotations

import numpy as np


def partition(owner, world):
    """perm / port_start as the device's whole-batch partition gives them
    (CLASSIFY_EACH_PACKET order, include/click/packetbatch.hh:259-307): owner
    d in [0, world) is output d, anything else the invalid list (output
    world). port_start has world + 2 entries."""
    owner = np.asarray(owner, dtype=np.int64)
    port = np.where((owner >= 0) & (owner < world), owner, world)
    perm = np.argsort(port, kind="stable").astype(np.uint32)
    counts = np.bincount(port, minlength=world + 1)
    port_start = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint32)
    return perm, port_start


SLOT_ALIGN = 16     # every frame's slot: its length rounded up to 16 B (fcgpu_exchange.hh xslot)


def _slot(ln):
    return (ln.astype(np.uint64) + (SLOT_ALIGN - 1)) & ~np.uint64(SLOT_ALIGN - 1)


def _owner_of(ps, m):
    return np.searchsorted(ps.astype(np.int64), np.arange(m), side="right") - 1


def plan(desc, perm, port_start, world, rank):
    """-> (meta uint32 [m, 4] = off, length, src_index, src_rank; seg_bytes uint64 [world])."""
    desc = np.asarray(desc, dtype=np.uint32).reshape(-1, 2)
    n = len(perm)
    m = int(min(int(port_start[world]), n))
    idx = np.asarray(perm[:m], dtype=np.int64)
    ln = desc[idx, 1].astype(np.uint64)
    slot = _slot(ln)
    at = np.cumsum(slot) - slot
    total = slot.sum(dtype=np.uint64)
    ps = np.minimum(np.asarray(port_start[:world + 1], dtype=np.int64), m)
    base = np.append(at, total)[ps] if m else np.zeros(world + 1, dtype=np.uint64)
    owner = _owner_of(ps, m)
    meta = np.zeros((m, 4), dtype=np.uint32)
    if m:
        meta[:, 0] = (at - base[owner]).astype(np.uint32)
        meta[:, 1] = ln.astype(np.uint32)
        meta[:, 2] = idx.astype(np.uint32)
        meta[:, 3] = rank
    return meta, np.diff(base).astype(np.uint64)


def pack(arena, desc, meta, port_start, seg_bytes, world):
    """The send buffer: owner d's segment at sum(seg_bytes[:d]), each frame in
    its 16-B slot, slot bytes past the frame zero."""
    arena = np.asarray(arena, dtype=np.uint8)
    desc = np.asarray(desc, dtype=np.uint32).reshape(-1, 2)
    m = len(meta)
    send = np.zeros(int(np.sum(seg_bytes, dtype=np.uint64)), dtype=np.uint8)
    if m == 0:
        return send
    segbase = np.concatenate([[0], np.cumsum(seg_bytes, dtype=np.uint64)])[:-1].astype(np.int64)
    ps = np.minimum(np.asarray(port_start[:world + 1], dtype=np.int64), m)
    dst = segbase[_owner_of(ps, m)] + meta[:, 0].astype(np.int64)
    src = desc[meta[:, 2].astype(np.int64), 0].astype(np.int64)
    ln = meta[:, 1].astype(np.int64)
    rep = np.repeat(np.arange(m), ln)
    k = np.arange(len(rep)) - np.repeat(np.cumsum(ln) - ln, ln)
    send[dst[rep] + k] = arena[src[rep] + k]
    return send


def unpack(meta, src_displ):
    """Received records -> (offset, length) descriptors into the received buffer."""
    meta = np.asarray(meta, dtype=np.uint32).reshape(-1, 4)
    displ = np.asarray(src_displ, dtype=np.uint64)
    ok = meta[:, 3] < len(displ)
    d = np.zeros((len(meta), 2), dtype=np.uint32)
    r = np.where(ok, meta[:, 3], 0).astype(np.int64)
    d[:, 0] = np.where(ok, displ[r] + meta[:, 0].astype(np.uint64), 0).astype(np.uint32)
    d[:, 1] = np.where(ok, meta[:, 1], 0)
    return d


def all_to_all(parts, world):
    """What each receiver gets from an all-to-all of the ranks' (send, meta,
    port_start, seg_bytes): per receiver r, (buffer, meta, src_displ) with the
    sources' segments for r concatenated in source-rank order."""
    out = []
    for r in range(world):
        bufs, metas, displ, at = [], [], [], 0
        for send, meta, port_start, seg_bytes in parts:
            m = len(meta)
            ps = np.minimum(np.asarray(port_start[:world + 1], dtype=np.int64), m)
            sb = np.concatenate([[0], np.cumsum(seg_bytes, dtype=np.uint64)]).astype(np.int64)
            bufs.append(send[sb[r]:sb[r + 1]])
            metas.append(meta[ps[r]:ps[r + 1]])
            displ.append(at)
            at += int(sb[r + 1] - sb[r])
        out.append((np.concatenate(bufs) if bufs else np.zeros(0, np.uint8),
                    np.concatenate(metas) if metas else np.zeros((0, 4), np.uint32), displ))
    return out
