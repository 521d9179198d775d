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


# ---- the fixed-capacity layout (fcgpu_exchange_build_fixed / _unpack_fixed) ----

def build_fixed(arena, desc, owner, world, rank, seg_recs, seg_bytes):
    """The fixed-capacity send side from each packet's owner (owner[i] >= world:
    stays): (meta uint32 [world * (seg_recs + 1), 4], send uint8 [world *
    seg_bytes], defined uint8 mask of send's written bytes, defined_meta bool
    [world * (seg_recs + 1)]). Owner d's segment: its header (packets, bytes
    low, bytes high, overflow) at row d (seg_recs + 1), then its records in
    input order (offset within the segment, length, source index, source
    rank), its frames from byte d seg_bytes in 16-B slots (slot bytes past the
    frame zero). An owner with more than seg_recs packets or seg_bytes slot
    bytes gets its header alone, overflow 1. Unwritten rows and bytes are not
    part of the format (the mask)."""
    arena = np.asarray(arena, dtype=np.uint8)
    desc = np.asarray(desc, dtype=np.uint32).reshape(-1, 2)
    owner = np.asarray(owner, dtype=np.int64)
    rows = seg_recs + 1
    meta = np.zeros((world * rows, 4), dtype=np.uint32)
    dm = np.zeros(world * rows, dtype=bool)
    send = np.zeros(world * seg_bytes, dtype=np.uint8)
    defined = np.zeros(world * seg_bytes, dtype=bool)
    for d in range(world):
        idx = np.nonzero(owner == d)[0]
        ln = desc[idx, 1].astype(np.uint64)
        slot = _slot(ln)
        total = int(slot.sum(dtype=np.uint64))
        over = len(idx) > seg_recs or total > seg_bytes
        meta[d * rows] = (len(idx), total & 0xFFFFFFFF, total >> 32, 1 if over else 0)
        dm[d * rows] = True
        if over or not len(idx):
            continue
        at = (np.cumsum(slot) - slot).astype(np.int64)
        r0 = d * rows + 1
        meta[r0:r0 + len(idx), 0] = at.astype(np.uint32)
        meta[r0:r0 + len(idx), 1] = ln.astype(np.uint32)
        meta[r0:r0 + len(idx), 2] = idx.astype(np.uint32)
        meta[r0:r0 + len(idx), 3] = rank
        dm[r0:r0 + len(idx)] = True
        for k, i in enumerate(idx):
            o, L, s = d * seg_bytes + int(at[k]), int(ln[k]), int(slot[k])
            send[o:o + L] = arena[int(desc[i, 0]):int(desc[i, 0]) + L]
            defined[o:o + s] = True
    return meta, send, defined, dm


def all_to_all_fixed(parts, world, seg_recs, seg_bytes):
    """Equal-split all-to-all of the ranks' (meta, send): receiver r gets every
    source s's segment r at position s."""
    rows = seg_recs + 1
    out = []
    for r in range(world):
        out.append((np.concatenate([m[r * rows:(r + 1) * rows] for m, _ in parts]),
                    np.concatenate([b[r * seg_bytes:(r + 1) * seg_bytes] for _, b in parts])))
    return out


def unpack_fixed(rmeta, world, seg_recs, seg_bytes, stall, step):
    """The receive side: (desc uint32 [count, 2], count, stall) -- descriptors
    in (source rank, source order) into the received frames (source s at s
    seg_bytes); count 0 and stall = step (if it was 0) when a segment
    overflowed or stall was already set."""
    rmeta = np.asarray(rmeta, dtype=np.uint32).reshape(-1, 4)
    rows = seg_recs + 1
    hdr = rmeta[::rows][:world]
    nbytes = hdr[:, 1].astype(np.uint64) | (hdr[:, 2].astype(np.uint64) << np.uint64(32))
    bad = (hdr[:, 3] & 1).astype(bool) | (hdr[:, 0] > seg_recs) | (nbytes > seg_bytes)
    if bad.any() or stall:
        return np.zeros((0, 2), np.uint32), 0, (stall or step)
    out = []
    for s in range(world):
        recs = rmeta[s * rows + 1:s * rows + 1 + int(hdr[s, 0])]
        d = np.zeros((len(recs), 2), np.uint32)
        d[:, 0] = (s * seg_bytes + recs[:, 0].astype(np.int64)).astype(np.uint32)
        d[:, 1] = recs[:, 1]
        out.append(d)
    desc = np.concatenate(out) if out else np.zeros((0, 2), np.uint32)
    return desc, len(desc), stall
