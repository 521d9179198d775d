"""Shared test helpers: batch variants and result comparison."""
from __future__ import annotations

import numpy as np

from fastclick_amd import synth
from fastclick_amd import _native as N


def repack(batch: synth.Batch, *, misalign_seed=None, gap=0) -> synth.Batch:
    """Copy frames into a fresh arena, optionally at randomly misaligned offsets
    (0..15 bytes past a 64-B boundary) to exercise the window-shift path."""
    rng = np.random.default_rng(misalign_seed) if misalign_seed is not None else None
    frames = batch.frames()
    offs, pos = [], 0
    for f in frames:
        pos = (pos + 63) & ~63
        if rng is not None:
            pos += int(rng.integers(0, 16))
        offs.append(pos)
        pos += max(len(f), 1) + gap
    arena = np.zeros(pos + synth.ARENA_PAD, np.uint8)
    for o, f in zip(offs, frames):
        arena[o:o + len(f)] = np.frombuffer(f, np.uint8)
    desc = np.stack([np.array(offs, np.uint32), batch.desc[:, 1].astype(np.uint32)], axis=1)
    return synth.Batch(arena=arena, desc=np.ascontiguousarray(desc), meta=dict(batch.meta))


def set_fragment(batch: synth.Batch, frac: float, seed=11, ip_off=14):
    """Mark ~frac of packets as non-first fragments (fragment offset != 0) with
    a consistent checksum."""
    rng = np.random.default_rng(seed)
    sel = np.nonzero(rng.random(batch.n) < frac)[0]
    A = batch.arena
    for i in sel:
        o = int(batch.desc[i, 0]) + ip_off
        fo = int(rng.integers(1, 0x1FFF))
        A[o + 6], A[o + 7] = (fo >> 8) & 0x1F, fo & 0xFF
        synth._refresh_cksum(A, o)
    return sel


def compare(got: dict, exp: dict, *, keys=("reason", "port", "hash"), anno=True, perm=True,
            ctx=""):
    for k in keys:
        g, e = got[k], exp[k]
        if not np.array_equal(g, e):
            bad = np.nonzero(g != e)[0]
            raise AssertionError(f"{ctx}: {k} mismatch at {len(bad)} packets, first {bad[:8]}: "
                                 f"got {g[bad[:8]]} expected {e[bad[:8]]}")
    if anno and "anno" in got:
        ok = exp["reason"] == N.R_OK
        for f in ("dst_ip", "length", "nh", "th", "vlan_tci", "ip6_nxt"):
            g, e = got["anno"][f][ok], exp["anno"][f][ok]
            if not np.array_equal(g, e):
                bad = np.nonzero(g != e)[0]
                raise AssertionError(f"{ctx}: anno.{f} mismatch at {len(bad)} valid packets")
    if perm and "perm" in got:
        assert np.array_equal(got["port_start"], exp["port_start"]), f"{ctx}: port_start"
        assert np.array_equal(got["perm"], exp["perm"]), f"{ctx}: perm"
    if perm and "tile_perm" in got:
        local = (exp["perm_tile"] % 256).astype(np.uint8)
        assert np.array_equal(got["tile_perm"], local), f"{ctx}: tile_perm"
    if perm and "perm_tile" in got:
        assert np.array_equal(got["tile_count"], exp["tile_count"]), f"{ctx}: tile_count"
        assert np.array_equal(got["perm_tile"], exp["perm_tile"]), f"{ctx}: perm_tile"
