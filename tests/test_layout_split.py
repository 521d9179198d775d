"""The header-split arena (bench.py --layout split, synth.header_split).

A NIC with header/data buffer split (DPDK RTE_ETH_RX_OFFLOAD_BUFFER_SPLIT)
puts each frame's first bytes in one buffer and the rest in another; the
descriptor then points at the header segment with the frame's full length
(what FromDPDKDevice's mbuf wrap hands on, elements/userlevel/
fromdpdkdevice.cc:374-456). With 64-B header segments in a dense ring, two
header windows share every 128-B line, where the wire layout of an IMIX batch
leaves 5/12 of them alone in theirs.

The chain never reads past the header segment for these frames
(synth.header_reach), so every result must be identical to the wire layout's:
the oracle on both layouts (CPU), and the HIP path on the split layout against
the oracle on the wire layout (GPU), for C3 (IMIX) and C5 (VLAN + IPv6).
"""
import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N

from helpers import compare


def cases():
    return [
        ("c3", synth.c3(6000, nflows=300), N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)),
        ("c5", synth.c5(6000), N.make_cfg(check_mode=N.CHECK_AUTO, offset=0, checksum=True,
                                          classify=N.CLS_LB_HASH, nports=16)),
        ("c3-errors", _with_errors(synth.c3(6000, nflows=300)),
         N.make_cfg(offset=14, checksum=True, classify=N.CLS_HASHSWITCH, nports=7, hs_offset=26, hs_length=8)),
    ]


def _with_errors(b):
    synth.inject_errors(b, 0.03, seed=5)
    return b


def test_header_split_layout():
    b = synth.c3(1000, nflows=50)
    s = synth.header_split(b, 64)
    assert s.n == b.n and s.arena.size == 64 * b.n + synth.ARENA_PAD
    assert (s.desc[:, 0] == np.arange(b.n) * 64).all() and (s.desc[:, 1] == b.desc[:, 1]).all()
    for i in range(0, b.n, 97):
        f, h = b.frame(i), bytes(s.arena[64 * i:64 * i + 64])
        assert h[:min(64, len(f))] == f[:64]
    assert int(synth.header_reach(b).max()) == 38
    # a chain that would read past the header segment is refused
    with pytest.raises(ValueError, match="do not fit"):
        synth.header_split(b, 32)


@pytest.mark.parametrize("case", range(3))
def test_oracle_split_equals_wire(oracle, case):
    name, b, cfg = cases()[case]
    s = synth.header_split(b, 64)
    exp = oracle.process_batch(cfg, b)
    got = oracle.process_batch(cfg, s)
    for k in ("reason", "port", "hash", "perm", "port_start", "counters"):
        assert np.array_equal(got[k], exp[k]), f"{name}: {k}"


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(3))
def test_gpu_split_equals_wire_oracle(oracle, case):
    from fastclick_amd import device
    name, b, cfg = cases()[case]
    s = synth.header_split(b, 64)
    exp = oracle.process_batch(cfg, b)
    for part in (N.PART_GLOBAL, N.PART_TILE):
        got = device.process_batch(s, cfg, anno=True, perm=True, partition=part)
        compare(got, exp, ctx=f"{name} split part={part}", anno=True, perm=True)
        assert np.array_equal(got["counters"], exp["counters"]), name


def test_bench_split_option():
    """bench.py --layout split builds the header-split batch and keys its PMC
    traffic apart from the wire layout's."""
    import bench
    a = bench.parse(["--workload", "c3", "--layout", "split", "--packets", "4096"])
    b, valid = bench.make_host_batch(a)
    assert valid == 4096 and b.arena.size == 64 * 4096 + synth.ARENA_PAD
    w = bench.parse(["--workload", "c3", "--packets", "4096"])
    assert bench.traffic_key(a, 4096) == "c3/fb64/split/n4096" != bench.traffic_key(w, 4096)
    f = bench.parse(["--workload", "c4", "--flow-capacity", "2000000", "--classify", "ipclass16"])
    assert bench.traffic_key(f, 1 << 20) == "c4/fb64/wire/n1048576/flow2000000hmp/ipclass16"
