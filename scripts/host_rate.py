"""Host-resident (PCIe-inclusive) rates, for DESIGN.md.

1. fcgpu_process_host on a 1M-packet C2 batch: gather first min(len,128) B of
   every frame into pinned staging, H2D, kernels, D2H of verdict/hash/perm.
2. The GPUIPCheckClassify element behind a BURST-32 source (Click-shaped
   packets, linked-list batches, annotation scatter, per-port relinking) at
   several BATCH (accumulation) sizes.
Prints one JSON line. `host_rate.py threads`: the element's thread sweep;
`host_rate.py span`: a host-resident ring through fcgpu_span_submit, copies
vs zero-copy (span_mpps).
"""
import ctypes as C
import json
import struct
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from fastclick_amd import synth, click as K, _native as N  # noqa: E402


def raw_host(n, threads=1, tile=False, pinned=False):
    b = synth.c2(n)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    ctx = N.Context(0, n, cfg)
    ctx.set_host_threads(threads)
    base = b.arena.ctypes.data
    ptrs = (C.c_void_p * n)(*[base + int(o) for o in b.desc[:, 0]])
    lens = np.ascontiguousarray(b.desc[:, 1], dtype=np.uint32)
    lib = N.load()

    def arr(count, dtype):
        dtype = np.dtype(dtype)
        if not pinned:
            return np.zeros(count, dtype)
        p = lib.fcgpu_host_alloc(count * dtype.itemsize)
        return np.ctypeslib.as_array((C.c_uint8 * (count * dtype.itemsize)).from_address(p)).view(dtype)
    v = arr(n, np.uint16); h = arr(n, np.uint32)
    if tile:
        tp = arr(n, np.uint8); tc = arr(((n + 255) // 256) * 17, np.uint16)
        kw = dict(verdict=v.ctypes.data, hash=h.ctypes.data, tile_perm=tp.ctypes.data,
                  tile_count=tc.ctypes.data, partition=N.PART_TILE)
    else:
        p = np.zeros(n, np.uint32); st = np.zeros(18, np.uint32)
        kw = dict(verdict=v.ctypes.data, hash=h.ctypes.data, perm=p.ctypes.data, port_start=st.ctypes.data)
    ctx.process_host(ptrs, lens.ctypes.data, n, **kw)
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.process_host(ptrs, lens.ctypes.data, n, **kw)
    dt = time.perf_counter() - t0
    ctx.close()
    return n * reps / dt / 1e6


def h2d_gbs(nbytes=72 << 20, reps=20):
    """Pinned host -> device copy rate on this box (the PCIe bound of the path)."""
    src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t0) / 1e9


def gather_only_mpps(n=1 << 20, reps=10):
    """The host gather alone (numpy fancy-index copy of 64-B windows), for scale."""
    b = synth.c2(n)
    idx = (b.desc[:, 0].astype(np.int64)[:, None] + np.arange(64)[None, :])
    out = np.empty((n, 64), np.uint8)
    t0 = time.perf_counter()
    for _ in range(reps):
        np.take(b.arena, idx, out=out)
    return n * reps / (time.perf_counter() - t0) / 1e6


def pcap_mpps(n=1 << 22, chunk_pkts=1 << 18, threads=1, mapped=False):
    """pcap ingress (fcpcap + fcgpu_span_submit): a C2 trace written as a pcap
    (16-B record header + 60-B frame per packet), read from the page cache
    into pinned chunks and copied as-is; verdict + hash come back. The file is
    read once untimed so it is in the page cache."""
    import tempfile
    from fastclick_amd.pcap import process_pcap
    b = synth.c2(1 << 16)
    fr = b.frame(0)
    rec = np.frombuffer(struct.pack("<IIII", 0, 0, len(fr), len(fr)) + fr, np.uint8)
    body = np.tile(rec, n)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    with tempfile.NamedTemporaryFile(suffix=".pcap", dir="/tmp") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        f.write(body.tobytes())
        f.flush()
        process_pcap(f.name, cfg, chunk_pkts=chunk_pkts, chunk_bytes=chunk_pkts * 80 + 4096, collect=False)
        best = 0.0
        for _ in range(3):
            out, cnt, secs = process_pcap(f.name, cfg, chunk_pkts=chunk_pkts, chunk_bytes=chunk_pkts * 80 + 4096,
                                          collect=False, threads=threads, mapped=mapped)
            reg = out["registered"]
            assert cnt == n and int(out["counters"][N.CTR_COUNT]) == n
            best = max(best, cnt / secs / 1e6)
    return best if not mapped else (best, reg)


def span_mpps(n=1 << 20, mode="copy", slots=3, reps=24):
    """A host-resident ring: n C2 frames already contiguous in pinned memory
    (64-B slots) and their descriptors, submitted with fcgpu_span_submit over
    `slots` slots (a stream each) with no per-packet host work -- the
    end-to-end host-resident rate of SURVEY 8(d): H2D of descriptors +
    headers, the kernels and the D2H of verdict, hash and tile partition,
    overlapped across streams (mode "copy"), or the kernels reading the span
    and writing the outputs in place over PCIe (mode "zerocopy"). Every
    submission's counters are checked at the end."""
    lib = N.load()
    b = synth.c2(n)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    ctx = N.Context(0, n, cfg)
    ptrs = []

    def pinned(nbytes, dtype):
        p = lib.fcgpu_host_alloc(nbytes)
        assert p
        ptrs.append(p)
        return p, np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(nbytes,)).view(dtype)
    try:
        ps, span = pinned(b.arena.size + 4096, np.uint8)
        span[:b.arena.size] = b.arena
        pd, desc = pinned(8 * n, np.uint32)
        desc[:] = np.ascontiguousarray(b.desc, dtype=np.uint32).reshape(-1)
        outs = []
        for _ in range(slots):
            pv, _ = pinned(2 * n, np.uint16)
            ph, _ = pinned(4 * n, np.uint32)
            ptc, _ = pinned(2 * 17 * (n // 256 + 1), np.uint16)
            ptp, _ = pinned(n + 256, np.uint8)
            outs.append(dict(verdict=pv, hash=ph, tile_count=ptc, tile_perm=ptp, partition=N.PART_TILE))
        assert lib.fcgpu_span_mode(ctx.h, N.SPAN_ZEROCOPY if mode == "zerocopy" else N.SPAN_COPY) == N.OK
        ctx.reset_counters()

        def run(k):
            for r in range(k):
                s = r % slots
                if r >= slots:
                    ctx.span_wait(s)
                ctx.span_submit(s, ps, b.arena.size, pd, n, **outs[s])
            for s in range(min(k, slots)):
                ctx.span_wait(s)
        run(slots)                      # warm-up: allocations, first launches
        t0 = time.perf_counter()
        run(reps)
        dt = time.perf_counter() - t0
        assert int(ctx.counters()[N.CTR_COUNT]) == n * (reps + slots)
        return n * reps / dt / 1e6
    finally:
        for p in ptrs:
            lib.fcgpu_host_free(p)
        ctx.close()


def span_sweep():
    """span_mpps for both modes at 1M / 256K / 64K packets per submission: one JSON line."""
    out = {}
    for n in (1 << 20, 1 << 18, 1 << 16):
        for mode in ("copy", "zerocopy"):
            out[f"span_{mode}_{n}"] = round(span_mpps(n, mode, reps=max(24, (24 << 20) // n)), 1)
            print(json.dumps(out), file=sys.stderr, flush=True)
    print(json.dumps(out))


def mbuf_mpps(n=1 << 18, reps=48, order="shuffled", streams=1):
    """mbuf ingress (fcgpu_process_mbufs): n C2 frames in a DPDK-style
    mempool in page-locked host memory (128-B header, 128-B headroom,
    2048-B data room per element); each call hands the device the array of n
    mbuf pointers, the GPU builds descriptors from the mbuf headers and reads
    the header windows over PCIe (zero copy); outputs stay on the device."""
    import mmap
    from tests.test_mbuf import make_pool
    from fastclick_amd.device import DeviceOutputs
    rng = np.random.default_rng(1)
    frames = synth.c2(n).frames()
    buf, arr, base, size, ptrs = make_pool(frames, rng)
    if order == "sequential":
        ptrs = np.sort(ptrs)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    # one context per rx queue (stream): the pool is registered by the first
    ctxs = [N.Context(0, n, cfg) for _ in range(streams)]
    try:
        for c in ctxs:            # the first registers the pool, the others share it
            c.pool_register(base, size)
        ss = [torch.cuda.Stream() for _ in range(streams)]
        outs = [DeviceOutputs(n, 16, device="cuda", perm=True, partition=N.PART_TILE) for _ in range(streams)]
        for k in range(streams):
            ctxs[k].process_mbufs(ptrs.ctypes.data, n, stream=ss[k].cuda_stream, **outs[k].ptrs())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for r in range(reps):
            k = r % streams
            ctxs[k].process_mbufs(ptrs.ctypes.data, n, stream=ss[k].cuda_stream, **outs[k].ptrs())
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        tot = sum(int(c.counters()[N.CTR_COUNT]) for c in ctxs)
        assert tot == n * (reps + streams), tot
    finally:
        for c in ctxs:
            c.close()
    return n * reps / dt / 1e6


def main():
    out = {"h2d_pinned_gbs": round(h2d_gbs(), 2),
           "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default (4)")}
    for t in (1, 4):
        out[f"pcap_ingress_mpps_4M_t{t}"] = round(pcap_mpps(threads=t), 2)
    m, reg = pcap_mpps(mapped=True)
    out["pcap_ingress_mpps_4M_mapped"] = round(m, 2)
    out["pcap_mapped_registered"] = bool(reg)
    out["mbuf_ingress_mpps_256k_shuffled"] = round(mbuf_mpps(), 2)
    out["mbuf_ingress_mpps_256k_sequential"] = round(mbuf_mpps(order="sequential"), 2)
    out["mbuf_ingress_mpps_256k_shuffled_2streams"] = round(mbuf_mpps(streams=2), 2)
    out["mbuf_ingress_mpps_256k_shuffled_4streams"] = round(mbuf_mpps(streams=4), 2)
    out["process_host_mpps_1M_global"] = round(raw_host(1 << 20), 2)
    # fcgpu_process_host's pipeline chunk (kChunk in fcgpu_internal.hh, overridable)
    out["chunk"] = int(os.environ.get("FCGPU_HOST_CHUNK", "131072"))
    for threads in (1, 4, 8):
        out[f"process_host_mpps_1M_tile_t{threads}"] = round(raw_host(1 << 20, threads, tile=True), 2)
        out[f"process_host_mpps_1M_tile_t{threads}_pinned"] = round(
            raw_host(1 << 20, threads, tile=True, pinned=True), 2)
    # the element behind a BURST-32 source: a 64K-packet C2 trace replayed
    # through a mempool-sized packet pool (fcclick_bench), single flow as the
    # C2-chain CPU baseline
    b = synth.c2(1 << 16)
    base = "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash, BATCH {})"
    # the harness floor (source + sinks, no element work)
    out["harness_floor_mpps"] = round(K.bench_element("Pass", b, burst=32, reps=40) / 1e6, 2)
    for batch in (4096, 8192, 16384, 32768, 65536):
        out[f"element_mpps_batch{batch}"] = round(K.bench_element(base.format(batch), b, burst=32, reps=40) / 1e6, 2)
    for t in (2, 4, 8):
        out[f"element_mpps_batch16384_threads{t}"] = round(
            K.bench_element(base.format(16384), b, burst=32, reps=40, threads=t) / 1e6, 2)
    out["element_mpps_batch16384_per_packet_push"] = round(
        K.bench_element(base.format(16384), b, burst=K.PER_PACKET, reps=20) / 1e6, 2)
    print(json.dumps(out))


def thread_sweep():
    """The element's host-side scaling: BATCH x threads (one element instance
    and GPU context per thread, all timed loops started together, aggregate =
    all packets over the union of the windows), beside the harness floor (a
    pass-through element) at the same thread counts. One JSON line."""
    b = synth.c2(1 << 16)
    base = "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash, BATCH {})"
    out = {"gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default (4)"),
           "affinity": len(os.sched_getaffinity(0))}
    for t in (1, 2, 4, 8, 12, 16):
        out[f"floor_t{t}"] = round(K.bench_element("Pass", b, burst=32, reps=40, threads=t) / 1e6, 1)
    for batch in (4096, 8192, 16384):
        for t in (1, 2, 4, 8, 12, 16):
            out[f"el_b{batch}_t{t}"] = round(
                K.bench_element(base.format(batch), b, burst=32, reps=40, threads=t) / 1e6, 1)
            print(json.dumps({k: v for k, v in out.items() if k.startswith(f"el_b{batch}")}), file=sys.stderr,
                  flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "threads":
        thread_sweep()
    elif len(sys.argv) > 1 and sys.argv[1] == "span":
        span_sweep()
    elif len(sys.argv) > 1 and sys.argv[1] == "pcap":
        out = {}
        for rep in range(2):
            for t in (1, 4):
                out[f"pcap_copy_t{t}_{rep}"] = round(pcap_mpps(threads=t), 1)
            out[f"pcap_mapped_{rep}"] = round(pcap_mpps(mapped=True)[0], 1)
            print(json.dumps(out), file=sys.stderr, flush=True)
        print(json.dumps(out))
    else:
        main()
