"""Fixed cost of a timed region: t0 -> one fcgpu_process_jobs launch -> wait
-> t1, for a 256-packet batch and for the bench's fused launch (20 rotating
1M-packet C2 batches), waiting with torch.cuda.synchronize (HIP's default
wait), or polling the stream (hipStreamQuery) first, or (idleN) after the
GPU sat idle N us; with --spin the process
sets hipSetDeviceFlags(hipDeviceScheduleSpin) before the device is
initialised. Reports the medians of the region, of the host enqueue (t0 ->
return of the launch call) and of the device time of the launch (events).
Prints one JSON line."""
import ctypes as C
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
spin = "--spin" in sys.argv
if spin:
    hip = C.CDLL("libamdhip64.so")
    assert hip.hipSetDeviceFlags(1) == 0      # hipDeviceScheduleSpin
import torch  # noqa: E402
from fastclick_amd import synth, _native as N  # noqa: E402
from fastclick_amd.device import DeviceBatch, DeviceOutputs  # noqa: E402

res = {"spin": spin}
cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
for n, nb in ((256, 1), (1 << 20, 20)):
    b = DeviceBatch.upload(synth.c2(n), device="cuda:0")
    bufs = [(b.arena, b.desc)] + [(b.arena.clone(), b.desc.clone()) for _ in range(min(nb, 16) - 1)]
    ctx = N.Context(0, n, cfg)
    outs = [DeviceOutputs(n, 16, device="cuda:0", perm=False, tile_perm=True, partition=N.PART_TILE)
            for _ in range(nb)]
    s = torch.cuda.Stream()
    jobs = ctx.jobs([(bufs[k % len(bufs)][0].data_ptr(), bufs[k % len(bufs)][1].data_ptr(), n, s.cuda_stream,
                      outs[k].ptrs()) for k in range(nb)])
    for _ in range(10):
        ctx.run_jobs(jobs)
    torch.cuda.synchronize()
    modes = ["sync", "poll"] + ([f"idle{g}" for g in (100, 1000, 10000)] if nb > 1 else [])
    for mode in modes:
        reg, enq, dev = [], [], []
        gap = int(mode[4:]) * 1e-6 if mode.startswith("idle") else 0
        for _ in range(100 if not gap else 30):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            if gap:   # the GPU idle for `gap` before the region (host busy-waits)
                tg = time.perf_counter() + gap
                while time.perf_counter() < tg:
                    pass
            t0 = time.perf_counter()
            e0.record(s)
            ctx.run_jobs(jobs)
            e1.record(s)
            t1 = time.perf_counter()
            if mode == "poll":
                while not s.query():
                    pass
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            reg.append((t2 - t0) * 1e6)
            enq.append((t1 - t0) * 1e6)
            dev.append(e0.elapsed_time(e1) * 1e3)
        key = f"n{n}x{nb}_{mode}"
        res[key] = {"region_us": round(statistics.median(reg), 2), "enqueue_us": round(statistics.median(enq), 2),
                    "device_us": round(statistics.median(dev), 2),
                    "region_min_us": round(min(reg), 2),
                    "region_p90_us": round(sorted(reg)[int(0.9 * len(reg))], 2)}
    ctx.close()
print(json.dumps(res))
