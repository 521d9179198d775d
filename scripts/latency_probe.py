"""Fixed cost of a timed region: t0 -> one small fcgpu_process_jobs launch ->
device synchronize -> t1, with HIP's default wait and with spin-wait
(hipSetDeviceFlags(hipDeviceScheduleSpin) before the device is initialised).
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
for n in (256, 1 << 20):
    b = DeviceBatch.upload(synth.c2(n), device="cuda:0")
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    ctx = N.Context(0, n, cfg)
    o = DeviceOutputs(n, 16, device="cuda:0", perm=False, tile_perm=True, partition=N.PART_TILE)
    s = torch.cuda.Stream()
    jobs = ctx.jobs([(b.arena.data_ptr(), b.desc.data_ptr(), n, s.cuda_stream, o.ptrs())])
    for _ in range(20):
        ctx.run_jobs(jobs)
    torch.cuda.synchronize()
    ts = []
    for _ in range(200):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.run_jobs(jobs)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    res[f"region_us_n{n}"] = round(statistics.median(ts), 2)
    ctx.close()
print(json.dumps(res))
