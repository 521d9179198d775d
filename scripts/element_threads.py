"""One element thread-count point (for rocprofv3 traces of the host path):
python scripts/element_threads.py THREADS [BATCH [ZEROCOPY [SLOTS]]] -> one JSON line."""
import json
import os
import resource
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from fastclick_amd import synth, click as K  # noqa: E402

t = int(sys.argv[1]) if len(sys.argv) > 1 else 8
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 0      # 0: the element's default (BATCH auto)
zc = {"1": "true", "true": "true", "0": "false", "false": "false"}.get(sys.argv[3].lower(), "auto") \
    if len(sys.argv) > 3 else "auto"
slots = int(sys.argv[4]) if len(sys.argv) > 4 else 2
b = synth.c2(1 << 16)
conf = f"GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash, BATCH {batch or 'auto'}, ZEROCOPY {zc}, SLOTS {slots})"
mpps = K.bench_element(conf, b, burst=32, reps=40, threads=t) / 1e6
# pushed for 2 s (the CPU baseline's method): no thread's tail of a fixed count;
# the process's CPU time over that run (user + sys, all threads: the element's
# and the HIP runtime's) against its wall time
r0, w0 = resource.getrusage(resource.RUSAGE_SELF), time.monotonic()
timed = K.bench_element(conf, b, burst=32, threads=t, seconds=2.0) / 1e6
r1, w1 = resource.getrusage(resource.RUSAGE_SELF), time.monotonic()
cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
with open("/proc/self/status") as f:
    nthreads = int(next(ln.split()[1] for ln in f if ln.startswith("Threads:")))
print(json.dumps({"threads": t, "batch": batch or "auto", "zerocopy": zc, "slots": slots, "mpps": round(mpps, 1),
                  "mpps_timed": round(timed, 1), "cpus_busy": round(cpu / (w1 - w0), 2),
                  "process_threads": nthreads, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default")}),
      flush=True)
