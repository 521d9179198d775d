"""Where an element thread's time goes (A/B build only): FCCLICK_LIB points at
a harness build instrumented with rdtsc (scripts/mock/cyc), this runs the
element at THREADS threads and prints the cycles per packet spent staging
and submitting, waiting for the device, and completing (annotation + output
runs + the downstream sinks). python scripts/el_cycles.py THREADS [BATCH]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from fastclick_amd import synth, click as K  # noqa: E402

t = int(sys.argv[1]) if len(sys.argv) > 1 else 16
batch = sys.argv[2] if len(sys.argv) > 2 else "auto"
b = synth.c2(1 << 16)
conf = f"GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash, BATCH {batch})"
lib = K.load()
mpps = K.bench_element(conf, b, burst=32, reps=40, threads=t) / 1e6
print(json.dumps({"threads": t, "batch": batch, "mpps": round(mpps, 1)}), flush=True)
lib.fcclick_print_cycles()
if os.environ.get("FCGPU_LIB"):
    from fastclick_amd import _native as N
    N.load().fcgpu_print_cycles()
