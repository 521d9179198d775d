"""One element thread-count point (for rocprofv3 traces of the host path):
python scripts/element_threads.py THREADS [BATCH [ZEROCOPY]] -> one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from fastclick_amd import synth, click as K  # noqa: E402

t = int(sys.argv[1]) if len(sys.argv) > 1 else 8
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
zc = len(sys.argv) > 3 and sys.argv[3].lower() in ("1", "true", "zc")
b = synth.c2(1 << 16)
conf = f"GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash, BATCH {batch}, ZEROCOPY {str(zc).lower()})"
mpps = K.bench_element(conf, b, burst=32, reps=40, threads=t) / 1e6
print(json.dumps({"threads": t, "batch": batch, "zerocopy": zc, "mpps": round(mpps, 1),
                  "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default")}), flush=True)
