"""The element's BATCH on one crossover chain (scripts/crossover.py chains):
python scripts/element_batch_sweep.py CHAIN THREADS B1,B2,... -> one JSON line
per batch size (2-s pushed Mpps, the crossover's method). Tuning aid."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from fastclick_amd import click as K  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from crossover import chains  # noqa: E402

name, threads, sizes = sys.argv[1], int(sys.argv[2]), sys.argv[3].split(",")
c = chains()[name]
b = c["batch"]()
for bs in sizes:
    conf = c["gpu"][:-1] + f", BATCH {bs})"
    mpps = K.bench_element(conf, b, burst=32, threads=threads, seconds=2.0) / 1e6
    print(json.dumps({"chain": name, "threads": threads, "batch": bs, "mpps": round(mpps, 1)}), flush=True)
