"""The wire-layout configs' own ceiling:
for C2, C3 and C5 (1M packets, the bench's wire layout), the bare
header-window gather of exactly those descriptors (scripts/kgather: k_rx's
own loads -- descriptors + 64-B windows by LDS-DMA -- and nothing else, and
the same with k_rx's per-packet stores) against k_rx in bench.py (200
steps, the same rotation), all on one box. Prints one JSON line per workload
with both times and "k_rx / bare gather".

python scripts/gather_bound.py [--workloads c2,c3,c5]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    from fastclick_amd import synth
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c2,c3,c5")
    ap.add_argument("--n", type=int, default=1 << 20)
    a = ap.parse_args()
    out = os.path.join(ROOT, "gpurun_out", "gather_bound")
    os.makedirs(out, exist_ok=True)
    gen = {"c2": synth.c2, "c3": synth.c3, "c5": synth.c5}
    for w in a.workloads.split(","):
        b = gen[w](a.n)
        path = os.path.join(out, f"desc_{w}.bin")
        np.ascontiguousarray(b.desc, dtype=np.uint32).tofile(path)
        r = subprocess.run([os.path.join(ROOT, "scripts", "kgather"), path, str(b.n), str(b.arena.nbytes), "20"],
                           capture_output=True, text=True, timeout=120)
        if r.returncode:
            raise SystemExit(r.stdout + r.stderr)
        g = {x["variant"]: x for x in (json.loads(line) for line in r.stdout.splitlines() if line.startswith("{"))}
        rb = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", w, "--steps", "200",
                             "--warmup", "20", "--no-cpu"], capture_output=True, text=True, timeout=300)
        if rb.returncode:
            raise SystemExit(rb.stderr[-2000:])
        line = json.loads([x for x in rb.stdout.splitlines() if x.startswith("{")][-1])
        k = line["roofline"]["kernel_ms"] * 1e3
        bare, bare_out = g["gather"]["us_per_batch"], g["gather+outputs"]["us_per_batch"]
        more = {k: g[k]["us_per_batch"] for k in ("gather+packed", "gather+vh", "gather+tperm") if k in g}
        print(json.dumps({"workload": w, "packets": b.n, "arena_bytes": int(b.arena.nbytes),
                          "k_rx_us": round(k, 2), "bare_gather_us": bare, "gather_plus_outputs_us": bare_out,
                          "k_rx_over_bare_gather": round(k / bare, 3),
                          "k_rx_over_gather_plus_outputs": round(k / bare_out, 3),
                          "k_rx_roofline_frac": line["roofline"]["frac"], "nbuf_gather": g["gather"]["nbuf"],
                          "store_variants_us": more,
                          "bench_hbm_batches": line["config"].get("hbm_batches")}), flush=True)


if __name__ == "__main__":
    main()
