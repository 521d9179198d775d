"""profiles/pmc_traffic.json from one session's rocprofv3 PMC passes of k_rx
(one 1M-packet C2 batch per launch): FETCH_SIZE (x2, the gfx950 half-count of
MI355X_MICROARCH.md's HBM section), WRITE_SIZE, TCC_EA0_RDREQ. Labelled with
the hash of the kernel sources it was measured on (bench.py reports the
figure as roofline.traffic only while the sources still hash the same).

    python scripts/pmc_traffic.py SESSION_DIR   (holds pmc_fetch/, pmc_write/, pmc_ea/)
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def per_dispatch(path, counter):
    vals = collections.defaultdict(float)
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        if r["Counter_Name"] == counter and "k_rx" in r["Kernel_Name"]:
            vals[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    ds = sorted(vals)[4:]          # the warmup launches out
    return sum(vals[d] for d in ds) / len(ds), len(ds)


def main(sess):
    fetch, nd = per_dispatch(os.path.join(sess, "pmc_fetch"), "FETCH_SIZE")
    write, _ = per_dispatch(os.path.join(sess, "pmc_write"), "WRITE_SIZE")
    rdreq, _ = per_dispatch(os.path.join(sess, "pmc_ea"), "TCC_EA0_RDREQ_sum")
    pk = 1 << 20
    out = {
        "packets": pk, "workload": "c2", "frame_bytes": 64, "kernel": "k_rx",
        "source_sha16": bench.kernel_source_sha(),
        "fetch_size_kb": round(fetch, 1),
        "hbm_read_bytes_per_launch": int(fetch * 1024 * 2),
        "ea_rdreq_per_launch": int(rdreq),
        "ea_rdreq_x128_bytes": int(rdreq * 128),
        "write_size_kb": round(write, 1),
        "hbm_write_bytes_per_launch": int(write * 1024),
        "hbm_bytes_per_launch": int(fetch * 1024 * 2),
        "algorithmic_read_bytes_per_launch": bench.PKT_BYTES_READ * pk,
        "correction": "read bytes = FETCH_SIZE(KB)*1024*2 (gfx950 half-count, MI355X_MICROARCH.md HBM)",
        "source": f"{os.path.relpath(sess, ROOT)}/pmc_fetch, pmc_write, pmc_ea (rocprofv3 --pmc, one pass each, "
                  f"{nd} k_rx dispatches of one 1M-packet C2 batch after 4 warmup launches, mean per dispatch)",
    }
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
