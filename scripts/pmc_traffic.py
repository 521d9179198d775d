"""profiles/pmc_traffic.json from rocprofv3 PMC passes of k_rx, one entry per
workload variant (bench.traffic_key: workload, frame size, layout, batch size
and every option that changes what k_rx reads or writes).

Each variant's three passes (one batch per launch, --fuse 1 --streams 1) are
FETCH_SIZE (x2: the gfx950 half-count of MI355X_MICROARCH.md's HBM section),
WRITE_SIZE and TCC_EA0_RDREQ, in <session>/pmc_fetch_<tag>/, pmc_write_<tag>/,
pmc_ea_<tag>/ (scripts/session.sh `pmcv`). Every entry is labelled with the
hash of the kernel sources it was measured on: bench.py reports it as
roofline.traffic only while the sources still hash the same. Entries of other
variants already in the file are kept.

    python scripts/pmc_traffic.py SESSION_DIR TAG="bench args" [TAG="bench args" ...]
"""
import collections
import csv
import json
import os
import shlex
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

OUT = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def per_dispatch(path, counter):
    if not os.path.isdir(path):      # scripts/session.sh writes rocprofv3 output under prof_<step>/
        path = os.path.join(os.path.dirname(path), "prof_" + os.path.basename(path))
    vals = collections.defaultdict(float)
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        if r["Counter_Name"] == counter and "k_rx" in r["Kernel_Name"]:
            vals[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    ds = sorted(vals)[4:]          # the warmup launches out
    return sum(vals[d] for d in ds) / len(ds), len(ds)


def entry(sess, tag, argv):
    args = bench.parse(shlex.split(argv))
    pk = args.packets
    fetch, nd = per_dispatch(os.path.join(sess, f"pmc_fetch_{tag}"), "FETCH_SIZE")
    write, _ = per_dispatch(os.path.join(sess, f"pmc_write_{tag}"), "WRITE_SIZE")
    rdreq, _ = per_dispatch(os.path.join(sess, f"pmc_ea_{tag}"), "TCC_EA0_RDREQ_sum")
    alg = bench.PKT_BYTES_READ * pk
    rd = int(fetch * 1024 * 2)
    return bench.traffic_key(args, pk), {
        "bench_args": argv, "packets": pk, "workload": args.workload, "frame_bytes": args.frame_bytes,
        "layout": args.layout, "kernel": "k_rx", "source_sha16": bench.kernel_source_sha(),
        "fetch_size_kb": round(fetch, 1),
        "hbm_read_bytes_per_launch": rd,
        "ea_rdreq_per_launch": int(rdreq),
        "ea_rdreq_x128_bytes": int(rdreq * 128),
        "write_size_kb": round(write, 1),
        "hbm_write_bytes_per_launch": int(write * 1024),
        "hbm_bytes_per_launch": rd,
        "algorithmic_read_bytes_per_launch": alg,
        "read_over_algorithmic": round(rd / alg, 4),
        "read_bytes_per_packet": round(rd / pk, 2),
        "correction": "read bytes = FETCH_SIZE(KB)*1024*2 (gfx950 half-count, MI355X_MICROARCH.md HBM)",
        "source": f"{os.path.relpath(sess, ROOT)}/prof_pmc_fetch_{tag}, prof_pmc_write_{tag}, prof_pmc_ea_{tag} "
                  f"(rocprofv3 --pmc, one pass each, {nd} k_rx dispatches of one {pk}-packet batch after "
                  f"4 warmup launches, mean per dispatch)",
    }


def main(sess, pairs):
    try:
        with open(OUT) as f:
            doc = json.load(f)
    except Exception:
        doc = {}
    entries = doc.get("entries", {}) if doc.get("format") == 2 else {}
    for p in pairs:
        tag, argv = p.split("=", 1)
        key, e = entry(sess, tag, argv)
        entries[key] = e
        print(key, json.dumps(e))
    doc = {"format": 2, "note": "one entry per bench.traffic_key; bench.py reads the entry of its own "
                                "variant while source_sha16 matches the kernel sources",
           "entries": dict(sorted(entries.items()))}
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
