"""Copy a session's evidence from gpurun_out/ into profiles/<name>/: every
step log, rocprofv3 kernel stats (+ a timeline of the last 20 k_rx launches),
PMC counter summaries per pass (mean per k_rx launch after the first 4), and
a table of the bench lines."""
import collections
import csv
import glob
import os
import shutil
import subprocess
import sys

src = "gpurun_out"
dst = os.path.join("profiles", sys.argv[1])
os.makedirs(dst, exist_ok=True)
for p in glob.glob(os.path.join(src, "*.log")):
    shutil.copy(p, dst)
pmc = []
for d in sorted(glob.glob(os.path.join(src, "prof_*"))):
    name = os.path.basename(d)[5:]
    out = os.path.join(dst, name)
    os.makedirs(out, exist_ok=True)
    for f in ("run_kernel_stats.csv",):
        if os.path.exists(os.path.join(d, f)):
            shutil.copy(os.path.join(d, f), out)
    tr = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(tr):
        with open(os.path.join(out, "timeline.txt"), "w") as fh:
            subprocess.run([sys.executable, "scripts/trace_steps.py", tr, "20"], stdout=fh)
        with open(os.path.join(out, "launches.txt"), "w") as fh:
            subprocess.run([sys.executable, "scripts/launch_table.py", tr], stdout=fh)
    cc = os.path.join(d, "run_counter_collection.csv")
    if os.path.exists(cc):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(cc)):
            if "k_rx" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            v = v[4:] or v
            pmc.append(f"{name:28s} {k:24s} launches={len(v):3d} mean={sum(v) / len(v):14.1f}")
if pmc:
    open(os.path.join(dst, "pmc_summary.txt"), "w").write("\n".join(pmc) + "\n")
with open(os.path.join(dst, "bench_table.txt"), "w") as fh:
    subprocess.run([sys.executable, "scripts/summarize_session.py", src], stdout=fh)
print(open(os.path.join(dst, "bench_table.txt")).read())
if pmc:
    print("\n".join(pmc))
