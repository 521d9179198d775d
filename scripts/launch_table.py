"""k_rx launches of a rocprofv3 kernel trace (run_kernel_trace.csv) with the
batches each carried (fused launches, fcgpu_process_jobs): batches = grid
workgroups / the workgroups of one batch. Prints every launch and the
per-batch time, which is what bench.py's roofline.kernel_ms reports.

usage: launch_table.py run_kernel_trace.csv [packets_per_batch]"""
import csv
import sys

path = sys.argv[1]
packets = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
wg_per_batch = (packets + 255) // 256
rows = [r for r in csv.DictReader(open(path)) if "k_rx" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
gcol = next(k for k in rows[0] if k.startswith("Grid_Size") and k.endswith("X")) if rows else None
tot_us, tot_b = 0.0, 0
for r in rows:
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    wgs = int(r[gcol]) // 256
    b = max(1, wgs // wg_per_batch)
    tot_us += dur
    tot_b += b
    print(f"launch dur {dur:9.2f} us  workgroups {wgs:7d}  batches {b:3d}  per batch {dur / b:7.2f} us")
if rows:
    print(f"{len(rows)} launches, {tot_b} batches: {tot_us / len(rows):.2f} us per launch on average, "
          f"{tot_us / tot_b:.2f} us per batch")
