"""Per-dispatch timeline of the last K k_rx launches in a rocprofv3 kernel
trace (run_kernel_trace.csv): start offset, duration, queue, and the gaps --
how a short timed region spends its time."""
import csv
import sys

path = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = [r for r in csv.DictReader(open(path)) if "k_rx" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-k:]
t0 = int(rows[0]["Start_Timestamp"])
durs = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    durs.append((e - s) / 1e3)
    print(f"start {(s - t0) / 1e3:8.2f} us  dur {(e - s) / 1e3:6.2f} us  queue {r['Queue_Id']}")
span = (int(rows[-1]["End_Timestamp"]) - t0) / 1e3
print(f"span {span:.2f} us for {len(rows)} launches = {span / len(rows):.2f} us/launch; "
      f"mean dur {sum(durs) / len(durs):.2f} us; first 5 mean {sum(durs[:5]) / 5:.2f}, last 5 mean {sum(durs[-5:]) / 5:.2f}")
