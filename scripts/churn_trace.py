"""Summarise a rocprofv3 kernel trace of scripts/flow_churn.py: per churn level
(misses per batch), the average device time of k_rx and of each new-flow
kernel. Usage: python scripts/churn_trace.py <run_kernel_trace.csv> [reps]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    levels = [0, 100, 1000, 10000, 100000, 1048576]
    rows = [r for r in csv.DictReader(open(path)) if "k_rx" in r["Kernel_Name"] or "k_flow" in r["Kernel_Name"]]
    calls = []
    for r in rows:
        name = "k_rx" if "k_rx" in r["Kernel_Name"] else r["Kernel_Name"].split("(")[0].split("::")[-1]
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        if name == "k_rx":
            calls.append({})
        calls[-1][name] = calls[-1].get(name, 0.0) + us
    calls = calls[2:]                      # the two calls that teach the base flows
    out = {}
    for li, k in enumerate(levels):
        acc = defaultdict(float)
        for c in calls[li * reps:(li + 1) * reps]:
            for n, v in c.items():
                acc[n] += v
        out[k] = {n: round(v / reps, 1) for n, v in acc.items()}
        fin = sum(v for n, v in out[k].items() if n != "k_rx")
        print(f"misses {k:>8}: k_rx {out[k].get('k_rx', 0):7.1f} us, new-flow pass {fin:7.1f} us  {out[k]}")


if __name__ == "__main__":
    main()
