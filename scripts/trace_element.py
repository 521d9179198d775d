"""Where a batch of the element's host path spends its time, from one
rocprofv3 --hip-trace --kernel-trace --memory-copy-trace run of
scripts/element_threads.py (prints one JSON line of medians / p90s, us):

  submit->start  host API call return -> the op starting on the GPU (queueing)
  op duration    H2D copy, k_rx, D2H copy
  gaps           H2D end -> k_rx start, k_rx end -> D2H start (cross-engine hand-off)
  round trip     H2D call -> D2H end
  wait           hipStreamSynchronize durations (thread blocked on its batch)
  think          a thread's time between its API calls (its own CPU work)

    python scripts/trace_element.py TRACE_DIR
"""
import collections
import csv
import json
import os
import statistics as st
import sys


def q(v, p):
    v = sorted(v)
    return round(v[min(len(v) - 1, int(p * len(v)))], 1) if v else None


def main(d):
    api = list(csv.DictReader(open(os.path.join(d, "run_hip_api_trace.csv"))))
    cps = list(csv.DictReader(open(os.path.join(d, "run_memory_copy_trace.csv"))))
    kts = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    ops = {}
    for r in cps:
        ops[int(r["Correlation_Id"])] = ("H2D" if "HOST_TO" in r["Direction"] else "D2H",
                                         int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    for r in kts:
        if "k_rx" in r["Kernel_Name"]:
            ops[int(r["Correlation_Id"])] = ("K", int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    sub = collections.defaultdict(list)
    wait, think = [], []
    per_thread = collections.defaultdict(list)
    for r in api:
        c, s, e = int(r["Correlation_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        per_thread[int(r["Thread_Id"])].append((s, e, r["Function"]))
        if c in ops:
            kind, os_, oe = ops[c]
            sub[kind].append((os_ - e) / 1e3)
        if r["Function"] == "hipStreamSynchronize":
            wait.append((e - s) / 1e3)
    for calls in per_thread.values():
        calls.sort()
        for a, b in zip(calls, calls[1:]):
            if b[0] > a[1]:
                think.append((b[0] - a[1]) / 1e3)
    # per stream, consecutive ops: the H2D -> K -> D2H chain of each batch
    by_stream = collections.defaultdict(list)
    for r in cps:
        by_stream[int(r["Stream_Id"])].append(ops[int(r["Correlation_Id"])])
    for r in kts:
        if "k_rx" in r["Kernel_Name"]:
            by_stream[int(r["Stream_Id"])].append(ops[int(r["Correlation_Id"])])
    gap_hk, gap_kd, rt = [], [], []
    for lst in by_stream.values():
        lst.sort(key=lambda x: x[1])
        for a, b, c in zip(lst, lst[1:], lst[2:]):
            if a[0] == "H2D" and b[0] == "K" and c[0] == "D2H":
                gap_hk.append((b[1] - a[2]) / 1e3)
                gap_kd.append((c[1] - b[2]) / 1e3)
                rt.append((c[2] - a[1]) / 1e3)
    dur = collections.defaultdict(list)
    for kind, s, e in ops.values():
        dur[kind].append((e - s) / 1e3)
    out = {
        "threads": len(per_thread),
        "submit_to_start_us": {k: {"med": q(v, .5), "p90": q(v, .9)} for k, v in sub.items()},
        "op_us": {k: {"med": q(v, .5), "p90": q(v, .9), "n": len(v)} for k, v in dur.items()},
        "gap_h2d_to_k_us": {"med": q(gap_hk, .5), "p90": q(gap_hk, .9)},
        "gap_k_to_d2h_us": {"med": q(gap_kd, .5), "p90": q(gap_kd, .9)},
        "gpu_round_trip_us": {"med": q(rt, .5), "p90": q(rt, .9)},
        "sync_wait_us": {"med": q(wait, .5), "p90": q(wait, .9), "mean": round(st.mean(wait), 1) if wait else None},
        "think_us": {"med": q(think, .5), "p90": q(think, .9)},
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
