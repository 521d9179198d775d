"""Host-resident crossover: the drop-in element against the CPU chain it
replaces, on the same box, the same thread counts, the same chain and
trace shape (VERDICT r03 "Next" #2).

Per chain, one JSON line per thread count T in --threads:
  cpu   oracle/_build/fc_cpu_baseline -- the scalar restatement of the
        reference elements (32-packet linked-list PacketBatches from a packet
        pool, atomic counters, one pipeline per thread)
  gpu   GPUIPCheckClassify through libfcclick (the same harness packets and
        32-packet source batches, default BATCH / ZEROCOPY / SLOTS), T element
        instances on T threads sharing the GPU

Chains (SURVEY 8(f) rows the element folds in, where the CPU pays more per
packet):
  prog16   C4 (uniform 5-tuples) + IPClassifier with 15 UDP dst-port ranges
           and '-' (the program the reference compiler printed)
  flow20k  C3 (IMIX 64/570/1500 B 7:4:1, 10k flows) + FlowIPManagerHMP
           (CAPACITY 20000) + AggregateHash + FlowSwitch hash x16
  udp      C2 + CheckUDPHeader (valid non-zero checksums: verified)
  base     C2 headline chain (CheckIPHeader + AggregateHash + FlowSwitch x16)

python scripts/crossover.py [--chains a,b] [--threads 1,8,16] [--seconds S]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (one HIP runtime for torch and libfcgpu)

from fastclick_amd import synth, click as K  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_build", "fc_cpu_baseline")


def ipclass16():
    with open(os.path.join(ROOT, "tests", "golden", "reftests.json")) as f:
        progs = {p["case"]: p for p in json.load(f)["programs"]}
    return progs["ipclass16"]["program"]


def chains():
    prog = ipclass16()
    base = "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16"
    return {
        "prog16": dict(cpu=["--flows", "4096", "--trace", "65536", "--program", "@prog"],
                       gpu=base + ", PROGRAM \"" + "|".join(prog.strip().splitlines()) + "\")",
                       batch=lambda: synth.c4(1 << 16, seed=4), prog=prog),
        "flow20k": dict(cpu=["--flows", "10000", "--imix", "--trace", "65536", "--flow-capacity", "20000"],
                        gpu=base + ", LB_MODE hash, FLOW_CAPACITY 20000)",
                        batch=lambda: synth.c3(1 << 16, seed=3)),
        "udp": dict(cpu=["--l4", "udp"], gpu=base + ", LB_MODE hash, L4 UDP)",
                    batch=lambda: synth.set_udp_checksums(synth.c2(1 << 16))),
        "base": dict(cpu=[], gpu=base + ", LB_MODE hash)", batch=lambda: synth.c2(1 << 16)),
    }


def run_cpu(args, threads, seconds, prog):
    cmd = [EXE, "--seconds", str(2 * seconds), "--threads", str(threads)]
    tmp = None
    for a in args:
        if a == "@prog":
            tmp = tempfile.NamedTemporaryFile("w", suffix=".prog", delete=False)
            tmp.write(prog)
            tmp.close()
            a = tmp.name
        cmd.append(a)
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=4 * seconds + 120)
        if out.returncode:
            raise RuntimeError(out.stderr)
        return json.loads(out.stdout.strip().splitlines()[-1])
    finally:
        if tmp:
            os.unlink(tmp.name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", default="prog16,flow20k,udp,base")
    ap.add_argument("--threads", default="1,8,16")
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-gpu", action="store_true")
    a = ap.parse_args()
    ths = [int(t) for t in a.threads.split(",")]
    allc = chains()
    for name in a.chains.split(","):
        c = allc[name]
        if not a.no_cpu:
            for t in ths:
                if t == 1 and len(ths) > 1:
                    continue                 # every multi-thread run reports its 1-thread rate too
                r = run_cpu(c["cpu"], t, a.seconds, c.get("prog"))
                rows = [(1, r["mpps_1core"])] + ([(t, r["mpps"])] if t > 1 else [])
                for tt, v in rows:
                    print(json.dumps({"chain": name, "side": "cpu", "threads": tt, "mpps": round(v, 1),
                                      "sample": r["sample"]}), flush=True)
        if not a.no_gpu:
            b = c["batch"]()
            for t in ths:
                # pushed for --seconds, as the CPU side is; and the fixed-count run of earlier rounds
                mpps = K.bench_element(c["gpu"], b, burst=32, threads=t, seconds=a.seconds) / 1e6
                reps = K.bench_element(c["gpu"], b, burst=32, reps=a.reps, threads=t) / 1e6
                print(json.dumps({"chain": name, "side": "gpu", "threads": t, "mpps": round(mpps, 1),
                                  "mpps_reps": round(reps, 1), "conf": c["gpu"][:160]}), flush=True)


if __name__ == "__main__":
    main()
