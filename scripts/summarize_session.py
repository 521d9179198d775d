"""Summarise a session's bench lines (gpurun_out/*.log) as a table."""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for p in sorted(glob.glob(os.path.join(d, "*.log"))):
    for line in open(p, errors="replace"):
        if line.startswith("{\"metric\""):
            j = json.loads(line)
            r = j.get("roofline") or {}
            c = j["config"]
            print(f"{os.path.basename(p)[:-4]:34s} {j['value']:9.1f} Mpps {j['ms_per_step']*1e3:7.2f} us/step "
                  f"k_rx {r.get('kernel_ms', 0)*1e3:6.2f} us frac {r.get('frac', 0):.3f} ({r.get('basis')}) "
                  f"kfrac {r.get('kernel_frac', 0):.3f} s={c.get('streams')} fb={c.get('frame_bytes')}")
