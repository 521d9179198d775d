"""Device cost of the flow re-shard's pack and unpack (fcgpu_exchange_*,
DESIGN section 6): a 1M-packet batch already classified to 8 owner ranks
(C4: 60-B frames in 64-B slots, uniform 5-tuples; C3: IMIX 64/570/1500 B), the
plan (3 kernels), the pack and the unpack timed with HIP events on the launch
stream, median of --reps. Prints one JSON line per workload with the per-kernel
times, Mpps and the algorithmic HBM bytes per packet:

  plan    perm 4 + desc 8 (twice: block sums, records) + record 16 + arena
          offset 4 written = 40 B
  pack    record 16 + arena offset 4 + frame L read + slot (L+3)&~3 written
  unpack  record 16 read + descriptor 8 written = 24 B
  build   (fcgpu_exchange_build, from the owner pass's verdicts) verdict 2 +
          descriptor 8 read twice (per-tile sums, then records and frames),
          record 16 written, frame L read + slot written

python scripts/exchange_rate.py [--reps 50]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fastclick_amd import _native as N, synth  # noqa: E402
from fastclick_amd.device import DeviceBatch, DeviceOutputs, run_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--world", type=int, default=8)
    a = ap.parse_args()
    world, n = a.world, 1 << 20
    for name, b in (("c4", synth.c4(n, seed=41)), ("c3", synth.c3(n, seed=42))):
        cfg = N.make_cfg(offset=14, checksum=True, hash_mode=N.HASH_FLOWID, classify=N.CLS_LB_HASH, nports=world)
        ctx = N.Context(0, n, cfg)
        db = DeviceBatch.upload(b, device="cuda:0")
        outs = DeviceOutputs(n, world, device="cuda:0", perm=True, port_start=True, partition=N.PART_GLOBAL)
        run_device(ctx, db, outs)
        meta = torch.empty((n, 4), dtype=torch.int32, device="cuda:0")
        seg = torch.empty(world, dtype=torch.int64, device="cuda:0")
        s = torch.cuda.current_stream().cuda_stream
        args = (db.desc.data_ptr(), outs.perm.data_ptr(), outs.port_start.data_ptr(), n, world, 0,
                meta.data_ptr(), seg.data_ptr())
        ctx.exchange_plan(*args, stream=s)
        total = int(seg.sum())
        m = int(outs.port_start[world])
        frame_bytes = int(db.desc[outs.perm[:m].long(), 1].long().sum())
        send = torch.empty(total, dtype=torch.uint8, device="cuda:0")
        rdesc = torch.empty((m, 2), dtype=torch.int32, device="cuda:0")
        displ = [0] * world
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        t = {"plan": [], "pack": [], "unpack": []}
        for r in range(a.reps + 3):
            ev[0].record()
            ctx.exchange_plan(*args, stream=s)
            ev[1].record()
            ctx.exchange_pack(db.arena.data_ptr(), outs.port_start.data_ptr(), meta.data_ptr(),
                              seg.data_ptr(), n, world, send.data_ptr(), total, stream=s)
            ev[2].record()
            ctx.exchange_unpack(meta.data_ptr(), m, displ, rdesc.data_ptr(), stream=s)
            ev[3].record()
            torch.cuda.synchronize()
            if r >= 3:
                for k, key in enumerate(("plan", "pack", "unpack")):
                    t[key].append(ev[k].elapsed_time(ev[k + 1]) * 1e3)
        med = {k: statistics.median(v) for k, v in t.items()}
        byt = {"plan": 40 * m, "pack": 20 * m + frame_bytes + total, "unpack": 24 * m}
        out = {"workload": name, "packets": n, "sent": m, "world": world, "frame_bytes": frame_bytes,
               "send_bytes": total, "us": {k: round(v, 2) for k, v in med.items()},
               "mpps": round(m / sum(med.values()), 1),
               "gbs": {k: round(byt[k] / med[k] / 1e3, 1) for k in med},
               "bytes_per_packet": {k: round(byt[k] / m, 1) for k in byt}}
        print(json.dumps(out), flush=True)
        # the one-pass send side from the verdicts (fcgpu_exchange_build)
        vouts = DeviceOutputs(n, world, device="cuda:0", verdict=True, hash=False)
        run_device(ctx, db, vouts)
        cap = int(db.arena.numel()) + 16 * n
        bmeta = torch.empty((n, 4), dtype=torch.int32, device="cuda:0")
        bsn = torch.empty(world, dtype=torch.int32, device="cuda:0")
        bsb = torch.empty(world, dtype=torch.int64, device="cuda:0")
        bsend = torch.empty(cap, dtype=torch.uint8, device="cuda:0")
        tb, tv = [], []
        for r in range(a.reps + 3):
            ev[0].record()
            run_device(ctx, db, vouts)
            ev[1].record()
            ctx.exchange_build(db.arena.data_ptr(), db.desc.data_ptr(), vouts.verdict.data_ptr(), n, world, 0,
                               bmeta.data_ptr(), bsn.data_ptr(), bsb.data_ptr(), bsend.data_ptr(), cap, stream=s)
            ev[2].record()
            torch.cuda.synchronize()
            if r >= 3:
                tv.append(ev[0].elapsed_time(ev[1]) * 1e3)
                tb.append(ev[1].elapsed_time(ev[2]) * 1e3)
        assert torch.equal(bsb.cpu(), seg.cpu()) and torch.equal(bmeta[:m].cpu(), meta[:m].cpu())
        assert torch.equal(bsend[:total].cpu(), send[:total].cpu())
        mb = statistics.median(tb)
        byt = 10 * n + 10 * n + 16 * m + frame_bytes + total     # verdict+desc twice, records, frames in and out
        print(json.dumps({"workload": name, "path": "build", "packets": n, "sent": m, "world": world,
                          "us": {"owner_pass_verdicts": round(statistics.median(tv), 2), "build": round(mb, 2)},
                          "build_gbs": round(byt / mb / 1e3, 1), "build_bytes_per_packet": round(byt / m, 1),
                          "mpps_build": round(m / mb, 1)}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
