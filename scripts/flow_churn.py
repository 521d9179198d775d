"""New-flow churn through the device flow table.

A 1M-packet C4 batch (independent uniform 5-tuples, checksum off so source
addresses can be rewritten in place) teaches the table its 1M flows; then, for
each churn level k, the source address of k random packets is replaced on the
device by a fresh random value before each call, so the batch carries exactly
k packets of flows the table has never seen (k misses). Per level: the whole
call (k_rx + the new-flow pass, device events around it) and k_rx alone
(the context's own launch events), averaged over `--reps` calls, and a check
that the table grew by the number of distinct new flows.

    python scripts/flow_churn.py [--reps 5]  -> one JSON line
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--levels", default="0,100,1000,10000,100000,1048576")
    args = ap.parse_args()
    import torch
    from fastclick_amd import synth, _native as N
    from fastclick_amd.device import DeviceBatch, DeviceOutputs

    dev = "cuda:0"
    n = 1 << 20
    host = synth.c4(n, seed=7)
    b = DeviceBatch.upload(host, device=dev)
    off = torch.from_numpy(host.desc[:, 0].astype("int64")).to(dev)   # frame offsets
    del host
    cfg = N.make_cfg(offset=14, checksum=False, hash_mode=N.HASH_FLOWID, classify=N.CLS_LB_HASH, nports=16)
    ctx = N.Context(0, n, cfg)
    ctx.flow_enable(1 << 23)
    o = DeviceOutputs(n, 16, device=dev, verdict=True, hash=True, anno=False, perm=False, tile_perm=True,
                      port_start=True, partition=N.PART_TILE, flowid=True)
    optr = o.ptrs()
    stream = torch.cuda.current_stream()
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)

    def call():
        ctx.process(b.arena.data_ptr(), b.desc.data_ptr(), n, stream=stream.cuda_stream, **optr)

    call()
    call()                                  # the base flows are known now
    torch.cuda.synchronize()
    out = {"packets": n, "reps": args.reps}
    for k in [int(x) for x in args.levels.split(",")]:
        tot, grown = 0.0, 0
        ctx.read_timing()
        for _ in range(args.reps):
            if k:
                idx = torch.randperm(n, generator=gen, device=dev)[:k]
                addr = off[idx] + 14 + 12
                val = torch.randint(0, 256, (k, 4), generator=gen, device=dev, dtype=torch.uint8)
                for j in range(4):
                    b.arena[addr + j] = val[:, j]
            before = ctx.flow_count()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ctx.set_timing(True)
            e0.record(stream)
            call()
            e1.record(stream)
            ctx.set_timing(False)
            torch.cuda.synchronize()
            tot += e0.elapsed_time(e1)
            grown += ctx.flow_count() - before
        ms, cnt = ctx.read_timing()
        out[f"k{k}_call_us"] = round(tot / args.reps * 1e3, 2)
        out[f"k{k}_k_rx_us"] = round(ms[0] / max(cnt[0], 1) * 1e3, 2)
        out[f"k{k}_new_flows"] = grown
        assert grown <= k * args.reps and (k == 0) == (grown == 0), (k, grown)
        print(f"k={k}: call {out[f'k{k}_call_us']} us, k_rx {out[f'k{k}_k_rx_us']} us, "
              f"{grown} new flows", file=sys.stderr, flush=True)
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
