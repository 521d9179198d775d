"""The RCCL path on one GPU: a world-1 "nccl" process group on cuda:0.

bench.py reduces the per-output / per-reason counters with
fastclick_amd.dist.reduce_counters (an all-reduce: FastClick's per-thread
counters summed on read, include/click/sync.hh:384) and gathers the
per-output counts with dist.output_offsets (an all-gather). At world size 1
both skip the collective unless forced; here they are forced, so the same RCCL
calls the 8-GPU run makes are issued, on device tensors, through a real
communicator -- and RCCL's own log (NCCL_DEBUG_SUBSYS=COLL) shows that each
call reached it. The rank runs in a child process (its own communicator, a
time limit of its own).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from fastclick_amd import dist as D, synth, device, _native as N

def rccl_version():
    try:
        return ".".join(map(str, torch.cuda.nccl.version()))
    except Exception:
        return "?"

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
try:
    # the device counters of a real batch: the path's own output
    b = synth.c4(8192 + 77, seed=31)
    synth.inject_errors(b, 0.02, seed=32)
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=16)
    got = device.process_batch(b, cfg, anno=False, perm=True, device_index=0)
    ctr = torch.from_numpy(got["counters"].astype(np.int64))
    rep = torch.zeros(N.CTR_SHARDS, N.NCOUNTERS, dtype=torch.int64, device=dev)
    rep[1] = ctr[:N.NCOUNTERS].to(dev)
    rep[2, N.CTR_PORT] = 5                        # a second replica: the sum must include it
    tot = D.reduce_counters(rep, force=True)
    counts = torch.from_numpy(np.diff(got["port_start"].astype(np.int64))).to(dev)
    before, gtot = D.output_offsets(counts, force=True)
    t = torch.tensor([1.25], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)      # bench.py's max-over-ranks time
    torch.cuda.synchronize()
    print(json.dumps(dict(backend=dist.get_backend(), world=dist.get_world_size(),
                          rccl=rccl_version(),
                          tot=tot.cpu().tolist(), want=(rep.sum(0)).cpu().tolist(),
                          before=before.cpu().tolist(), gtot=gtot.cpu().tolist(),
                          counts=counts.cpu().tolist(), tmax=float(t.item()),
                          on_device=tot.is_cuda and gtot.is_cuda)), flush=True)
finally:
    dist.destroy_process_group()
"""


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_gpu_rccl_world1_counter_allreduce_and_gather():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,COLL")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True,
                       timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    # RCCL's log shares stdout: the child's result is its JSON line
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["backend"] == "nccl" and out["world"] == 1 and out["on_device"]
    assert out["tot"] == out["want"]
    assert out["before"] == [0] * len(out["counts"]) and out["gtot"] == out["counts"]
    assert out["tmax"] == 1.25
    log = r.stderr + r.stdout
    # RCCL saw the communicator and each forced collective
    assert "NCCL INFO" in log, log[-2000:]
    for op in ("AllReduce", "AllGather"):
        assert op in log, f"no {op} in RCCL's log:\n" + log[-2000:]
    print(f"RCCL {out['rccl']}: world-1 communicator on cuda:0; AllReduce + AllGather issued")
    for ln in log.splitlines():           # the evidence, in the test's own output (-v -s)
        if "NCCL INFO" in ln and any(k in ln for k in ("AllReduce", "AllGather", "Init COMPLETE", "RCCL version")):
            print(ln)
