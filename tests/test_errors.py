"""Failure handling (SURVEY 8(b) "Errors") and the launch guard.

- Every k_rx launch passes a host-side guard (rx_launch_ok): a launch missing
  an output its partition shape stores through, or with null inputs, is
  refused with an error instead of faulting the device (the r03_s17 fault:
  a shared launch with a null tile_count). fcgpu_launch_guard_selftest()
  runs the guard over malformed launches on the host; on the GPU, malformed
  jobs come back as FCGPU_EINVAL and the context keeps working.
- A batch the GPU fails is re-submitted once through copies
  (FCGPU_SUBMIT_COPY); a batch that fails twice leaves unprocessed on
  ERROR_OUTPUT or is killed, and is counted in gpu_errors / drop_details /
  drops -- the reference's element never loses a valid packet silently
  (elements/ip/checkipheader.cc:143-161 drops only invalid ones). Failures are
  injected with fcgpu_inject_fault (include/fastclick_gpu.h).
- The shared zero-copy queue (FCGPU_SPAN_AUTO) fuses only batches whose
  launch inputs are identical (configuration, check mode, checksum, compiled
  program) and takes them at submit time; a failed shared launch is reported
  by each owner's wait, and frees the slots.
"""
import ctypes as C

import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N

CONF = ("GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4, LB_MODE hash, DETAILS true, BATCH 2048, "
        "ZEROCOPY false, BADSRC 192.0.2.255)")


def test_launch_guard_selftest():
    lib = N.load()
    assert lib.fcgpu_launch_guard_selftest() == 0


def test_inject_fault_arguments():
    lib = N.load()
    assert lib.fcgpu_inject_fault(4, 0, 1) == N.EINVAL
    for k in (N.FAULT_SUBMIT, N.FAULT_WAIT, N.FAULT_LAUNCH, N.FAULT_ALLOC):
        assert lib.fcgpu_inject_fault(k, 0, 0) == N.OK


def test_error_output_keyword():
    from fastclick_amd import click as K
    K.check_config(CONF[:-1] + ", ERROR_OUTPUT 5)")
    for bad in ("ERROR_OUTPUT -2", "ERROR_OUTPUT x", "ERROR_OUTPUT 66"):
        with pytest.raises(K.ConfigError, match="ERROR_OUTPUT"):
            K.check_config(CONF[:-1] + f", {bad})")


def _batch():
    b = synth.c4(3 * 2048 + 300, seed=1501)
    synth.inject_errors(b, 0.03, seed=1502)
    return b


def _exp(oracle, b):
    from fastclick_amd import click as K
    return oracle.process_batch(K.element_cfg(CONF), b)


@pytest.fixture
def no_faults():
    lib = N.load()
    yield lib
    for k in (N.FAULT_SUBMIT, N.FAULT_WAIT, N.FAULT_LAUNCH, N.FAULT_ALLOC):
        lib.fcgpu_inject_fault(k, 0, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["submit", "wait"])
def test_gpu_element_retry_recovers(oracle, no_faults, where):
    """One failure (at submission, or reported by the completion wait): the
    batch goes again through copies and every packet leaves as without it."""
    from fastclick_amd import click as K
    lib = no_faults
    b = _batch()
    e = _exp(oracle, b)
    ref = K.run_element(CONF, b, nsinks=5)
    lib.fcgpu_inject_fault(N.FAULT_SUBMIT if where == "submit" else N.FAULT_WAIT, 0, 1)
    r = K.run_element(CONF, b, nsinks=5)
    assert r["error"] == ""
    assert np.array_equal(r["port"], e["port"].astype(np.uint32))
    for k in ("port", "agg", "dst", "len", "nh"):
        assert np.array_equal(r[k], ref[k]), k
    h = r["handlers"]
    assert h["gpu_retries"] == "1" and h["gpu_errors"] == "0" and h["error"] == ""
    assert h["count"] == ref["handlers"]["count"] and h["drops"] == ref["handlers"]["drops"]
    assert h["drop_details"] == ref["handlers"]["drop_details"]


@pytest.mark.gpu
@pytest.mark.parametrize("where,error_output", [("submit", -1), ("wait", -1), ("wait", 5)])
def test_gpu_element_failed_twice_is_counted(oracle, no_faults, where, error_output):
    """Two failures in a row: the batch's packets are killed (or leave on
    ERROR_OUTPUT, unprocessed, in input order), counted in gpu_errors, in
    drop_details' extra line and (killed) in drops; the run reports the error;
    every other batch is processed as usual."""
    from fastclick_amd import click as K
    lib = no_faults
    b = _batch()
    e = _exp(oracle, b)
    conf = CONF if error_output < 0 else CONF[:-1] + f", ERROR_OUTPUT {error_output})"
    # device batches: 3 x 2048 packets, then the last 300 at flush. Submissions
    # 0-3 go out before the last one completes; submission 4 is its
    # re-submission: skip 3, fail 2 -> the last batch fails twice
    lib.fcgpu_inject_fault(N.FAULT_SUBMIT if where == "submit" else N.FAULT_WAIT, 3, 2)
    r = K.run_element(conf, b, nsinks=6, allow_error=True)
    assert "injected fault" in r["error"]
    lost = np.arange(3 * 2048, b.n)
    rest = np.arange(3 * 2048)
    if error_output < 0:
        assert (r["port"][lost] == 0xFFFFFFFF).all()
    else:
        assert (r["port"][lost] == error_output).all()
        seq = r["seq"][lost].astype(np.int64)
        assert (np.diff(seq) > 0).all()         # input order
        assert (r["nh"][lost] == -1).all()      # unprocessed: no header marks
        assert np.array_equal(r["len"][lost], b.desc[lost, 1].astype(np.uint32))
    assert np.array_equal(r["port"][rest], e["port"][rest].astype(np.uint32))
    h = r["handlers"]
    assert h["gpu_errors"] == str(len(lost)) and h["gpu_retries"] == "1"
    ok_rest = e["reason"][rest] == N.R_OK
    assert int(h["count"]) == int(ok_rest.sum())
    killed = len(lost) if error_output < 0 else 0
    assert int(h["drops"]) == int((~ok_rest).sum()) + killed
    lines = h["drop_details"].strip("\n").split("\n")
    assert len(lines) == 7 and lines[6].endswith("GPU failure") and int(lines[6].split()[0]) == len(lost)


def _block(lib, ctx, b, cap):
    from tests.test_span_modes import Block
    return Block(lib, ctx, b, cap)


@pytest.mark.gpu
def test_gpu_shared_queue_mixed_configs(oracle):
    """Four AUTO contexts whose configurations differ only in the check mode
    or the checksum flag, their batches queued together: each batch is
    checked with its own context's configuration (the launch fuses only
    identical ones). While a batch of its is queued, a context refuses
    fcgpu_configure / fcgpu_set_program / fcgpu_program_jit."""
    from tests.test_span_modes import OUTS
    lib = N.load()
    b = synth.c4(3000 + 17, seed=1511)
    synth.inject_errors(b, 0.05, seed=1512)
    cfgs = [N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=8),
            N.make_cfg(offset=14, checksum=False, classify=N.CLS_LB_HASH, nports=8),
            N.make_cfg(offset=14, check_mode=N.MARK_IP4, classify=N.CLS_LB_HASH, nports=8),
            N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=8)]
    exps = [oracle.process_batch(c, b) for c in cfgs]
    assert not np.array_equal(exps[0]["reason"], exps[1]["reason"])
    assert not np.array_equal(exps[1]["reason"], exps[2]["reason"])
    ctxs, blks = [], []
    try:
        for c in cfgs:
            h = C.c_void_p()
            assert lib.fcgpu_open(0, 4096, C.byref(h)) == N.OK
            assert lib.fcgpu_configure(h, C.byref(c)) == N.OK
            assert lib.fcgpu_span_mode(h, N.SPAN_AUTO) == N.OK
            ctxs.append(h)
        for h in ctxs:
            blks.append(_block(lib, h, b, 4096))
        # one queued (fewer than four pending: not launched yet)
        assert lib.fcgpu_span_zerocopy_active(ctxs[0]) == 1
        rc = lib.fcgpu_span_submit_block(ctxs[0], 0, blks[0].pin, blks[0].in_bytes, 0, blks[0].frames_off, b.n,
                                         blks[0].out, OUTS, N.PART_TILE)
        assert rc == N.OK
        assert lib.fcgpu_configure(ctxs[0], C.byref(cfgs[1])) == N.EINVAL
        assert b"queued" in lib.fcgpu_last_error(ctxs[0])
        assert lib.fcgpu_program_jit(ctxs[0], 1) == N.EINVAL
        assert lib.fcgpu_set_program(ctxs[0], N.PROG_IPFILTER, None, 0, 0) == N.EINVAL
        for k in range(1, 4):
            rc = lib.fcgpu_span_submit_block(ctxs[k], 0, blks[k].pin, blks[k].in_bytes, 0, blks[k].frames_off,
                                             b.n, blks[k].out, OUTS, N.PART_TILE)
            assert rc == N.OK, lib.fcgpu_last_error(ctxs[k])
        for k in range(4):
            assert lib.fcgpu_span_wait(ctxs[k], 0) == N.OK, lib.fcgpu_last_error(ctxs[k])
            L, n = blks[k].L, b.n
            v = blks[k].res[L.verdict:L.verdict + 2 * n].view(np.uint16)
            assert np.array_equal(v & 0xff, exps[k]["reason"].astype(np.uint16)), k
            # MarkIPHeader checks nothing: a header-error packet's ports may lie
            # past its end (bytes no staging defines; IPFlowID reads them anyway)
            a = exps[k]["anno"]
            inside = a["th"].astype(np.int64) + 4 <= b.desc[:, 1].astype(np.int64)
            assert inside.sum() > 0.9 * n
            assert np.array_equal((v >> 8)[inside], exps[k]["port"].astype(np.uint16)[inside]), k
        # waited: reconfiguring is allowed again
        assert lib.fcgpu_configure(ctxs[0], C.byref(cfgs[0])) == N.OK
    finally:
        for x in blks:
            x.free()
        for h in ctxs:
            lib.fcgpu_close(h)


@pytest.mark.gpu
def test_gpu_shared_queue_launch_failure(oracle, no_faults):
    """A failed shared launch: every batch it carried reports the error through
    its owner's wait (submission itself returned OK), the slots are free
    again, and a re-submission through copies (FCGPU_SUBMIT_COPY) gives the
    oracle's results."""
    from tests.test_span_modes import OUTS
    lib = no_faults
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=8)
    b = synth.c4(2000 + 9, seed=1521)
    synth.inject_errors(b, 0.05, seed=1522)
    e = oracle.process_batch(cfg, b)
    ctxs, blks = [], []
    try:
        for _ in range(4):
            h = C.c_void_p()
            assert lib.fcgpu_open(0, 4096, C.byref(h)) == N.OK
            assert lib.fcgpu_configure(h, C.byref(cfg)) == N.OK
            assert lib.fcgpu_span_mode(h, N.SPAN_AUTO) == N.OK
            ctxs.append(h)
            blks.append(_block(lib, h, b, 4096))
        lib.fcgpu_inject_fault(N.FAULT_LAUNCH, 0, 1)
        for k, h in enumerate(ctxs):
            rc = lib.fcgpu_span_submit_block(h, 1, blks[k].pin, blks[k].in_bytes, 0, blks[k].frames_off, b.n,
                                             blks[k].out, OUTS, N.PART_TILE)
            assert rc == N.OK, lib.fcgpu_last_error(h)
        for h in ctxs:
            assert lib.fcgpu_span_wait(h, 1) == N.ERUNTIME
            assert lib.fcgpu_span_wait(h, 1) == N.OK      # free again
        for k, h in enumerate(ctxs):
            blks[k].res[:] = 0xEE
            rc = lib.fcgpu_span_submit_block(h, 1, blks[k].pin, blks[k].in_bytes, 0, blks[k].frames_off, b.n,
                                             blks[k].out, OUTS | N.SUBMIT_COPY, N.PART_TILE)
            assert rc == N.OK, lib.fcgpu_last_error(h)
            assert lib.fcgpu_span_wait(h, 1) == N.OK
            L = blks[k].L
            v = blks[k].res[L.verdict:L.verdict + 2 * b.n].view(np.uint16)
            assert np.array_equal(v & 0xff, e["reason"].astype(np.uint16))
    finally:
        for x in blks:
            x.free()
        for h in ctxs:
            lib.fcgpu_close(h)


@pytest.mark.gpu
def test_gpu_malformed_jobs_refused(oracle):
    """Malformed submissions through the C ABI come back as FCGPU_EINVAL with a
    message -- a tile partition asked for without its tile_count (what the
    kernel stores through), null frames or descriptors, a bad partition
    value, a batch past max_batch -- and the context then processes a good
    batch as the oracle does (nothing faulted on the device)."""
    import torch
    from fastclick_amd import device
    lib = N.load()
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_HASH, nports=8)
    b = synth.c4(1500, seed=1531)
    ctx = N.Context(0, 2048, cfg)
    try:
        dev = torch.device("cuda:0")
        arena = torch.from_numpy(b.arena).to(dev)
        desc = torch.from_numpy(np.ascontiguousarray(b.desc, dtype=np.uint32)).to(dev)
        verdict = torch.zeros(b.n, dtype=torch.int16, device=dev)
        tperm = torch.zeros(b.n + 256, dtype=torch.uint8, device=dev)
        tcount = torch.zeros(9 * 8, dtype=torch.int16, device=dev)

        def job(n=b.n, arena_p=arena.data_ptr(), desc_p=desc.data_ptr(), part=N.PART_TILE, tp=True, tc=True):
            j = N.fcgpu_job()
            j.arena, j.desc, j.n = arena_p, desc_p, n
            j.out.verdict = verdict.data_ptr()
            j.out.partition = part
            j.out.tile_perm = tperm.data_ptr() if tp else None
            j.out.tile_count = tcount.data_ptr() if tc else None
            return j
        torch.cuda.synchronize()
        for bad in (job(tc=False), job(arena_p=None), job(desc_p=None), job(part=7), job(n=4096)):
            rc = lib.fcgpu_process_jobs(ctx.h, C.byref(bad), 1, None)
            assert rc in (N.EINVAL, N.ENOMEM), rc
            assert lib.fcgpu_last_error(ctx.h)
        jobs = (N.fcgpu_job * 2)(job(), job(tc=False))
        assert lib.fcgpu_process_jobs(ctx.h, jobs, 2, None) == N.EINVAL
        torch.cuda.synchronize()
        got = device.process_batch(b, cfg)
        exp = oracle.process_batch(cfg, b)
        assert np.array_equal(got["reason"], exp["reason"]) and np.array_equal(got["port"], exp["port"])
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_element_retries_under_busy_shared_queue(oracle, no_faults):
    """Sixteen element threads on the UDP chain share the GPU's zero-copy
    queue (ZEROCOPY auto: FCGPU_SPAN_AUTO with >= 4 contexts). Six of that
    queue's launches fail mid-run (fcgpu_inject_fault LAUNCH, after 40 good
    ones), so their batches' owners re-submit them through copies
    (FCGPU_SUBMIT_COPY) while the other threads keep the queue busy -- the
    interleaving of round 5's hung staging experiment.
    The device blocks those re-submissions use were reserved at initialize
    (fcgpu_span_reserve), so none allocates or synchronises the device.
    Every packet is accounted for: each thread's outputs received exactly the
    oracle's per-output counts, every failed batch went through once more and
    succeeded, and the run ends (the test's timeout)."""
    from fastclick_amd import click as K
    lib = no_faults
    conf = "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash, L4 UDP)"
    b = synth.c3(65536, nflows=2000, seed=1541)
    synth.set_udp_checksums(b)
    synth.inject_errors(b, 0.03, seed=1542)
    e = oracle.process_batch(K.element_cfg(conf), b)
    per_port = np.bincount(e["port"].astype(np.int64), minlength=17)
    assert per_port.sum() == b.n and per_port[16] > 0
    threads, reps = 16, 4
    lib.fcgpu_inject_fault(N.FAULT_LAUNCH, 40, 6)
    pk, hs = K.run_element_threads(conf, b, threads=threads, reps=reps, nsinks=17)
    retries = sum(int(h["gpu_retries"]) for h in hs)
    assert retries >= 6, retries                          # each failed launch carried >= 1 batch
    for t, h in enumerate(hs):
        assert h["gpu_errors"] == "0" and h["error"] == "", (t, h)
        assert np.array_equal(pk[t], per_port * reps), t
        # "count": packets past the IP check (fcgpu_counters_derive): the
        # L4 check's drops are counted there too, as CheckIPHeader counts them
        ip_drop = np.isin(e["reason"], [N.R_MINISCULE, N.R_BAD_VERSION, N.R_BAD_HLEN, N.R_BAD_IP_LEN,
                                        N.R_BAD_CKSUM, N.R_BAD_SADDR, N.R_BAD_IP6, N.R_VLAN_REJECT])
        assert int(h["count"]) == int((~ip_drop).sum()) * reps, t
        assert int(h["drops"]) == int(ip_drop.sum()) * reps, t
