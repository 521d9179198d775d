"""Decision programs: IPFilter / IPClassifier / Classifier.

The reference compiles its rule language into a step program and prints it
through the element's `program` handler (elements/ip/ipfilter.cc:1402,
elements/standard/classification.cc:978-991, :1104-1140). tests/golden/prog.npz
holds, from the compiled reference (gen_golden.py, set "prog"):
  * the program text of an IPClassifier with nine rules and of a Classifier
    with six, exactly as `print c.program` printed them;
  * the output every packet of a 3000-frame set left on (254 = no rule
    matched -> killed; 255 = CheckIPHeader rejected it first).
The C oracle's interpreter is pinned to those outputs; the HIP interpreter is
checked against the goldens and against the oracle on random programs.
"""
import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N
from tests.helpers import compare, repack
from tests.test_golden import load, batch_of

NOMATCH, INVALID = 254, 255
KINDS = {"ipc": N.PROG_IPFILTER, "cls": N.PROG_CLASSIFIER}


def _program(g, name):
    from fastclick_amd import click
    text = bytes(g[f"{name}_prog"]).decode()
    steps, oe = click.parse_program(text)
    return text, (KINDS[name], steps, oe), int(g[f"{name}_nout"])


def _outputs(r):
    return np.where(r["reason"] == N.R_OK, r["port"],
                    np.where(r["reason"] == N.R_NO_MATCH, NOMATCH, INVALID)).astype(np.uint8)


def _cfg(nout, **kw):
    return N.make_cfg(offset=14, checksum=True, classify=N.CLS_PROGRAM, nports=nout, **kw)


# ---------------------------------------------------------------- parser (CPU)

def test_parse_reference_program_text():
    g = load("prog")
    text, (kind, steps, oe), nout = _program(g, "ipc")
    assert oe == -1 and len(steps) == text.count("yes->")
    # step 0 of the IPClassifier: "264/00110000%00ff0000" = IP protocol == UDP
    assert (steps[0].offset, steps[0].value, steps[0].mask) == (264, 0x1100, 0xFF00)
    assert any(s.flags & N.STEP_SHORT_YES for s in steps)
    # [X] (no output) is kept distinct from every real output
    assert any(s.no == -2147483647 for s in steps)
    _, (_, csteps, coe), cnout = _program(g, "cls")
    assert coe == -1 and cnout == 6 and len(csteps) > 0


def test_parse_errors_and_all():
    from fastclick_amd import click
    assert click.parse_program("all->[3]\nsafe length 0\nalignment offset 0\n") == ([], 3)
    bad = [" 0 264/0011000%00ff0000  yes->[0]  no->[1]",          # short hex
           " 1 264/00110000%00ff0000  yes->[0]  no->[1]",          # index != 0
           " 0 264/00110000%00ff0000  yes->step 3  no->[1]",       # jump past the end
           " 0 264/00110000%00ff0000  yes->[0]",                   # no "no->"
           ""]
    for t in bad:
        with pytest.raises(click.ConfigError):
            click.parse_program(t)
    # '|' separates lines too (configuration strings)
    steps, oe = click.parse_program(" 0 256/45000000%ff000000  yes->[0]  no->[1]|safe length 260")
    assert len(steps) == 1 and steps[0].value == 0x45 and steps[0].mask == 0xFF


def test_element_program_keyword_errors():
    from fastclick_amd import click
    ok = "GPUIPCheckClassify(OFFSET 14, N 2, PROGRAM \" 0 265/11000000%ff000000  yes->[0]  no->[1]\")"
    click.check_config(ok)
    for conf in ["GPUIPCheckClassify(OFFSET 14, N 1, PROGRAM \" 0 265/11000000%ff000000  yes->[0]  no->[1]\")",
                 "GPUIPCheckClassify(OFFSET 14, N 2, PROGRAM \"garbage\")",
                 "GPUIPCheckClassify(OFFSET 14, N 2, PROGRAM_KIND ETHER)",
                 "GPUIPCheckClassify(OFFSET 14, N 2, PROGRAM \"all->[5]\")"]:
        with pytest.raises(click.ConfigError):
            click.check_config(conf)


# ------------------------------------------------------- oracle vs reference

@pytest.mark.parametrize("name", ["ipc", "cls"])
def test_oracle_program_golden(oracle, name):
    g = load("prog")
    _, prog, nout = _program(g, name)
    r = oracle.process_batch(_cfg(nout), batch_of(g), program=prog)
    exp = g[f"{name}_out"]
    got = _outputs(r)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, f"{name}: {len(bad)} packets differ, first {bad[:8]}: {got[bad[:8]]} vs {exp[bad[:8]]}"
    # every rule and the no-match path are exercised
    assert len(np.unique(exp)) == nout + 2
    # counters: unmatched packets are counted (CheckIPHeader passed them) but
    # are not CheckIPHeader drops
    c = r["counters"]
    assert c[N.CTR_COUNT] == (exp != INVALID).sum()
    assert c[N.CTR_DROPS] == (exp == INVALID).sum()
    assert c[N.CTR_REASON + N.reason_slot(N.R_NO_MATCH)] == (exp == NOMATCH).sum()
    assert c[N.CTR_PORT + nout] == (exp >= NOMATCH).sum()


# ------------------------------------------------------------------- GPU

def random_program(rng, batch, kind, nout, nsteps):
    """Random forward-jumping program whose comparison values are taken from
    real packets (so both branches are taken), with out-of-range outputs, [X]
    and short->yes steps mixed in."""
    A = batch.arena
    off = batch.desc[:, 0].astype(np.int64)
    steps = []
    for k in range(nsteps):
        if kind == N.PROG_IPFILTER:
            base = int(rng.choice([0, 256, 512]))
            o = base + int(rng.integers(0, 44 if base else 16)) + (int(rng.integers(0, 200)) if rng.random() < 0.05 else 0)
            frame_off = 14 + (o - 256) if base == 256 else 34 + (o - 512) if base == 512 else o - 2
        else:
            o = int(rng.integers(0, 80)) + (int(rng.integers(0, 200)) if rng.random() < 0.05 else 0)
            frame_off = o
        p = int(rng.integers(0, batch.n))
        fo = int(off[p]) + max(frame_off, 0)
        word = int.from_bytes(A[fo:fo + 4].tobytes(), "little")
        mb = [int(rng.choice([0, 0xFF, 0xF0, 0x0F, 0x80, 0x1F])) for _ in range(4)]
        mask = int.from_bytes(bytes(mb), "little")
        value = word & mask if rng.random() < 0.7 else int(rng.integers(0, 1 << 32)) & mask

        def jump():
            r = rng.random()
            if r < 0.55 and k + 1 < nsteps:
                return int(rng.integers(k + 1, nsteps))
            if r < 0.85:
                return -int(rng.integers(0, nout))
            return -2147483647 if r < 0.92 else -nout - int(rng.integers(0, 3))   # [X] / missing output
        steps.append((o, value, mask, jump(), jump(), int(rng.random() < 0.3)))
    return steps


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from fastclick_amd import device
    N.load()
    return device


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ipc", "cls"])
def test_gpu_program_golden(dev, name):
    g = load("prog")
    _, prog, nout = _program(g, name)
    for part in (N.PART_GLOBAL, N.PART_TILE):
        r = dev.process_batch(batch_of(g), _cfg(nout), partition=part, program=prog)
        got = _outputs(r)
        exp = g[f"{name}_out"]
        bad = np.nonzero(got != exp)[0]
        assert len(bad) == 0, f"{name} part={part}: {len(bad)} differ, first {bad[:8]}: {got[bad[:8]]} vs {exp[bad[:8]]}"


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [N.PROG_IPFILTER, N.PROG_CLASSIFIER])
@pytest.mark.parametrize("mode", ["c4", "mix", "misaligned"])
def test_gpu_random_programs_vs_oracle(dev, oracle, kind, mode):
    rng = np.random.default_rng(100 + kind * 10 + len(mode))
    if mode == "mix":
        b = synth.c5(20_000, seed=5)
        base = dict(check_mode=N.CHECK_AUTO, checksum=True)
    else:
        b = synth.c4(20_000, seed=4)
        synth.add_ip_options(b, 0.1, seed=6)
        synth.inject_errors(b, 0.02, seed=7)
        if mode == "misaligned":
            b = repack(b, misalign_seed=8)
        base = dict(offset=14, checksum=True)
    outcomes = set()
    for trial in range(6):
        nout = int(rng.integers(1, 65))
        nsteps = int(rng.integers(1, 120 if trial < 5 else 2000))
        prog = (kind, random_program(rng, b, kind, nout, nsteps), -1)
        cfg = N.make_cfg(classify=N.CLS_PROGRAM, nports=nout, **base)
        exp = oracle.process_batch(cfg, b, program=prog)
        for part in (N.PART_GLOBAL, N.PART_TILE):
            got = dev.process_batch(b, cfg, partition=part, program=prog)
            compare(got, exp, ctx=f"kind={kind} {mode} trial={trial} part={part}")
            assert np.array_equal(got["counters"], exp["counters"])
        outcomes |= set(np.unique(exp["reason"]).tolist())
    assert N.R_NO_MATCH in outcomes and N.R_OK in outcomes


@pytest.mark.gpu
def test_gpu_program_output_everything(dev, oracle):
    b = synth.c4(5000, seed=9)
    synth.inject_errors(b, 0.05, seed=10)
    for oe in (0, 3):
        cfg = _cfg(4)
        prog = (N.PROG_IPFILTER, [], oe)
        exp = oracle.process_batch(cfg, b, program=prog)
        got = dev.process_batch(b, cfg, partition=N.PART_TILE, program=prog)
        compare(got, exp, ctx=f"all->[{oe}]")
        assert (got["port"][got["reason"] == N.R_OK] == oe).all()


@pytest.mark.gpu
def test_gpu_program_required(dev):
    b = synth.c1(100)
    with pytest.raises(RuntimeError, match="fcgpu_set_program"):
        dev.process_batch(b, _cfg(2))


@pytest.mark.gpu
@pytest.mark.parametrize("jit", ["true", "false"])
@pytest.mark.parametrize("name", ["ipc", "cls"])
def test_element_program_golden(name, jit):
    """IPClassifier/Classifier through the element (program compiled to code,
    or interpreted): packets leave on the rule's output in input order,
    unmatched packets are killed, invalid ones leave on N."""
    from fastclick_amd import click
    g = load("prog")
    text, _, nout = _program(g, name)
    kind = "IPFILTER" if name == "ipc" else "CLASSIFIER"
    conf = (f"GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N {nout}, PROGRAM_KIND {kind}, PROGRAM_JIT {jit}, "
            f"PROGRAM \"{text.replace(chr(10), '|')}\")")
    res = click.run_element(conf, batch_of(g), nsinks=nout + 1)
    exp = g[f"{name}_out"].astype(np.int64)
    port = res["port"].astype(np.int64)
    want = np.where(exp == NOMATCH, 0xFFFFFFFF, np.where(exp == INVALID, nout, exp))
    assert np.array_equal(port, want)
    seq = res["seq"].astype(np.int64)
    for k in range(nout + 1):
        sel = np.nonzero(port == k)[0]
        assert np.all(np.diff(seq[sel]) > 0), f"output {k} order"


# ---------------------------------- programs and cases the reference's tests pin

def _reftests():
    import json
    import os
    from tests.test_golden import HERE
    with open(os.path.join(HERE, "reftests.json")) as f:
        return json.load(f)


def _run_reftest_programs(run):
    from fastclick_amd import click
    g = load("prog")
    b = batch_of(g)
    for case in _reftests()["programs"]:
        steps, oe = click.parse_program(case["program"])
        kind = KINDS["cls" if case["kind"] == "cls" else "ipc"]
        r = run(_cfg(case["nout"]), b, (kind, steps, oe))
        exp = np.array(case["outputs"], np.int64)
        assert len(exp) == b.n
        got = _outputs(r).astype(np.int64)
        bad = np.nonzero(got != exp)[0]
        assert len(bad) == 0, f"{case['case']} ({case['test']}): {len(bad)} differ, first {bad[:8]}"


def _run_short_cases(run):
    """IPFilter-01/02/03/08: truncated IP packets behind a header-marking
    source (FromIPSummaryDump sets the IP header like MarkIPHeader), raw IP
    (nh 0) or Ethernet-encapsulated (nh 14)."""
    from fastclick_amd import click
    for case in _reftests()["short"]:
        for fname, text in case["programs"].items():
            steps, oe = click.parse_program(text)
            nout = 2 if ", 1 -" in case["filters"][fname] else 1
            for nh in (0, 14):
                pk = [p for p in case["packets"] if p["filter"] == fname and p["nh"] == nh]
                if not pk:
                    continue
                b = synth.from_frames([bytes.fromhex(p["bytes"]) for p in pk])
                cfg = N.make_cfg(check_mode=N.MARK_IP4, offset=nh, hash_mode=N.HASH_NONE,
                                 classify=N.CLS_PROGRAM, nports=nout)
                r = run(cfg, b, (N.PROG_IPFILTER, steps, oe))
                for j, p in enumerate(pk):
                    want = (N.R_NO_MATCH, nout) if p["expect"] == "X" else (N.R_OK, p["expect"])
                    got = (int(r["reason"][j]), int(r["port"][j]))
                    assert got == want, f"{case['case']} {fname} ts={p['ts']} len={len(p['bytes']) // 2}: {got} vs {want}"


def test_oracle_reference_test_programs(oracle):
    _run_reftest_programs(lambda cfg, b, prog: oracle.process_batch(cfg, b, program=prog))


def test_oracle_reference_short_packet_cases(oracle):
    _run_short_cases(lambda cfg, b, prog: oracle.process_batch(cfg, b, program=prog))


@pytest.mark.gpu
def test_gpu_reference_test_programs(dev):
    for part in (N.PART_GLOBAL, N.PART_TILE):
        _run_reftest_programs(lambda cfg, b, prog: dev.process_batch(b, cfg, partition=part, program=prog))


@pytest.mark.gpu
def test_gpu_reference_short_packet_cases(dev):
    for part in (N.PART_GLOBAL, N.PART_TILE):
        _run_short_cases(lambda cfg, b, prog: dev.process_batch(b, cfg, partition=part, program=prog))


def chain_program(rng, nout, nsteps):
    """Programs shaped like the reference's compilation of port-range rules:
    mostly runs of mask tests on one transport/network word (contiguous bit
    ranges of the big-endian word, some wider than a jump table takes), mixed
    with tests on other words, forward jumps, outputs, [X] and short->yes.
    fcgpu_set_program turns the runs into jump tables; the oracle walks the
    steps as given."""
    steps = []
    for k in range(nsteps):
        o = int(rng.choice([512, 512, 512, 516, 264, 260, 268]))
        width = int(rng.integers(1, 13))
        lo = int(rng.integers(0, 33 - width))
        m_be = ((1 << width) - 1) << lo
        mask = int.from_bytes(m_be.to_bytes(4, "big"), "little")
        value = int(rng.integers(0, 1 << 32)) & mask

        def jump():
            r = rng.random()
            if r < 0.6 and k + 1 < nsteps:
                return int(rng.integers(k + 1, min(nsteps, k + 6)))
            if r < 0.9:
                return -int(rng.integers(0, nout))
            return -2147483647
        steps.append((o, value, mask, jump(), jump(), int(rng.random() < 0.3)))
    return steps


@pytest.mark.gpu
def test_gpu_chain_programs_tables_vs_oracle(dev, oracle):
    """Jump-table steps (runs on one word) give the oracle's outputs, including
    packets whose tested word is cut short (the table step then falls back to
    the original steps' length-checked rules)."""
    rng = np.random.default_rng(4242)
    b = synth.c4(30_000, seed=44)
    # ~15 % datagrams with 0..7 transport bytes: ip_len, frame length, checksum
    A = b.arena
    for i in np.nonzero(rng.random(b.n) < 0.15)[0]:
        k = int(rng.integers(0, 8))
        o = int(b.desc[i, 0]) + 14
        L = 20 + k
        A[o + 2], A[o + 3] = L >> 8, L & 0xFF
        b.desc[i, 1] = 14 + L
        synth._refresh_cksum(A, o)
    synth.inject_errors(b, 0.01, seed=45)
    outcomes = set()
    for trial in range(8):
        nout = int(rng.integers(2, 20))
        nsteps = int(rng.integers(3, 60 if trial < 6 else 400))
        prog = (N.PROG_IPFILTER, chain_program(rng, nout, nsteps), -1)
        cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_PROGRAM, nports=nout)
        exp = oracle.process_batch(cfg, b, program=prog)
        got = dev.process_batch(b, cfg, partition=N.PART_TILE, program=prog)
        compare(got, exp, ctx=f"chain trial={trial}")
        assert np.array_equal(got["counters"], exp["counters"])
        outcomes |= set(np.unique(exp["port"]).tolist())
    assert len(outcomes) > 5


# ---------------------------------------------------- programs compiled to code

@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ipc", "cls"])
def test_gpu_program_jit_golden(dev, name):
    """fcgpu_program_jit: the reference-compiled programs as straight-line code
    (hiprtc) give the reference's outputs, for both partition shapes."""
    g = load("prog")
    _, prog, nout = _program(g, name)
    for part in (N.PART_GLOBAL, N.PART_TILE):
        r = dev.process_batch(batch_of(g), _cfg(nout), partition=part, program=prog, program_jit=True)
        got = _outputs(r)
        exp = g[f"{name}_out"]
        bad = np.nonzero(got != exp)[0]
        assert len(bad) == 0, f"jit {name} part={part}: {len(bad)} differ, first {bad[:8]}"


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["c4", "mix"])
def test_gpu_random_programs_jit_vs_oracle(dev, oracle, mode):
    """Random programs (table steps, short words, [X], outputs past N) as
    code: the same outputs and counters as the oracle, program by program."""
    import torch
    from fastclick_amd.device import DeviceBatch, DeviceOutputs, run_device
    rng = np.random.default_rng(700 + len(mode))
    if mode == "mix":
        b = synth.c5(20_000, seed=15)
        base = dict(check_mode=N.CHECK_AUTO, checksum=True)
    else:
        b = synth.c4(20_000, seed=14)
        synth.add_ip_options(b, 0.1, seed=16)
        synth.inject_errors(b, 0.02, seed=17)
        base = dict(offset=14, checksum=True)
    for trial, kind in enumerate([N.PROG_IPFILTER, N.PROG_CLASSIFIER, N.PROG_IPFILTER]):
        nout = int(rng.integers(2, 40))
        prog = (kind, random_program(rng, b, kind, nout, int(rng.integers(20, 200))), -1)
        cfg = N.make_cfg(classify=N.CLS_PROGRAM, nports=nout, **base)
        exp = oracle.process_batch(cfg, b, program=prog)
        ctx = N.Context(0, b.n, cfg)
        try:
            ctx.set_program(*prog)
            ctx.program_jit(True)
            assert ctx.program_jit_active()
            db = DeviceBatch.upload(b, device="cuda:0")
            for part in (N.PART_GLOBAL, N.PART_TILE):
                outs = DeviceOutputs(b.n, nout, device="cuda:0", anno=True, perm=True, port_start=True,
                                     partition=part)
                run_device(ctx, db, outs)
                torch.cuda.synchronize()
                got = outs.numpy()
                compare(got, exp, ctx=f"jit {mode} trial={trial} part={part}")
        finally:
            ctx.close()


@pytest.mark.gpu
def test_gpu_program_jit_cycle_and_reconfigure(dev, oracle):
    """A program with a backward jump stays interpreted (fcgpu_program_jit
    refuses it, the interpreter's bounded walk still answers as the oracle);
    an acyclic program installed afterwards is compiled; a later flow table
    adds its kernels on first launch; switching JIT off goes back to the
    interpreter -- all with the oracle's outputs."""
    import torch
    from fastclick_amd.device import DeviceBatch, DeviceOutputs, run_device
    b = synth.c4(8_000, seed=21)
    # step 1 -> 2 -> 1 for odd source ports: the walk gives up (unmatched)
    cyc = [(256 + 9, 17, 0xff, 1, -1, 0), (512, 0, 0x1, -1, 2, 0), (256 + 12, 0, 0, 1, 1, 0)]
    steps = [(256 + 9, 17, 0xff, 1, -1, 0), (512 + 2, 0, 0x100, -0, -2, 0)]
    cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_PROGRAM, nports=3)
    ctx = N.Context(0, b.n, cfg)
    try:
        db = DeviceBatch.upload(b, device="cuda:0")

        def run_check(prog, flow=False):
            exp = oracle.process_batch(cfg, b, program=prog)
            outs = DeviceOutputs(b.n, 3, device="cuda:0", perm=True, partition=N.PART_TILE, flowid=flow)
            run_device(ctx, db, outs)
            torch.cuda.synchronize()
            got = outs.numpy()
            assert np.array_equal(got["reason"], exp["reason"]) and np.array_equal(got["port"], exp["port"])

        ctx.set_program(N.PROG_IPFILTER, cyc, -1)
        with pytest.raises(RuntimeError, match="cycle"):
            ctx.program_jit(True)
        assert not ctx.program_jit_active()
        run_check((N.PROG_IPFILTER, cyc, -1))
        ctx.set_program(N.PROG_IPFILTER, steps, -1)
        assert ctx.program_jit_active()
        run_check((N.PROG_IPFILTER, steps, -1))
        ctx.flow_enable(1 << 16)
        run_check((N.PROG_IPFILTER, steps, -1), flow=True)
        ctx.program_jit(False)
        assert not ctx.program_jit_active()
        run_check((N.PROG_IPFILTER, steps, -1), flow=True)
    finally:
        ctx.close()
