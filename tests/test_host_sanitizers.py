"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

SURVEY §5: the reference ships no sanitizer build; this repo runs its own
host-side parsers (FromDump-compatible pcap reader, decision-program text,
element keywords) and the oracle under ASan/UBSan on seeded random and
mutated inputs (tests/host_fuzz.cc), and the pcap reader's parallel reads
under ThreadSanitizer. The HIP kernels are not instrumented
(GPU sanitizers are not available on the pool); libfcgpu.so is linked
uninstrumented only for fcgpu_default_cfg and the element's symbols, and no
HIP call is made.
"""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "fastclick_amd", "lib")


def _build_and_run(tmp_path, sanitize, runs):
    san = [f"-fsanitize={sanitize}", "-fno-omit-frame-pointer", "-g", "-O1"]
    if sanitize != "thread":
        san.append("-fno-sanitize-recover=all")
    tag = sanitize.replace(",", "_")
    obj = tmp_path / f"fc_oracle_{tag}.o"
    subprocess.run(["gcc", *san, "-std=gnu11", "-I", os.path.join(ROOT, "include"), "-c",
                    os.path.join(ROOT, "oracle", "fc_oracle.c"), "-o", str(obj)], check=True)
    exe = tmp_path / f"host_fuzz_{tag}"
    subprocess.run(["g++", *san, "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "host_fuzz.cc"),
                    os.path.join(ROOT, "fastclick_amd", "csrc", "host", "pcap_reader.cc"), str(obj),
                    "-L", LIB, "-lfcgpu", f"-Wl,-rpath,{LIB}", "-lpthread", "-o", str(exe)], check=True)
    with open(os.path.join(ROOT, "tests", "golden", "reftests.json")) as f:
        progs = [p["program"].strip().replace("\n", "|") for p in json.load(f)["programs"]]
    pf = tmp_path / "programs.txt"
    pf.write_text("\n".join(progs) + "\n")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1",
               TMPDIR=str(tmp_path))
    for seed, seconds in runs:
        out = subprocess.run([str(exe), str(pf), str(seconds), str(seed)], capture_output=True, text=True,
                             env=env, timeout=300)
        assert out.returncode == 0, out.stderr[-4000:]
        assert "host_fuzz ok" in out.stdout, out.stdout + out.stderr[-2000:]


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="no host compiler")
@pytest.mark.skipif(not os.path.exists(os.path.join(LIB, "libfcgpu.so")), reason="libfcgpu.so not built")
def test_host_code_under_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, "address,undefined", [(1, 4), (2, 4)])


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="no host compiler")
@pytest.mark.skipif(not os.path.exists(os.path.join(LIB, "libfcgpu.so")), reason="libfcgpu.so not built")
def test_host_code_under_tsan(tmp_path):
    """The pcap reader's parallel pread() pieces (fcpcap_set_threads)."""
    _build_and_run(tmp_path, "thread", [(3, 3)])


ELEMENT_CONFS = [
    # compact 8-B-packed records, DESC32 descriptors (the headline chain)
    "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash, BATCH {b})",
    # records to the frame's end (the UDP checksum), 16-B packing
    "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash, L4 UDP, BATCH {b})",
    # whole captures, (offset, length) descriptors (a decision program: the
    # reference compiler's 16-rule IPClassifier, tests/golden/reftests.json)
    "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, PROGRAM \"{prog}\", BATCH {b})",
    # VLAN / IPv6 dispatch, full annotations, paint and strip
    "GPUIPCheckClassify(MODE AUTO, N 16, LB_MODE hash, COLOR 3, STRIP true, BATCH {b})",
]


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_element_data_path_under_asan_ubsan(tmp_path):
    """The element's data path -- staging (the per-packet and the run fast
    paths), submission, completion, annotation and the output runs -- under
    ASan/UBSan over the stand-in library whose batches complete at once
    (scripts/mock_fcgpu.cc; no HIP call), for compact records, records to the
    frame's end, whole captures and the VLAN/IPv6 dispatch, in copy- and
    zero-copy-sized batches and at several BATCH sizes (slots opened, filled
    and submitted mid-PacketBatch)."""
    san = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g", "-O1", "-fno-sanitize-recover=all"]
    exe = tmp_path / "element_bench_asan"
    subprocess.run(["g++", *san, "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "scripts", "mock_fcgpu.cc"),
                    os.path.join(ROOT, "fastclick_amd", "csrc", "host", "fcclick_capi.cc"),
                    os.path.join(ROOT, "fastclick_amd", "csrc", "host", "pcap_reader.cc"),
                    os.path.join(ROOT, "scripts", "mock_element_bench.cc"), "-lpthread", "-o", str(exe)],
                   check=True)
    with open(os.path.join(ROOT, "tests", "golden", "reftests.json")) as f:
        prog = "|".join({p["case"]: p for p in json.load(f)["programs"]}["ipclass16"]["program"].strip().splitlines())
    for zc in ("0", "1"):
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
                   UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", MOCK_ZEROCOPY=zc)
        for conf in ELEMENT_CONFS:
            for b in ("auto", "1000", "37"):
                c = conf.format(b=b, prog=prog)
                out = subprocess.run([str(exe), "2", b, "2", c], capture_output=True, text=True, env=env,
                                     timeout=300)
                assert out.returncode == 0, (c, out.stderr[-4000:])
                assert '"element_mpps"' in out.stdout, (c, out.stdout, out.stderr[-2000:])
