"""The FastClick package element (fastclick_pkg/) compiled against the
reference's own headers.

The reference's configure is not run; fastclick_pkg/gen_config.py makes the
two headers it would generate (click/config.h, click/config-userlevel.h) by
config.status's `#undef` substitution over the reference's config.h.in and
config-userlevel.h.in, for a userlevel x86-64 build with batching, flows and
IPv6. The element, its ClickPolicy over FastClick's Packet / PacketBatch /
Timer / per_thread, and the shared RxCore then compile to an object with
g++ against /root/reference/include (-Wall -Wextra -Werror) -- every FastClick
declaration the package uses, with the argument types it passes. A mutated
copy with one API misuse must fail, so the check is not vacuous.

CPU only; skipped where the reference tree is absent (the GPU box).
Reference interface: include/click/batchelement.hh:29-125,
include/click/packetbatch.hh:631, include/click/sync.hh:56-203,
include/click/timer.hh:158.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
PKG = os.path.join(ROOT, "fastclick_pkg")

pytestmark = pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "config.h.in")),
                                reason="reference tree not present")


def _config(tmp):
    sys.path.insert(0, PKG)
    try:
        import gen_config
    finally:
        sys.path.pop(0)
    out = os.path.join(tmp, "cfg")
    gen_config.generate(REF, out)
    return out


def _compile(cfg, src, inc_first=None):
    cmd = ["g++", "-std=gnu++17", "-O1", "-Wall", "-Wextra", "-Werror", "-c", "-o", os.devnull,
           "-DHAVE_CONFIG_H", "-DCLICK_USERLEVEL"]
    if inc_first:
        cmd.append(f"-I{inc_first}")
    cmd += [f"-I{cfg}", f"-I{REF}/include", f"-I{ROOT}/fastclick_amd/csrc/host", f"-I{ROOT}/include", src]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=300)


def test_generated_config_defines_the_build(tmp_path):
    cfg = _config(str(tmp_path))
    text = open(os.path.join(cfg, "click", "config.h")).read()
    for line in ("#define HAVE_BATCH 1", "#define HAVE_FLOW 1", "#define HAVE_IP6 1",
                 "#define CLICK_BYTE_ORDER CLICK_LITTLE_ENDIAN", "#define __MTCLICK__ 1"):
        assert line in text
    assert "/* #undef HAVE_DPDK */" in open(os.path.join(cfg, "click", "config-userlevel.h")).read()
    assert "#undef HAVE_" not in text.replace("/* #undef", "")


def test_package_element_compiles_against_reference_headers(tmp_path):
    cfg = _config(str(tmp_path))
    r = _compile(cfg, os.path.join(PKG, "gpuipcheckclassify.cc"))
    assert r.returncode == 0, r.stderr[-4000:]


@pytest.mark.parametrize("old,new", [
    # PacketBatch::make_from_simple_list(Packet*, Packet*, unsigned) (packetbatch.hh:631)
    ("PacketBatch::make_from_simple_list(h, t, n)", "PacketBatch::make_from_simple_list(h, n)"),
    # per_thread<T>::get_value_for_thread(int) returns T& (sync.hh)
    ("State &s = _state.get_value_for_thread(thread);", "State *s = _state.get_value_for_thread(thread);"),
    # Packet::set_anno_u32(int, uint32_t) exists; a misspelled accessor must not compile
    ("p->set_anno_u32(o, v);", "p->set_anno_uint32(o, v);"),
])
def test_api_misuse_fails_to_compile(tmp_path, old, new):
    cfg = _config(str(tmp_path))
    mut = tmp_path / "mut"
    mut.mkdir()
    for f in ("gpuipcheckclassify.hh", "gpuipcheckclassify.cc"):
        shutil.copy(os.path.join(PKG, f), mut / f)
    hit = False
    for f in ("gpuipcheckclassify.hh", "gpuipcheckclassify.cc"):
        text = (mut / f).read_text()
        if old in text:
            (mut / f).write_text(text.replace(old, new))
            hit = True
    assert hit, f"the package no longer contains `{old}`"
    r = _compile(cfg, str(mut / "gpuipcheckclassify.cc"), inc_first=str(mut))
    assert r.returncode != 0, f"`{new}` compiled"
