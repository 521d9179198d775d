"""The C-ABI libraries load on a CPU-only host and export every symbol that
include/*.h declares (no compute calls: there is no GPU here)."""
import ctypes as C
import os
import re

import pytest

from fastclick_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(fc(?:gpu|click|pcap)_[a-z_0-9]+)\s*\(",
                                 src, flags=re.M)))


def test_fcgpu_exports_every_declared_symbol():
    names = declared("fastclick_gpu.h")
    assert len(names) >= 15
    lib = N.load()
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(N.FCGPU_SYMBOLS), set(names) ^ set(N.FCGPU_SYMBOLS)
    assert lib.fcgpu_abi_version() == N.ABI_VERSION


def test_struct_layouts_match_header():
    assert C.sizeof(N.fcgpu_anno) == 16
    assert C.sizeof(N.fcgpu_out) == 9 * 8 + 8
    # 12 u32 scalars + 2x16 u32 lists + nbad6 + 16x16 B + process_eh, l4_mode, l4_checksum
    assert C.sizeof(N.fcgpu_cfg) == 4 * 12 + 4 * 32 + 4 + 256 + 6 * 4
    lib = N.load()
    cfg = N.fcgpu_cfg()
    lib.fcgpu_default_cfg(C.byref(cfg))
    assert cfg.size == C.sizeof(N.fcgpu_cfg)
    assert cfg.checksum == 0          # CheckIPHeader default: CHECKSUM false
    assert cfg.native_vlan == 0 and cfg.nbad6 == 1 and bytes(cfg.bad6[0]) == b"\xff" * 16
    assert cfg.l4_mode == N.L4_NONE and cfg.l4_checksum == 1   # CheckUDPHeader default CHECKSUM true


def test_field_offsets_match_c_compiler(tmp_path):
    """Every ctypes field offset equals offsetof() from the C header (gcc)."""
    import subprocess
    structs = {"fcgpu_cfg": N.fcgpu_cfg, "fcgpu_anno": N.fcgpu_anno, "fcgpu_out": N.fcgpu_out,
               "fcgpu_step": N.fcgpu_step, "fcgpu_job": N.fcgpu_job, "fcgpu_block_layout": N.fcgpu_block_layout,
               "fcgpu_mbuf_layout": N.fcgpu_mbuf_layout, "fcgpu_flow_config": N.fcgpu_flow_config,
               "fcgpu_flow_stat": N.fcgpu_flow_stat, "fcgpu_anno8": N.fcgpu_anno8, "fcgpu_xmeta": N.fcgpu_xmeta}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "fastclick_gpu.h"', "int main(void) {"]
    for sname, st in structs.items():
        lines.append(f'printf("{sname} sizeof %zu\\n", sizeof({sname}));')
        for fname, _ in st._fields_:
            lines.append(f'printf("{sname} {fname} %zu\\n", offsetof({sname}, {fname}));')
    lines.append("return 0; }")
    src = tmp_path / "off.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "off"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    out = subprocess.check_output([str(exe)], text=True).split("\n")
    seen = 0
    for line in filter(None, out):
        sname, fname, val = line.split()
        st = structs[sname]
        want = C.sizeof(st) if fname == "sizeof" else getattr(st, fname).offset
        assert int(val) == want, (sname, fname, val, want)
        seen += 1
    assert seen == sum(len(st._fields_) + 1 for st in structs.values())


def test_header_constants_match_python():
    """Every numeric #define FCGPU_X in fastclick_gpu.h has N.X with the same value."""
    src = open(os.path.join(ROOT, "include", "fastclick_gpu.h")).read()
    seen = 0
    for name, val in re.findall(r"^#define\s+FCGPU_(\w+)\s+([^/\n]+)", src, flags=re.M):
        expr = re.sub(r"(\d)u\b", r"\1", val.strip())
        if not re.fullmatch(r"[\d\sx+\-*()<a-fA-F]+", expr):
            continue
        assert hasattr(N, name), name
        assert getattr(N, name) == eval(expr, {}), (name, val)
        seen += 1
    assert seen >= 30


def test_open_without_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = N.load()
    h = C.c_void_p()
    rc = lib.fcgpu_open(0, 1024, C.byref(h))
    assert rc == N.ENODEV
    assert b"no HIP device" in lib.fcgpu_last_error(None)


def test_fcclick_exports_every_declared_symbol():
    if not os.path.exists(os.path.join(ROOT, "include", "fcclick.h")):
        pytest.skip("no host harness header")
    from fastclick_amd import click as K
    names = declared("fcclick.h")
    lib = K.load()
    for n in names:
        assert hasattr(lib, n), n


def test_fcpcap_exports_every_declared_symbol():
    from fastclick_amd import click as K
    names = declared("fcpcap.h")
    assert len(names) >= 8
    lib = K.load()
    for n in names:
        assert hasattr(lib, n), n


def test_every_header_is_checked():
    """include/ holds exactly the three C-ABI headers the tests above cover."""
    assert sorted(f for f in os.listdir(os.path.join(ROOT, "include")) if f.endswith(".h")) == \
        ["fastclick_gpu.h", "fcclick.h", "fcpcap.h"]


def test_lb_fastmod_exhaustive():
    """The device computes ((H>>16)^(H&0xffff)) % n as x - umulhi(x, ceil(2^32/n)) * n
    (fcgpu_device.hh lb_port); exact for every 16-bit x and every n <= 64."""
    import numpy as np
    x = np.arange(1 << 16, dtype=np.uint64)
    for n in range(2, 65):
        m = ((1 << 32) + n - 1) // n
        q = (x * np.uint64(m)) >> np.uint64(32)
        assert np.array_equal(x - q * np.uint64(n), x % np.uint64(n)), n
