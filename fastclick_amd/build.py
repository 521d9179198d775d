"""In-tree build of the native libraries (hipcc for gfx950, g++ for the host side).

    libfcgpu.so   HIP kernels + C ABI (include/fastclick_gpu.h)
    libfcclick.so Click-shaped host harness + GPUIPCheckClassify element,
                  linked against libfcgpu.so (include/fcclick.h)

Outputs land in fastclick_amd/lib/ (git-ignored, shipped to the GPU box with
the working tree).
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib")
INC = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

FCGPU_SRC = [os.path.join(CSRC, "fcgpu_api.hip")]
FCGPU_DEPS = FCGPU_SRC + [os.path.join(CSRC, "fcgpu_device.hh"), os.path.join(CSRC, "fcgpu_flow.hh"),
                          os.path.join(CSRC, "capture.hh"), os.path.join(INC, "fastclick_gpu.h")]
FCCLICK_SRC = [os.path.join(CSRC, "host", f) for f in ("fcclick_capi.cc", "pcap_reader.cc")]
FCCLICK_DEPS = FCCLICK_SRC + [os.path.join(CSRC, "host", f) for f in
                              ("click_model.hh", "click_args.hh", "gpu_core.hh", "gpu_element.hh",
                               "program_text.hh")] + \
    [os.path.join(CSRC, "capture.hh")] + [os.path.join(INC, f) for f in ("fcclick.h", "fcpcap.h", "fastclick_gpu.h")]


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.exists(d) and os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    print("+", " ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)


def build_fcgpu(force=False):
    out = os.path.join(LIB, "libfcgpu.so")
    if force or _stale(out, FCGPU_DEPS):
        os.makedirs(LIB, exist_ok=True)
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
              f"-I{INC}", *FCGPU_SRC, "-o", out])
    return out


def build_fcclick(force=False):
    out = os.path.join(LIB, "libfcclick.so")
    if not all(os.path.exists(p) for p in FCCLICK_SRC):
        return None
    if force or _stale(out, FCCLICK_DEPS + [os.path.join(LIB, "libfcgpu.so")]):
        _run(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra",
              f"-I{INC}", *FCCLICK_SRC, "-o", out, f"-L{LIB}", "-lfcgpu",
              "-Wl,-rpath,$ORIGIN"])
    return out


def build_all(force=False):
    build_fcgpu(force)
    build_fcclick(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
