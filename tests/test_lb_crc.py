"""LoadBalancer LB_MODE hash_crc (include/click/loadbalancer.hh:563-569).

The reference computes ipv4_hash_crc (include/click/dpdk_glue.hh:13-27) with
DPDK's rte_hash_crc_4byte, which on x86 is the SSE4.2 crc32 instruction
(_mm_crc32_u32). DPDK is not in this image, so the reference itself cannot
run here: the oracle's CRC32-C restatement is pinned instead to that very
instruction, on random words and on the IPFlow5ID word sequence, by a small C
program compiled with -msse4.2 (parity of the port formula otherwise
follows the reference's source; no reference run pins it). The device is
then compared with the oracle.
"""
import os
import platform
import subprocess

import numpy as np
import pytest

from fastclick_amd import synth
from fastclick_amd import _native as N
from tests.helpers import compare, set_fragment

HW = r"""
#include <nmmintrin.h>
#include <stdio.h>
#include <stdint.h>
int main(void) {
    uint32_t d, c;
    while (scanf("%u %u", &d, &c) == 2) printf("%u\n", _mm_crc32_u32(c, d));
    return 0;
}
"""


@pytest.mark.skipif(platform.machine() not in ("x86_64", "AMD64"), reason="SSE4.2 crc32 is x86")
def test_oracle_crc32c_matches_sse42_instruction(oracle, tmp_path):
    src = tmp_path / "crc.c"
    src.write_text(HW)
    exe = tmp_path / "crc"
    subprocess.check_call(["gcc", "-O2", "-msse4.2", str(src), "-o", str(exe)])
    rng = np.random.default_rng(3)
    d = rng.integers(0, 1 << 32, 3000, dtype=np.uint64)
    c = rng.integers(0, 1 << 32, 3000, dtype=np.uint64)
    c[:100] = 0
    inp = "\n".join(f"{a} {b}" for a, b in zip(d.tolist(), c.tolist()))
    hw = [int(x) for x in subprocess.run([str(exe)], input=inp, capture_output=True, text=True,
                                          check=True).stdout.split()]
    lib = oracle.load()
    sw = [lib.fco_crc32c_u32(int(a), int(b)) for a, b in zip(d.tolist(), c.tolist())]
    assert sw == hw


@pytest.mark.gpu
def test_gpu_lb_crc_vs_oracle(oracle):
    from fastclick_amd import device
    b = synth.c4(60_000, seed=81)
    set_fragment(b, 0.05, seed=82)
    synth.add_ip_options(b, 0.05, seed=83)
    synth.inject_errors(b, 0.02, seed=84)
    for nports in (16, 7):
        cfg = N.make_cfg(offset=14, checksum=True, classify=N.CLS_LB_CRC, nports=nports)
        exp = oracle.process_batch(cfg, b)
        for part in (N.PART_GLOBAL, N.PART_TILE):
            got = device.process_batch(b, cfg, partition=part)
            compare(got, exp, ctx=f"lb_crc n={nports} part={part}")
        assert len(np.unique(exp["port"][exp["reason"] == N.R_OK])) == nports


def test_element_lb_crc_config():
    from fastclick_amd import click as K
    K.check_config("GPUIPCheckClassify(OFFSET 14, N 8, LB_MODE hash_crc)")
    with pytest.raises(K.ConfigError, match="hash_crc"):
        K.check_config("GPUIPCheckClassify(MODE AUTO, N 8, LB_MODE hash_crc)")
