"""Occupancy of the hot kernels, from the compiler's resource report (hipcc -Rpass-analysis=kernel-resource-usage,
CPU only).  Round 5 lost 15 us of decode3 to a silent VGPR increase (112 -> 129: three waves per SIMD instead of
four); these floors catch that at build time.  The floors are the occupancies the timings in DESIGN.md were
measured at."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "data-compression_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

FLOORS = {
    "dc_encode.hip": {r"encode_fused_kernelILi7ELb0E": 7},
    # every segment length the hot paths run (16: CT6 / CT11 and mid sizes; 20: CT5/CT7 above 2.5 M chunks, the
    # headline bench), and the dense-job decode3 instance
    # headline bench), and the dense-job decode3 instance.  parse3<7,20> holds 5 waves per SIMD (its 20-chunk
    # segments: 3971 jobs at 2^26 = 3.9 per SIMD, all resident in one round)
    "dc_decode3.hip": {r"parse3_kernelILi7ELi16E": 6, r"parse3_kernelILi7ELi20E": 5,
                       r"decode3_kernelILi7ELi(16|20)ELi1040E": 4, r"parse3_kernelILi6ELi16E": 6},
}


def _occupancy(src):
    out = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-gpu-rdc",
                          "-fPIC", "-c", os.path.join(CSRC, src), "-o", os.devnull,
                          "-Rpass-analysis=kernel-resource-usage"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    occ, name = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"Occupancy \[waves/SIMD\]: (\d+)", line)
        if m and name:
            occ[name] = int(m.group(1))
    return occ


@pytest.mark.skipif(not os.path.exists(HIPCC) and not shutil.which("hipcc"), reason="no hipcc")
@pytest.mark.parametrize("src", sorted(FLOORS))
def test_hot_kernel_occupancy(src):
    occ = _occupancy(src)
    for pat, floor in FLOORS[src].items():
        hits = {k: v for k, v in occ.items() if re.search(pat, k)}
        assert hits, f"{pat} not in the resource report of {src}"
        for k, v in hits.items():
            assert v >= floor, f"{k}: {v} waves per SIMD, below {floor}"
