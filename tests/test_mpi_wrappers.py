"""Float MPI send/recv wrappers (include/dc_mpi.h, data-compression_amd/csrc/dc_mpi.c): the float
counterparts of the reference's MPI_Send_bitwise_double / MPI_Recv_bitwise_double
(impl/dataCompression.c:226-353).  tests/native/mpi_wrapper_check.c sends one U10 buffer through each
pair (CT5/6/11/7) from rank 0 to rank 1 and compares what arrives bit for bit with the same round trip
done locally through the reference C ABI."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "data-compression_amd", "lib")
CHECK = os.path.join(LIB, "mpi_wrapper_check")
MPIRUN = "/opt/conda/bin/mpirun"
SYMS = [f"MPI_{d}_bitwise_float{s}" for d in ("Send", "Recv") for s in ("", "_np", "_op", "_mask")]


@pytest.mark.skipif(not os.path.isfile(os.path.join(LIB, "libdcamd_mpi.so")), reason="make -C data-compression_amd mpi")
def test_mpi_wrapper_exports():
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(LIB, "libdcamd_mpi.so")], capture_output=True,
                         text=True, check=True).stdout
    names = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    for s in SYMS:
        assert s in names, s
    hdr = open(os.path.join(ROOT, "include", "dc_mpi.h")).read()
    for s in SYMS:
        assert re.search(r"\b%s\s*\(" % s, hdr), s


@pytest.mark.gpu
@pytest.mark.skipif(not (os.path.isfile(CHECK) and os.path.isfile(MPIRUN)), reason="MPI wrapper check not built")
@pytest.mark.parametrize("n", [1 << 20, 4099])
def test_mpi_wrappers_round_trip(n):
    env = dict(os.environ, DC_ABS_ERROR_BOUND="0.001", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([MPIRUN, "-np", "2", CHECK, str(n)], capture_output=True, text=True, timeout=200, env=env)
    ok = re.findall(r"MPI_WRAPPER ct=(\d+) n=\d+ OK", r.stdout)
    assert r.returncode == 0 and sorted(ok) == ["11", "5", "6", "7"], r.stdout[-2000:] + r.stderr[-2000:]
