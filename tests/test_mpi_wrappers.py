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
SYMS += [f"MPI_{d}_bitwise_double{s}{c}" for d in ("Send", "Recv") for s in ("", "_np", "_op") for c in ("", "_cn")]
SYMS += ["MPI_Bcast_bitwise_double", "MPI_Bcast_bitwise_crc", "MPI_Bcast_bitwise_mask_crc", "MPI_Bcast_bitwise_crc_hamming"]
CHECK64 = os.path.join(LIB, "mpi_wrapper_check64")


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


@pytest.mark.gpu
@pytest.mark.skipif(not (os.path.isfile(CHECK64) and os.path.isfile(MPIRUN)), reason="MPI wrapper check not built")
@pytest.mark.parametrize("n,ber", [(1 << 20, "0"), (1 << 20, "1e-6"), (4099, "0")])
def test_mpi_double_wrappers(n, ber):
    """The reference's double wrappers (dc_mpi64.c): send/recv (+ _cn) equal the local round trip bit for
    bit; MPI_Bcast_bitwise_double and the CRC / Hamming broadcasts deliver the clean decode to rank 1 -- with DC_BER=1e-6 through
    simulated CRC failures and resends (CT8/9) and real bit flips + Hamming correction / resend (CT10)."""
    env = dict(os.environ, DC_ABS_ERROR_BOUND="0.001", HSA_ENABLE_IPC_MODE_LEGACY="0", DC_BER=ber)
    r = subprocess.run([MPIRUN, "-np", "2", CHECK64, str(n)], capture_output=True, text=True, timeout=200, env=env)
    ok = re.findall(r"MPI_WRAPPER64 (\w+) ct=(\d+) n=\d+ OK", r.stdout)
    assert r.returncode == 0 and len(ok) == 10, r.stdout[-2000:] + r.stderr[-2000:]
