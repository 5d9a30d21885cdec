"""The reference's float MPI applications linked unchanged against libdcamd (SURVEY 8(b) link closure,
BASELINE configs[0]: pingpong CT7 @1e-3 on a 16384-float buffer under mpirun -np 2).

oracle/build_apps.sh compiles impl/pingpong.c and impl/himenoBMTxps.c from /root/reference (in this
container only) into oracle/_ref/apps/: `<app>_ref` with the reference codec compiled in, `<app>_dcamd`
with this repo's include/dataCompression.h and -ldcamd.  The binaries travel to the GPU box with the
tree; the reference sources do not.  On the GPU box both pingpong builds run the same input and must
print the same compression ratio and the same round-trip error (`gosa`) for every deterministic CT
(1/5/6/7/11; 8/9/10 flip random bits seeded by time()).

himenoBMTxps is link-checked only: with impl/param.h's two z-ranks each rank "receives" a halo from
MPI_PROC_NULL at the physical boundary, decompresses a 0-byte stream and copies the never-written
result (plus an uninitialised min) into p (impl/himenoBMTxps.c:644-706), so even the reference build
prints a different Gosa on every run (inf, 2.8e20, 3.4e7 in three runs here) -- no fixed output to
compare against."""
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APPS = os.path.join(ROOT, "oracle", "_ref", "apps")
MPIRUN = "/opt/conda/bin/mpirun"
HAVE_REF = os.path.isfile("/root/reference/impl/pingpong.c") and os.path.isfile("/opt/conda/bin/mpicc")


def _app(name):
    return os.path.join(APPS, name)


@pytest.mark.skipif(not HAVE_REF, reason="reference sources / mpicc not present (GPU box)")
def test_apps_link_unchanged():
    """pingpong and himenoBMTxps compile and link against include/ + libdcamd with no source change."""
    subprocess.check_call([os.path.join(ROOT, "oracle", "build_apps.sh")], stdout=subprocess.DEVNULL,
                          stderr=subprocess.DEVNULL)
    for app in ("pingpong", "himenoBMTxps", "k-means", "mm", "lu"):
        exe = _app(app + "_dcamd")
        assert os.path.isfile(exe), exe
        undef = subprocess.run(["nm", "-u", exe], capture_output=True, text=True, check=True).stdout
        # every codec symbol the app needs comes from libdcamd, none from a reference object
        exported = set()
        for so in ("libdcamd.so", "libdcamd_mpi.so"):
            lib = subprocess.run(["nm", "-D", "--defined-only",
                                  os.path.join(ROOT, "data-compression_amd", "lib", so)],
                                 capture_output=True, text=True, check=True).stdout
            exported |= {ln.split()[-1] for ln in lib.splitlines() if ln.strip()}
        for sym in re.findall(r"\bU (\S+)", undef):
            s = sym.split("@")[0]
            if re.match(r"(my|toSmall|med_|do_crc|hamming|bit_flip|block_size|floattostr|doubletostr|get_random|"
                        r"transform_|readfrombinary|writetobinary|MPI_Bcast_bitwise|MPI_Send_bitwise|MPI_Recv_bitwise)", s):
                assert s in exported, s


def _run_pingpong(exe, ct, path, env):
    # the app copies argv[2] into a char[64] (impl/pingpong.c:79-81): run in its directory, short name
    r = subprocess.run([MPIRUN, "-np", "2", exe, str(ct), os.path.basename(path)], capture_output=True, text=True,
                       timeout=120, env=env, cwd=os.path.dirname(path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return r.stdout


def _metrics(out):
    rate = re.findall(r"Compression rate \(([a-z_]+)\): ([0-9.]+)", out)
    gosa = re.findall(r"gosa = ([0-9.eE+-]+)", out)
    return rate, gosa


@pytest.mark.gpu
@pytest.mark.skipif(not (os.path.isfile(_app("pingpong_dcamd")) and os.path.isfile(MPIRUN)),
                    reason="oracle/_ref/apps not built (run oracle/build_apps.sh where /root/reference exists)")
@pytest.mark.parametrize("ct", [1, 5, 6, 7, 11])
def test_pingpong_dcamd_matches_reference(ct, tmp_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
    import dcamd
    x = dcamd.gen_u10(16384)                              # configs[0]: U10 2^14, %.9g round-trips fscanf
    path = str(tmp_path / "u10.txt")
    with open(path, "w") as f:
        f.write("".join("%.9g\n" % v for v in x))
    env = dict(os.environ, DC_ABS_ERROR_BOUND="0.001", HSA_ENABLE_IPC_MODE_LEGACY="0")
    out_ref = _run_pingpong(_app("pingpong_ref"), ct, path, env)
    out_gpu = _run_pingpong(_app("pingpong_dcamd"), ct, path, env)
    rr, gr = _metrics(out_ref)
    rg, gg = _metrics(out_gpu)
    assert (rr or ct == 1) and gr, out_ref[-1500:]     # CT1 prints no bit-wise rate line
    assert rr == rg, (out_ref[-1500:], out_gpu[-1500:])
    assert gr == gg, (out_ref[-1500:], out_gpu[-1500:])



@pytest.mark.gpu
@pytest.mark.skipif(not (os.path.isfile(_app("k-means_dcamd")) and os.path.isfile(MPIRUN)),
                    reason="oracle/_ref/apps not built (run oracle/build_apps.sh where /root/reference exists)")
@pytest.mark.parametrize("ct", [5, 6, 7, 8, 9])
def test_kmeans_dcamd_matches_reference(ct, tmp_path):
    """impl/k-means.c unchanged: 1000 iterations broadcasting 100 cluster centres (x and y) per iteration
    through the double codecs (CT5/6/7) and MPI_Bcast_bitwise_crc / _mask_crc (CT8/9), on
    impl/dataset/testfloat_8_8_128.txt.  Both builds print the same mean error (gosa) and compression
    ratio (CT8/9 resend counts are random, seeded by time(), as in the reference)."""
    ds = tmp_path / "dataset"
    ds.mkdir()
    shutil.copyfile(os.path.join(ROOT, "tests", "golden", "kat_testfloat_8_8_128.txt"), ds / "testfloat_8_8_128.txt")
    env = dict(os.environ, DC_ABS_ERROR_BOUND="0.001", HSA_ENABLE_IPC_MODE_LEGACY="0")
    outs = []
    for exe in (_app("k-means_ref"), _app("k-means_dcamd")):
        r = subprocess.run([MPIRUN, "-np", "2", exe, str(ct)], capture_output=True, text=True, timeout=300, env=env,
                           cwd=str(tmp_path))
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        outs.append((re.findall(r"gosa = ([0-9.eE+-]+)", r.stdout), re.findall(r"compress ratio = ([0-9.eE+-]+)", r.stdout)))
    assert outs[0][0] and outs[0][1], outs
    assert outs[0] == outs[1], outs
