"""Pin the CPU oracle's double codecs (oracle/dc_oracle64.c) to the reference's double KATs and to
golden vectors of the compiled reference (tests/golden/make_golden64.py)."""
import hashlib
import os

import numpy as np
import pytest

from conftest import BOUNDS, CASES64, GOLDEN, golden64


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES64)
def test_prepasses64(oracle, bound, case):
    g = golden64(bound)
    mn, xs = oracle.to_small64(g[f"{case}/input"])
    assert mn == g[f"{case}/min"]
    mean, t = oracle.med64(xs)
    assert mean == g[f"{case}/mean"] and t == g[f"{case}/type"]
    assert oracle.mask20(mean) == g[f"{case}/mask20"]


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES64)
@pytest.mark.parametrize("ct", [5, 6, 7, 11])
def test_encoder64_bit_exact(oracle, bound, case, ct):
    g = golden64(bound)
    _, xs = oracle.to_small64(g[f"{case}/input"])
    t, m20 = int(g[f"{case}/type"]), int(g[f"{case}/mask20"])
    s, nb, pos = oracle.compress64(ct, xs, bound, t, m20)
    ref = g[f"{case}/ct{ct}/stream"]
    assert nb == ref.size and pos == g[f"{case}/ct{ct}/pos"]
    assert np.array_equal(s, ref)


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES64)
@pytest.mark.parametrize("ct", [5, 6, 7, 11])
def test_decoder64(oracle, bound, case, ct):
    g = golden64(bound)
    key = f"{case}/ct{ct}"
    n = g[f"{case}/input"].size
    t, m20 = int(g[f"{case}/type"]), int(g[f"{case}/mask20"])
    spec, got = oracle.decompress64(ct, g[key + "/stream"], n, bound, t, m20)
    assert got == n
    if bool(g[key + "/ref_consistent"]):
        assert np.array_equal(spec.view(np.uint64), g[key + "/ref_decoded"].view(np.uint64))
    elif key + "/ref_decoded" in g:      # Q2: the reference never writes the last value
        ref = g[key + "/ref_decoded"]
        assert np.array_equal(spec[:-1].view(np.uint64), ref[:-1].view(np.uint64)) or case == "unit32k"


def test_quirk_cases_are_the_known_ones():
    """Only the Q1 analogue (CT7, mean in [2^-9, 0.5)) and Q2 (last m=0 token on a byte boundary)
    make the reference decoder disagree with the grammar."""
    for bound in BOUNDS:
        g = golden64(bound)
        bad = sorted(k[:-len("/ref_consistent")] for k in g if k.endswith("/ref_consistent") and not bool(g[k]))
        assert set(bad) <= {"unit32k/ct7", "eq16k/ct6", "q2/ct6", "q2/ct7", "eq16k/ct7"}, bad


@pytest.mark.parametrize("stem,ct,ext", [("testdouble_8_8_128", 6, "bnp"), ("testdouble_8_8_8_128", 11, "bop")])
def test_double_kats(oracle, stem, ct, ext):
    """impl/dataset/<stem>.txt.bc (CT6 / CT11 at 1e-6, after toSmallDataset_double) and the decoded
    text (%f of decoded + min) shipped in the reference tree."""
    x = np.fromfile(os.path.join(GOLDEN, f"kat64_{stem}.bi"), np.float64)
    kat = np.fromfile(os.path.join(GOLDEN, f"kat64_{stem}.bc"), np.uint8)
    mn, xs = oracle.to_small64(x)
    s, nb, pos = oracle.compress64(ct, xs, 1e-6)
    assert nb == kat.size and np.array_equal(s, kat)
    d, n = oracle.decompress64(ct, kat, x.size, 1e-6)
    assert n == x.size
    txt = "".join("%f\n" % v for v in d + mn).encode()
    ref = open(os.path.join(GOLDEN, f"kat64_{stem}.{ext}.txt"), "rb").read()
    assert hashlib.sha256(txt).hexdigest() == hashlib.sha256(ref).hexdigest()


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("ct", [5, 6, 11])
def test_append64(oracle, bound, ct):
    g = golden64(bound)
    xs = g["append/input"]
    s1, nb1, p1 = oracle.compress64(ct, xs[:333], bound)
    assert nb1 == g[f"append/ct{ct}/first_bytes"] and p1 == g[f"append/ct{ct}/first_pos"]
    s2, nb2, p2 = oracle.compress64(ct, xs[333:], bound, prefix=s1, prefix_pos=p1)
    assert np.array_equal(s2, g[f"append/ct{ct}/stream"]) and p2 == g[f"append/ct{ct}/pos"]



@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES64)
def test_ct1_double_oracle(oracle, bound, case):
    """myCompress_double (:3815) arrays of the oracle equal the compiled reference's; the decoder
    restores raws exactly and rebuilds codes from the decoded history."""
    g = golden64(bound)
    x = g[f"{case}/input"]
    raw, codes, pos = oracle.bytewise_compress64(x, bound)
    assert np.array_equal(raw.view(np.uint64), g[f"{case}/ct1/raw"].view(np.uint64))
    assert codes == g[f"{case}/ct1/codes"].tobytes() and np.array_equal(pos, g[f"{case}/ct1/pos"])
    d = oracle.bytewise_decompress64(raw, codes, pos, x.size)
    israw = np.ones(x.size, bool)
    israw[pos - 1] = False
    assert np.array_equal(d[israw].view(np.uint64), x[israw].view(np.uint64))
