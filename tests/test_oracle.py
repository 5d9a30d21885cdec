"""Pin the CPU oracle (oracle/dc_oracle.c) to the reference's golden vectors and KATs.

Fixtures were produced by the compiled reference impl/dataCompression.c (tests/golden/make_golden.py).
"""
import os

import numpy as np
import pytest

from conftest import BOUNDS, CASES, GOLDEN, golden


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES)
def test_prepasses(oracle, bound, case):
    g = golden(bound)
    x = g[f"{case}/input"]
    mn, xs = oracle.to_small(x)
    assert mn == g[f"{case}/min"]
    mean, t = oracle.med(xs)
    assert mean == g[f"{case}/mean"] and t == g[f"{case}/type"]
    assert oracle.mask17(mean) == g[f"{case}/mask17"]


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("ct", [5, 6, 7, 11])
def test_encoder_bit_exact(oracle, bound, case, ct):
    g = golden(bound)
    _, xs = oracle.to_small(g[f"{case}/input"])
    t, m17 = int(g[f"{case}/type"]), int(g[f"{case}/mask17"])
    s, nb, pos = oracle.compress(ct, xs, bound, t, m17)
    ref = g[f"{case}/ct{ct}/stream"]
    assert nb == ref.size and pos == g[f"{case}/ct{ct}/pos"]
    assert np.array_equal(s, ref)


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("ct", [5, 6, 7, 11])
def test_decoders(oracle, bound, case, ct):
    g = golden(bound)
    key = f"{case}/ct{ct}"
    s = g[key + "/stream"]
    n = g[f"{case}/input"].size
    t, m17 = int(g[f"{case}/type"]), int(g[f"{case}/mask17"])
    spec, got = oracle.decompress(ct, s, n, bound, t, m17)
    assert got == n
    if key + "/ref_decoded" in g:
        ref = g[key + "/ref_decoded"]
        cref, nc, stuck = oracle.decompress_cref(ct, s, n, bound, t, m17)
        # the faithful restatement reproduces every element the reference writes
        assert np.array_equal(cref[:nc].view(np.uint32), ref[:nc].view(np.uint32))
        if bool(g[key + "/ref_consistent"]):
            assert np.array_equal(spec.view(np.uint32), ref.view(np.uint32))
            assert nc == n and stuck == 0


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES)
def test_bytewise_ct1(oracle, bound, case):
    g = golden(bound)
    x = g[f"{case}/input"]
    raw, codes, pos = oracle.bytewise_compress(x, bound)
    assert np.array_equal(raw.view(np.uint32), g[f"{case}/ct1/raw"].view(np.uint32))
    assert codes == g[f"{case}/ct1/codes"].tobytes()
    assert np.array_equal(pos, g[f"{case}/ct1/pos"])
    dec = oracle.bytewise_decompress(raw, codes, pos, x.size)
    # raw elements come back verbatim
    israw = np.ones(x.size, bool)
    israw[pos - 1] = False
    assert np.array_equal(dec[israw], x[israw])


@pytest.mark.parametrize("bound", BOUNDS)
def test_crc32(oracle, bound):
    import zlib
    g = golden(bound)
    for case in CASES:
        for ct in (5, 6, 7, 11):
            s = g[f"{case}/ct{ct}/stream"]
            assert oracle.crc32(s) == g[f"{case}/ct{ct}/crc"] == zlib.crc32(s.tobytes())


@pytest.mark.parametrize("bound", BOUNDS)
def test_hamming(oracle, bound):
    g = golden(bound)
    s = g["hamming/stream"]
    bs = int(g["hamming/block_size"])
    assert oracle.block_size(s.size, 1e-6) == bs == 125000
    nblk = (s.size + bs - 1) // bs
    for i in range(nblk):
        blk = s[i * bs: min(s.size, (i + 1) * bs)]
        r, c = oracle.hamming_encode(blk)
        assert r == g[f"hamming/r{i}"] and c == g[f"hamming/c{i}"].tobytes()
        t, fixed, c2, _ = oracle.hamming_decode(blk, c, r)
        assert t == 0 and np.array_equal(fixed, blk)
        bad = blk.copy()
        bad[1234] ^= 0x10
        t, fixed, c2, _ = oracle.hamming_decode(bad, c, r)
        assert t == 3 and np.array_equal(fixed, blk)
        bad[777] ^= 0x01
        t, _, _, _ = oracle.hamming_decode(bad, c, r)
        assert t == 1
        cp = bytearray(c)
        cp[r] ^= 1
        t, fixed, c3, _ = oracle.hamming_decode(blk, bytes(cp), r)
        assert t == 2 and c3 == c


@pytest.mark.parametrize("bound", BOUNDS)
def test_append_mode(oracle, bound):
    g = golden(bound)
    xs = g["append/input"]
    for ct in (5, 6, 11):
        s1, nb1, pos1 = oracle.compress(ct, xs[:333], bound)
        assert nb1 == g[f"append/ct{ct}/first_bytes"] and pos1 == g[f"append/ct{ct}/first_pos"]
        s2, nb2, pos2 = oracle.compress(ct, xs[333:], bound, prefix=s1, prefix_pos=pos1)
        assert np.array_equal(s2, g[f"append/ct{ct}/stream"]) and pos2 == g[f"append/ct{ct}/pos"]


def test_kat_testfloat(oracle):
    """impl/dataset/testfloat_8_8_128.txt.bc is the reference's own CT5 stream at 1e-6."""
    x = np.loadtxt(os.path.join(GOLDEN, "kat_testfloat_8_8_128.txt"), dtype=np.float32)
    kat = np.fromfile(os.path.join(GOLDEN, "kat_testfloat_8_8_128.txt.bc"), np.uint8)
    mn, xs = oracle.to_small(x)
    s, nb, pos = oracle.compress(5, xs, 1e-6)
    assert np.array_equal(s, kat)
    dec, n = oracle.decompress(5, kat, x.size, 1e-6)
    txt = open(os.path.join(GOLDEN, "kat_testfloat_8_8_128.txt.bc.txt")).read().split()
    assert txt == ["%f" % v for v in (dec + mn).astype(np.float32)]
    assert abs(nb * 8 / (x.size * 32) - 1 / 1.392546) < 1e-6     # impl/pingpong.csv:36


def test_kat_float_eq(oracle):
    kat = np.fromfile(os.path.join(GOLDEN, "kat_float_eq_8192.txt.bc"), np.uint8)
    x = np.full(8192, np.float32(0.123456789))
    _, xs = oracle.to_small(x)
    for ct in (5, 11):
        s, nb, pos = oracle.compress(ct, xs, 1e-6)
        assert np.array_equal(s, kat)


def test_thresholds(oracle):
    lt, le = oracle.thr(1e-3)
    assert np.float32(lt) < 1e-3 <= np.nextafter(np.float32(lt), np.float32(1))
    assert oracle.bound_binary(1e-3) == 10 and oracle.bound_binary(1e-6) == 20


def test_u10_generator(oracle):
    from pyoracle import gen_u10_np
    for off in (0, 12345):
        assert np.array_equal(oracle.gen_u10(4096, 42, off), gen_u10_np(4096, 42, off))
