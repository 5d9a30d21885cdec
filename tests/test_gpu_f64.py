"""GPU parity of the DOUBLE codecs (dc_f64.hip through the reference C ABI
myCompress_bitwise_double* / myDecompress_bitwise_double*, impl/dataCompression.c:355-3308) against the
compiled reference's golden vectors, the reference's double KATs and the CPU oracle.  Bit-exact."""
import ctypes as C
import hashlib
import os

import numpy as np
import pytest

from conftest import BOUNDS, CASES64, GOLDEN, golden64

pytestmark = pytest.mark.gpu
CTS = [5, 6, 7, 11]


def _tm(g, case):
    return int(g[f"{case}/type"]), int(g[f"{case}/mask20"])


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES64)
def test_prepasses64_gpu(dc, bound, case):
    g = golden64(bound)
    mn, xs = dc.to_small64(g[f"{case}/input"])
    assert mn == g[f"{case}/min"]
    mean, t = dc.med64(xs)
    assert mean == g[f"{case}/mean"] and t == g[f"{case}/type"]


@pytest.mark.parametrize("kind", ["neg_zero_first", "zero_at_0", "nan_at_0", "nans", "inf", "snan"])
@pytest.mark.parametrize("n", [1, 5, 4097, (1 << 18) + 3])
def test_to_small64_edge_cases(dc, oracle, kind, n):
    """toSmallDataset_double bit for bit against the oracle (x86): signed zeros, NaN at data[0] and elsewhere
    (quieted payloads propagate through the subtraction), infinities (inf - inf: the default NaN)."""
    rs = np.random.RandomState(n)
    x = rs.rand(n) * 10 + 1
    if kind == "neg_zero_first" and n > 3:
        x[n // 2] = -0.0; x[n // 2 + 1::11] = 0.0
    elif kind == "zero_at_0":
        x[0] = 0.0; x[1::7] = -0.0
    elif kind == "nan_at_0":
        x[0] = np.nan; x[1::3] = -3.0
    elif kind == "nans":
        x[1::4] = np.nan; x[-1] = 0.5
    elif kind == "inf":
        x[::9] = np.inf; x[n // 3] = -np.inf
    elif kind == "snan":
        x[1::5] = np.nan
        x.view(np.uint64)[1::5] = np.uint64(0x7FF0000000000123)
    mn, xs = dc.to_small64(x)
    omn, oxs = oracle.to_small64(x)
    assert np.float64(mn).view(np.uint64) == np.float64(omn).view(np.uint64)
    assert np.array_equal(xs.view(np.uint64), oxs.view(np.uint64))


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES64)
@pytest.mark.parametrize("ct", CTS)
def test_encoder64_golden(dc, oracle, bound, case, ct):
    g = golden64(bound)
    dc.set_bound(bound)
    _, xs = oracle.to_small64(g[f"{case}/input"])
    t, m20 = _tm(g, case)
    s, nb, pos = dc.compress64(ct, xs, t, m20)
    ref = g[f"{case}/ct{ct}/stream"]
    assert nb == ref.size and pos == g[f"{case}/ct{ct}/pos"]
    assert np.array_equal(s, ref)


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES64)
@pytest.mark.parametrize("ct", CTS)
def test_decoder64_golden(dc, oracle, bound, case, ct):
    g = golden64(bound)
    dc.set_bound(bound)
    key = f"{case}/ct{ct}"
    s = g[key + "/stream"]
    n = g[f"{case}/input"].size
    t, m20 = _tm(g, case)
    out = dc.decompress64(ct, s, n, t, m20)
    spec, got = oracle.decompress64(ct, s, n, bound, t, m20)
    assert got == n
    assert np.array_equal(out.view(np.uint64), spec.view(np.uint64))
    if bool(g[key + "/ref_consistent"]):
        assert np.array_equal(out.view(np.uint64), g[key + "/ref_decoded"].view(np.uint64))


@pytest.mark.parametrize("stem,ct,ext", [("testdouble_8_8_128", 6, "bnp"), ("testdouble_8_8_8_128", 11, "bop")])
def test_double_kats_gpu(dc, stem, ct, ext):
    """The reference tree's double KATs: stream bytes and the decoded text (%f of decoded + min)."""
    dc.set_bound(1e-6)
    x = np.fromfile(os.path.join(GOLDEN, f"kat64_{stem}.bi"), np.float64)
    kat = np.fromfile(os.path.join(GOLDEN, f"kat64_{stem}.bc"), np.uint8)
    mn, xs = dc.to_small64(x)
    s, nb, pos = dc.compress64(ct, xs)
    assert nb == kat.size and np.array_equal(s, kat)
    d = dc.decompress64(ct, kat, x.size)
    txt = "".join("%f\n" % v for v in d + mn).encode()
    ref = open(os.path.join(GOLDEN, f"kat64_{stem}.{ext}.txt"), "rb").read()
    assert hashlib.sha256(txt).hexdigest() == hashlib.sha256(ref).hexdigest()


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("ct", [5, 6, 11])
def test_append64_gpu(dc, bound, ct):
    g = golden64(bound)
    dc.set_bound(bound)
    xs = g["append/input"]
    s1, nb1, p1 = dc.compress64(ct, xs[:333])
    assert nb1 == g[f"append/ct{ct}/first_bytes"] and p1 == g[f"append/ct{ct}/first_pos"]
    s2, nb2, p2 = dc.compress64(ct, xs[333:], prefix=s1, prefix_pos=p1)
    assert np.array_equal(s2, g[f"append/ct{ct}/stream"]) and p2 == g[f"append/ct{ct}/pos"]


def _inputs(oracle):
    rs = np.random.RandomState(5)
    n = 1 << 18
    return {
        "u10": oracle.gen_u10_64(n),
        "ramp": 0.37 * np.arange(n, dtype=np.float64),                       # '110' chains across chunks
        "const": np.full(n, 0.123456789),                                    # periodic '100' stream
        "runs": np.repeat(rs.rand(n // 500) * 7.0, 500),                     # '101' copies crossing chunks
        "mixed": np.concatenate([oracle.gen_u10_64(n // 4), np.full(n // 4, 2.5), np.arange(n // 4) * 1e-4,
                                 rs.rand(n // 4) * 1e9]),
    }


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("ct", CTS)
def test_roundtrip64_vs_oracle(dc, oracle, bound, ct):
    dc.set_bound(bound)
    for name, x in _inputs(oracle).items():
        mn, xs = oracle.to_small64(x)
        mean, t = oracle.med64(xs)
        m20 = oracle.mask20(mean)
        s, nb, pos = dc.compress64(ct, xs, t, m20)
        so, nbo, poso = oracle.compress64(ct, xs, bound, t, m20)
        assert nb == nbo and pos == poso and np.array_equal(s, so), name
        d = dc.decompress64(ct, s, xs.size, t, m20)
        ref, got = oracle.decompress64(ct, s, xs.size, bound, t, m20)
        assert got == xs.size
        assert np.array_equal(d.view(np.uint64), ref.view(np.uint64)), name


@pytest.mark.parametrize("ct", CTS)
def test_ragged64(dc, oracle, ct):
    bound = 1e-3
    dc.set_bound(bound)
    x = oracle.gen_u10_64(70000, seed=9)
    for n in (1, 2, 3, 4, 5, 63, 64, 65, 255, 1023, 1024, 1025, 2047, 4097, 65537):
        xs = np.ascontiguousarray(x[:n])
        s, nb, pos = dc.compress64(ct, xs, 2, 0x40000)
        so, nbo, poso = oracle.compress64(ct, xs, bound, 2, 0x40000)
        assert nb == nbo and pos == poso and np.array_equal(s, so), n
        d = dc.decompress64(ct, s, n, 2, 0x40000)
        ref, _ = oracle.decompress64(ct, s, n, bound, 2, 0x40000)
        assert np.array_equal(d.view(np.uint64), ref.view(np.uint64)), n


@pytest.mark.parametrize("ct", [5, 7, 11])
def test_sentinel_and_signed64(dc, oracle, ct):
    """-1.0 inputs (the encoder's history sentinel, :3191) take the exact serial encoder; negative values
    produce sign-1 raw tokens that parse as 3-bit codes -- both follow the reference bit for bit."""
    bound = 1e-3
    dc.set_bound(bound)
    rs = np.random.RandomState(3)
    x = rs.rand(5000) * 4.0 - 1.0
    x[[0, 7, 100, 2500]] = -1.0
    s, nb, pos = dc.compress64(ct, x, 2, 0x40000)
    so, nbo, poso = oracle.compress64(ct, x, bound, 2, 0x40000)
    assert nb == nbo and pos == poso and np.array_equal(s, so)
    d = dc.decompress64(ct, s, x.size, 2, 0x40000)
    ref, got = oracle.decompress64(ct, s, x.size, bound, 2, 0x40000)
    assert np.array_equal(d[:got].view(np.uint64), ref[:got].view(np.uint64))


def test_device_api64_chained(dc, oracle):
    """dc64_encode_device -> dc64_decode_device with the bit count handed over on the device."""
    import torch
    bound = 1e-3
    dc.set_bound(bound)
    n = 1 << 20
    x = oracle.gen_u10_64(n)
    mn, xs = oracle.to_small64(x)
    mean, t = oracle.med64(xs)
    m20 = oracle.mask20(mean)
    dx = torch.from_numpy(xs).cuda()
    cap = int(dc.L.dc64_stream_capacity(n))
    st = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    nbits = torch.zeros(1, dtype=torch.int64, device="cuda")
    out = torch.empty(n, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    dc.encode64_device(7, dx.data_ptr(), n, st.data_ptr(), t, m20, total_ptr=nbits.data_ptr())
    dc.decode64_device(7, st.data_ptr(), -1, n, out.data_ptr(), t, m20, d_nbits=nbits.data_ptr(), max_bytes=cap)
    flags = dc.decode64_finish()
    nb = dc.encode64_result()
    so, nbo, _ = oracle.compress64(7, xs, bound, t, m20)
    assert (nb + 7) // 8 == nbo and np.array_equal(st[:nbo].cpu().numpy(), so)
    ref, _ = oracle.decompress64(7, so, n, bound, t, m20)
    assert np.array_equal(out.cpu().numpy().view(np.uint64), ref.view(np.uint64))
    assert flags == 0                        # the parallel path decoded it (no exact serial fallback)


def test_decode64_paths(dc, oracle, monkeypatch):
    """Random data decodes on the speculative-entry path (flags 0); the chunk-map path (forced with
    DC64_FORCE_MAP=1, taken by itself when link repair does not converge) decodes the same streams --
    U10, a constant input (periodic '100' stream) and '101' runs -- bit-exactly."""
    bound = 1e-3
    dc.set_bound(bound)
    rs = np.random.RandomState(8)
    cases = [oracle.gen_u10_64(1 << 19), np.full(1 << 19, 0.123456789), np.repeat(rs.rand(1 << 10) * 7.0, 512)]
    for force in ("0", "1"):
        monkeypatch.setenv("DC64_FORCE_MAP", force)
        for i, x in enumerate(cases):
            mn, xs = oracle.to_small64(x)
            s, nb, pos = dc.compress64(5, xs)
            d = dc.decompress64(5, s, xs.size)
            flags = int(dc.L.dc64_last_decode_flags())
            ref, _ = oracle.decompress64(5, s, xs.size, bound)
            assert np.array_equal(d.view(np.uint64), ref.view(np.uint64)), (force, i)
            if force == "1":
                assert flags & 2, flags
            elif i == 0:
                assert flags == 0, flags


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES64)
def test_ct1_double_gpu(dc, oracle, bound, case):
    """myCompress_double / myDecompress_double on the GPU: arrays equal the compiled reference's
    (golden), the decode equals the oracle's bit for bit."""
    g = golden64(bound)
    dc.set_bound(bound)
    x = g[f"{case}/input"]
    raw, codes, pos = dc.ct1_compress64(x)
    assert np.array_equal(raw.view(np.uint64), g[f"{case}/ct1/raw"].view(np.uint64))
    assert codes == g[f"{case}/ct1/codes"].tobytes() and np.array_equal(pos, g[f"{case}/ct1/pos"])
    d = dc.ct1_decompress64(raw, codes, pos, x.size)
    ref = oracle.bytewise_decompress64(raw, codes, pos, x.size)
    assert np.array_equal(d.view(np.uint64), ref.view(np.uint64))


def test_ct1_double_large(dc, oracle):
    bound = 1e-3
    dc.set_bound(bound)
    rs = np.random.RandomState(4)
    x = np.concatenate([oracle.gen_u10_64(1 << 18), np.arange(1 << 17) * 0.25, np.repeat(rs.rand(256), 512)])
    raw, codes, pos = dc.ct1_compress64(x)
    r2, c2, p2 = oracle.bytewise_compress64(x, bound)
    assert np.array_equal(raw.view(np.uint64), r2.view(np.uint64)) and codes == c2 and np.array_equal(pos, p2)
    d = dc.ct1_decompress64(raw, codes, pos, x.size)
    assert np.array_equal(d.view(np.uint64), oracle.bytewise_decompress64(raw, codes, pos, x.size).view(np.uint64))


@pytest.mark.parametrize("kind,n", [("u10", 1 << 24), ("u10", 1 << 26), ("ramp", 1 << 21), ("signed", 1 << 20),
                                    ("nan", 100003), ("zeros", 1 << 22), ("wide", 1 << 20), ("tiny", 1 << 20)])
def test_med64_exact_parallel(dc, oracle, kind, n):
    """med_dataset_double's left-to-right double sum (impl/dataCompression.c:3564-3590) by the binade-
    transducer kernels (dc_aux.hip) must equal the serial sum bit for bit (mean and type)."""
    import torch
    rs = np.random.RandomState(n % 997)
    if kind == "u10":
        x = oracle.gen_u10_64(n)
    elif kind == "ramp":
        x = np.arange(n, dtype=np.float64) * 0.0005
    elif kind == "signed":
        x = rs.randn(n) * 3
    elif kind == "nan":
        x = oracle.gen_u10_64(n)
        x[n // 3] = np.nan
    elif kind == "zeros":
        x = np.zeros(n)
        x[::7919] = -0.0
    elif kind == "wide":
        x = rs.rand(n) * np.exp2(rs.randint(-200, 200, n).astype(np.float64))
    else:
        x = rs.rand(n) * 1e-300
    d = torch.from_numpy(np.ascontiguousarray(x, np.float64)).cuda()
    torch.cuda.synchronize()
    mean = C.c_double(0)
    t = C.c_int(0)
    dc.check(dc.L.dc64_med_device(C.c_void_p(d.data_ptr()), n, C.byref(mean), C.byref(t)), "dc64_med_device")
    om, ot = oracle.med64(x)
    assert np.array_equal(np.float64(mean.value).view(np.uint64), np.float64(om).view(np.uint64)), (mean.value, om)
    assert t.value == ot
