"""The fused pre-passes (dc_prep_device: toSmallDataset_float's minimum and med_dataset_float of x - min, without
writing x - min) and the encode of x - min made while loading x (dc_encode_sub_device), against the oracle's
separate passes (impl/dataCompression.c:3543-3562 toSmallDataset_float, :3593-3620 med_dataset_float, then the
encoder of :2030-2284 on data_small) -- bit for bit: minimum, mean, type, stream bytes and length."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _x(oracle, kind, n):
    rs = np.random.RandomState(n % 991)
    if kind == "u10":
        return oracle.gen_u10(n)
    if kind == "shifted":                          # a negative minimum: x - min moves every binade
        return (oracle.gen_u10(n) - np.float32(7.25)).astype(np.float32)
    if kind == "ramp":
        return (np.float32(0.0005) * np.arange(n, dtype=np.float32) + np.float32(3.0)).astype(np.float32)
    if kind == "signed":
        return (rs.randn(n) * 3).astype(np.float32)
    if kind == "wide":                             # exponents over ~60 binades
        return (rs.rand(n) * np.exp2(rs.randint(-30, 30, n))).astype(np.float32)
    x = (rs.rand(n) * 10 + 1).astype(np.float32)
    m = n // 2
    if kind == "min_first":
        x[0] = -5.0
    elif kind == "zero_min":                       # the minimum is a zero: the first one's sign
        x[m] = -0.0; x[m + 1::11] = 0.0
    elif kind == "nans":
        x[1::97] = np.nan; x[min(5, n - 1)] = -2.0
    elif kind == "snan":
        x.view(np.uint32)[3::101] = np.uint32(0x7F800123)
    elif kind == "inf":                            # +inf values, finite minimum: x - min = +inf there
        x[::501] = np.inf
    elif kind == "equal":                          # every chunk all zeros after the subtraction
        x[:] = 2.5
    elif kind == "zero_prefix":
        x[: n // 3] = 1.0; x[n // 3] = 0.5
    elif kind == "nan_at_0":                       # non-finite minimum: the separate passes
        x[0] = np.nan
    elif kind == "neg_inf":
        x[n // 3] = -np.inf
    elif kind == "minus_one":                      # x - min = -1.0f nowhere, but a -1 input is fine after it
        x[::7] = -1.0
    return x


KINDS = ["u10", "shifted", "ramp", "signed", "wide", "min_first", "zero_min", "nans", "snan", "inf", "equal",
         "zero_prefix", "nan_at_0", "neg_inf", "minus_one"]


@pytest.mark.parametrize("n", [1, 5, 4097, (1 << 20) + 3])
@pytest.mark.parametrize("kind", KINDS)
def test_prep_matches_separate_passes(dc, oracle, kind, n):
    import torch
    x = _x(oracle, kind, n)
    d = torch.from_numpy(x).cuda()
    torch.cuda.synchronize()
    mn, mean, t = dc.prep_device(d.data_ptr(), n)
    omn, xs = oracle.to_small(x)
    om, ot = oracle.med(xs)
    assert np.float32(mn).view(np.uint32) == np.float32(omn).view(np.uint32), (mn, omn)
    assert np.float32(mean).view(np.uint32) == np.float32(om).view(np.uint32), (mean, om)
    assert t == ot


@pytest.mark.parametrize("kind,n", [("u10", 1 << 22), ("wide", 1 << 20), ("shifted", (1 << 20) + 77)])
def test_prep_windows(dc, oracle, kind, n, monkeypatch):
    """the narrow binade window and the forced wide one (DC_MED_WIDE=1) on the fused statistics"""
    import torch
    x = _x(oracle, kind, n)
    d = torch.from_numpy(x).cuda()
    torch.cuda.synchronize()
    omn, xs = oracle.to_small(x)
    om, ot = oracle.med(xs)
    for force in ("0", "1"):
        monkeypatch.setenv("DC_MED_WIDE", force)
        mn, mean, t = dc.prep_device(d.data_ptr(), n)
        assert np.float32(mean).view(np.uint32) == np.float32(om).view(np.uint32), (force, mean, om)
        assert t == ot and np.float32(mn) == np.float32(omn)


def _encode_sub(dc, d, n, mn, ct, t, m17):
    import torch
    st = torch.zeros(dc.stream_capacity(n), dtype=torch.uint8, device="cuda")
    dc.encode_sub_device(ct, d.data_ptr(), n, mn, st.data_ptr(), type_=t, mask17=m17)
    bits = dc.encode_result()
    nb = (bits + 7) // 8
    return st[:nb].cpu().numpy(), nb, bits


@pytest.mark.parametrize("ct", [5, 6, 7, 11])
@pytest.mark.parametrize("kind,n", [("u10", 1 << 20), ("shifted", 300001), ("ramp", 200000), ("nans", 100003),
                                    ("min_first", 4097), ("equal", 70000), ("zero_min", 65537), ("nan_at_0", 5000),
                                    ("inf", 9001), ("u10", 5)])
def test_encode_sub_matches_oracle(dc, oracle, ct, kind, n):
    import torch
    dc.set_bound(1e-3)
    x = _x(oracle, kind, n)
    d = torch.from_numpy(x).cuda()
    torch.cuda.synchronize()
    mn, mean, t = dc.prep_device(d.data_ptr(), n)
    omn, xs = oracle.to_small(x)
    if ct in (5, 7, 11) and (np.isnan(xs).any() or (xs < 0).any() or (xs == -1.0).any()):
        pytest.skip("outside the codec's domain (the reference's -1.0f sentinel / negative inputs)")
    if ct == 7 and not 1 <= t <= 7:
        pytest.skip("CT7 needs a type in 1..7 (an infinite maximum gives 0)")
    m17 = oracle.mask17(mean) if ct == 7 else 0
    t = t if ct == 7 else 0
    s, nb, bits = _encode_sub(dc, d, n, mn, ct, t, m17)
    so, nbo, poso = oracle.compress(ct, xs, 1e-3, t, m17)
    assert nb == nbo and np.array_equal(s, so)


def test_encode_sub_other_variants(dc, oracle):
    """the variants that do not subtract while loading (here the helping instantiation; also the count + pack
    launches and the wait-free retry) take x - min written out first: the same stream"""
    import torch
    dc.set_bound(1e-3)
    n = (1 << 20) + 5
    x = _x(oracle, "shifted", n)
    d = torch.from_numpy(x).cuda()
    torch.cuda.synchronize()
    mn, mean, t = dc.prep_device(d.data_ptr(), n)
    omn, xs = oracle.to_small(x)
    m17 = oracle.mask17(mean)
    s1, nb1, _ = _encode_sub(dc, d, n, mn, 7, t, m17)
    ds = torch.from_numpy(xs).cuda()
    st = torch.zeros(dc.stream_capacity(n), dtype=torch.uint8, device="cuda")
    dc.encode_device(7, ds.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17)
    bits = dc.encode_result()
    assert nb1 == (bits + 7) // 8 and np.array_equal(s1, st[:nb1].cpu().numpy())
    prev = dc.L.dc_set_encode_help(1)                          # the helping instantiation: written out first
    try:
        s2, nb2, _ = _encode_sub(dc, d, n, mn, 7, t, m17)
    finally:
        dc.L.dc_set_encode_help(prev)
    assert nb2 == nb1 and np.array_equal(s2, s1)


def test_prep_chain_u10_2p26_vs_oracle(dc, oracle):
    """The bench workload through the fused chain (raw U10 2^26 floats in HBM): minimum, mean, type and the stream of
    x - min equal the oracle's separate passes (toSmallDataset_float, med_dataset_float, the CT7 encoder)."""
    import torch
    dc.set_bound(1e-3)
    n = 1 << 26
    x = oracle.gen_u10(n)
    d = torch.from_numpy(x).cuda()
    torch.cuda.synchronize()
    mn, mean, t = dc.prep_device(d.data_ptr(), n)
    omn, xs = oracle.to_small(x)
    om, ot = oracle.med(xs)
    assert np.float32(mn) == np.float32(omn) and np.float32(mean).view(np.uint32) == np.float32(om).view(np.uint32)
    assert t == ot
    m17 = oracle.mask17(mean)
    s, nb, bits = _encode_sub(dc, d, n, mn, 7, t, m17)
    del d
    torch.cuda.empty_cache()
    so, nbo, _ = oracle.compress(7, xs, 1e-3, t, m17)
    assert nb == nbo == 162634383 and np.array_equal(s, so)


def test_prep_chain_u10_2p28_vs_golden_hash(dc, oracle):
    """2^28 raw floats (the sweep's largest size): the fused chain's stream has the oracle's bit count and hash
    (tests/golden/bench_hashes.json, tests/golden/make_bench_hashes.py)"""
    import json, os
    import torch
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bench_hashes.json")))["ct7_u10_2^28_0.001_w1"]
    dc.set_bound(1e-3)
    n = 1 << 28
    d = torch.from_numpy(oracle.gen_u10(n)).cuda()
    torch.cuda.synchronize()
    mn, mean, t = dc.prep_device(d.data_ptr(), n)
    m17 = oracle.mask17(mean)
    st = torch.zeros(dc.stream_capacity(n), dtype=torch.uint8, device="cuda")
    dc.encode_sub_device(7, d.data_ptr(), n, mn, st.data_ptr(), type_=t, mask17=m17)
    bits = dc.encode_result()
    h = dc.hash_device(st.data_ptr(), (bits + 7) // 8)
    del d, st
    torch.cuda.empty_cache()
    assert bits == int(g["nbits"]) and h == int(g["stream"])
