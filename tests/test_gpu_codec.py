"""GPU parity: libdcamd (gfx950 kernels, called through the reference C ABI) vs the golden
vectors of the compiled reference and the CPU oracle.  Integer/byte work -> bit-exact."""
import numpy as np
import pytest

from conftest import BOUNDS, CASES, golden

pytestmark = pytest.mark.gpu
CTS = [5, 6, 7, 11]


def _prep(g, case):
    return int(g[f"{case}/type"]), int(g[f"{case}/mask17"])


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES)
def test_prepasses_gpu(dc, bound, case):
    g = golden(bound)
    x = g[f"{case}/input"]
    mn, xs = dc.to_small(x)
    assert mn == g[f"{case}/min"]
    mean, t = dc.med(xs)
    assert mean == g[f"{case}/mean"] and t == g[f"{case}/type"]


@pytest.mark.parametrize("kind", ["pos_zero_first", "neg_zero_first", "zero_at_0", "neg_zero_at_0", "nan_at_0",
                                  "nans", "inf", "neg", "all_nan_tail", "equal", "snan"])
@pytest.mark.parametrize("n", [1, 2, 5, 4097, 1 << 20, (1 << 20) + 3])
def test_to_small_edge_cases(dc, oracle, kind, n):
    """toSmallDataset_float's minimum (impl/dataCompression.c: data[0], replaced only by a strictly smaller
    value, NaNs never) bit for bit against the oracle: signed zeros (the first zero's sign wins when the
    minimum is zero), NaN at data[0] and elsewhere, infinities, negatives, ragged sizes."""
    rs = np.random.RandomState(n)
    x = (rs.rand(n).astype(np.float32) * 10 + 1).astype(np.float32)
    m = n // 2
    if kind == "pos_zero_first" and n > 3:
        x[m] = 0.0; x[m + 1:] = np.where(rs.rand(n - m - 1) < 0.01, np.float32(-0.0), x[m + 1:])
    elif kind == "neg_zero_first" and n > 3:
        x[m] = -0.0; x[m + 1:] = np.where(rs.rand(n - m - 1) < 0.01, np.float32(0.0), x[m + 1:])
    elif kind == "zero_at_0":
        x[0] = 0.0; x[1::7] = -0.0
    elif kind == "neg_zero_at_0":
        x[0] = -0.0; x[1::5] = 0.0
    elif kind == "nan_at_0":
        x[0] = np.nan; x[1::3] = -3.0
    elif kind == "nans":
        x[1::4] = np.nan; x[-1] = 0.5
    elif kind == "inf":
        x[::9] = np.inf; x[n // 3] = -np.inf
    elif kind == "neg":
        x -= 20.0; x[-1] = -100.0
    elif kind == "all_nan_tail":
        x[1:] = np.nan
    elif kind == "equal":
        x[:] = 2.5
    elif kind == "snan":                                  # signalling NaNs with payloads: quieted, kept
        x.view(np.uint32)[1::5] = np.uint32(0x7F800123)
    mn, xs = dc.to_small(x)
    omn, oxs = oracle.to_small(x)
    assert np.float32(mn).view(np.uint32) == np.float32(omn).view(np.uint32)
    assert np.array_equal(xs.view(np.uint32), oxs.view(np.uint32))


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("ct", CTS)
def test_encoder_golden(dc, oracle, bound, case, ct):
    g = golden(bound)
    dc.set_bound(bound)
    _, xs = oracle.to_small(g[f"{case}/input"])
    t, m17 = _prep(g, case)
    s, nb, pos = dc.compress(ct, xs, t, m17)
    ref = g[f"{case}/ct{ct}/stream"]
    assert nb == ref.size and pos == g[f"{case}/ct{ct}/pos"]
    assert np.array_equal(s, ref)


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("ct", CTS)
def test_decoder_golden(dc, oracle, bound, case, ct):
    g = golden(bound)
    dc.set_bound(bound)
    key = f"{case}/ct{ct}"
    s = g[key + "/stream"]
    n = g[f"{case}/input"].size
    t, m17 = _prep(g, case)
    out = dc.decompress(ct, s, n, t, m17)
    spec, got = oracle.decompress(ct, s, n, bound, t, m17)
    assert got == n
    assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))
    if bool(g[key + "/ref_consistent"]):
        assert np.array_equal(out.view(np.uint32), g[key + "/ref_decoded"].view(np.uint32))


@pytest.mark.parametrize("bound", BOUNDS)
def test_crc_hamming_gpu(dc, bound):
    g = golden(bound)
    for case in CASES:
        for ct in CTS:
            s = g[f"{case}/ct{ct}/stream"]
            assert dc.crc32(s) == g[f"{case}/ct{ct}/crc"]
    s = g["hamming/stream"]
    bs = int(g["hamming/block_size"])
    for i in range((s.size + bs - 1) // bs):
        blk = s[i * bs: min(s.size, (i + 1) * bs)]
        r, c = dc.hamming_encode(blk)
        assert r == g[f"hamming/r{i}"] and c == g[f"hamming/c{i}"].tobytes()
        bad = blk.copy()
        bad[4321] ^= 0x04
        t, fixed, _ = dc.hamming_decode(bad, c, r)
        assert t == 3 and np.array_equal(fixed, blk)
        bad[99] ^= 0x80
        t, _, _ = dc.hamming_decode(bad, c, r)
        assert t == 1


@pytest.mark.parametrize("bound", BOUNDS)
def test_append_mode_gpu(dc, bound):
    g = golden(bound)
    dc.set_bound(bound)
    xs = g["append/input"]
    for ct in (5, 6, 11):
        s1, nb1, pos1 = dc.compress(ct, xs[:333])
        assert nb1 == g[f"append/ct{ct}/first_bytes"] and pos1 == g[f"append/ct{ct}/first_pos"]
        s2, nb2, pos2 = dc.compress(ct, xs[333:], prefix=s1, prefix_pos=pos1)
        assert np.array_equal(s2, g[f"append/ct{ct}/stream"]) and pos2 == g[f"append/ct{ct}/pos"]


def _inputs(oracle, kind, n):
    if kind == "u10":
        return oracle.gen_u10(n)
    if kind == "eq":
        return np.full(n, np.float32(0.123456789))
    if kind == "unit":
        return np.random.RandomState(n).rand(n).astype(np.float32)
    if kind == "ramp":
        return (np.float32(0.0005) * np.arange(n, dtype=np.float32)).astype(np.float32)
    if kind == "himeno":
        return np.tile(oracle.gen_himeno_plane(256, 256), max(1, n // 65536))[:n]
    if kind == "mixed":
        rs = np.random.RandomState(3)
        x = oracle.gen_u10(n)
        runs = rs.randint(0, n, 64)
        for r in runs:                    # constant runs -> long copy chains across chunks
            x[r:r + 3000] = x[r]
        return x
    raise ValueError(kind)


@pytest.mark.parametrize("bound", [1e-3, 1e-6])
@pytest.mark.parametrize("kind,n", [("u10", 1 << 20), ("eq", 1 << 20), ("unit", 300001), ("ramp", 200000),
                                    ("himeno", 1 << 18), ("mixed", 500000)])
@pytest.mark.parametrize("ct", CTS)
def test_roundtrip_vs_oracle(dc, oracle, bound, kind, n, ct):
    dc.set_bound(bound)
    x = _inputs(oracle, kind, n)
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = dc.compress(ct, xs, t, m17)
    so, nbo, poso = oracle.compress(ct, xs, bound, t, m17)
    assert nb == nbo and pos == poso and np.array_equal(s, so)
    out = dc.decompress(ct, s, n, t, m17)
    spec, got = oracle.decompress(ct, s, n, bound, t, m17)
    assert got == n
    assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))


@pytest.mark.parametrize("bound", [1e-3, 1e-6])
@pytest.mark.parametrize("kind,n", [("u10", 1 << 18), ("eq", 1 << 18), ("himeno", 1 << 16), ("mixed", 1 << 17),
                                    ("ramp", 100003)])
@pytest.mark.parametrize("ct", CTS)
def test_both_decoder_builds(dc, oracle, bound, kind, n, ct):
    """The same stream through the 1024-bit-chunk and the 256-bit-chunk builds of the decoder (the
    library picks one per decode from the stream capacity): both equal the oracle bit for bit."""
    dc.set_bound(bound)
    x = _inputs(oracle, kind, n)
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = dc.compress(ct, xs, t, m17)
    spec, got = oracle.decompress(ct, s, n, bound, t, m17)
    assert got == n
    old = dc.set_small_chunk_max_bytes(0)
    try:
        for thr, cb in ((0, 1024), (1 << 40, 256)):
            dc.set_small_chunk_max_bytes(thr)
            out = dc.decompress(ct, s, n, t, m17)
            assert dc.chunk_bits() == cb
            assert np.array_equal(out.view(np.uint32), spec.view(np.uint32)), f"chunk bits {cb}"
    finally:
        dc.set_small_chunk_max_bytes(old)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 63, 64, 65, 4095, 4096, 4097, 8191, 12345, 65537])
@pytest.mark.parametrize("ct", CTS)
def test_ragged_sizes(dc, oracle, n, ct):
    dc.set_bound(1e-3)
    x = oracle.gen_u10(n, seed=n)
    x[::7] = x[0]                         # some predictable / zero tokens
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = dc.compress(ct, xs, t, m17)
    so, nbo, poso = oracle.compress(ct, xs, 1e-3, t, m17)
    assert nb == nbo and pos == poso and np.array_equal(s, so)
    out = dc.decompress(ct, s, n, t, m17)
    spec, _ = oracle.decompress(ct, s, n, 1e-3, t, m17)
    assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))


def test_empty_input(dc):
    s, nb, pos = dc.compress(5, np.zeros(0, np.float32))
    assert nb == 0 and pos == 8


def test_kat_testfloat_gpu(dc, oracle):
    import os
    from conftest import GOLDEN
    x = np.loadtxt(os.path.join(GOLDEN, "kat_testfloat_8_8_128.txt"), dtype=np.float32)
    kat = np.fromfile(os.path.join(GOLDEN, "kat_testfloat_8_8_128.txt.bc"), np.uint8)
    dc.set_bound(1e-6)
    mn, xs = dc.to_small(x)
    s, nb, pos = dc.compress(5, xs)
    assert np.array_equal(s, kat)
    dec = dc.decompress(5, kat, x.size)
    txt = open(os.path.join(GOLDEN, "kat_testfloat_8_8_128.txt.bc.txt")).read().split()
    assert txt == ["%f" % v for v in (dec + mn).astype(np.float32)]


def test_negative_one_rejected(dc):
    dc.set_bound(1e-3)
    x = np.array([0.5, 1.0, -1.0, 2.0], np.float32)
    import ctypes
    s, nb, pos = dc.compress(5, x)       # the ABI reports the error and leaves the stream untouched
    assert nb == 0


@pytest.mark.parametrize("bound", [1e-3, 1e-6])
@pytest.mark.parametrize("ct", CTS)
def test_signed_inputs(dc, oracle, bound, ct):
    """The ABI does not require toSmallDataset: negative values put a 1 sign bit into raw tokens
    (and misaligned speculative parses read arbitrary sign bits)."""
    dc.set_bound(bound)
    rs = np.random.RandomState(7)
    x = (rs.randn(400000) * 3).astype(np.float32)
    x[x == -1.0] = 0.5
    x[1000:1300] = x[1000]
    t, m17 = oracle.type_mask(np.abs(x))
    s, nb, pos = dc.compress(ct, x, t, m17)
    so, nbo, poso = oracle.compress(ct, x, bound, t, m17)
    assert nb == nbo and pos == poso and np.array_equal(s, so)
    out = dc.decompress(ct, s, x.size, t, m17)
    spec, got = oracle.decompress(ct, s, x.size, bound, t, m17)
    if ct == 6:
        assert got == x.size
    # CT5/7/11: a sign bit parses as a 3-bit code, so the stream decodes to other values (and may end
    # early); the reference decoder's output is still the contract
    assert np.array_equal(out[:got].view(np.uint32), spec[:got].view(np.uint32))


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES)
def test_ct1_golden(dc, oracle, bound, case):
    """CT1 byte-wise codec (myCompress :3980 / myDecompress :3943) vs the compiled reference's arrays."""
    g = golden(bound)
    dc.set_bound(bound)
    x = g[f"{case}/input"]
    raw, codes, pos = dc.ct1_compress(x)
    assert np.array_equal(raw.view(np.uint32), g[f"{case}/ct1/raw"].view(np.uint32))
    assert codes == g[f"{case}/ct1/codes"].tobytes()
    assert np.array_equal(pos, g[f"{case}/ct1/pos"])
    out = dc.ct1_decompress(raw, codes, pos, x.size)
    ref = oracle.bytewise_decompress(raw, codes, pos, x.size)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("kind,n", [("u10", 1 << 20), ("ramp", 300000), ("himeno", 1 << 18), ("mixed", 500000),
                                    ("eq", 100000)])
def test_ct1_roundtrip(dc, oracle, kind, n):
    dc.set_bound(1e-3)
    x = _inputs(oracle, kind, n)
    raw, codes, pos = dc.ct1_compress(x)
    r2, c2, p2 = oracle.bytewise_compress(x, 1e-3)
    assert np.array_equal(raw.view(np.uint32), r2.view(np.uint32)) and codes == c2 and np.array_equal(pos, p2)
    out = dc.ct1_decompress(raw, codes, pos, n)
    ref = oracle.bytewise_decompress(raw, codes, pos, n)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("ct", CTS)
def test_shard_encode_with_start_bit(dc, oracle, ct):
    """Multi-GPU building blocks on one device: a shard's bit count (count kernels only), then the
    shard encoded at start_bit = global offset mod 8 with its predictor halo, equals the global
    stream's bits of that shard."""
    import torch
    dc.set_bound(1e-3)
    n = 300000
    x = oracle.gen_u10(n)
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = oracle.compress(ct, xs, 1e-3, t, m17)
    cut = 123457
    _, nbc, posc = oracle.compress(ct, xs[:cut], 1e-3, t, m17)
    b0 = nbc * 8 if posc == 8 else (nbc - 1) * 8 + (8 - posc)
    total = nb * 8 if pos == 8 else (nb - 1) * 8 + (8 - pos)
    pad = (4 - cut % 4) % 4                                        # 16-byte aligned shard start
    dx2 = torch.from_numpy(np.concatenate([np.zeros(pad, np.float32), xs])).cuda()
    shard = dx2[pad + cut:]
    assert shard.data_ptr() % 16 == 0
    bits1 = dc.encode_bits(ct, shard.data_ptr(), n - cut, idx0=cut, type_=t, mask17=m17)
    assert bits1 == total - b0
    cap = dc.stream_capacity(n - cut)
    out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    dc.encode_device(ct, shard.data_ptr(), n - cut, out.data_ptr(), idx0=cut, type_=t, mask17=m17, start_bit=b0 % 8)
    tb = dc.encode_result()
    assert tb == b0 % 8 + bits1
    got = out[: (tb + 7) // 8].cpu().numpy()
    bits = np.unpackbits(s)[b0:total]
    want = np.packbits(np.concatenate([np.zeros(b0 % 8, np.uint8), bits]))
    assert np.array_equal(got, want)


@pytest.mark.parametrize("kind,n", [("u10", 1 << 24), ("u10", 1 << 20), ("ramp", 1 << 21), ("unit", 3000001),
                                    ("himeno", 1 << 18), ("signed", 1 << 20), ("nan", 100000), ("tiny", 1 << 20),
                                    ("zeros", 1 << 22), ("zeros_u10", (1 << 21) + 77), ("wide", 1 << 20),
                                    ("u10", 1 << 26)])
def test_med_exact_parallel(dc, oracle, kind, n):
    """med_dataset_float's left-to-right float sum, computed by the binade-transducer scan, must equal
    the serial sum bit for bit (mean and type)."""
    import torch
    rs = np.random.RandomState(n % 1000)
    if kind == "signed":
        x = (rs.randn(n) * 3).astype(np.float32)
    elif kind == "nan":
        x = oracle.gen_u10(n)
        x[n // 2] = np.nan
    elif kind == "tiny":
        x = (rs.rand(n) * 1e-30).astype(np.float32)
    elif kind == "zeros":                      # the EQ input after toSmallDataset: zero chunks are skipped
        x = np.zeros(n, np.float32)
        x[::7919] = -0.0
    elif kind == "zeros_u10":                  # a zero prefix, then values (the skip ends mid-block)
        x = oracle.gen_u10(n)
        x[: n // 3] = 0.0
    elif kind == "wide":                       # exponents over ~60 binades: many serial chunks
        x = (rs.rand(n) * np.exp2(rs.randint(-30, 30, n))).astype(np.float32)
    else:
        x = _inputs(oracle, kind, n)
    d = torch.from_numpy(x).cuda()
    torch.cuda.synchronize()
    mean, t = dc.med_device(d.data_ptr(), n)
    om, ot = oracle.med(x)
    assert np.array_equal(np.float32(mean).view(np.uint32), np.float32(om).view(np.uint32)), (mean, om)
    assert t == ot


@pytest.mark.parametrize("kind,n", [("u10", 1 << 22), ("ramp", 1 << 21), ("signed", 1 << 20), ("wide", 1 << 20),
                                    ("zeros_u10", (1 << 20) + 77)])
def test_med_windows(dc, oracle, kind, n, monkeypatch):
    """The exact mean by the narrow binade window (tried first) and by the wide one (DC_MED_WIDE=1, or after
    the narrow compose missed more than 16 chunks): the same serial sum bit for bit."""
    import torch
    rs = np.random.RandomState(n % 997)
    if kind == "signed":
        x = (rs.randn(n) * 3).astype(np.float32)
    elif kind == "wide":
        x = (rs.rand(n) * np.exp2(rs.randint(-30, 30, n))).astype(np.float32)
    elif kind == "zeros_u10":
        x = oracle.gen_u10(n)
        x[: n // 3] = 0.0
    else:
        x = _inputs(oracle, kind, n)
    d = torch.from_numpy(x).cuda()
    torch.cuda.synchronize()
    om, ot = oracle.med(x)
    for force in ("0", "1"):
        monkeypatch.setenv("DC_MED_WIDE", force)
        mean, t = dc.med_device(d.data_ptr(), n)
        assert np.array_equal(np.float32(mean).view(np.uint32), np.float32(om).view(np.uint32)), (force, mean, om)
        assert t == ot
        if force == "1":
            assert dc.L.dc_med_last_wide() == 1
        elif kind in ("u10", "ramp"):
            assert dc.L.dc_med_last_wide() == 0          # the narrow window holds these sums


@pytest.mark.parametrize("n", [5000, 1 << 20])
def test_med_wide_fresh(dc, oracle, n, monkeypatch):
    """DC_MED_WIDE=1 on the FIRST call for an array: the wide window must compute its own chunk
    sums and binade estimates, not take those an earlier call on other data left in the scratch.  The
    previous call here runs on a different array (other values, other size), then the forced-wide call on
    a new one; both equal the serial sums."""
    import torch
    rs = np.random.RandomState(n % 101)
    prev = (rs.rand(3 * n + 7) * 1e4).astype(np.float32)         # other binades, other chunk count
    x = oracle.gen_u10(n)
    dp = torch.from_numpy(prev).cuda()
    dx = torch.from_numpy(x).cuda()
    torch.cuda.synchronize()
    monkeypatch.setenv("DC_MED_WIDE", "1")
    for arr, d in ((prev, dp), (x, dx), (prev, dp)):
        om, ot = oracle.med(arr)
        mean, t = dc.med_device(d.data_ptr(), len(arr))
        assert np.float32(mean).view(np.uint32) == np.float32(om).view(np.uint32), (len(arr), mean, om)
        assert t == ot
        assert dc.L.dc_med_last_wide() == 1


@pytest.mark.parametrize("ber", [1e-6, 1e-4])
def test_ct9_ber_flow(dc, oracle, ber):
    """CT9 (bitmask + CRC) with real bit flips: the sender's CRC-32 of the CT7
    stream, floor(bits*BER) flipped bits on the received copy (positions of dcamd.flip_positions),
    the receiver's CRC detects the damage, the retransmitted clean stream passes and decodes exactly
    like the oracle.  CRC-32 pinned to zlib (= the reference's do_crc32)."""
    import zlib
    import torch
    import dcamd
    dc.set_bound(1e-3)
    n = 1 << 20
    x = oracle.gen_u10(n)
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    dx = torch.from_numpy(xs).cuda()
    cap = dc.stream_capacity(n)
    snd = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    rcv = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    crc = torch.zeros(2, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    dc.encode_device(7, dx.data_ptr(), n, snd.data_ptr(), type_=t, mask17=m17)
    nbits = dc.encode_result()
    nb = (nbits + 7) // 8
    dc.crc32_device_async(snd.data_ptr(), nb, crc.data_ptr())
    dc.synchronize()
    rcv.copy_(snd)
    torch.cuda.synchronize()
    nflip = int(nbits * ber)
    assert nflip > 0
    dc.flip_bits_device(rcv.data_ptr(), nbits, nflip, 12345)
    dc.crc32_device_async(rcv.data_ptr(), nb, crc.data_ptr() + 4)
    dc.synchronize()
    clean = snd[:nb].cpu().numpy()
    got = rcv[:nb].cpu().numpy()
    want = np.unpackbits(clean)
    for p in dcamd.flip_positions(nbits, nflip, 12345):
        want[p] ^= 1
    assert np.array_equal(got, np.packbits(want))
    c = crc.cpu().numpy().view(np.uint32)
    assert c[0] == zlib.crc32(clean.tobytes())
    assert c[1] == zlib.crc32(got.tobytes())
    assert c[0] != c[1]                                     # damage detected -> resend
    rcv.copy_(snd)
    torch.cuda.synchronize()
    dc.crc32_device_async(rcv.data_ptr(), nb, crc.data_ptr() + 4)
    dc.synchronize()
    c = crc.cpu().numpy().view(np.uint32)
    assert c[0] == c[1]
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    dc.decode_device(7, rcv.data_ptr(), nb, n, out.data_ptr(), type_=t, mask17=m17)
    dc.decode_finish()
    ref, _ = oracle.decompress(7, clean, n, 1e-3, t, m17)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("ct", CTS)
@pytest.mark.parametrize("kind", ["u10", "ramp", "mixed"])
@pytest.mark.parametrize("mode", ["known", "deferred"])
def test_shard_decode(dc, oracle, ct, kind, mode):
    """Multi-GPU decode building block: a shard of one global stream, from its start bit,
    decodes exactly like that part of the whole stream -- with the three values before it given up
    front ("known"), or supplied afterwards to re-decode the prefix that depends on them
    ("deferred": the 12-byte exchange of the multi-GPU flow)."""
    import torch
    dc.set_bound(1e-3)
    n = 300000
    x = _inputs(oracle, kind, n)
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = oracle.compress(ct, xs, 1e-3, t, m17)
    ref, _ = oracle.decompress(ct, s, n, 1e-3, t, m17)
    total = nb * 8 if pos == 8 else (nb - 1) * 8 + (8 - pos)
    for cut in (123457, 3, 262144 + 5):
        _, nbc, posc = oracle.compress(ct, xs[:cut], 1e-3, t, m17)
        b0 = nbc * 8 if posc == 8 else (nbc - 1) * 8 + (8 - posc)
        ds = torch.from_numpy(np.concatenate([s, np.zeros(64, np.uint8)])).cuda()
        out = torch.full((n - cut,), -7.0, dtype=torch.float32, device="cuda")
        hin = torch.from_numpy(ref[cut - 3:cut][::-1].copy()).cuda()          # b1, b2, b3
        torch.cuda.synchronize()
        dc.decode_shard_device(ct, ds.data_ptr(), nb, b0, total - b0, n - cut, out.data_ptr(), type_=t, mask17=m17,
                               hin_ptr=hin.data_ptr() if mode == "known" else None)
        dc.decode_finish()
        if mode == "deferred":
            dc.decode_shard_fix(hin.data_ptr())
        got = out.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref[cut:].view(np.uint32)), (cut, np.flatnonzero(got != ref[cut:])[:10])


@pytest.mark.parametrize("ct", CTS)
@pytest.mark.parametrize("size,ijk,v", [("M", 3, 1), ("M", 3, 128), ("M", 1, 1), ("M", 2, 64),
                                        ("L", 3, 1), ("L", 3, 6), ("L", 1, 255), ("L", 2, 100)])
def test_halo_plane_device(dc, oracle, ct, size, ijk, v):
    """Fused Himeno halo path: the plane of a device-resident p[129][129][131]
    (impl/param.h, M size) or p[257][257][8] (the L size's i/j extent, a thin z slab per rank as the
    bench's halo step) gathered in transform_3d_array_to_1d_array order, toSmallDataset_float'ed and
    encoded on the GPU equals the oracle stream of the host-side plane; the decode writes plane + min
    back into p exactly as impl/himenoBMTxps.c:699-706."""
    _halo_plane_case(dc, oracle, ct, size, ijk, v, noise=True)


@pytest.mark.parametrize("ct", CTS)
@pytest.mark.parametrize("ijk,v", [(3, 1), (3, 5), (1, 255), (2, 100)])
def test_halo_plane_device_initmt(dc, oracle, ct, ijk, v):
    """The L-size plane exactly as BASELINE config 4 produces it: initmt's p = i^2/(imax-1)^2 with no noise,
    so a z-plane is rows of one repeated value -- a runs-mode stream of '101' copy runs (the bench's --halo
    stream) -- through the fused device encode and decode, against the oracle."""
    _halo_plane_case(dc, oracle, ct, "L", ijk, v, noise=False)


def _halo_plane_case(dc, oracle, ct, size, ijk, v, noise):
    import torch
    dc.set_bound(1e-3)
    if size == "M":
        mi, mj, mk = 129, 129, 131
        imax, jmax, kmax = 128, 128, 130
    else:
        mi, mj, mk = 257, 257, 8
        imax, jmax, kmax = 256, 256, 7
    ii = np.arange(mi, dtype=np.float32)[:, None, None]
    rs = np.random.RandomState(ijk * 1000 + v)
    p = (ii * ii / np.float32((imax - 1) * (imax - 1)) + np.zeros((mi, mj, mk), np.float32)).astype(np.float32)
    if noise:
        p += (rs.rand(mi, mj, mk).astype(np.float32) * np.float32(0.01))
    A, B = {1: (jmax, kmax), 2: (imax, kmax), 3: (imax, jmax)}[ijk]
    a, b = np.meshgrid(np.arange(A), np.arange(B), indexing="ij")
    idx = {1: (v, a, b), 2: (a, v, b), 3: (a, b, v)}[ijk]
    plane = p[idx].reshape(-1).copy()
    mn, xs = oracle.to_small(plane)
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = oracle.compress(ct, xs, 1e-3, t, m17)
    dp = torch.from_numpy(p).cuda()
    n = A * B
    st = torch.zeros(dc.stream_capacity(n), dtype=torch.uint8, device="cuda")
    bits = torch.zeros(1, dtype=torch.int64, device="cuda")
    dmin = torch.zeros(1, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ty, mk17 = dc.halo_encode_device(ct, dp.data_ptr(), (mi, mj, mk), ijk, v, (imax, jmax, kmax), st.data_ptr(),
                                     bits.data_ptr(), dmin.data_ptr(), type_=0, mask17=0)
    if ct == 7:
        assert (ty, mk17) == (t, m17)
    tb = dc.encode_result()
    assert (tb + 7) // 8 == nb
    assert np.array_equal(st[:nb].cpu().numpy(), s)
    assert np.float32(dmin.cpu().numpy()[0]) == np.float32(mn)
    q = torch.zeros_like(dp)
    dc.halo_decode_device(ct, st.data_ptr(), nb, 0, ty, mk17, dmin.data_ptr(), q.data_ptr(), (mi, mj, mk), ijk, v,
                          (imax, jmax, kmax))
    dc.synchronize()
    dec, _ = oracle.decompress(ct, s, n, 1e-3, t, m17)
    want = (dec + np.float32(mn)).astype(np.float32)
    got = q.cpu().numpy()[idx].reshape(-1)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("ct", [5, 6, 7, 11])
@pytest.mark.parametrize("noise", [False, True])
@pytest.mark.parametrize("ijk,planes", [(3, (1, 5)), (1, (1, 254)), (2, (7, 200))])
@pytest.mark.parametrize("unfused", [0, 1])
def test_halo_decode2_pair(dc, oracle, ct, noise, ijk, planes, unfused):
    """(r06) two planes decoded at once on two streams (dc_halo_decode2_device) write the same values into p as two
    dc_halo_decode_device calls (async halo mode, as the bench's step); by default each plane's values kernel adds
    the minimum and scatters into p itself (unfused=1: the separate scatter pass)"""
    import torch
    dc.set_bound(1e-3)
    mi, mj, mk = 257, 257, 8
    imax, jmax, kmax = 256, 256, 7
    ii = np.arange(mi, dtype=np.float32)[:, None, None]
    kk = np.arange(mk, dtype=np.float32)[None, None, :]
    p = (ii * ii / np.float32((imax - 1) * (imax - 1)) + np.float32(0.01) * kk + np.zeros((mi, mj, mk), np.float32))
    if noise:
        p = p + np.random.RandomState(3).rand(mi, mj, mk).astype(np.float32) * np.float32(0.01)
    p = p.astype(np.float32)
    dp = torch.from_numpy(p).cuda()
    A, B = {1: (jmax, kmax), 2: (imax, kmax), 3: (imax, jmax)}[ijk]
    n = A * B
    a, b = np.meshgrid(np.arange(A), np.arange(B), indexing="ij")
    st = [torch.zeros(dc.stream_capacity(n), dtype=torch.uint8, device="cuda") for _ in range(2)]
    bits = torch.zeros(2, dtype=torch.int64, device="cuda")
    mins = torch.zeros(2, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ty = [0, 0]
    m17 = [0, 0]
    for h, v in enumerate(planes):
        ty[h], m17[h] = dc.halo_encode_device(ct, dp.data_ptr(), (mi, mj, mk), ijk, v, (imax, jmax, kmax),
                                              st[h].data_ptr(), bits.data_ptr() + 8 * h, mins.data_ptr() + 4 * h)
        dc.encode_result()
    if ct == 7 and (ty[0], m17[0]) != (ty[1], m17[1]):
        pytest.skip("CT7: the two planes have different masks (one decode2 call takes one)")
    q1 = torch.zeros_like(dp)
    q2 = torch.zeros_like(dp)
    prev = dc.L.dc_set_halo_async(1)
    prev_u = dc.L.dc_set_halo_unfused(unfused)
    try:
        for h, v in enumerate(planes):
            dc.halo_decode_device(ct, st[h].data_ptr(), -1, bits.data_ptr() + 8 * h, ty[h], m17[h],
                                  mins.data_ptr() + 4 * h, q1.data_ptr(), (mi, mj, mk), ijk, v, (imax, jmax, kmax))
        dc.halo_decode2_device(ct, st[0].data_ptr(), st[1].data_ptr(), bits.data_ptr(), bits.data_ptr() + 8, ty[0],
                               m17[0], mins.data_ptr(), mins.data_ptr() + 4, q2.data_ptr(), (mi, mj, mk), ijk,
                               planes[0], planes[1], (imax, jmax, kmax))
        dc.synchronize()
        status = dc.decode_status()
    finally:
        dc.L.dc_set_halo_unfused(prev_u)
        dc.L.dc_set_halo_async(prev)
    if status != 0:
        # a plane the small-stream decoder declines (a '110'/'111' carry across its blocks, status 512 | why):
        # the documented fallback, both planes decoded again synchronously
        assert status & 512 and ijk != 3, hex(status)
        dc.decode_status_clear()
        for h, v in enumerate(planes):
            dc.halo_decode_device(ct, st[h].data_ptr(), -1, bits.data_ptr() + 8 * h, ty[h], m17[h],
                                  mins.data_ptr() + 4 * h, q2.data_ptr(), (mi, mj, mk), ijk, v, (imax, jmax, kmax))
        dc.synchronize()
    else:
        assert torch.equal(q1, q2)                        # (every other element of p stays 0 in both)
    q2h = q2.cpu().numpy()
    for h, v in enumerate(planes):                        # and against the oracle's decode + min
        k = (int(bits[h]) + 7) // 8
        s = st[h][:k].cpu().numpy()
        dec, _ = oracle.decompress(ct, s, n, 1e-3, ty[h], m17[h])
        want = (dec + mins[h].cpu().numpy()).astype(np.float32)
        idx = {1: (v, a, b), 2: (a, v, b), 3: (a, b, v)}[ijk]
        assert np.array_equal(q2h[idx].reshape(-1).view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("ct", [5, 6, 7, 11])
@pytest.mark.parametrize("ijk,v0,v1", [(3, 1, 5), (1, 1, 255), (2, 7, 100)])
def test_halo_encode2_pair(dc, oracle, ct, ijk, v0, v1):
    """(r06) two planes encoded at once on two streams (dc_halo_encode2_device): the same bit counts, streams and
    minima as two dc_halo_encode_device calls"""
    import torch
    dc.set_bound(1e-3)
    mi, mj, mk = 257, 257, 8
    imax, jmax, kmax = 256, 256, 7
    rs = np.random.RandomState(ct * 100 + ijk)
    p = (rs.rand(mi, mj, mk).astype(np.float32) * np.float32(3) - np.float32(1)).astype(np.float32)
    dp = torch.from_numpy(p).cuda()
    A, B = {1: (jmax, kmax), 2: (imax, kmax), 3: (imax, jmax)}[ijk]
    n = A * B
    t, m17 = (3, 0x0813f) if ct == 7 else (0, 0)           # (CT7 with a given mask: the fused path)
    outs = []
    for pairwise in (False, True):
        st = [torch.zeros(dc.stream_capacity(n), dtype=torch.uint8, device="cuda") for _ in range(2)]
        bits = torch.zeros(2, dtype=torch.int64, device="cuda")
        mins = torch.zeros(2, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        if pairwise:
            dc.halo_encode2_device(ct, dp.data_ptr(), (mi, mj, mk), ijk, v0, v1, (imax, jmax, kmax), st[0].data_ptr(),
                                   st[1].data_ptr(), bits.data_ptr(), bits.data_ptr() + 8, mins.data_ptr(),
                                   mins.data_ptr() + 4, type_=t, mask17=m17)
        else:
            for h, v in enumerate((v0, v1)):
                dc.halo_encode_device(ct, dp.data_ptr(), (mi, mj, mk), ijk, v, (imax, jmax, kmax), st[h].data_ptr(),
                                      bits.data_ptr() + 8 * h, mins.data_ptr() + 4 * h, type_=t, mask17=m17)
        dc.synchronize()
        assert dc.encode_status() == 0
        b = bits.cpu().tolist()
        outs.append((b, [st[h][:(b[h] + 7) // 8].cpu().numpy() for h in range(2)], mins.cpu().numpy().view(np.uint32)))
    (b0, s0, m0), (b1, s1, m1) = outs
    assert b0 == b1 and np.array_equal(m0, m1)
    assert all(np.array_equal(x, y) for x, y in zip(s0, s1))


@pytest.mark.parametrize("ct", [5, 6, 11])
@pytest.mark.parametrize("dims", [(9, 7, 5), (33, 20, 6), (40, 45, 30), (130, 129, 3)])
@pytest.mark.parametrize("kind", ["noise", "zero_min", "nan"])
def test_halo_small_planes(dc, oracle, ct, dims, kind):
    """(r06) halo planes of every size class of the gather's minimum (one workgroup finishing it alone, a few, many):
    the minimum's bits and the stream against the oracle's toSmallDataset_float + compress, for the three plane
    orientations, one encode and the pair encode"""
    import torch
    dc.set_bound(1e-3)
    mi, mj, mk = dims
    imax, jmax, kmax = mi - 1, mj - 1, mk - 1
    rs = np.random.RandomState(sum(dims) + len(kind))
    p = (rs.rand(mi, mj, mk).astype(np.float32) * np.float32(2) - np.float32(0.5)).astype(np.float32)
    if kind == "zero_min":
        p = np.abs(p).astype(np.float32)
        p[1, 1, :] = -0.0
        p[2, 1, :] = 0.0
    elif kind == "nan":
        p[::3, 1::2, :] = np.nan
    dp = torch.from_numpy(p).cuda()
    for ijk in (1, 2, 3):
        A, B = {1: (jmax, kmax), 2: (imax, kmax), 3: (imax, jmax)}[ijk]
        ext = {1: mi, 2: mj, 3: mk}[ijk]
        v0, v1 = 1, ext - 2
        n = A * B
        a, b = np.meshgrid(np.arange(A), np.arange(B), indexing="ij")
        st = [torch.zeros(dc.stream_capacity(n), dtype=torch.uint8, device="cuda") for _ in range(2)]
        bits = torch.zeros(2, dtype=torch.int64, device="cuda")
        mins = torch.zeros(2, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        dc.halo_encode2_device(ct, dp.data_ptr(), (mi, mj, mk), ijk, v0, v1, (imax, jmax, kmax), st[0].data_ptr(),
                               st[1].data_ptr(), bits.data_ptr(), bits.data_ptr() + 8, mins.data_ptr(),
                               mins.data_ptr() + 4)
        dc.synchronize()
        assert dc.encode_status() == 0
        for h, v in enumerate((v0, v1)):
            idx = {1: (v, a, b), 2: (a, v, b), 3: (a, b, v)}[ijk]
            omn, xs = oracle.to_small(p[idx].reshape(-1).copy())
            assert mins.cpu().numpy().view(np.uint32)[h] == np.float32(omn).view(np.uint32), (ijk, h)
            if ct == 6 and np.isnan(xs).any():
                continue
            so, nbo, _ = oracle.compress(ct, xs, 1e-3, 0, 0)
            k = (int(bits[h]) + 7) // 8
            assert k == nbo and np.array_equal(st[h][:k].cpu().numpy(), so), (ijk, h)


@pytest.mark.parametrize("ct", [5, 6, 11])
@pytest.mark.parametrize("pair_encode", [False, True])
def test_halo_graph_replay(dc, oracle, ct, pair_encode):
    """(r06) the halo step recorded into a HIP graph (dc_capture_begin/end) and replayed (dc_graph_launch): each replay
    re-reads the array rewritten in place and gives the streams, bit counts, minima and decoded planes of the same
    calls issued directly; direct encodes after the replays stay correct (their epochs restart)"""
    import torch
    dc.set_bound(1e-3)
    mi, mj, mk = 257, 257, 8
    imax, jmax, kmax = 256, 256, 7
    n = imax * jmax
    planes = [1, kmax - 2]
    rs = np.random.RandomState(ct)
    fields = [(rs.rand(mi, mj, mk).astype(np.float32) * np.float32(2 + k) - np.float32(k)).astype(np.float32)
              for k in range(3)]
    dp = torch.from_numpy(fields[0]).cuda()

    def bufs():
        return ([torch.zeros(dc.stream_capacity(n), dtype=torch.uint8, device="cuda") for _ in range(2)],
                torch.zeros(2, dtype=torch.int64, device="cuda"), torch.zeros(2, dtype=torch.float32, device="cuda"),
                torch.zeros(mi, mj, mk, dtype=torch.float32, device="cuda"))

    def step(b):
        st, bits, mins, q = b
        if pair_encode:
            dc.halo_encode2_device(ct, dp.data_ptr(), (mi, mj, mk), 3, planes[0], planes[1], (imax, jmax, kmax),
                                   st[0].data_ptr(), st[1].data_ptr(), bits.data_ptr(), bits.data_ptr() + 8,
                                   mins.data_ptr(), mins.data_ptr() + 4)
        else:
            for h, v in enumerate(planes):
                dc.halo_encode_device(ct, dp.data_ptr(), (mi, mj, mk), 3, v, (imax, jmax, kmax), st[h].data_ptr(),
                                      bits.data_ptr() + 8 * h, mins.data_ptr() + 4 * h)
        dc.halo_decode2_device(ct, st[0].data_ptr(), st[1].data_ptr(), bits.data_ptr(), bits.data_ptr() + 8, 0, 0,
                               mins.data_ptr(), mins.data_ptr() + 4, q.data_ptr(), (mi, mj, mk), 3, planes[0], planes[1],
                               (imax, jmax, kmax))

    def result(b):
        st, bits, mins, q = b
        bb = bits.cpu().tolist()
        return (bb, [st[h][:(bb[h] + 7) // 8].cpu().numpy() for h in range(2)], mins.cpu().numpy().view(np.uint32),
                q[:imax, :jmax, planes].cpu().numpy().view(np.uint32))

    def same(a, b):
        return a[0] == b[0] and all(np.array_equal(x, y) for x, y in zip(a[1], b[1])) and \
            np.array_equal(a[2], b[2]) and np.array_equal(a[3], b[3])

    prev = dc.L.dc_set_halo_async(1)
    g = None
    try:
        torch.cuda.synchronize()
        gb = bufs()
        step(gb)                                   # (sizes the buffers: capture after one direct step)
        dc.synchronize()
        dc.capture_begin()
        step(gb)
        g = dc.capture_end()
        for k in (1, 2, 0, 2):
            dp.copy_(torch.from_numpy(fields[k]))
            torch.cuda.synchronize()
            db = bufs()
            torch.cuda.synchronize()
            step(db)                               # the same step issued directly
            dc.synchronize()
            want = result(db)
            dc.graph_launch(g)
            dc.synchronize()
            assert dc.decode_status() == 0 and dc.encode_status() == 0
            got = result(gb)
            assert same(got, want), k
            for h, v in enumerate(planes):         # and the streams against the oracle's encode of x - min
                omn, xs = oracle.to_small(fields[k][:imax, :jmax, v].reshape(-1).copy())
                so, nbo, _ = oracle.compress(ct, xs, 1e-3, 0, 0)
                assert np.float32(omn).view(np.uint32) == got[2][h]
                assert (got[0][h] + 7) // 8 == nbo and np.array_equal(got[1][h], so)
    finally:
        if g is not None:
            dc.graph_destroy(g)
        dc.L.dc_set_halo_async(prev)
    # a decode other than an async halo plane's cannot be recorded: dc_capture_end fails and nothing is kept
    x = torch.from_numpy(fields[0][:, :, 1].reshape(-1).copy()).cuda()
    s = torch.zeros(dc.stream_capacity(x.numel()), dtype=torch.uint8, device="cuda")
    tb = torch.zeros(1, dtype=torch.int64, device="cuda")
    dc.encode_device(ct, x.data_ptr(), x.numel(), s.data_ptr(), total_ptr=tb.data_ptr())
    nb = (dc.encode_result() + 7) // 8
    out = torch.zeros_like(x)
    dc.capture_begin()
    with pytest.raises(Exception):
        dc.decode_device(ct, s.data_ptr(), nb, x.numel(), out.data_ptr())
    with pytest.raises(Exception):
        dc.capture_end()
    dc.decode_device(ct, s.data_ptr(), nb, x.numel(), out.data_ptr())     # (the library works on after it)
    dc.decode_finish()
    spec, _ = oracle.decompress(ct, s[:nb].cpu().numpy(), x.numel(), 1e-3, 0, 0)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), spec.view(np.uint32))


@pytest.mark.parametrize("ct", [5, 6, 11])
@pytest.mark.parametrize("kind", ["initmt", "noise", "negative", "zero_min", "nan", "inf"])
@pytest.mark.parametrize("ijk,v", [(3, 1), (1, 255), (2, 7)])
def test_halo_fused_vs_separate(dc, oracle, ct, kind, ijk, v):
    """(r06) The halo encode's fused passes (the gather with toSmallDataset's minimum partials, min_final, the encoder
    subtracting the minimum while loading) against its separate passes (dc_set_halo_unfused(1)) and the oracle:
    the same minimum (bits), bit count and stream -- planes with negative values, a zero minimum, NaNs (quieted as
    x86 does) and infinities (a NaN or infinite minimum takes the x86 subtraction in the encoder)."""
    import torch
    dc.set_bound(1e-3)
    mi, mj, mk = 257, 257, 8
    imax, jmax, kmax = 256, 256, 7
    rs = np.random.RandomState(hash((kind, ijk, v)) % 1000)
    ii = np.arange(mi, dtype=np.float32)[:, None, None]
    p = (ii * ii / np.float32((imax - 1) * (imax - 1)) + np.zeros((mi, mj, mk), np.float32)).astype(np.float32)
    if kind != "initmt":
        p += (rs.rand(mi, mj, mk).astype(np.float32) * np.float32(0.01))
    if kind == "negative":
        p -= np.float32(3.5)
    elif kind == "zero_min":
        p[5, 3, :] = -0.0; p[7, 9, :] = 0.0; p[0, :, :] += np.float32(0.5); p[:, 0, :] += np.float32(0.5)
    elif kind == "nan":
        p[3::17, 5::13, :] = np.nan
    elif kind == "inf":
        p[2::19, :, :] = np.inf
    A, B = {1: (jmax, kmax), 2: (imax, kmax), 3: (imax, jmax)}[ijk]
    a, b = np.meshgrid(np.arange(A), np.arange(B), indexing="ij")
    idx = {1: (v, a, b), 2: (a, v, b), 3: (a, b, v)}[ijk]
    plane = p[idx].reshape(-1).copy()
    n = A * B
    omn, xs = oracle.to_small(plane)
    dp = torch.from_numpy(p).cuda()
    res = []
    for unfused in (0, 1):
        prev = dc.L.dc_set_halo_unfused(unfused)
        try:
            st = torch.zeros(dc.stream_capacity(n), dtype=torch.uint8, device="cuda")
            bits = torch.zeros(1, dtype=torch.int64, device="cuda")
            dmin = torch.zeros(1, dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            dc.halo_encode_device(ct, dp.data_ptr(), (mi, mj, mk), ijk, v, (imax, jmax, kmax), st.data_ptr(),
                                  bits.data_ptr(), dmin.data_ptr(), type_=0, mask17=0)
            tb = dc.encode_result()
            res.append((tb, st[:(tb + 7) // 8].cpu().numpy(), dmin.cpu().numpy().view(np.uint32)[0]))
        finally:
            dc.L.dc_set_halo_unfused(prev)
    (b0, s0, m0), (b1, s1, m1) = res
    assert m0 == m1 == np.float32(omn).view(np.uint32)
    assert b0 == b1 and np.array_equal(s0, s1)
    if ct != 6 or not np.isnan(xs).any():
        so, nbo, _ = oracle.compress(ct, xs, 1e-3, 0, 0)
        assert (b0 + 7) // 8 == nbo and np.array_equal(s0, so)




@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("ct", CTS)
def test_decoder_golden_chunk_map_forced(dc, oracle, bound, ct):
    """The chunk-map decoder is the fallback of every decline: with both knobs at -1 (segment decoder off,
    small-stream decoder off) every golden stream goes straight to it and must still equal the grammar
    decoder (-1 is honoured by both knobs, halo planes included)."""
    g = golden(bound)
    dc.set_bound(bound)
    m3 = dc.L.dc_set_decode3_min_bytes(-1)
    rm = dc.L.dc_set_runs_max_bytes(-1)
    try:
        for case in CASES:
            s = g[f"{case}/ct{ct}/stream"]
            n = g[f"{case}/input"].size
            t, m17 = _prep(g, case)
            out = dc.decompress(ct, s, n, t, m17)
            assert not dc.L.dc_last_decode_launched_v3() and not dc.L.dc_last_decode_launched_runs()
            spec, _ = oracle.decompress(ct, s, n, bound, t, m17)
            assert np.array_equal(out.view(np.uint32), spec.view(np.uint32)), case
    finally:
        dc.L.dc_set_decode3_min_bytes(m3)
        dc.L.dc_set_runs_max_bytes(rm)


@pytest.mark.parametrize("nbytes", [0, 1, 3, 4, 5, 4096, 65537, (1 << 22) + 7])
def test_hash_device_matches_host(dc, nbytes):
    """dc_hash_device (bench.py's self-check) equals its host twin dcamd.hash_words on ragged lengths: bytes
    past nbytes do not count."""
    import torch
    import dcamd
    rng = np.random.RandomState(nbytes & 0xFFFF)
    h = rng.randint(0, 256, size=nbytes + 9, dtype=np.uint8)
    d = torch.from_numpy(h).cuda()
    torch.cuda.synchronize()
    assert dc.hash_device(d.data_ptr(), nbytes) == dcamd.hash_words(h, nbytes)
    if nbytes:
        h2 = h.copy()
        h2[nbytes - 1] ^= 1
        assert dcamd.hash_words(h2, nbytes) != dcamd.hash_words(h, nbytes)


def test_copy_rate_device(dc):
    """dc_copy_rate_device (bench.py's achievable ceiling): every variant copies the buffer exactly and the
    best rate is a plausible HBM rate."""
    import torch
    n = 1 << 24
    a = torch.arange(n, dtype=torch.int32, device="cuda")
    b = torch.zeros_like(a)
    torch.cuda.synchronize()
    gbs, v = dc.copy_rate(a.data_ptr(), b.data_ptr(), 4 * n, 3)
    assert torch.equal(a, b)
    assert 0 <= v < 4 and 500.0 < gbs < 8000.0


@pytest.mark.parametrize("nbytes", [0, 1, 15, 16, 17, 4095, 16383, 16384, 16385, 40000, (1 << 20) + 7, 3 * 16384 * 1024 + 5])
def test_crc32_stream_device_zlib(dc, nbytes):
    """The fused CRC's block kernel + combine (dc_crc32_stream_device) equals zlib on ragged lengths (bytes past
    nbytes, here nonzero, do not count)."""
    import zlib
    import torch
    rng = np.random.RandomState(nbytes & 0xFFFF)
    h = rng.randint(0, 256, size=nbytes + 64, dtype=np.uint8)
    d = torch.from_numpy(h).cuda()
    c = torch.zeros(4, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    dc.crc32_stream_device(d.data_ptr(), nbytes, c.data_ptr())
    dc.synchronize()
    assert (int(c[0].item()) & 0xFFFFFFFF) == zlib.crc32(h[:nbytes].tobytes())


@pytest.mark.parametrize("ct", [5, 6, 7, 11])
@pytest.mark.parametrize("n", [1, 5, 4096, 4097, 70001, (1 << 20) + 5])
def test_encode_crc_device(dc, oracle, ct, n):
    """dc_encode_crc_device: the stream equals the plain encode's (and the oracle's), and the CRC its tiles build
    from the words they store equals zlib's CRC-32 of the stream bytes."""
    import zlib
    import torch
    dc.set_bound(1e-3)
    _, xs = oracle.to_small(oracle.gen_u10(n))
    t, m17 = oracle.type_mask(xs)
    dx = torch.from_numpy(xs).cuda()
    cap = dc.stream_capacity(n)
    st = torch.full((cap,), 0x5A, dtype=torch.uint8, device="cuda")
    nb = torch.zeros(1, dtype=torch.int64, device="cuda")
    c = torch.zeros(4, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    for _ in range(2):                                   # (twice: the block accumulators are reused)
        dc.encode_crc_device(ct, dx.data_ptr(), n, st.data_ptr(), nb.data_ptr(), c.data_ptr(), type_=t, mask17=m17)
        bits = dc.encode_result()
        nbytes = (bits + 7) // 8
        s = st[:nbytes].cpu().numpy()
        so, nbo, _ = oracle.compress(ct, xs, 1e-3, t, m17)
        assert nbo == nbytes and np.array_equal(s, so)
        assert (int(c[0].item()) & 0xFFFFFFFF) == zlib.crc32(s.tobytes())


def test_crc_resend_crc_device(dc):
    """The CT9 resend with the receiver's CRC of the copy computed as it is written: a damaged copy is replaced
    (count[0] = 1), the copy's CRC equals the sender's (count[1] = 0); an intact copy is left alone."""
    import zlib
    import torch
    nbytes = 5 * 16384 + 77
    h = np.random.RandomState(7).randint(0, 256, size=nbytes + 64, dtype=np.uint8)
    src = torch.from_numpy(h).cuda()
    dst = src.clone()
    dst[12345] ^= 4
    crc2 = torch.zeros(2, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    dc.crc32_stream_device(src.data_ptr(), nbytes, crc2.data_ptr())
    dc.crc32_stream_device(dst.data_ptr(), nbytes, crc2.data_ptr() + 4)
    dc.synchronize()
    assert int(crc2[0].item()) != int(crc2[1].item())
    dc.crc_resend_crc_device(crc2.data_ptr(), src.data_ptr(), dst.data_ptr(), nbytes, cnt.data_ptr())
    dc.synchronize()
    assert cnt.tolist() == [1, 0]
    assert torch.equal(dst[:nbytes], src[:nbytes])
    assert (int(crc2[1].item()) & 0xFFFFFFFF) == zlib.crc32(h[:nbytes].tobytes())
    dc.crc_resend_crc_device(crc2.data_ptr(), src.data_ptr(), dst.data_ptr(), nbytes, cnt.data_ptr())
    dc.synchronize()
    assert cnt.tolist() == [1, 0]


@pytest.mark.parametrize("nbytes", [1, 16, 4095, 32768, 32769, 65536 + 48, (1 << 20) + 7, 5 * (1 << 22) + 13])
def test_crc32_copy_device(dc, nbytes):
    """The CT9 send (dc_crc32_copy_device): the destination holds the source's bytes (and nothing past them
    changes), the CRC is zlib's of the bytes sent -- full 32 KiB blocks staged, the last block by bytes."""
    import zlib
    import torch
    rng = np.random.RandomState(nbytes & 0xFFFF)
    h = rng.randint(0, 256, size=nbytes + 64, dtype=np.uint8)
    src = torch.from_numpy(h).cuda()
    dst = torch.full((nbytes + 64,), 0x5A, dtype=torch.uint8, device="cuda")
    c = torch.zeros(4, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    dc.crc32_copy_device(src.data_ptr(), dst.data_ptr(), nbytes, c.data_ptr())
    dc.synchronize()
    assert (int(c[0].item()) & 0xFFFFFFFF) == zlib.crc32(h[:nbytes].tobytes())
    assert torch.equal(dst[:nbytes], src[:nbytes])
    assert bool((dst[nbytes:] == 0x5A).all())


@pytest.mark.parametrize("nbytes", [1, 100, 32768, 32768 * 5 + 17, (1 << 22) + 3])
def test_crc32_pair_device(dc, nbytes):
    """The CT9 checks in one pass (dc_crc32_pair_device): both CRCs zlib's of their own buffer, the buffers
    untouched -- one byte apart, and identical."""
    import zlib
    import torch
    rng = np.random.RandomState(nbytes & 0xFFFF)
    h = rng.randint(0, 256, size=nbytes + 64, dtype=np.uint8)
    a = torch.from_numpy(h).cuda()
    b = a.clone()
    b[nbytes // 2] ^= 0x10
    c = torch.zeros(4, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    dc.crc32_pair_device(a.data_ptr(), b.data_ptr(), nbytes, c.data_ptr(), c.data_ptr() + 4)
    dc.synchronize()
    hb = h.copy()
    hb[nbytes // 2] ^= 0x10
    assert (int(c[0].item()) & 0xFFFFFFFF) == zlib.crc32(h[:nbytes].tobytes())
    assert (int(c[1].item()) & 0xFFFFFFFF) == zlib.crc32(hb[:nbytes].tobytes())
    dc.crc32_pair_device(a.data_ptr(), a.data_ptr(), nbytes, c.data_ptr() + 8, c.data_ptr() + 12)
    dc.synchronize()
    assert int(c[2].item()) == int(c[3].item()) == int(c[0].item())


@pytest.mark.parametrize("ct", [5, 6, 7, 11])
@pytest.mark.parametrize("log2n", [12, 20, 24])
def test_encode_send_device(dc, oracle, ct, log2n):
    """The CT9 send without a copy pass (dc_encode_send_device): the receiver's buffer holds exactly the
    sender's stream (the oracle's bytes), nothing past it written."""
    import torch
    n = 1 << log2n
    dc.set_bound(1e-3)
    _, xs = oracle.to_small(oracle.gen_u10(n))
    t, m17 = oracle.type_mask(xs)
    cap = dc.stream_capacity(n)
    x = torch.from_numpy(xs).cuda()
    st = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    rcv = torch.full((cap,), 0x5A, dtype=torch.uint8, device="cuda")
    nbits = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    dc.encode_send_device(ct, x.data_ptr(), n, st.data_ptr(), rcv.data_ptr(), nbits.data_ptr(), type_=t, mask17=m17)
    nb = (dc.encode_result() + 7) // 8
    torch.cuda.synchronize()
    s, onb, _ = oracle.compress(ct, xs, 1e-3, t, m17)
    assert nb == onb
    assert np.array_equal(st[:nb].cpu().numpy(), s)
    assert torch.equal(rcv[:nb], st[:nb])
    w = (nb + 3) // 4 * 4                                # (the last word's padding bytes are the stream's zeros)
    assert bool((rcv[w:] == 0x5A).all())


@pytest.mark.parametrize("nbytes", [3 * 32768 * 32 + 5, (1 << 22) + 1])
def test_crc_resend_crc_device_large(dc, nbytes):
    """The resend at sizes of many 32 KiB blocks with a ragged tail: replaced once, its CRC zlib's, gated after."""
    import zlib
    import torch
    h = np.random.RandomState(11).randint(0, 256, size=nbytes + 64, dtype=np.uint8)
    src = torch.from_numpy(h).cuda()
    dst = src.clone()
    dst[nbytes // 2] ^= 1
    dst[nbytes - 1] ^= 128
    crc2 = torch.zeros(2, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    dc.crc32_device_async(src.data_ptr(), nbytes, crc2.data_ptr())
    dc.crc32_device_async(dst.data_ptr(), nbytes, crc2.data_ptr() + 4)
    dc.crc_resend_crc_device(crc2.data_ptr(), src.data_ptr(), dst.data_ptr(), nbytes, cnt.data_ptr())
    dc.synchronize()
    assert cnt.tolist() == [1, 0]
    assert torch.equal(dst[:nbytes], src[:nbytes])
    assert (int(crc2[1].item()) & 0xFFFFFFFF) == zlib.crc32(h[:nbytes].tobytes())

