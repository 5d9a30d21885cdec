"""GPU parity of the segment decoder (csrc/dc_decode3.hip): forced on for every stream size, its
decode must equal the oracle's grammar decoder bit for bit, and it must take (not decline) every stream
of ordinary density.  Streams it declines (runs mode: mostly 3-bit codes) must still decode exactly
through the chunk-map decoder it hands them to."""
import numpy as np
import pytest

from conftest import BOUNDS, CASES, golden

pytestmark = pytest.mark.gpu
CTS = [5, 6, 7, 11]


@pytest.fixture
def v3(dc):
    old = dc.set_decode3_min_bytes(0)             # every stream through the segment decoder
    yield dc
    dc.set_decode3_min_bytes(old)


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
        for r in rs.randint(0, n, 64):           # constant runs -> prediction chains across chunks
            x[r:r + 3000] = x[r]
        return x
    if kind == "sparse":                          # every 5th value near a predictor: '101'..'111' codes
        x = oracle.gen_u10(n)
        x[1::5] = x[0::5][: x[1::5].size]
        x[2::7] = 0.0
        return x
    raise ValueError(kind)


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("ct", CTS)
def test_decode3_golden(v3, oracle, bound, case, ct):
    g = golden(bound)
    v3.set_bound(bound)
    key = f"{case}/ct{ct}"
    s = g[key + "/stream"]
    n = g[f"{case}/input"].size
    t, m17 = int(g[f"{case}/type"]), int(g[f"{case}/mask17"])
    out = v3.decompress(ct, s, n, t, m17)
    spec, got = oracle.decompress(ct, s, n, bound, t, m17)
    assert got == n
    assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))
    if bool(g[key + "/ref_consistent"]):
        assert np.array_equal(out.view(np.uint32), g[key + "/ref_decoded"].view(np.uint32))


@pytest.mark.parametrize("bound", [1e-3, 1e-6])
@pytest.mark.parametrize("kind,n", [("u10", 1 << 20), ("u10", 100003), ("eq", 1 << 18), ("unit", 300001),
                                    ("ramp", 200000), ("himeno", 1 << 18), ("mixed", 500000), ("sparse", 400009)])
@pytest.mark.parametrize("ct", CTS)
def test_decode3_roundtrip(v3, oracle, bound, kind, n, ct):
    v3.set_bound(bound)
    x = _inputs(oracle, kind, n)
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = v3.compress(ct, xs, t, m17)
    out = v3.decompress(ct, s, n, t, m17)
    spec, got = oracle.decompress(ct, s, n, bound, t, m17)
    assert got == n
    assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))
    if kind == "u10":
        # (a constant input, the Himeno rows and a slow ramp are locally periodic: paths read out of phase
        # meet late or never; denser streams can overflow a job's output buffer: the segment decoder hands
        # both to the chunk-map decoder)
        assert v3.last_decode_was_v3(), "an ordinary stream left the segment decoder"


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 63, 64, 65, 255, 256, 257, 4095, 4096, 4097, 8191, 12345, 65537,
                               262143])
@pytest.mark.parametrize("ct", CTS)
def test_decode3_ragged(v3, oracle, n, ct):
    v3.set_bound(1e-3)
    x = oracle.gen_u10(n, seed=n)
    x[::7] = x[0]
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = v3.compress(ct, xs, t, m17)
    out = v3.decompress(ct, s, n, t, m17)
    spec, _ = oracle.decompress(ct, s, n, 1e-3, t, m17)
    assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))


@pytest.mark.parametrize("ct", CTS)
@pytest.mark.parametrize("log2n", [22, 24])
def test_decode3_device_chain(dc, oracle, ct, log2n):
    """encode_device -> decode_device with the bit count left on the device (the bench's path, default
    thresholds): the segment decoder runs and equals the oracle."""
    import torch
    n = 1 << log2n
    dc.set_bound(1e-3)
    x = oracle.gen_u10(n)
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    dev = torch.device("cuda", 0)
    xd = torch.from_numpy(xs).to(dev)
    cap = dc.stream_capacity(n)
    st = torch.zeros(cap, dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    nbits = torch.zeros(1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    dc.encode_device(ct, xd.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17, total_ptr=nbits.data_ptr())
    dc.decode_device(ct, st.data_ptr(), -1, n, out.data_ptr(), type_=t, mask17=m17, d_nbits=nbits.data_ptr(),
                     max_bytes=cap)
    dc.decode_finish()
    assert dc.last_decode_was_v3()
    nb = (int(nbits.item()) + 7) // 8
    s = st[:nb].cpu().numpy()
    spec, got = oracle.decompress(ct, s, n, 1e-3, t, m17)
    assert got == n
    assert np.array_equal(out.cpu().numpy().view(np.uint32), spec.view(np.uint32))


@pytest.mark.parametrize("ct", [5, 7, 11])
@pytest.mark.parametrize("n,kind", [(1 << 18, "zeros"), (100003, "zeros"), (5, "zeros"), (1 << 18, "one"),
                                    (1 << 18, "last"), (65537, "tiny")])
def test_decode3_zero_runs(v3, oracle, ct, n, kind):
    """Runs-mode streams of '100' codes only (constant input after toSmallDataset, BASELINE config 3) decode
    to zeros inside the segment decoder; one value outside the bound anywhere (first, last) makes it hand
    the stream to the chunk-map decoder -- both exact against the oracle's grammar decoder."""
    v3.set_bound(1e-3)
    x = np.full(n, np.float32(0.123456789))
    if kind == "one":
        x[n // 3] = np.float32(5.0)
    elif kind == "last":
        x[-1] = np.float32(5.0)
    elif kind == "tiny":                                  # values inside the bound: still '100' codes
        x[::17] = np.float32(0.123456789 + 4e-4)
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = v3.compress(ct, xs, t, m17)
    out = v3.decompress(ct, s, n, t, m17)
    spec, got = oracle.decompress(ct, s, n, 1e-3, t, m17)
    assert got == n
    assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))
    if kind in ("zeros", "tiny"):
        assert v3.last_decode_was_v3() and not out.view(np.uint32).any()
    else:
        assert not v3.last_decode_was_v3()


@pytest.mark.parametrize("seg", [4, 8, 16, 20, 24])
@pytest.mark.parametrize("kind,n", [("u10", 1 << 20), ("u10", 12345), ("mixed", 500000), ("sparse", 400009),
                                    ("u10", 4097)])
@pytest.mark.parametrize("ct", CTS)
def test_decode3_segment_lengths(v3, oracle, seg, kind, n, ct):
    """Every parse segment length (4, 8, 16, 20, 24 chunks: the pre-walk, the record stores, the jobs per parse
    job, decode jobs starting inside a segment) decodes exactly; ordinary streams stay in the segment decoder at
    each (the maps parse keeps 16-chunk parse jobs when the length does not divide 128 decode jobs)."""
    old = v3.set_decode3_seg(seg)
    try:
        v3.set_bound(1e-3)
        x = _inputs(oracle, kind, n)
        _, xs = oracle.to_small(x)
        t, m17 = oracle.type_mask(xs)
        s, nb, pos = v3.compress(ct, xs, t, m17)
        out = v3.decompress(ct, s, n, t, m17)
        spec, got = oracle.decompress(ct, s, n, 1e-3, t, m17)
        assert got == n
        assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))
        if kind == "u10":
            assert v3.last_decode_was_v3(), "an ordinary stream left the segment decoder"
    finally:
        v3.set_decode3_seg(old)


@pytest.mark.parametrize("ct,lg,bound", [(11, 24, 1e-3), (6, 24, 1e-3), (6, 25, 1e-3), (5, 24, 1e-3),
                                         (7, 24, 1e-3), (6, 20, 1e-6), (6, 24, 1e-6), (11, 22, 1e-6)])
def test_default_segment_length_mid_sizes(v3, oracle, ct, lg, bound):
    """The default segment length (dc_decode3_seg) and exit publication keep mid-size U10 streams in the
    segment decoder: 8-chunk segments declined CT11 from 2^24 floats and CT6 from 2^25, and CT6 at a bound
    of 1e-6 declined at every size (a job exit moved after it was published), so those take 16-chunk
    segments and CT6 publishes after its in-job repairs; device stream, decode against the oracle's."""
    import torch
    v3.set_bound(bound)
    n = 1 << lg
    _, xs = oracle.to_small(oracle.gen_u10(n))
    t, m17 = oracle.type_mask(xs)
    s, nb, _ = oracle.compress(ct, xs, bound, t, m17)
    spec, got = oracle.decompress(ct, s, n, bound, t, m17)
    assert got == n
    d_s = torch.from_numpy(np.concatenate([s, np.zeros(64, np.uint8)])).cuda()
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    v3.decode_device(ct, d_s.data_ptr(), nb, n, out.data_ptr(), type_=t, mask17=m17, max_bytes=d_s.numel())
    v3.decode_finish()
    assert v3.last_decode_was_v3(), "the stream left the segment decoder"
    assert np.array_equal(out.cpu().numpy().view(np.uint32), spec.view(np.uint32))


@pytest.mark.parametrize("ct", [5, 7])
@pytest.mark.parametrize("lg", [20, 24])
def test_decode3_dense_streams(v3, oracle, ct, lg):
    """Dense streams (CT7 at a bound of 1e-2: fewer than ~16 bits per value, more values per 64-chunk decode
    job than the 1040-value buffer) stay on the segment decoder: the dense instantiation (2080 values per
    job) takes them -- from the device path (bit count on the device: first decode declines DENSE and is
    redone dense inside dc_decode_finish, later ones start dense) and from the host ABI (length known)."""
    import torch
    v3.set_bound(1e-2)
    try:
        n = 1 << lg
        _, xs = oracle.to_small(oracle.gen_u10(n))
        t, m17 = oracle.type_mask(xs)
        s, nb, _ = oracle.compress(ct, xs, 1e-2, t, m17)
        ref, _ = oracle.decompress(ct, s, n, 1e-2, t, m17)
        out = v3.decompress(ct, s, n, t, m17)                     # host ABI: nbytes known
        assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))
        assert v3.L.dc_last_decode_was_v3()
        dx = torch.from_numpy(xs).cuda()
        cap = v3.stream_capacity(n)
        st = torch.zeros(cap, dtype=torch.uint8, device="cuda")
        d_nbits = torch.zeros(1, dtype=torch.int64, device="cuda")
        o = torch.empty(n, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        for _ in range(2):                                        # device path, twice (the hint sticks)
            o.fill_(-7.0)
            torch.cuda.synchronize()
            v3.encode_device(ct, dx.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17, total_ptr=d_nbits.data_ptr())
            v3.decode_device(ct, st.data_ptr(), -1, n, o.data_ptr(), type_=t, mask17=m17, d_nbits=d_nbits.data_ptr(),
                             max_bytes=cap)
            v3.decode_finish()
            assert v3.L.dc_last_decode_was_v3()
            assert np.array_equal(o.cpu().numpy().view(np.uint32), ref.view(np.uint32))
        assert nb * 8 < 18 * n                                    # (the case is dense)
    finally:
        v3.set_bound(1e-3)


@pytest.fixture
def v3maps(dc):
    old = dc.set_decode3_min_bytes(0)
    oldm = dc.L.dc_set_decode3_maps(1)             # every stream parsed by entry -> exit maps
    yield dc
    dc.L.dc_set_decode3_maps(oldm)
    dc.set_decode3_min_bytes(old)


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("ct", CTS)
def test_maps_parse_golden(v3maps, oracle, bound, case, ct):
    """The maps parse (dc_decode_maps.hip) in place of parse3 on every golden stream: the segment decoder's values
    from its records equal the grammar decoder (runs-mode streams decline to the other decoders as before)."""
    g = golden(bound)
    v3maps.set_bound(bound)
    s = g[f"{case}/ct{ct}/stream"]
    n = g[f"{case}/input"].size
    t, m17 = int(g[f"{case}/type"]), int(g[f"{case}/mask17"])
    out = v3maps.decompress(ct, s, n, t, m17)
    spec, _ = oracle.decompress(ct, s, n, bound, t, m17)
    assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))


def _slow_sync(kind, n):
    i = np.arange(n, dtype=np.float64)
    if kind == "sine":
        x = np.sin(i * 1e-3) * 50.0 + np.sin(i * 0.37) * 0.5
    elif kind == "normal":
        x = np.random.default_rng(1).standard_normal(n)
    else:                                          # a noisy ramp
        x = i * 1e-4 + np.random.default_rng(2).random(n) * 1e-2
    x = x.astype(np.float32)
    return x - x.min()


@pytest.mark.parametrize("ct,kind,bound", [(7, "ramp", 1e-3), (5, "ramp", 1e-3), (7, "sine", 1e-5), (5, "sine", 1e-5),
                                           (11, "normal", 1e-3), (6, "sine", 1e-5)])
@pytest.mark.parametrize("lg", [16, 20])
def test_slow_sync_streams(v3, oracle, ct, kind, bound, lg):
    """Streams whose parse paths merge slowly (tools/experiments/sync_kinds.py: 20-200 kbit) stay on the segment
    decoder: parse3 declines them (paths not met) and dc_decode_finish parses them by maps; the values equal the
    grammar decoder.  Decoded twice: the second decode of the same parameters starts with the maps parse."""
    v3.set_bound(bound)
    try:
        n = 1 << lg
        xs = _slow_sync(kind, n)
        t, m17 = oracle.type_mask(xs)
        s, nb, _ = oracle.compress(ct, xs, bound, t, m17)
        ref, _ = oracle.decompress(ct, s, n, bound, t, m17)
        for _ in range(2):
            out = v3.decompress(ct, s, n, t, m17)
            assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))
            assert v3.L.dc_last_decode_was_v3()
    finally:
        v3.set_bound(1e-3)


@pytest.mark.parametrize("ct", [5, 7])
def test_slow_sync_large_seg20(dc, oracle, ct):
    """A noisy ramp large enough for 20-chunk parse segments (2^25 floats: > 2.5 M chunks of capacity) declines
    parse3 and is parsed by maps, which keep 16-chunk parse jobs (dc_maps_seg) -- decode3 after them uses the
    same; the values equal the grammar decoder's."""
    import torch
    dc.set_bound(1e-3)
    n = 1 << 25
    xs = _slow_sync("ramp", n)
    t, m17 = oracle.type_mask(xs)
    s, nb, _ = oracle.compress(ct, xs, 1e-3, t, m17)
    ref, _ = oracle.decompress(ct, s, n, 1e-3, t, m17)
    cap = dc.stream_capacity(n)
    d_s = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    d_s[:nb] = torch.from_numpy(s).cuda()
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    for force in (0, 1):                              # as parse3 leaves it, then parsed by maps for certain
        old = dc.L.dc_set_decode3_maps(force)
        try:
            out.fill_(-1.0)
            dc.decode_device(ct, d_s.data_ptr(), nb, n, out.data_ptr(), type_=t, mask17=m17, max_bytes=cap)
            dc.decode_finish()
            assert dc.L.dc_last_decode_was_v3()
            if force:
                assert dc.L.dc_last_decode_used_maps()
            assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
        finally:
            dc.L.dc_set_decode3_maps(old)
