"""The one-workgroup decoder of small streams (dc_decode_tiny.hip: at most 2^14 values and 2^19 bits) against the
oracle's grammar decoder, bit for bit, at the sizes and contents the reference's apps send (impl/pingpong.c: 2^14
floats; the decoders of impl/dataCompression.c:1703-2027 CT7, :2922-3135 CT5, :2459-2630 CT6, :698-797 CT11).  A
stream it declines (runs of predictions: constant or copy-run data, the -1.0f history sentinel) must still decode
exactly, on the decoder the host falls back to."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def tiny_on(dc):
    """the one-workgroup decoder is opt-in (dc_set_decode_tiny(1)): on for these tests"""
    prev = dc.L.dc_set_decode_tiny(1)
    yield
    dc.L.dc_set_decode_tiny(prev)


def _x(oracle, kind, n):
    rs = np.random.RandomState(n % 977 + 1)
    if kind == "u10":
        return oracle.gen_u10(n)
    if kind == "unit":
        return rs.rand(n).astype(np.float32)
    if kind == "ramp":
        return (np.float32(0.0005) * np.arange(n, dtype=np.float32)).astype(np.float32)
    if kind == "sine":                                   # smooth: many predictions, pending prefixes
        return (np.sin(np.arange(n, dtype=np.float32) * np.float32(0.01)) * np.float32(5) + np.float32(5)).astype(np.float32)
    if kind == "eq":                                     # runs mode: the tiny decoder declines, the fallback decodes
        return np.full(n, np.float32(0.123456789))
    if kind == "wide":
        return (rs.rand(n) * np.exp2(rs.randint(-20, 20, n))).astype(np.float32)
    if kind == "mixed":
        x = oracle.gen_u10(n)
        for r in rs.randint(0, n, 8):
            x[r:r + 300] = x[r]
        return x
    raise ValueError(kind)


@pytest.mark.parametrize("bound", [1e-3, 1e-6])
@pytest.mark.parametrize("kind", ["u10", "unit", "ramp", "sine", "eq", "wide", "mixed"])
@pytest.mark.parametrize("n", [1, 3, 4, 5, 100, 1000, 4097, 12345, 16383, 16384])
@pytest.mark.parametrize("ct", [5, 6, 7, 11])
def test_tiny_vs_oracle(dc, oracle, ct, n, kind, bound):
    dc.set_bound(bound)
    dc.L.dc_set_decode3_maps(-1)                          # (forget the parameters an earlier stream declined for)
    x = _x(oracle, kind, n)
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = dc.compress(ct, xs, t, m17)
    out = dc.decompress(ct, s, n, t, m17)
    spec, got = oracle.decompress(ct, s, n, bound, t, m17)
    assert got == n
    assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))
    if kind in ("u10", "unit") and bound == 1e-3 and n >= 12345 and ct != 11:
        # (smaller streams: the small-stream decoder; CT11's 32-bit tokens resynchronise slowly and its link chains
        # may pass the rounds: the segment decoder then)
        assert dc.L.dc_last_decode_was_tiny() == 1, "a small ordinary stream left the one-workgroup decoder"


def test_tiny_decline_goes_to_segment_decoder(dc, oracle):
    """a stream the one-workgroup decoder declines for its link rounds (CT11 on data whose 32-bit tokens stay out of
    phase) is decoded by the segment decoder, and later streams of these parameters start there"""
    dc.set_bound(1e-3)
    dc.L.dc_set_decode3_maps(-1)                          # (forget remembered parameters)
    n = 16384
    xs = oracle.to_small((np.random.RandomState(5).rand(n)).astype(np.float32))[1]
    s, nb, pos = dc.compress(11, xs, 0, 0)
    for _ in range(2):
        out = dc.decompress(11, s, n, 0, 0)
        spec, got = oracle.decompress(11, s, n, 1e-3, 0, 0)
        assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))
    dc.L.dc_set_decode3_maps(-1)


def test_tiny_switch(dc, oracle):
    """dc_set_decode_tiny(0) keeps small streams on the segment decoder: the same values"""
    dc.set_bound(1e-3)
    n = 16384
    xs = oracle.to_small(oracle.gen_u10(n))[1]
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = dc.compress(7, xs, t, m17)
    a = dc.decompress(7, s, n, t, m17)
    assert dc.L.dc_last_decode_was_tiny() == 1
    prev = dc.L.dc_set_decode_tiny(0)
    try:
        b = dc.decompress(7, s, n, t, m17)
        assert dc.L.dc_last_decode_was_tiny() == 0
    finally:
        dc.L.dc_set_decode_tiny(prev)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
