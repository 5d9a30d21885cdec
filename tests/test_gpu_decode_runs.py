"""GPU parity of the small-stream decoder (csrc/dc_decode_runs.hip): every stream of at most 8192 chunks
(256 KiB) -- the Himeno halo planes (runs-mode '101' copy runs, BASELINE config 4), constant inputs ('100'
runs), ordinary data, prediction chains across chunk and block boundaries -- decoded through it (forced by
the capacity threshold) must equal the oracle's grammar decoder bit for bit, and stay on this path (no
hand-over to the chunk-map decoder) for the streams it is built for."""
import numpy as np
import pytest

from test_gpu_decode3 import _inputs

pytestmark = pytest.mark.gpu
CTS = [5, 6, 7, 11]


@pytest.fixture
def rd(dc):
    old = dc.set_runs_max_bytes(1 << 30)            # every stream that fits through the small-stream decoder
    yield dc
    dc.set_runs_max_bytes(old)


@pytest.mark.parametrize("bound", [1e-3, 1e-6])
@pytest.mark.parametrize("kind,n", [("u10", 16384), ("u10", 4097), ("eq", 65536), ("himeno", 65536),
                                    ("mixed", 50000), ("sparse", 40009), ("ramp", 20000), ("unit", 30001)])
@pytest.mark.parametrize("ct", CTS)
def test_runs_roundtrip(rd, oracle, bound, kind, n, ct):
    rd.set_bound(bound)
    x = _inputs(oracle, kind, n)
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = rd.compress(ct, xs, t, m17)
    out = rd.decompress(ct, s, n, t, m17)
    spec, got = oracle.decompress(ct, s, n, bound, t, m17)
    assert got == n
    assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))
    if nb <= 8192 * 32 and kind in ("u10", "eq", "himeno"):
        assert rd.last_decode_was_runs(), "a stream the small-stream decoder is built for left it"


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 31, 32, 33, 85, 86, 87, 255, 256, 257, 1023, 1024, 1025, 4095, 12345])
@pytest.mark.parametrize("ct", CTS)
def test_runs_ragged(rd, oracle, n, ct):
    rd.set_bound(1e-3)
    x = oracle.gen_u10(n, seed=n)
    x[::7] = x[0]
    x[n // 2:n // 2 + 40] = x[n // 2]                # a copy run in the middle
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = rd.compress(ct, xs, t, m17)
    out = rd.decompress(ct, s, n, t, m17)
    spec, _ = oracle.decompress(ct, s, n, 1e-3, t, m17)
    assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))


@pytest.mark.parametrize("ct", [5, 7, 11])
def test_runs_long_copy_chains(rd, oracle, ct):
    """Copy runs longer than a chunk and than a thread's block (the carry scan of slot maps): rows of 700
    equal values, each row's first value a new one -- the Himeno plane's structure with longer rows."""
    rd.set_bound(1e-3)
    rows = [np.full(700, np.float32(v)) for v in oracle.gen_u10(90, seed=5)]
    x = np.concatenate(rows).astype(np.float32)
    n = x.size
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = rd.compress(ct, xs, t, m17)
    out = rd.decompress(ct, s, n, t, m17)
    spec, _ = oracle.decompress(ct, s, n, 1e-3, t, m17)
    assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))
    assert rd.last_decode_was_runs()


def test_runs_device_chain_default_threshold(dc, oracle):
    """2^12 floats with default thresholds (16 KiB + 68 of capacity): encode_device -> decode_device from
    the device bit count goes through the small-stream decoder and equals the oracle."""
    import torch
    n = 1 << 12
    dc.set_bound(1e-3)
    _, xs = oracle.to_small(oracle.gen_u10(n))
    t, m17 = oracle.type_mask(xs)
    xd = torch.from_numpy(xs).cuda()
    cap = dc.stream_capacity(n)
    st = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    nbits = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    dc.encode_device(7, xd.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17, total_ptr=nbits.data_ptr())
    dc.decode_device(7, st.data_ptr(), -1, n, out.data_ptr(), type_=t, mask17=m17, d_nbits=nbits.data_ptr(),
                     max_bytes=cap)
    dc.decode_finish()
    assert dc.last_decode_was_runs()
    nb = (int(nbits.item()) + 7) // 8
    spec, _ = oracle.decompress(7, st[:nb].cpu().numpy(), n, 1e-3, t, m17)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), spec.view(np.uint32))
