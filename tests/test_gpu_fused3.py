"""GPU parity of the single-launch parse + decode (fused3_kernel, csrc/dc_decode3.hip) and of
its dynamic form (fused3d_kernel: decode jobs handed out from 8 queues, records handed to other CUs in the launch;
mode 2): switched on (dc_set_fused3) for 16-chunk-segment streams, every segment length it can take (16, 20, 24, 32,
64 chunks) must decode bit for bit as the oracle's grammar decoder, from host and device bit counts, for the
golden streams, ragged sizes, prediction-heavy streams and the zero-run streams it fills itself."""
import os

import numpy as np
import pytest

from conftest import BOUNDS, CASES, golden
from test_gpu_decode3 import _inputs

pytestmark = pytest.mark.gpu
CTS = [5, 6, 7, 11]
SEGS = [16, 20, 24, 32, 64]


@pytest.fixture(params=[1, 2], ids=["static", "dynamic"])
def f3(dc, request):
    old_min = dc.set_decode3_min_bytes(0)         # every stream through the segment decoder ...
    old_seg = dc.set_decode3_seg(16)               # ... with 16-chunk segments: the fused launch's streams
    old_f = dc.set_fused3(request.param)
    dc.L.dc_set_decode3_maps(-1)                   # (no parameters remembered for the maps parse or dense buffer)
    yield dc
    dc.set_fused3(old_f)
    dc.set_decode3_seg(old_seg)
    dc.set_decode3_min_bytes(old_min)
    os.environ.pop("DC_FUSED3_SEG", None)


def _dense(ct, nb, n):
    """The host's up-front choice of the dense job buffer (dc_host.c decode_device_h): such streams keep the
    two launches (the fused kernel has the ordinary buffer only)."""
    return nb * 8 < 18 * n and (ct == 6 or nb * 8 >= 6 * n)


def _check(dc, oracle, ct, xs, bound, ordinary=True):
    n = xs.size
    t, m17 = oracle.type_mask(xs)
    s, nb, pos = dc.compress(ct, xs, t, m17)
    out = dc.decompress(ct, s, n, t, m17)
    spec, got = oracle.decompress(ct, s, n, bound, t, m17)
    assert got == n
    assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))
    fused = dc.last_decode_fused()
    # (a stream of parameters whose parse paths once did not meet starts with the maps parse: dc_host.c maps_key)
    if ordinary and dc.last_decode_was_v3() and not dc.L.dc_last_decode_used_maps():
        assert fused == (not _dense(ct, nb, n)), "an ordinary stream did not take the fused launch"
    return out, fused


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("ct", CTS)
def test_fused3_golden(f3, oracle, bound, case, ct):
    g = golden(bound)
    f3.set_bound(bound)
    key = f"{case}/ct{ct}"
    s = g[key + "/stream"]
    n = g[f"{case}/input"].size
    t, m17 = int(g[f"{case}/type"]), int(g[f"{case}/mask17"])
    out = f3.decompress(ct, s, n, t, m17)
    spec, got = oracle.decompress(ct, s, n, bound, t, m17)
    assert got == n
    assert np.array_equal(out.view(np.uint32), spec.view(np.uint32))
    if bool(g[key + "/ref_consistent"]):
        assert np.array_equal(out.view(np.uint32), g[key + "/ref_decoded"].view(np.uint32))


@pytest.mark.parametrize("seg", SEGS)
@pytest.mark.parametrize("kind,n", [("u10", 1 << 20), ("u10", 12345), ("u10", 4097), ("mixed", 500000),
                                    ("sparse", 400009), ("unit", 300001)])
@pytest.mark.parametrize("ct", CTS)
def test_fused3_segment_lengths(f3, oracle, seg, kind, n, ct):
    """Every fused segment length (the parse jobs' record stores -- 20- and 24-chunk segments end on an 8-byte
    store -- and each decode job's first token when decode jobs start inside a segment) decodes exactly."""
    os.environ["DC_FUSED3_SEG"] = str(seg)
    f3.set_bound(1e-3)
    _, xs = oracle.to_small(_inputs(oracle, kind, n))
    # (prediction-heavy streams may need the maps parse or the dense buffer: the two launches take them)
    out, fused = _check(f3, oracle, ct, xs, 1e-3, ordinary=kind == "u10")
    if kind == "u10":
        assert f3.last_decode_was_v3(), "an ordinary stream left the segment decoder"
    if fused:
        assert f3.fused3_last_seg() == seg


@pytest.mark.parametrize("n", [1, 3, 64, 65, 4095, 4097, 65537, 262143])
@pytest.mark.parametrize("ct", CTS)
def test_fused3_ragged(f3, oracle, n, ct):
    f3.set_bound(1e-3)
    x = oracle.gen_u10(n, seed=n)
    x[::7] = x[0]
    _, xs = oracle.to_small(x)
    _check(f3, oracle, ct, xs, 1e-3, ordinary=n >= 64)     # (streams under 16 bytes: the chunk-map decoder)


@pytest.mark.parametrize("ct", [5, 7, 11])
@pytest.mark.parametrize("n,kind", [(1 << 18, "zeros"), (100003, "zeros"), (5, "zeros"), (1 << 18, "one"),
                                    (1 << 18, "last"), (65537, "tiny")])
def test_fused3_zero_runs(f3, oracle, ct, n, kind):
    """Runs-mode streams: the fused launch writes the zeros while checking the pattern; one value outside the
    bound declines it to the chunk-map decoder, which writes the output again -- both exact."""
    f3.set_bound(1e-3)
    x = np.full(n, np.float32(0.123456789))
    if kind == "one":
        x[n // 3] = np.float32(5.0)
    elif kind == "last":
        x[-1] = np.float32(5.0)
    elif kind == "tiny":
        x[::17] = np.float32(0.123456789 + 4e-4)
    _, xs = oracle.to_small(x)
    out, fused = _check(f3, oracle, ct, xs, 1e-3)
    assert fused
    if kind in ("zeros", "tiny"):
        assert f3.last_decode_was_v3() and not out.view(np.uint32).any()
    else:
        assert not f3.last_decode_was_v3()


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("ct", CTS)
@pytest.mark.parametrize("log2n", [22, 24])
def test_fused3_device_chain(dc, oracle, ct, log2n, mode):
    """encode_device -> decode_device with the bit count on the device (the bench's path, default thresholds,
    the fused launch switched on; its segment length from the stream's capacity) equals the oracle."""
    import torch
    old = dc.set_fused3(mode)
    try:
        n = 1 << log2n
        dc.set_bound(1e-3)
        _, xs = oracle.to_small(oracle.gen_u10(n))
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
        spec, got = oracle.decompress(ct, st[:nb].cpu().numpy(), n, 1e-3, t, m17)
        assert got == n
        assert np.array_equal(out.cpu().numpy().view(np.uint32), spec.view(np.uint32))
    finally:
        dc.set_fused3(old)


@pytest.mark.parametrize("mode", [1, 2])
def test_fused3_bench_size(dc, oracle, mode):
    """The bench's workload (CT7, U10 2^26, bound 1e-3, host bit count: the model picks the segment length)
    through the fused launch, back to back twice (epochs; fused3d: its queue heads reset between launches),
    against the oracle."""
    import torch
    old = dc.set_fused3(mode)
    try:
        n = 1 << 26
        dc.set_bound(1e-3)
        _, xs = oracle.to_small(oracle.gen_u10(n))
        t, m17 = oracle.type_mask(xs)
        s, nb, _ = oracle.compress(7, xs, 1e-3, t, m17)
        spec, got = oracle.decompress(7, s, n, 1e-3, t, m17)
        d_s = torch.from_numpy(np.concatenate([s, np.zeros(64, np.uint8)])).cuda()
        out = torch.empty(n, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        for _ in range(3):
            out.fill_(-1.0)
            dc.decode_device(7, d_s.data_ptr(), nb, n, out.data_ptr(), type_=t, mask17=m17, max_bytes=d_s.numel())
            dc.decode_finish()
            assert dc.last_decode_was_v3() and dc.last_decode_fused()
            assert np.array_equal(out.cpu().numpy().view(np.uint32), spec.view(np.uint32))
    finally:
        dc.set_fused3(old)
