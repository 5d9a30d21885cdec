"""GPU parity at the BASELINE.json sizes (configs 2, 3 and 5, and the bench's own CT7 U10 2^26 shape).

Every case runs the device API the bench times (dc_encode_device / dc_decode_device on HBM-resident
buffers) and compares, bit for bit, against the CPU oracle (the C restatement of impl/dataCompression.c,
pinned to the compiled reference's fixtures in test_oracle.py):
  * the stream: its bit length (-> bytes and pos) and every byte (orc_compress),
  * the decode of that stream (orc_decompress_spec, the reference decoder's grammar),
  * that the decode completed on the fast path (dc_decode_status == 0) where the bench relies on it.
At 2^28 floats the single-pass encoder has 65,536 tiles (4x the bench's 16,384): its scanner workgroup and the
tiles' look-backs over the scanner's inclusive states run 4x as long (encode_fused_kernel, dc_encode.hip).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _u10(oracle, n):
    return oracle.gen_u10(n)


def _eq(n):
    # tools/float_eq_262144.txt (every line 0.123456789) tiled x1024 -> 2^28 (BASELINE configs[2])
    return np.full(n, np.float32(0.123456789), np.float32)


def _device_roundtrip(dc, oracle, ct, xs, bound, t, m17):
    import torch
    n = xs.size
    dx = torch.from_numpy(xs).cuda()
    cap = dc.stream_capacity(n)
    st = torch.empty(cap, dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    nbits_d = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    dc.encode_device(ct, dx.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17, total_ptr=nbits_d.data_ptr())
    nbits = dc.encode_result()
    nb = (nbits + 7) // 8
    # decode straight from the encoder's device bit count (the bench's chaining)
    dc.decode_device(ct, st.data_ptr(), -1, n, out.data_ptr(), type_=t, mask17=m17, d_nbits=nbits_d.data_ptr(),
                     max_bytes=cap)
    status = dc.decode_status()
    dc.decode_finish()
    s = st[:nb].cpu().numpy()
    o = out.cpu().numpy()
    del dx, st, out
    torch.cuda.empty_cache()
    return s, nbits, o, status


def _check(dc, oracle, ct, x, bound, want_fast=True):
    dc.set_bound(bound)
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    s, nbits, out, status = _device_roundtrip(dc, oracle, ct, xs, bound, t, m17)
    so, nbo, poso = oracle.compress(ct, xs, bound, t, m17)
    pos = 8 - (nbits & 7) if nbits & 7 else 8
    assert (nbits + 7) // 8 == nbo and pos == poso
    assert np.array_equal(s, so)
    del so
    ref, got = oracle.decompress(ct, s, xs.size, bound, t, m17)
    assert got == xs.size
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))
    if want_fast:
        assert status == 0, f"decoder left the fast path (status 0x{status:x})"
    return nbits


def test_config3_ct7_eq_2p28(dc, oracle):
    """BASELINE configs[2]: CT7 on float_eq tiled to 2^28 -> 100,663,296 bytes of '100' tokens."""
    n = 1 << 28
    nbits = _check(dc, oracle, 7, _eq(n), 1e-3, want_fast=False)
    assert nbits == 3 * n


def test_ct7_u10_2p28(dc, oracle):
    """The 2^28 end of the north_star sweep on real data (65,536 encoder tiles, 2^28 decode)."""
    _check(dc, oracle, 7, _u10(oracle, 1 << 28), 1e-3)


def test_ct7_u10_2p26(dc, oracle):
    """The bench workload itself (BASELINE metric): CT7 U10 2^26 @1e-3 -> 162,634,383 bytes."""
    nbits = _check(dc, oracle, 7, _u10(oracle, 1 << 26), 1e-3)
    assert (nbits + 7) // 8 == 162634383


def test_config2_ct6_u10_2p26(dc, oracle):
    """BASELINE configs[1]: CT6 (bit-wise, no prediction) on 2^26 U10 -> 171,129,120 bytes."""
    nbits = _check(dc, oracle, 6, _u10(oracle, 1 << 26), 1e-3)
    assert (nbits + 7) // 8 == 171129120


def test_config5_ct9_ber_2p26(dc, oracle):
    """BASELINE configs[4]: CT9 = CT7 stream + CRC-32 at BER 1e-6 with floor(bits*BER) real bit flips on
    2^26 U10: the receiver's CRC differs (damage detected), the resent clean stream passes and decodes
    bit-identically to the oracle's decode of the oracle's own stream."""
    import zlib
    import torch
    dc.set_bound(1e-3)
    n = 1 << 26
    _, xs = oracle.to_small(_u10(oracle, n))
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
    nflip = int(nbits * 1e-6)
    assert nflip == 1301
    dc.flip_bits_device(rcv.data_ptr(), nbits, nflip, 777)
    dc.crc32_device_async(rcv.data_ptr(), nb, crc.data_ptr() + 4)
    dc.synchronize()
    clean = snd[:nb].cpu().numpy()
    c = crc.cpu().numpy().view(np.uint32)
    assert c[0] == zlib.crc32(clean.tobytes())
    assert c[0] != c[1]
    so, nbo, _ = oracle.compress(7, xs, 1e-3, t, m17)
    assert nbo == nb and np.array_equal(clean, so)
    rcv.copy_(snd)
    torch.cuda.synchronize()
    dc.crc32_device_async(rcv.data_ptr(), nb, crc.data_ptr() + 4)
    dc.synchronize()
    c = crc.cpu().numpy().view(np.uint32)
    assert c[0] == c[1]
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    dc.decode_device(7, rcv.data_ptr(), nb, n, out.data_ptr(), type_=t, mask17=m17)
    assert dc.decode_status() == 0
    dc.decode_finish()
    ref, _ = oracle.decompress(7, clean, n, 1e-3, t, m17)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_decode_status_reports_chained_slow_path(dc, oracle):
    """Several decodes queued before one finish: if one of them left the fast path the status word says
    so (dc_decode_status), and dc_decode_finish refuses to pretend the earlier decode completed."""
    import torch
    import dcamd
    dc.set_bound(1e-3)
    n = 1 << 16
    xs = np.full(n, np.float32(0.0))                   # a constant CT6 stream: locally periodic -> slow path
    s, nb, _ = dc.compress(6, xs)
    ds = torch.from_numpy(s).cuda()
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    dc.decode_device(6, ds.data_ptr(), nb, n, out.data_ptr())
    st1 = dc.decode_status()
    dc.decode_device(6, ds.data_ptr(), nb, n, out.data_ptr())
    if st1 == 0:
        dc.decode_finish()
        pytest.skip("this stream stays on the fast path")
    assert dc.decode_status() != 0
    with pytest.raises(dcamd.DCError):
        dc.decode_finish()
    dc.decode_device(6, ds.data_ptr(), nb, n, out.data_ptr())     # a single decode is completed exactly
    dc.decode_finish()
    ref, _ = oracle.decompress(6, s, n, 1e-3)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_encode_stream_orders_after_library_stream(dc, oracle):
    """dc_set_encode_stream: an encode on the caller's stream waits for work queued on the library stream
    (the halo path / host ABI fill the encoder's input on the library stream)."""
    import ctypes
    import torch
    dc.set_bound(1e-3)
    n = 1 << 20
    x = oracle.gen_u10(n)
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    es = torch.cuda.Stream()
    dc.check(dc.L.dc_set_encode_stream(ctypes.c_void_p(es.cuda_stream)), "dc_set_encode_stream")
    try:
        for ct in (5, 7):
            s, nb, pos = dc.compress(ct, xs, t, m17)            # host ABI: H2D + encode
            so, nbo, poso = oracle.compress(ct, xs, 1e-3, t, m17)
            assert nb == nbo and pos == poso and np.array_equal(s, so)
    finally:
        dc.L.dc_set_encode_stream(None)


def test_back_to_back_encodes_2p26(dc, oracle):
    """The bench's timed loop: 48 single-pass encodes of the CT7 2^26 workload back to back on one stream.
    The encoder's error word is sticky (only dc_encode_result's retry clears it), so any look-back or hand-off
    timeout in any of them shows; every stream must equal the first, which equals the oracle's."""
    import torch
    dc.set_bound(1e-3)
    n = 1 << 26
    _, xs = oracle.to_small(_u10(oracle, n))
    t, m17 = oracle.type_mask(xs)
    dx = torch.from_numpy(xs).cuda()
    cap = dc.stream_capacity(n)
    st = torch.empty(cap, dtype=torch.uint8, device="cuda")
    first = torch.empty_like(st)
    torch.cuda.synchronize()
    dc.encode_device(7, dx.data_ptr(), n, first.data_ptr(), type_=t, mask17=m17)
    nbits = dc.encode_result()
    assert dc.encode_status() == 0
    nb = (nbits + 7) // 8
    so, nbo, _ = oracle.compress(7, xs, 1e-3, t, m17)
    assert nb == nbo and np.array_equal(first[:nb].cpu().numpy(), so)
    del so
    same = True
    for _ in range(48):
        st.zero_()
        torch.cuda.synchronize()          # (the library stream is non-blocking: no order with torch's)
        dc.encode_device(7, dx.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17)
        dc.synchronize()
        same &= bool(torch.equal(st[:nb], first[:nb]))
    status = dc.encode_status()
    assert status == 0, f"encoder error word 0x{status:x}"
    assert same
    del dx, st, first
    torch.cuda.empty_cache()


@pytest.mark.parametrize("help_", [0, 1])
@pytest.mark.parametrize("per_cu,lds,log2n", [(1, 0, 22), (4, 0, 24), (2, 65536, 24), (6, 0, 22)])
def test_encode_beside_occupying_kernel(dc, oracle, per_cu, lds, log2n, help_):
    """The single-pass encoder while another kernel holds CU slots on a second stream of the same process
    (forward progress under co-residency).  Its tiles wait only for lower tiles, which in-order
    dispatch has made resident, so the neighbour slows it but cannot wedge it; a wait that did reach its bound
    (20 ms AND 8192 polls: dc_encode.hip WaitBound) would have taken the exact three-launch fallback.  Either way
    the stream equals the oracle's, and the encoder's error word is clear after dc_encode_result."""
    import torch
    n = 1 << log2n
    dc.set_bound(1e-3)
    _, xs = oracle.to_small(_u10(oracle, n))
    t, m17 = oracle.type_mask(xs)
    dx = torch.from_numpy(xs).cuda()
    cap = dc.stream_capacity(n)
    st = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    retries0 = int(dc.L.dc_encode_retries())
    side = torch.cuda.Stream()
    old = dc.L.dc_set_encode_help(help_)            # (1: the helping instantiation, as ranks sharing a GPU run)
    try:
        for _ in range(3):
            dc.occupy_device(side.cuda_stream, 4000.0, per_cu * 256, lds)    # 4 ms beside each encode
            dc.encode_device(7, dx.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17)
            nbits = dc.encode_result()
            assert dc.encode_status() == 0
    finally:
        dc.L.dc_set_encode_help(old)
    torch.cuda.synchronize()
    so, nbo, _ = oracle.compress(7, xs, 1e-3, t, m17)
    assert (nbits + 7) // 8 == nbo
    assert np.array_equal(st[:nbo].cpu().numpy(), so)
    print(f"encoder fallbacks beside the neighbour: {int(dc.L.dc_encode_retries()) - retries0}")
