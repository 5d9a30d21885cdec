"""Single-token helpers and character-level Hamming routines of the reference header
(impl/dataCompression.h:64-156), exported by libdcamd from csrc/dc_host_token.c, checked against the
reference's own functions compiled from impl/dataCompression.c (oracle/_ref/libref_<bound>.so, built by
oracle/build_ref.sh).  Host code only: no GPU call."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle  # noqa: E402

libc = C.CDLL("libc.so.6")
libc.malloc.restype = C.c_void_p
libc.malloc.argtypes = [C.c_size_t]
libc.free.argtypes = [C.c_void_p]

BOUNDS = [1e-3, 1e-6]


def _ref(bound):
    try:
        return pyoracle.RefLib(bound).L
    except FileNotFoundError:
        pytest.skip("compiled reference (oracle/_ref) not built")


def _ours(bound):
    import dcamd
    L = dcamd.Lib().L
    L.dc_set_abs_error_bound.argtypes = [C.c_double]
    L.dc_set_abs_error_bound(bound)
    return L


def _setup(L, dbl=False):
    t = C.c_double if dbl else C.c_float
    sfx = "double" if dbl else "float"
    ap = [t, C.POINTER(C.c_void_p), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    getattr(L, "compress_bitwise_" + sfx).argtypes = ap
    getattr(L, "compress_bitwise_%s_mask" % sfx).argtypes = ap + [C.c_int, C.c_char_p]
    getattr(L, "decompress_bitwise_%s_np" % sfx).argtypes = [C.c_void_p, C.c_int]
    getattr(L, "decompress_bitwise_%s_np" % sfx).restype = t
    getattr(L, "decompress_bitwise_" + sfx).argtypes = [C.c_void_p, C.c_int, t, t, t]
    getattr(L, "decompress_bitwise_" + sfx).restype = t
    getattr(L, "decompress_bitwise_%s_mask" % sfx).argtypes = [C.c_void_p, C.c_int, t, t, t, C.c_int, C.c_char_p]
    getattr(L, "decompress_bitwise_%s_mask" % sfx).restype = t


def _append(L, fn, vals, *extra):
    p = C.c_void_p(None)
    nb = C.c_int(0)
    pos = C.c_int(8)
    for v in vals:
        getattr(L, fn)(v, C.byref(p), C.byref(nb), C.byref(pos), *extra)
    out = C.string_at(p.value, nb.value) if nb.value else b""
    libc.free(p)
    return out, nb.value, pos.value


def _inputs(dbl):
    rng = np.random.default_rng(7)
    dt = np.float64 if dbl else np.float32
    u10 = (rng.random(300) * 10).astype(dt)
    spec = np.array([0.0, 1e-40 if not dbl else 1e-310, 1e-3, 0.0009999, 3.5, 3.880054, 1.0, 2.0, 7.99, 1e6, 3e38 if not dbl else 1e300],
                    dt)
    return np.concatenate([u10, spec])


def _mask(mean, dbl):
    if dbl:
        u = int(np.array([mean], np.float64).view(np.uint64)[0])
        return "".join("1" if (u >> (63 - i)) & 1 else "0" for i in range(20)).encode()
    u = int(np.array([mean], np.float32).view(np.uint32)[0])
    return "".join("1" if (u >> (31 - i)) & 1 else "0" for i in range(17)).encode()


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("dbl", [False, True])
def test_compress_token_helpers_vs_reference(bound, dbl):
    R, O = _ref(bound), _ours(bound)
    for L in (R, O):
        _setup(L, dbl)
    sfx = "double" if dbl else "float"
    xs = [float(v) for v in _inputs(dbl)]
    assert _append(O, "compress_bitwise_" + sfx, xs) == _append(R, "compress_bitwise_" + sfx, xs)
    for t, mean in ((2, 3.880054), (1, 0.75), (3, 200.0)):
        m = _mask(mean, dbl)
        a = _append(O, "compress_bitwise_%s_mask" % sfx, xs, t, m)
        b = _append(R, "compress_bitwise_%s_mask" % sfx, xs, t, m)
        assert a == b, (t, mean)


def _token_strings(L, sfx, x, extra):
    """one element's token as a '0'/'1' string (encoded by the library under test)"""
    s, nb, pos = _append(L, "compress_bitwise_%s%s" % (sfx, "_mask" if extra else ""), [x], *extra)
    nbits = nb * 8 - (pos % 8 if pos != 8 else 0)
    bits = "".join(format(b, "08b") for b in s)[:nbits]
    return bits


def _cstr(bits, cap):
    """a malloc'd string (the reference reallocs it for raw tokens)"""
    p = libc.malloc(cap)
    C.memmove(p, bits.encode(), len(bits))
    return p


@pytest.mark.parametrize("bound", BOUNDS)
@pytest.mark.parametrize("dbl", [False, True])
def test_decompress_token_helpers_vs_reference(bound, dbl):
    R, O = _ref(bound), _ours(bound)
    for L in (R, O):
        _setup(L, dbl)
    sfx = "double" if dbl else "float"
    width = 64 if dbl else 32
    view = np.uint64 if dbl else np.uint32
    dt = np.float64 if dbl else np.float32

    def same(a, b):
        return np.array([a], dt).view(view)[0] == np.array([b], dt).view(view)[0]

    hist = (1.25, 0.5, 0.125)
    checked = 0
    for x in _inputs(dbl):
        x = float(x)
        bits = _token_strings(O, sfx, x, ())
        for fn, args in (("decompress_bitwise_%s_np" % sfx, ()), ("decompress_bitwise_" + sfx, hist)):
            pr, po = _cstr(bits, width + 1), _cstr(bits, width + 1)
            a = getattr(R, fn)(pr, len(bits), *args)
            b = getattr(O, fn)(po, len(bits), *args)
            assert same(a, b), (fn, x, bits)
            libc.free(po)          # the reference's copy may have moved (realloc): leaked, as the reference does
            checked += 1
        for t, mean in ((2, 3.880054), (1, 0.75)):
            m = _mask(mean, dbl)
            if bits[1:1 + t] == "1" * t:
                continue          # outside the type's domain (a raw exponent starting with `type` ones, :3593-3614)
            mb = _token_strings(O, sfx, x, (t, m))
            pr, po = _cstr(mb, width + 1), _cstr(mb, width + 1)
            a = getattr(R, "decompress_bitwise_%s_mask" % sfx)(pr, len(mb), *hist, t, m)
            b = getattr(O, "decompress_bitwise_%s_mask" % sfx)(po, len(mb), *hist, t, m)
            assert same(a, b), ("mask", x, t, mb)
            libc.free(po)
            checked += 1
    for code in ("100", "101", "110", "111"):          # the three predictors on the caller's history
        for fn, extra in (("decompress_bitwise_" + sfx, ()), ("decompress_bitwise_%s_mask" % sfx, (2, _mask(3.88, dbl)))):
            pr, po = _cstr(code, 4), _cstr(code, 4)
            a = getattr(R, fn)(pr, 3, *hist, *extra)
            b = getattr(O, fn)(po, 3, *hist, *extra)
            assert same(a, b), (fn, code)
            libc.free(pr)
            libc.free(po)
    assert checked > 500


def _ham_setup(L):
    L.hamming_code.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int]
    L.hamming_verify.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_char_p]
    L.error_info.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_int)]
    L.hamming_rectify.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int]
    L.cast_bits_to_char.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
    L.hamming_verify_bit.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_char_p]
    L.hamming_rectify_bit.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int]
    L.hmLength.argtypes = [C.c_int]


@pytest.mark.parametrize("nbytes", [1, 7, 40, 200])
def test_hamming_char_routines_vs_reference(nbytes):
    R, O = _ref(1e-3), _ours(1e-3)
    for L in (R, O):
        _ham_setup(L)
    rng = np.random.default_rng(nbytes)
    raw = bytes(rng.integers(0, 256, nbytes, dtype=np.uint8))
    k = nbytes * 8
    r = R.hmLength(k)
    assert O.hmLength(k) == r

    def run(L, flips):
        data = C.create_string_buffer(k + 1)
        L.cast_bits_to_char(raw, data, nbytes)
        c = C.create_string_buffer(r + 2)
        L.hamming_code(data, c, k, r)
        code = c.raw[:r + 1]
        d2 = bytearray(data.raw[:k])
        c2 = bytearray(code)
        for f in flips:                      # flip Hamming positions (check or data chars)
            if f < 0:
                c2[r] ^= 1                    # '0' <-> '1'
            else:
                d2[f] ^= 1
        db = C.create_string_buffer(bytes(d2) + b"\0")
        cb = C.create_string_buffer(bytes(c2) + b"\0")
        v = C.create_string_buffer(r + 2)
        L.hamming_verify(db, cb, k, r, v)
        pos = C.c_int(0)
        et = L.error_info(v, r, C.byref(pos))
        if et == 3:
            L.hamming_rectify(db, cb, k, r, pos.value)
        # byte-level twins on the same flips
        bb = bytearray(raw)
        for f in flips:
            if f >= 0:
                bb[f >> 3] ^= 1 << (7 - (f & 7))
        bbuf = C.create_string_buffer(bytes(bb), len(bb))
        cb2 = C.create_string_buffer(bytes(c2) + b"\0")
        v2 = C.create_string_buffer(r + 2)
        L.hamming_verify_bit(bbuf, cb2, nbytes, r, v2)
        pos2 = C.c_int(0)
        et2 = L.error_info(v2, r, C.byref(pos2))
        if et2 == 3:
            L.hamming_rectify_bit(bbuf, cb2, nbytes, r, pos2.value)
        return (code, v.raw[:r + 1], et, pos.value, db.raw[:k], cb.raw[:r + 1],
                v2.raw[:r + 1], et2, pos2.value, bbuf.raw[:nbytes], cb2.raw[:r + 1])

    for flips in ([], [3], [k - 1], [0, 5], [-1]):
        if any(f >= k for f in flips):
            continue
        assert run(O, flips) == run(R, flips), flips


def test_readfrombinary(tmp_path):
    O = _ours(1e-3)
    O.readfrombinary_float.argtypes = [C.c_char_p, C.c_int]
    O.readfrombinary_float.restype = C.c_void_p
    O.readfrombinary_double.argtypes = [C.c_char_p, C.c_int]
    O.readfrombinary_double.restype = C.c_void_p
    f = np.arange(37, dtype=np.float32) * 0.5
    d = np.arange(11, dtype=np.float64) * 0.25
    pf, pd = tmp_path / "a.bin", tmp_path / "b.bin"
    f.tofile(pf)
    d.tofile(pd)
    p = O.readfrombinary_float(str(pf).encode(), f.size)
    assert np.array_equal(np.frombuffer(C.string_at(p, f.nbytes), np.float32), f)
    libc.free(p)
    p = O.readfrombinary_double(str(pd).encode(), d.size)
    assert np.array_equal(np.frombuffer(C.string_at(p, d.nbytes), np.float64), d)
    libc.free(p)
    assert O.readfrombinary_float(str(tmp_path / "missing").encode(), 4) is None


def test_get_double_bin_vs_reference():
    """getDoubleBin (c:5232-5242) as the reference compiles: the low 32-bit word, twice."""
    R, O = _ref(1e-6), _ours(1e-6)
    for L in (R, O):
        L.getDoubleBin.argtypes = [C.c_double, C.c_char_p]
    r = np.random.default_rng(3)
    vals = [0.0, -0.0, 1.0, -2.0, 1e-3, 123.456, 1.0 + 2.0 ** -21, 2.0 ** -30 + 1] + list(r.normal(0, 50, 200))
    for v in vals:
        a, b = C.create_string_buffer(64), C.create_string_buffer(64)
        R.getDoubleBin(float(v), a)
        O.getDoubleBin(float(v), b)
        assert a.raw == b.raw, v
