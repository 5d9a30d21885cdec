"""ctypes bindings for the parity oracle (TEST INFRASTRUCTURE ONLY).

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Two back ends:

* ``Oracle``  -- oracle/build/liboracle.so, the C restatement in dc_oracle.c (travels to the GPU box).
* ``RefLib``  -- oracle/_ref/libref_<bound>.so, the reference's own impl/dataCompression.c compiled
  by oracle/build_ref.sh (built in the dev container; the .so also travels to the GPU box, the
  reference sources never do).
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBORACLE = os.path.join(HERE, "build", "liboracle.so")
REFDIR = os.path.join(HERE, "_ref")

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_libc = C.CDLL(None)
_libc.free.argtypes = [C.c_void_p]
_libc.malloc.argtypes = [C.c_size_t]
_libc.malloc.restype = C.c_void_p


def bound_tag(bound):
    return "%g" % bound


def build():
    """Build liboracle.so (and the reference libs when /root/reference is present)."""
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE])
    subprocess.check_call(["make", "-s", "-C", HERE, "ref"])


class Oracle:
    def __init__(self, path=LIBORACLE):
        if not os.path.exists(path):
            build()
        L = self.L = C.CDLL(path)
        L.orc_bound_binary.argtypes = [C.c_double]
        L.orc_thr_lt.argtypes = [C.c_double]
        L.orc_thr_lt.restype = C.c_float
        L.orc_thr_le.argtypes = [C.c_double]
        L.orc_thr_le.restype = C.c_float
        L.orc_to_small.argtypes = [_f32p, C.c_long, _f32p]
        L.orc_to_small.restype = C.c_float
        L.orc_med.argtypes = [_f32p, C.c_long, C.POINTER(C.c_int)]
        L.orc_med.restype = C.c_float
        L.orc_mask17.argtypes = [C.c_float]
        L.orc_mask17.restype = C.c_uint32
        L.orc_compress.argtypes = [C.c_int, _f32p, C.c_long, C.c_double, C.c_int, C.c_uint32,
                                   C.POINTER(C.c_void_p), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.orc_decompress_spec.argtypes = [C.c_int, _u8p, C.c_long, C.c_long, C.c_double, C.c_int,
                                          C.c_uint32, _f32p]
        L.orc_decompress_spec.restype = C.c_long
        L.orc_decompress_cref.argtypes = [C.c_int, _u8p, C.c_long, C.c_long, C.c_double, C.c_int,
                                          C.c_uint32, _f32p, C.POINTER(C.c_int)]
        L.orc_decompress_cref.restype = C.c_long
        L.orc_bytewise_compress.argtypes = [_f32p, C.c_int, C.c_double, _f32p, C.c_char_p, _i32p]
        L.orc_bytewise_decompress.argtypes = [_f32p, C.c_char_p, _i32p, C.c_int, C.c_int, _f32p]
        L.orc_crc32.argtypes = [_u8p, C.c_long]
        L.orc_crc32.restype = C.c_uint32
        L.orc_hm_length.argtypes = [C.c_long]
        L.orc_hamming_encode.argtypes = [_u8p, C.c_long, C.POINTER(C.c_int), C.c_char_p]
        L.orc_hamming_decode.argtypes = [_u8p, C.c_char_p, C.c_long, C.c_int, C.POINTER(C.c_long)]
        L.orc_block_size.argtypes = [C.c_int, C.c_double]
        L.orc_gen_u10.argtypes = [_f32p, C.c_long, C.c_uint64, C.c_long]
        L.orc_gen_himeno_plane.argtypes = [_f32p, C.c_int, C.c_int]
        # double codecs (dc_oracle64.c)
        L.orc64_to_small.argtypes = [_f64p, C.c_long, _f64p]
        L.orc64_to_small.restype = C.c_double
        L.orc64_med.argtypes = [_f64p, C.c_long, C.POINTER(C.c_int)]
        L.orc64_med.restype = C.c_double
        L.orc64_mask20.argtypes = [C.c_double]
        L.orc64_mask20.restype = C.c_uint32
        L.orc64_compress.argtypes = [C.c_int, _f64p, C.c_long, C.c_double, C.c_int, C.c_uint32,
                                     C.POINTER(C.c_void_p), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.orc64_decompress_spec.argtypes = [C.c_int, _u8p, C.c_long, C.c_long, C.c_double, C.c_int,
                                            C.c_uint32, _f64p]
        L.orc64_decompress_spec.restype = C.c_long
        L.orc64_gen_u10.argtypes = [_f64p, C.c_long, C.c_uint64, C.c_long]
        L.orc64_bytewise_compress.argtypes = [_f64p, C.c_int, C.c_double, _f64p, C.c_char_p, _i32p]
        L.orc64_bytewise_decompress.argtypes = [_f64p, C.c_char_p, _i32p, C.c_int, C.c_int, _f64p]

    # -- helpers
    def bound_binary(self, b):
        return self.L.orc_bound_binary(b)

    def thr(self, b):
        return self.L.orc_thr_lt(b), self.L.orc_thr_le(b)

    def to_small(self, x):
        x = np.ascontiguousarray(x, np.float32)
        out = np.empty_like(x)
        mn = self.L.orc_to_small(x, x.size, out)
        return np.float32(mn), out

    def med(self, x):
        x = np.ascontiguousarray(x, np.float32)
        t = C.c_int(0)
        mean = self.L.orc_med(x, x.size, C.byref(t))
        return np.float32(mean), t.value

    def mask17(self, mean):
        return int(self.L.orc_mask17(float(mean)))

    def type_mask(self, xs):
        mean, t = self.med(xs)
        return t, self.mask17(mean)

    def compress(self, ct, x, bound, type_=0, mask17=0, prefix=None, prefix_pos=8):
        """Returns (stream uint8 array, bytes, pos).  prefix: existing stream to append to."""
        x = np.ascontiguousarray(x, np.float32)
        p = C.c_void_p(None)
        nbytes = C.c_int(0)
        pos = C.c_int(8)
        if prefix is not None and len(prefix):
            buf = _libc.malloc(len(prefix))
            C.memmove(buf, bytes(prefix), len(prefix))
            p = C.c_void_p(buf)
            nbytes.value = len(prefix)
            pos.value = prefix_pos
        self.L.orc_compress(ct, x, x.size, bound, type_, mask17, C.byref(p), C.byref(nbytes), C.byref(pos))
        out = np.frombuffer(C.string_at(p.value, nbytes.value), np.uint8).copy() if nbytes.value else np.zeros(0, np.uint8)
        _libc.free(p)
        return out, nbytes.value, pos.value

    def decompress(self, ct, s, num, bound, type_=0, mask17=0):
        s = np.ascontiguousarray(s, np.uint8)
        out = np.zeros(num, np.float32)
        n = self.L.orc_decompress_spec(ct, s if s.size else np.zeros(1, np.uint8), s.size, num, bound,
                                       type_, mask17, out)
        return out, n

    def decompress_cref(self, ct, s, num, bound, type_=0, mask17=0):
        s = np.ascontiguousarray(s, np.uint8)
        out = np.zeros(num, np.float32)
        st = C.c_int(0)
        n = self.L.orc_decompress_cref(ct, s if s.size else np.zeros(1, np.uint8), s.size, num, bound,
                                       type_, mask17, out, C.byref(st))
        return out, n, st.value

    def bytewise_compress(self, x, bound):
        x = np.ascontiguousarray(x, np.float32)
        raw = np.zeros(max(x.size, 1), np.float32)
        codes = C.create_string_buffer(max(x.size, 1))
        pos = np.zeros(max(x.size, 1), np.int32)
        nf = self.L.orc_bytewise_compress(x, x.size, bound, raw, codes, pos)
        nc = x.size - nf
        return raw[:nf].copy(), codes.raw[:nc], pos[:nc].copy()

    def bytewise_decompress(self, raw, codes, pos, num):
        raw = np.ascontiguousarray(raw, np.float32) if len(raw) else np.zeros(1, np.float32)
        pos = np.ascontiguousarray(pos, np.int32) if len(pos) else np.zeros(1, np.int32)
        out = np.zeros(num, np.float32)
        self.L.orc_bytewise_decompress(raw, codes or b"\0", pos, len(codes), num, out)
        return out

    def crc32(self, s):
        s = np.ascontiguousarray(s, np.uint8)
        return int(self.L.orc_crc32(s if s.size else np.zeros(1, np.uint8), s.size))

    def hamming_encode(self, s):
        s = np.ascontiguousarray(s, np.uint8)
        r = C.c_int(0)
        c = C.create_string_buffer(80)
        self.L.orc_hamming_encode(s, s.size, C.byref(r), c)
        return r.value, c.raw[: r.value + 1]

    def hamming_decode(self, s, c, r):
        s = np.array(s, np.uint8)
        cb = C.create_string_buffer(bytes(c), len(c) + 1)
        ep = C.c_long(0)
        t = self.L.orc_hamming_decode(s, cb, s.size, r, C.byref(ep))
        return t, s, cb.raw[: r + 1], ep.value

    def block_size(self, nbytes, ber=1e-6):
        return self.L.orc_block_size(nbytes, ber)

    def gen_u10(self, n, seed=42, offset=0):
        out = np.empty(n, np.float32)
        self.L.orc_gen_u10(out, n, seed, offset)
        return out

    # -- double codecs
    def to_small64(self, x):
        x = np.ascontiguousarray(x, np.float64)
        out = np.empty_like(x)
        mn = self.L.orc64_to_small(x, x.size, out)
        return np.float64(mn), out

    def med64(self, x):
        x = np.ascontiguousarray(x, np.float64)
        t = C.c_int(0)
        mean = self.L.orc64_med(x, x.size, C.byref(t))
        return np.float64(mean), t.value

    def mask20(self, mean):
        return int(self.L.orc64_mask20(float(mean)))

    def compress64(self, ct, x, bound, type_=0, mask20=0, prefix=None, prefix_pos=8):
        x = np.ascontiguousarray(x, np.float64)
        p = C.c_void_p(None)
        nbytes = C.c_int(0)
        pos = C.c_int(8)
        if prefix is not None and len(prefix):
            buf = _libc.malloc(len(prefix))
            C.memmove(buf, bytes(prefix), len(prefix))
            p = C.c_void_p(buf)
            nbytes.value = len(prefix)
            pos.value = prefix_pos
        self.L.orc64_compress(ct, x, x.size, bound, type_, mask20, C.byref(p), C.byref(nbytes), C.byref(pos))
        out = np.frombuffer(C.string_at(p.value, nbytes.value), np.uint8).copy() if nbytes.value else np.zeros(0, np.uint8)
        _libc.free(p)
        return out, nbytes.value, pos.value

    def decompress64(self, ct, s, num, bound, type_=0, mask20=0):
        s = np.ascontiguousarray(s, np.uint8)
        out = np.zeros(num, np.float64)
        n = self.L.orc64_decompress_spec(ct, s if s.size else np.zeros(1, np.uint8), s.size, num, bound,
                                         type_, mask20, out)
        return out, n

    def bytewise_compress64(self, x, bound):
        x = np.ascontiguousarray(x, np.float64)
        raw = np.zeros(max(x.size, 1), np.float64)
        codes = C.create_string_buffer(max(x.size, 1))
        pos = np.zeros(max(x.size, 1), np.int32)
        nf = self.L.orc64_bytewise_compress(x, x.size, bound, raw, codes, pos)
        nc = x.size - nf
        return raw[:nf].copy(), codes.raw[:nc], pos[:nc].copy()

    def bytewise_decompress64(self, raw, codes, pos, num):
        raw = np.ascontiguousarray(raw, np.float64) if len(raw) else np.zeros(1, np.float64)
        pos = np.ascontiguousarray(pos, np.int32) if len(pos) else np.zeros(1, np.int32)
        out = np.zeros(num, np.float64)
        self.L.orc64_bytewise_decompress(raw, codes or b"\0", pos, len(codes), num, out)
        return out

    def gen_u10_64(self, n, seed=42, offset=0):
        out = np.empty(n, np.float64)
        self.L.orc64_gen_u10(out, n, seed, offset)
        return out

    def gen_himeno_plane(self, imax=256, jmax=256):
        out = np.empty(imax * jmax, np.float32)
        self.L.orc_gen_himeno_plane(out, imax, jmax)
        return out


def gen_u10_np(n, seed=42, offset=0):
    """numpy restatement of orc_gen_u10."""
    i = np.arange(offset, offset + n, dtype=np.uint64) + np.uint64(1)
    with np.errstate(over="ignore"):
        z = np.uint64(0x9E3779B97F4A7C15) * i + np.uint64(seed)
        z ^= z >> np.uint64(30)
        z *= np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(27)
        z *= np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return ((z >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)) * np.float32(10.0)


class RefLib:
    """The reference's own dataCompression.c compiled for one absErrorBound (oracle/_ref)."""

    def __init__(self, bound):
        path = os.path.join(REFDIR, "libref_%s.so" % bound_tag(bound))
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.bound = bound
        L = self.L = C.CDLL(path)
        pp = [_f32p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        for nm in ("myCompress_bitwise", "myCompress_bitwise_np", "myCompress_bitwise_op"):
            getattr(L, nm).argtypes = pp
        L.myCompress_bitwise_mask.argtypes = pp + [C.c_int, C.c_char_p]
        for nm in ("myDecompress_bitwise", "myDecompress_bitwise_np", "myDecompress_bitwise_op"):
            getattr(L, nm).argtypes = [_u8p, C.c_int, C.c_int]
            getattr(L, nm).restype = C.c_void_p
        L.myDecompress_bitwise_mask.argtypes = [_u8p, C.c_int, C.c_int, C.c_int, C.c_char_p]
        L.myDecompress_bitwise_mask.restype = C.c_void_p
        L.toSmallDataset_float.argtypes = [_f32p, C.POINTER(C.c_void_p), C.c_int]
        L.toSmallDataset_float.restype = C.c_float
        L.med_dataset_float.argtypes = [_f32p, C.c_int, C.POINTER(C.c_int)]
        L.med_dataset_float.restype = C.c_float
        L.floattostr.argtypes = [C.POINTER(C.c_float), C.c_char_p]
        L.do_crc32.argtypes = [_u8p, C.c_int]
        L.do_crc32.restype = C.c_uint32
        L.hamming_encode.argtypes = [_u8p, C.POINTER(C.c_void_p), C.c_int, C.POINTER(C.c_int)]
        L.hamming_decode.argtypes = [_u8p, C.c_char_p, C.c_int, C.c_int]
        L.hmLength.argtypes = [C.c_int]
        L.block_size.argtypes = [C.c_int]
        L.myCompress.argtypes = [_f32p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_int]
        L.myDecompress.argtypes = [_f32p, C.c_char_p, _i32p, C.c_int]
        L.myDecompress.restype = C.c_void_p
        dp = [_f64p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        for nm in ("myCompress_bitwise_double", "myCompress_bitwise_double_np", "myCompress_bitwise_double_op"):
            getattr(L, nm).argtypes = dp
        L.myCompress_bitwise_double_mask.argtypes = dp + [C.c_int, C.c_char_p]
        for nm in ("myDecompress_bitwise_double", "myDecompress_bitwise_double_np", "myDecompress_bitwise_double_op"):
            getattr(L, nm).argtypes = [_u8p, C.c_int, C.c_int]
            getattr(L, nm).restype = C.c_void_p
        L.myDecompress_bitwise_double_mask.argtypes = [_u8p, C.c_int, C.c_int, C.c_int, C.c_char_p]
        L.myDecompress_bitwise_double_mask.restype = C.c_void_p
        L.myCompress_double.argtypes = [_f64p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_int]
        L.toSmallDataset_double.argtypes = [_f64p, C.POINTER(C.c_void_p), C.c_int]
        L.toSmallDataset_double.restype = C.c_double
        L.med_dataset_double.argtypes = [_f64p, C.c_int, C.POINTER(C.c_int)]
        L.med_dataset_double.restype = C.c_double

    @staticmethod
    def mask_chars(mask17):
        return "".join("1" if (mask17 >> (16 - i)) & 1 else "0" for i in range(17)).encode()

    def compress(self, ct, x, type_=0, mask17=0):
        x = np.ascontiguousarray(x, np.float32)
        p = C.c_void_p(None)
        nb = C.c_int(0)
        pos = C.c_int(8)
        args = (x, x.size, C.byref(p), C.byref(nb), C.byref(pos))
        if ct == 5:
            self.L.myCompress_bitwise(*args)
        elif ct == 6:
            self.L.myCompress_bitwise_np(*args)
        elif ct == 11:
            self.L.myCompress_bitwise_op(*args)
        elif ct == 7:
            self.L.myCompress_bitwise_mask(*args, type_, self.mask_chars(mask17))
        else:
            raise ValueError(ct)
        out = np.frombuffer(C.string_at(p.value, nb.value), np.uint8).copy() if nb.value else np.zeros(0, np.uint8)
        _libc.free(p)
        return out, nb.value, pos.value

    def decompress(self, ct, s, num, type_=0, mask17=0):
        s = np.ascontiguousarray(s, np.uint8)
        if ct == 5:
            p = self.L.myDecompress_bitwise(s, s.size, num)
        elif ct == 6:
            p = self.L.myDecompress_bitwise_np(s, s.size, num)
        elif ct == 11:
            p = self.L.myDecompress_bitwise_op(s, s.size, num)
        elif ct == 7:
            p = self.L.myDecompress_bitwise_mask(s, s.size, num, type_, self.mask_chars(mask17))
        else:
            raise ValueError(ct)
        out = np.frombuffer(C.string_at(p, 4 * num), np.float32).copy()
        _libc.free(p)
        return out

    @staticmethod
    def mask_chars20(mask20):
        return "".join("1" if (mask20 >> (19 - i)) & 1 else "0" for i in range(20)).encode()

    _D = {5: "", 6: "_np", 11: "_op", 7: "_mask"}

    def compress64(self, ct, x, type_=0, mask20=0):
        x = np.ascontiguousarray(x, np.float64)
        p = C.c_void_p(None)
        nb = C.c_int(0)
        pos = C.c_int(8)
        args = (x, x.size, C.byref(p), C.byref(nb), C.byref(pos))
        f = getattr(self.L, "myCompress_bitwise_double" + self._D[ct])
        f(*args, type_, self.mask_chars20(mask20)) if ct == 7 else f(*args)
        out = np.frombuffer(C.string_at(p.value, nb.value), np.uint8).copy() if nb.value else np.zeros(0, np.uint8)
        _libc.free(p)
        return out, nb.value, pos.value

    def decompress64(self, ct, s, num, type_=0, mask20=0):
        s = np.ascontiguousarray(s, np.uint8)
        f = getattr(self.L, "myDecompress_bitwise_double" + self._D[ct])
        p = f(s, s.size, num, type_, self.mask_chars20(mask20)) if ct == 7 else f(s, s.size, num)
        out = np.frombuffer(C.string_at(p, 8 * num), np.float64).copy()
        _libc.free(p)
        return out

    def bytewise64(self, x):
        x = np.ascontiguousarray(x, np.float64)
        pf, pc, pp = C.c_void_p(None), C.c_void_p(None), C.c_void_p(None)
        nf = self.L.myCompress_double(x, C.byref(pf), C.byref(pc), C.byref(pp), x.size)
        nc = x.size - nf
        raw = np.frombuffer(C.string_at(pf.value, 8 * nf), np.float64).copy() if nf else np.zeros(0, np.float64)
        codes = C.string_at(pc.value, nc) if nc else b""
        pos = np.frombuffer(C.string_at(pp.value, 4 * nc), np.int32).copy() if nc else np.zeros(0, np.int32)
        for q in (pf, pc, pp):
            _libc.free(q)
        return raw, codes, pos

    def to_small64(self, x):
        x = np.ascontiguousarray(x, np.float64)
        p = C.c_void_p(None)
        mn = self.L.toSmallDataset_double(x, C.byref(p), x.size)
        out = np.frombuffer(C.string_at(p.value, 8 * x.size), np.float64).copy()
        _libc.free(p)
        return np.float64(mn), out

    def med64(self, x):
        x = np.ascontiguousarray(x, np.float64)
        t = C.c_int(0)
        mean = self.L.med_dataset_double(x, x.size, C.byref(t))
        return np.float64(mean), t.value

    def to_small(self, x):
        x = np.ascontiguousarray(x, np.float32)
        p = C.c_void_p(None)
        mn = self.L.toSmallDataset_float(x, C.byref(p), x.size)
        out = np.frombuffer(C.string_at(p.value, 4 * x.size), np.float32).copy()
        _libc.free(p)
        return np.float32(mn), out

    def med(self, x):
        x = np.ascontiguousarray(x, np.float32)
        t = C.c_int(0)
        mean = self.L.med_dataset_float(x, x.size, C.byref(t))
        return np.float32(mean), t.value

    def crc32(self, s):
        s = np.ascontiguousarray(s, np.uint8)
        return int(self.L.do_crc32(s, s.size))

    def hamming_encode(self, s):
        s = np.ascontiguousarray(s, np.uint8)
        p = C.c_void_p(None)
        r = C.c_int(0)
        self.L.hamming_encode(s, C.byref(p), s.size, C.byref(r))
        c = C.string_at(p.value, r.value + 1)
        _libc.free(p)
        return r.value, c

    def bytewise(self, x):
        x = np.ascontiguousarray(x, np.float32)
        pf, pc, pp = C.c_void_p(None), C.c_void_p(None), C.c_void_p(None)
        nf = self.L.myCompress(x, C.byref(pf), C.byref(pc), C.byref(pp), x.size)
        nc = x.size - nf
        raw = np.frombuffer(C.string_at(pf.value, 4 * nf), np.float32).copy() if nf else np.zeros(0, np.float32)
        codes = C.string_at(pc.value, nc) if nc else b""
        pos = np.frombuffer(C.string_at(pp.value, 4 * nc), np.int32).copy() if nc else np.zeros(0, np.int32)
        for q in (pf, pc, pp):
            _libc.free(q)
        return raw, codes, pos
