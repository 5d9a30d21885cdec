"""Python binding of libdcamd (ctypes) -- used by tests/, bench.py and __graft_entry__.

The library is the product: the reference's C ABI (include/dataCompression.h) implemented on
gfx950 kernels, plus the device-pointer API of include/dc_gpu.h.  This module only marshals
numpy arrays / torch tensors into those C entry points; it computes nothing itself and raises if
the shared object is missing.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("DCAMD_LIB") or os.path.join(HERE, "lib", "libdcamd.so")   # override: A/B experiments

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_libc = C.CDLL(None)
_libc.free.argtypes = [C.c_void_p]
_libc.malloc.argtypes = [C.c_size_t]
_libc.malloc.restype = C.c_void_p

# symbols include/dataCompression.h + include/dc_gpu.h promise (checked by tests/test_library.py)
ABI_SYMBOLS = [
    "myCompress_bitwise", "myCompress_bitwise_np", "myCompress_bitwise_op", "myCompress_bitwise_mask",
    "myDecompress_bitwise", "myDecompress_bitwise_np", "myDecompress_bitwise_op", "myDecompress_bitwise_mask",
    "toSmallDataset_float", "med_dataset_float", "do_crc32", "hmLength", "hamming_encode", "hamming_decode",
    "bit_flip", "block_size", "get_random_int", "floattostr", "strtofloat", "doubletostr", "strtodbl",
    "getFloatBin", "to_absErrorBound_binary", "add_bit_to_bytes", "bit_set", "myCompress", "myDecompress",
    "myCompress_bitwise_double", "myCompress_bitwise_double_np", "myCompress_bitwise_double_op",
    "myCompress_bitwise_double_mask", "myDecompress_bitwise_double", "myDecompress_bitwise_double_np",
    "myDecompress_bitwise_double_op", "myDecompress_bitwise_double_mask", "toSmallDataset_double",
    "med_dataset_double", "myCompress_double", "myDecompress_double", "writetobinary_double",
    "readfrombinary_writetotxt_double",
]
EXT_SYMBOLS = [
    "dc_init", "dc_last_error", "dc_get_stream", "dc_synchronize", "dc_set_abs_error_bound",
    "dc_get_abs_error_bound", "dc_stream_capacity", "dc_encode_device", "dc_encode_result",
    "dc_decode_device", "dc_decode_finish", "dc_to_small_device", "dc_med_device", "dc_prep_device", "dc_encode_sub_device", "dc_last_decode_was_tiny", "dc_set_halo_unfused", "dc_halo_decode2_device", "dc_halo_encode2_device", "dc_capture_begin", "dc_capture_end", "dc_graph_launch", "dc_graph_destroy", "dc_last_decode_launched_tiny", "dc_set_decode_tiny", "dc_crc32_device",
    "dc_decode_chunk_bits_value", "dc_ct1_encode_device", "dc_ct1_decode_device", "dc_encode_bits_device",
    "dc_crc32_device_async", "dc_crc32_copy_device", "dc_encode_send_device", "dc_crc32_pair_device", "dc_encode_crc_device", "dc_crc32_stream_device", "dc_crc_resend_crc_device",
    "dc_hash_device", "dc_copy_rate_device", "dc_flip_bits_device", "dc_decode_shard_device", "dc_decode_shard_fix",
    "dc_halo_encode_device", "dc_halo_decode_device",
    "dc64_stream_capacity", "dc64_encode_device", "dc64_encode_result", "dc64_decode_device", "dc64_decode_finish",
    "dc64_last_decode_flags", "dc64_to_small_device", "dc64_med_device", "dc_set_encode_stream",
    "dc_decode_status", "dc_abi_status", "dc_med_sum_device", "dc_type_from_max", "dc_set_small_chunk_max_bytes",
    "dc_set_decode3_min_bytes", "dc_set_decode3_seg", "dc_set_fused3", "dc_fused3_stamps", "dc_fused3_last_seg", "dc_decode3_last_fused", "dc_last_decode_was_v3", "dc_last_decode_launched_v3",
    "dc_encode_status", "dc_encode_clear_status", "dc_encode_mode", "dc_encode_retries", "dc_crc_resend_device",
    "dc_merge_shards_device", "dc_merge_status", "dc_extract_shard_device", "dc_occupy_device", "dc_set_encode_help", "dc_decode_shard3_device", "dc_decode_shard3_fix",
    "dc_decode_status_clear", "dc_set_runs_max_bytes", "dc_last_decode_was_runs",
    "dc_last_decode_launched_runs", "dc_last_decode_used_maps", "dc_med_last_wide", "dc_set_decode3_maps", "dc_set_halo_async", "dc_med_shard_stats", "dc_med_shard_trans",
    "dc_med_shard_binades",
]


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE])


class DCError(RuntimeError):
    pass


class Lib:
    """Thin ctypes view of libdcamd.so."""

    def __init__(self, path=LIB):
        if not os.path.exists(path):
            raise ImportError(f"libdcamd.so not built ({path}); run `make -C data-compression_amd`")
        L = self.L = C.CDLL(path)
        self.path = path
        vp, ll, u32 = C.c_void_p, C.c_longlong, C.c_uint32
        L.dc_init.argtypes = [C.c_int]
        L.dc_last_error.restype = C.c_char_p
        L.dc_get_stream.restype = vp
        L.dc_set_abs_error_bound.argtypes = [C.c_double]
        L.dc_get_abs_error_bound.restype = C.c_double
        L.dc_stream_capacity.argtypes = [ll]
        L.dc_stream_capacity.restype = C.c_size_t
        L.dc_encode_device.argtypes = [C.c_int, vp, ll, ll, C.c_int, u32, C.c_int, vp, vp]
        L.dc_encode_crc_device.argtypes = [C.c_int, vp, ll, ll, C.c_int, u32, vp, vp, vp]
        L.dc_crc32_stream_device.argtypes = [vp, ll, vp]
        L.dc_crc_resend_crc_device.argtypes = [vp, vp, vp, ll, vp]
        L.dc_encode_result.argtypes = [C.POINTER(C.c_ulonglong)]
        L.dc_encode_bits_device.argtypes = [C.c_int, vp, ll, ll, C.c_int, u32, C.POINTER(C.c_ulonglong)]
        L.dc_decode_device.argtypes = [C.c_int, vp, ll, vp, ll, ll, C.c_int, u32, vp]
        L.dc_decode_shard_device.argtypes = [C.c_int, vp, ll, C.c_ulonglong, C.c_ulonglong, ll, C.c_int, u32, vp, vp]
        L.dc_decode_shard_fix.argtypes = [vp]
        L.dc_merge_shards_device.argtypes = [vp, ll, C.c_int, vp, vp, ll, vp]
        L.dc_merge_status.argtypes = [C.POINTER(C.c_uint), C.c_int]
        L.dc_extract_shard_device.argtypes = [vp, ll, vp, C.c_int, vp, ll, vp]
        L.dc_occupy_device.argtypes = [vp, C.c_double, C.c_int, C.c_int]
        L.dc_decode_shard3_device.argtypes = [C.c_int, vp, vp, ll, ll, C.c_int, u32, vp, C.c_int]
        L.dc_decode_shard3_fix.argtypes = [vp]
        L.dc_to_small_device.argtypes = [vp, ll, vp, C.POINTER(C.c_float)]
        L.dc_med_device.argtypes = [vp, ll, C.POINTER(C.c_float), C.POINTER(C.c_int)]
        L.dc_prep_device.argtypes = [vp, ll, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_int)]
        L.dc_encode_sub_device.argtypes = [C.c_int, vp, ll, C.c_float, C.c_int, u32, vp, vp]
        L.dc_med_sum_device.argtypes = [vp, ll, C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.dc_med_shard_stats.argtypes = [vp, ll, C.POINTER(C.c_double), C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.dc_med_shard_trans.argtypes = [vp, ll, C.c_double, C.POINTER(C.c_int), C.POINTER(C.c_longlong),
                                         C.POINTER(C.c_ubyte)]
        L.dc_type_from_max.argtypes = [C.c_float]
        L.dc_decode_status.argtypes = [C.POINTER(C.c_uint)]
        L.dc_crc32_device.argtypes = [vp, ll, C.POINTER(C.c_uint32)]
        L.dc_hash_device.argtypes = [vp, ll, C.POINTER(C.c_ulonglong)]
        L.dc_copy_rate_device.argtypes = [vp, vp, ll, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int)]
        L.dc_decode_chunk_bits_value.restype = ll
        L.dc_set_small_chunk_max_bytes.argtypes = [ll]
        L.dc_set_small_chunk_max_bytes.restype = ll
        L.dc_set_decode3_min_bytes.argtypes = [ll]
        L.dc_set_decode3_min_bytes.restype = ll
        L.dc_set_runs_max_bytes.argtypes = [ll]
        L.dc_set_runs_max_bytes.restype = ll
        pp = [_f32p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        for nm in ("myCompress_bitwise", "myCompress_bitwise_np", "myCompress_bitwise_op"):
            getattr(L, nm).argtypes = pp
        L.myCompress_bitwise_mask.argtypes = pp + [C.c_int, C.c_char_p]
        for nm in ("myDecompress_bitwise", "myDecompress_bitwise_np", "myDecompress_bitwise_op"):
            getattr(L, nm).argtypes = [_u8p, C.c_int, C.c_int]
            getattr(L, nm).restype = vp
        L.myDecompress_bitwise_mask.argtypes = [_u8p, C.c_int, C.c_int, C.c_int, C.c_char_p]
        L.myDecompress_bitwise_mask.restype = vp
        L.toSmallDataset_float.argtypes = [_f32p, C.POINTER(C.c_void_p), C.c_int]
        L.toSmallDataset_float.restype = C.c_float
        L.med_dataset_float.argtypes = [_f32p, C.c_int, C.POINTER(C.c_int)]
        L.med_dataset_float.restype = C.c_float
        L.do_crc32.argtypes = [_u8p, C.c_int]
        L.do_crc32.restype = C.c_uint32
        L.hamming_encode.argtypes = [_u8p, C.POINTER(C.c_void_p), C.c_int, C.POINTER(C.c_int)]
        L.hamming_decode.argtypes = [_u8p, C.c_char_p, C.c_int, C.c_int]
        L.hmLength.argtypes = [C.c_int]
        L.block_size.argtypes = [C.c_int]
        L.myCompress.argtypes = [_f32p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_int]
        L.myCompress.restype = C.c_int
        L.myDecompress.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.myDecompress.restype = vp
        # double codecs
        dp = [_f64p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        for nm in ("myCompress_bitwise_double", "myCompress_bitwise_double_np", "myCompress_bitwise_double_op"):
            getattr(L, nm).argtypes = dp
        L.myCompress_bitwise_double_mask.argtypes = dp + [C.c_int, C.c_char_p]
        for nm in ("myDecompress_bitwise_double", "myDecompress_bitwise_double_np", "myDecompress_bitwise_double_op"):
            getattr(L, nm).argtypes = [_u8p, C.c_int, C.c_int]
            getattr(L, nm).restype = vp
        L.myDecompress_bitwise_double_mask.argtypes = [_u8p, C.c_int, C.c_int, C.c_int, C.c_char_p]
        L.myDecompress_bitwise_double_mask.restype = vp
        L.toSmallDataset_double.argtypes = [_f64p, C.POINTER(C.c_void_p), C.c_int]
        L.toSmallDataset_double.restype = C.c_double
        L.med_dataset_double.argtypes = [_f64p, C.c_int, C.POINTER(C.c_int)]
        L.med_dataset_double.restype = C.c_double
        L.myCompress_double.argtypes = [_f64p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                        C.c_int]
        L.myCompress_double.restype = C.c_int
        L.myDecompress_double.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.myDecompress_double.restype = vp
        L.dc64_stream_capacity.argtypes = [ll]
        L.dc64_stream_capacity.restype = C.c_size_t
        L.dc64_encode_device.argtypes = [C.c_int, vp, ll, C.c_int, u32, C.c_int, vp, vp]
        L.dc64_encode_result.argtypes = [C.POINTER(C.c_ulonglong)]
        L.dc64_decode_device.argtypes = [C.c_int, vp, ll, vp, ll, ll, C.c_int, u32, vp]
        L.dc64_last_decode_flags.restype = C.c_uint
        L.dc64_to_small_device.argtypes = [vp, ll, vp, C.POINTER(C.c_double)]
        L.dc64_med_device.argtypes = [vp, ll, C.POINTER(C.c_double), C.POINTER(C.c_int)]

    # ---- state
    def init(self, device=0):
        rc = self.L.dc_init(device)
        if rc:
            raise DCError(f"dc_init: {rc} {self.err()}")

    def err(self):
        m = self.L.dc_last_error()
        return m.decode() if m else ""

    def check(self, rc, what):
        if rc:
            raise DCError(f"{what} -> {rc}: {self.err()}")

    def set_bound(self, b):
        self.L.dc_set_abs_error_bound(b)

    # ---- reference ABI on host arrays
    @staticmethod
    def mask_chars(mask17):
        return "".join("1" if (mask17 >> (16 - i)) & 1 else "0" for i in range(17)).encode()

    def compress(self, ct, x, type_=0, mask17=0, prefix=None, prefix_pos=8):
        x = np.ascontiguousarray(x, np.float32)
        p = C.c_void_p(None)
        nb = C.c_int(0)
        pos = C.c_int(8)
        if prefix is not None and len(prefix):
            buf = _libc.malloc(len(prefix))
            C.memmove(buf, bytes(prefix), len(prefix))
            p = C.c_void_p(buf)
            nb.value = len(prefix)
            pos.value = prefix_pos
        args = (x if x.size else np.zeros(1, np.float32), x.size, C.byref(p), C.byref(nb), C.byref(pos))
        fn = {5: self.L.myCompress_bitwise, 6: self.L.myCompress_bitwise_np, 11: self.L.myCompress_bitwise_op}
        if ct == 7:
            self.L.myCompress_bitwise_mask(*args, type_, self.mask_chars(mask17))
        else:
            fn[ct](*args)
        out = np.frombuffer(C.string_at(p.value, nb.value), np.uint8).copy() if nb.value else np.zeros(0, np.uint8)
        if p.value:
            _libc.free(p)
        return out, nb.value, pos.value

    def decompress(self, ct, s, num, type_=0, mask17=0):
        s = np.ascontiguousarray(s, np.uint8)
        sarg = s if s.size else np.zeros(1, np.uint8)
        if ct == 7:
            p = self.L.myDecompress_bitwise_mask(sarg, s.size, num, type_, self.mask_chars(mask17))
        else:
            fn = {5: self.L.myDecompress_bitwise, 6: self.L.myDecompress_bitwise_np, 11: self.L.myDecompress_bitwise_op}
            p = fn[ct](sarg, s.size, num)
        out = np.frombuffer(C.string_at(p, 4 * num), np.float32).copy() if num else np.zeros(0, np.float32)
        _libc.free(p)
        return out

    # ---- double codecs (myCompress_bitwise_double* / myDecompress_bitwise_double*)
    _D = {5: "", 6: "_np", 11: "_op", 7: "_mask"}

    @staticmethod
    def mask_chars20(mask20):
        return "".join("1" if (mask20 >> (19 - i)) & 1 else "0" for i in range(20)).encode()

    def compress64(self, ct, x, type_=0, mask20=0, prefix=None, prefix_pos=8):
        x = np.ascontiguousarray(x, np.float64)
        p = C.c_void_p(None)
        nb = C.c_int(0)
        pos = C.c_int(8)
        if prefix is not None and len(prefix):
            buf = _libc.malloc(len(prefix))
            C.memmove(buf, bytes(prefix), len(prefix))
            p = C.c_void_p(buf)
            nb.value = len(prefix)
            pos.value = prefix_pos
        args = (x if x.size else np.zeros(1, np.float64), x.size, C.byref(p), C.byref(nb), C.byref(pos))
        f = getattr(self.L, "myCompress_bitwise_double" + self._D[ct])
        f(*args, type_, self.mask_chars20(mask20)) if ct == 7 else f(*args)
        out = np.frombuffer(C.string_at(p.value, nb.value), np.uint8).copy() if nb.value else np.zeros(0, np.uint8)
        if p.value:
            _libc.free(p)
        return out, nb.value, pos.value

    def decompress64(self, ct, s, num, type_=0, mask20=0):
        s = np.ascontiguousarray(s, np.uint8)
        sarg = s if s.size else np.zeros(1, np.uint8)
        f = getattr(self.L, "myDecompress_bitwise_double" + self._D[ct])
        p = f(sarg, s.size, num, type_, self.mask_chars20(mask20)) if ct == 7 else f(sarg, s.size, num)
        out = np.frombuffer(C.string_at(p, 8 * num), np.float64).copy() if num else np.zeros(0, np.float64)
        _libc.free(p)
        return out

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

    def ct1_compress64(self, x):
        x = np.ascontiguousarray(x, np.float64)
        pf, pc, pp = C.c_void_p(None), C.c_void_p(None), C.c_void_p(None)
        nf = self.L.myCompress_double(x if x.size else np.zeros(1, np.float64), C.byref(pf), C.byref(pc), C.byref(pp),
                                      x.size)
        nc = x.size - nf
        raw = np.frombuffer(C.string_at(pf.value, 8 * nf), np.float64).copy() if nf else np.zeros(0, np.float64)
        codes = C.string_at(pc.value, nc) if nc else b""
        pos = np.frombuffer(C.string_at(pp.value, 4 * nc), np.int32).copy() if nc else np.zeros(0, np.int32)
        for q in (pf, pc, pp):
            if q.value:
                _libc.free(q)
        return raw, codes, pos

    def ct1_decompress64(self, raw, codes, pos, num):
        raw = np.ascontiguousarray(raw, np.float64)
        pos = np.ascontiguousarray(pos, np.int32)
        posx = np.concatenate([pos, np.zeros(1, np.int32)])   # terminator, as ct1_decompress
        cb = C.create_string_buffer(bytes(codes), len(codes) + 1)
        p = self.L.myDecompress_double(raw.ctypes.data if raw.size else None, C.cast(cb, C.c_void_p), posx.ctypes.data,
                                       num)
        out = np.frombuffer(C.string_at(p, 8 * num), np.float64).copy() if num else np.zeros(0, np.float64)
        _libc.free(p)
        return out

    def encode64_device(self, ct, x_ptr, n, out_ptr, type_=0, mask20=0, start_bit=0, total_ptr=None):
        self.check(self.L.dc64_encode_device(ct, x_ptr, n, type_, mask20, start_bit, out_ptr, total_ptr),
                   "dc64_encode_device")

    def encode64_result(self):
        v = C.c_ulonglong(0)
        self.check(self.L.dc64_encode_result(C.byref(v)), "dc64_encode_result")
        return v.value

    def decode64_device(self, ct, s_ptr, nbytes, num, out_ptr, type_=0, mask20=0, d_nbits=None, max_bytes=None):
        self.check(self.L.dc64_decode_device(ct, s_ptr, nbytes, d_nbits, max_bytes if max_bytes is not None else nbytes,
                                             num, type_, mask20, out_ptr), "dc64_decode_device")

    def decode64_finish(self):
        self.check(self.L.dc64_decode_finish(), "dc64_decode_finish")
        return int(self.L.dc64_last_decode_flags())

    # ---- CT1 byte-wise codec (myCompress / myDecompress)
    def ct1_compress(self, x):
        x = np.ascontiguousarray(x, np.float32)
        pf, pc, pp = C.c_void_p(None), C.c_void_p(None), C.c_void_p(None)
        nf = self.L.myCompress(x if x.size else np.zeros(1, np.float32), C.byref(pf), C.byref(pc), C.byref(pp), x.size)
        nc = x.size - nf
        raw = np.frombuffer(C.string_at(pf.value, 4 * nf), np.float32).copy() if nf else np.zeros(0, np.float32)
        codes = C.string_at(pc.value, nc) if nc else b""
        pos = np.frombuffer(C.string_at(pp.value, 4 * nc), np.int32).copy() if nc else np.zeros(0, np.int32)
        for q in (pf, pc, pp):
            if q.value:
                _libc.free(q)
        return raw, codes, pos

    def ct1_decompress(self, raw, codes, pos, num):
        raw = np.ascontiguousarray(raw, np.float32)
        pos = np.ascontiguousarray(pos, np.int32)
        # the reference reads one displacement entry past the last code: give it a terminator
        posx = np.concatenate([pos, np.zeros(1, np.int32)])
        cb = C.create_string_buffer(bytes(codes), len(codes) + 1)
        p = self.L.myDecompress(raw.ctypes.data if raw.size else None, C.cast(cb, C.c_void_p),
                                posx.ctypes.data, num)
        out = np.frombuffer(C.string_at(p, 4 * num), np.float32).copy() if num else np.zeros(0, np.float32)
        _libc.free(p)
        return out

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
        return int(self.L.do_crc32(s if s.size else np.zeros(1, np.uint8), s.size))

    def hamming_encode(self, s):
        s = np.ascontiguousarray(s, np.uint8)
        p = C.c_void_p(None)
        r = C.c_int(0)
        self.L.hamming_encode(s, C.byref(p), s.size, C.byref(r))
        c = C.string_at(p.value, r.value + 1)
        _libc.free(p)
        return r.value, c

    def hamming_decode(self, s, c, r):
        s = np.array(s, np.uint8)
        cb = C.create_string_buffer(bytes(c), len(c) + 1)
        t = self.L.hamming_decode(s, cb, s.size, r)
        return t, s, cb.raw[: r + 1]

    # ---- device API on torch tensors (library stream; caller synchronizes torch first)
    def stream_capacity(self, n):
        return int(self.L.dc_stream_capacity(n))

    def encode_device(self, ct, x_ptr, n, out_ptr, idx0=0, type_=0, mask17=0, start_bit=0, total_ptr=None):
        self.check(self.L.dc_encode_device(ct, x_ptr, n, idx0, type_, mask17, start_bit, out_ptr, total_ptr),
                   "dc_encode_device")

    def encode_crc_device(self, ct, x_ptr, n, out_ptr, total_ptr, crc_ptr, idx0=0, type_=0, mask17=0):
        """dc_encode_crc_device: the encode (start bit 0) plus the stream's zlib CRC-32 into *crc_ptr (device)."""
        self.check(self.L.dc_encode_crc_device(ct, x_ptr, n, idx0, type_, mask17, out_ptr, total_ptr, crc_ptr),
                   "dc_encode_crc_device")

    def crc32_copy_device(self, src_ptr, dst_ptr, nbytes, crc_ptr):
        """dc_crc32_copy_device: the CT9 send -- src copied to dst with the CRC-32 of the bytes sent (device)."""
        self.check(self.L.dc_crc32_copy_device(C.c_void_p(src_ptr), C.c_void_p(dst_ptr), C.c_longlong(nbytes),
                                               C.c_void_p(crc_ptr)), "dc_crc32_copy_device")

    def encode_send_device(self, ct, x_ptr, n, out_ptr, mirror_ptr, total_ptr=None, idx0=0, type_=0, mask17=0):
        """dc_encode_send_device: the encode (start bit 0) with its stream also written into the receiver's
        buffer mirror_ptr -- the CT9 send without a copy pass."""
        self.check(self.L.dc_encode_send_device(C.c_int(ct), C.c_void_p(x_ptr), C.c_longlong(n), C.c_longlong(idx0),
                                                C.c_int(type_), C.c_uint32(mask17), C.c_void_p(out_ptr),
                                                C.c_void_p(mirror_ptr), C.c_void_p(total_ptr)),
                   "dc_encode_send_device")

    def crc32_pair_device(self, a_ptr, b_ptr, nbytes, crc_a_ptr, crc_b_ptr):
        """dc_crc32_pair_device: the CRC-32 of two equally long device buffers in one pass (device results)."""
        self.check(self.L.dc_crc32_pair_device(C.c_void_p(a_ptr), C.c_void_p(b_ptr), C.c_longlong(nbytes),
                                               C.c_void_p(crc_a_ptr), C.c_void_p(crc_b_ptr)), "dc_crc32_pair_device")

    def crc32_stream_device(self, s_ptr, nbytes, crc_ptr):
        self.check(self.L.dc_crc32_stream_device(s_ptr, nbytes, crc_ptr), "dc_crc32_stream_device")

    def crc_resend_crc_device(self, d_crc2_ptr, src_ptr, dst_ptr, nbytes, d_count_ptr):
        self.check(self.L.dc_crc_resend_crc_device(d_crc2_ptr, src_ptr, dst_ptr, nbytes, d_count_ptr),
                   "dc_crc_resend_crc_device")

    def encode_bits(self, ct, x_ptr, n, idx0=0, type_=0, mask17=0):
        v = C.c_ulonglong(0)
        self.check(self.L.dc_encode_bits_device(ct, x_ptr, n, idx0, type_, mask17, C.byref(v)), "dc_encode_bits_device")
        return v.value

    def encode_status(self):
        v = C.c_uint(0)
        self.check(self.L.dc_encode_status(C.byref(v)), "dc_encode_status")
        return v.value

    def encode_result(self):
        v = C.c_ulonglong(0)
        self.check(self.L.dc_encode_result(C.byref(v)), "dc_encode_result")
        return v.value

    def decode_device(self, ct, s_ptr, nbytes, num, out_ptr, type_=0, mask17=0, d_nbits=None, max_bytes=None):
        self.check(self.L.dc_decode_device(ct, s_ptr, nbytes, d_nbits, max_bytes if max_bytes is not None else nbytes,
                                           num, type_, mask17, out_ptr), "dc_decode_device")

    def decode_shard_device(self, ct, s_ptr, stream_bytes, start_bit, nbits, num, out_ptr, type_=0, mask17=0,
                            hin_ptr=None):
        """Decode the shard at bits [start_bit, start_bit + nbits) of a device stream (dc_gpu.h)."""
        self.check(self.L.dc_decode_shard_device(ct, s_ptr, stream_bytes, start_bit, nbits, num, type_, mask17, hin_ptr,
                                                 out_ptr), "dc_decode_shard_device")

    def halo_encode_device(self, ct, p_ptr, dims, ijk, v, ext, stream_ptr, bits_ptr, min_ptr, type_=0, mask17=0):
        """Fused Himeno halo-plane encode (dc_gpu.h); dims = (mi, mj, mk), ext = (imax, jmax, kmax)."""
        t, m = C.c_int(0), C.c_uint32(0)
        self.check(self.L.dc_halo_encode_device(ct, C.c_void_p(p_ptr), *dims, ijk, v, *ext, type_, C.c_uint32(mask17),
                                                C.c_void_p(stream_ptr), C.c_void_p(bits_ptr), C.c_void_p(min_ptr),
                                                C.byref(t), C.byref(m)), "dc_halo_encode_device")
        return t.value, m.value

    def halo_decode_device(self, ct, stream_ptr, nbytes, bits_ptr, type_, mask17, min_ptr, p_ptr, dims, ijk, v, ext):
        self.check(self.L.dc_halo_decode_device(ct, C.c_void_p(stream_ptr), C.c_longlong(nbytes), C.c_void_p(bits_ptr),
                                                type_, C.c_uint32(mask17), C.c_void_p(min_ptr), C.c_void_p(p_ptr), *dims,
                                                ijk, v, *ext), "dc_halo_decode_device")

    def capture_begin(self):
        """dc_capture_begin: record the following library calls into a HIP graph"""
        self.check(self.L.dc_capture_begin(), "dc_capture_begin")

    def capture_end(self):
        """dc_capture_end: the recorded graph (an opaque handle for graph_launch / graph_destroy)"""
        h = C.c_void_p()
        self.check(self.L.dc_capture_end(C.byref(h)), "dc_capture_end")
        return h

    def graph_launch(self, h):
        self.check(self.L.dc_graph_launch(h), "dc_graph_launch")

    def graph_destroy(self, h):
        self.check(self.L.dc_graph_destroy(h), "dc_graph_destroy")

    def halo_encode2_device(self, ct, p_ptr, dims, ijk, v0, v1, ext, s0_ptr, s1_ptr, bits0_ptr, bits1_ptr, min0_ptr,
                            min1_ptr, type_=0, mask17=0):
        """dc_halo_encode2_device: two planes of one array encoded at once (two streams)."""
        self.check(self.L.dc_halo_encode2_device(ct, C.c_void_p(p_ptr), *dims, ijk, v0, v1, *ext, type_, C.c_uint32(mask17),
                                                 C.c_void_p(s0_ptr), C.c_void_p(s1_ptr), C.c_void_p(bits0_ptr),
                                                 C.c_void_p(bits1_ptr), C.c_void_p(min0_ptr), C.c_void_p(min1_ptr)),
                   "dc_halo_encode2_device")

    def halo_decode2_device(self, ct, s0_ptr, s1_ptr, bits0_ptr, bits1_ptr, type_, mask17, min0_ptr, min1_ptr, p_ptr,
                            dims, ijk, v0, v1, ext):
        """dc_halo_decode2_device: two planes of one array decoded at once (two streams; async halo mode)."""
        self.check(self.L.dc_halo_decode2_device(ct, C.c_void_p(s0_ptr), C.c_void_p(s1_ptr), C.c_void_p(bits0_ptr),
                                                 C.c_void_p(bits1_ptr), type_, C.c_uint32(mask17), C.c_void_p(min0_ptr),
                                                 C.c_void_p(min1_ptr), C.c_void_p(p_ptr), *dims, ijk, v0, v1, *ext),
                   "dc_halo_decode2_device")

    def decode_shard_fix(self, hin_ptr):
        self.check(self.L.dc_decode_shard_fix(hin_ptr), "dc_decode_shard_fix")

    def decode_finish(self):
        self.check(self.L.dc_decode_finish(), "dc_decode_finish")

    def merge_shards_device(self, gathered_ptr, slot_bytes, world, counts_ptr, out_ptr, out_bytes, total_ptr):
        """World all-gathered shards (slots of slot_bytes) + their device bit counts -> the global stream
        and its device bit count (dc_gpu.h); no host read."""
        self.check(self.L.dc_merge_shards_device(gathered_ptr, slot_bytes, world, counts_ptr, out_ptr, out_bytes,
                                                 total_ptr), "dc_merge_shards_device")

    def extract_shard_device(self, global_ptr, global_bytes, counts_ptr, rank, out_ptr, out_bytes, nbits_ptr):
        self.check(self.L.dc_extract_shard_device(global_ptr, global_bytes, counts_ptr, rank, out_ptr, out_bytes,
                                                  nbits_ptr), "dc_extract_shard_device")

    def occupy_device(self, stream_ptr, us, blocks, lds=0):
        """A neighbour holding CU slots: `blocks` workgroups resident for `us` microseconds (asynchronous)."""
        self.check(self.L.dc_occupy_device(stream_ptr, float(us), int(blocks), int(lds)), "dc_occupy_device")

    def merge_status(self, reset=False):
        v = C.c_uint(0)
        self.check(self.L.dc_merge_status(C.byref(v), 1 if reset else 0), "dc_merge_status")
        return v.value

    def decode_shard3_device(self, ct, s_ptr, nbits_ptr, max_bytes, num, out_ptr, type_=0, mask17=0, has_history=1):
        """A shard encoded at start bit 0 through the segment decoder, its first predictions pending."""
        self.check(self.L.dc_decode_shard3_device(ct, s_ptr, nbits_ptr, max_bytes, num, type_, mask17, out_ptr,
                                                  1 if has_history else 0),
                   "dc_decode_shard3_device")

    def decode_shard3_fix(self, hin_ptr):
        self.check(self.L.dc_decode_shard3_fix(hin_ptr), "dc_decode_shard3_fix")

    def decode_status_clear(self):
        self.check(self.L.dc_decode_status_clear(), "dc_decode_status_clear")

    def set_small_chunk_max_bytes(self, v):
        """Streams of at most v bytes of capacity use the 256-bit-chunk decoder build (< 0: default 1 MiB,
        0: never); returns the previous value."""
        return int(self.L.dc_set_small_chunk_max_bytes(int(v)))

    def set_decode3_min_bytes(self, v):
        """Streams of at least v bytes of capacity use the segment decoder (< -1: default 16 KiB + 1,
        -1: never, 0: always); returns the previous value."""
        return int(self.L.dc_set_decode3_min_bytes(int(v)))

    def set_decode3_seg(self, seg):
        """Force the segment decoder's parse segment length (4, 8 or 16 chunks; 0: by size); returns the
        previous setting."""
        return int(self.L.dc_set_decode3_seg(int(seg)))

    def set_fused3(self, on):
        """1: decode 16-chunk-segment streams with the single-launch parse + decode (fused3_kernel), 2: its
        dynamic form (fused3d_kernel, decode jobs from 8 queues), 0: with parse3 + decode3 (the default); returns
        the previous setting."""
        return int(self.L.dc_set_fused3(int(on)))

    def last_decode_fused(self):
        """1 if the last segment-decoder launch was the fused parse + decode."""
        return bool(self.L.dc_decode3_last_fused())

    def fused3_last_seg(self):
        """The segment length (chunks) of the last fused launch."""
        return int(self.L.dc_fused3_last_seg())

    def fused3_stamps(self, max_jobs):
        """The last fused launch's stamps (DC_FUSED3_STAMPS set): an (n, 4) uint64 array of s_memrealtime
        ticks per fused job (start, parse end, prefix known, decode end)."""
        buf = np.zeros((int(max_jobs), 4), dtype=np.uint64)
        self.L.dc_fused3_stamps.restype = C.c_longlong
        n = int(self.L.dc_fused3_stamps(C.c_void_p(buf.ctypes.data), C.c_longlong(int(max_jobs))))
        return buf[:max(n, 0)]

    def set_runs_max_bytes(self, v):
        """Streams of at most v bytes of capacity use the small-stream decoder (< -1: default 16 KiB + 256,
        -1: never); returns the previous value."""
        return int(self.L.dc_set_runs_max_bytes(int(v)))

    def last_decode_was_runs(self):
        """Whether the last finished decode's values came from the small-stream decoder."""
        return bool(self.L.dc_last_decode_was_runs())

    def last_decode_was_v3(self):
        """Whether the last finished decode's values came from the segment decoder."""
        return bool(self.L.dc_last_decode_was_v3())

    def chunk_bits(self):
        """Chunk bits of the decoder build the last decode ran."""
        return int(self.L.dc_decode_chunk_bits_value())

    def decode_status(self):
        """Fast-path status word OR-ed over every decode since the last finish (0: all on the fast path)."""
        v = C.c_uint(0)
        self.check(self.L.dc_decode_status(C.byref(v)), "dc_decode_status")
        return v.value

    def abi_status(self):
        return int(self.L.dc_abi_status())

    def med_sum_device(self, x_ptr, n, s_init=0.0):
        """Exact running float sum of med_dataset_float continued from s_init, and the max (multi-GPU mean)."""
        sm, mx = C.c_float(0), C.c_float(0)
        self.check(self.L.dc_med_sum_device(C.c_void_p(x_ptr), n, C.c_float(s_init), C.byref(sm), C.byref(mx)),
                   "dc_med_sum_device")
        return np.float32(sm.value), np.float32(mx.value)

    def med_shard_stats(self, x_ptr, n):
        """A shard's double sum (an estimate of what it adds to the running float sum), its max (NaNs never
        win) and its first element."""
        sm, mx, x0 = C.c_double(0), C.c_float(0), C.c_float(0)
        self.check(self.L.dc_med_shard_stats(C.c_void_p(x_ptr), n, C.byref(sm), C.byref(mx), C.byref(x0)),
                   "dc_med_shard_stats")
        return float(sm.value), np.float32(mx.value), np.float32(x0.value)

    def med_shard_trans(self, x_ptr, n, s_est):
        """A shard's whole-shard transducer for the binades of the window its running sum is estimated to
        enter at s_est: (e_lo, units [MW, 2] int64, flags [MW] uint8), see include/dc_gpu.h."""
        mw = int(self.L.dc_med_shard_binades())
        e_lo = C.c_int(0)
        units = (C.c_longlong * (2 * mw))()
        flags = (C.c_ubyte * mw)()
        self.check(self.L.dc_med_shard_trans(C.c_void_p(x_ptr), n, C.c_double(s_est), C.byref(e_lo), units, flags),
                   "dc_med_shard_trans")
        return int(e_lo.value), np.array(units[:], np.int64).reshape(mw, 2), np.array(flags[:], np.uint8)

    def type_from_max(self, mx):
        return int(self.L.dc_type_from_max(C.c_float(float(mx))))

    def synchronize(self):
        self.check(self.L.dc_synchronize(), "dc_synchronize")

    def to_small_device(self, x_ptr, n, out_ptr):
        """dc_to_small_device: out = x - min (toSmallDataset_float on device data); returns the minimum."""
        mn = C.c_float(0)
        self.check(self.L.dc_to_small_device(x_ptr, n, out_ptr, C.byref(mn)), "dc_to_small_device")
        return np.float32(mn.value)

    def prep_device(self, x_ptr, n):
        """dc_prep_device: (min, mean, type) = toSmallDataset_float's minimum and med_dataset_float of x - min, fused
        (x - min never written)."""
        mn, m, t = C.c_float(0), C.c_float(0), C.c_int(0)
        self.check(self.L.dc_prep_device(x_ptr, n, C.byref(mn), C.byref(m), C.byref(t)), "dc_prep_device")
        return np.float32(mn.value), np.float32(m.value), t.value

    def encode_sub_device(self, ct, x_ptr, n, mn, out_ptr, type_=0, mask17=0, total_ptr=None):
        """dc_encode_sub_device: the stream of x - mn (toSmallDataset_float's array), subtracted while loading."""
        self.check(self.L.dc_encode_sub_device(ct, x_ptr, n, float(mn), type_, mask17, out_ptr, total_ptr),
                   "dc_encode_sub_device")

    def med_device(self, x_ptr, n):
        m, t = C.c_float(0), C.c_int(0)
        self.check(self.L.dc_med_device(x_ptr, n, C.byref(m), C.byref(t)), "dc_med_device")
        return np.float32(m.value), t.value

    def hash_device(self, ptr, nbytes):
        """dc_hash_device: sum of splitmix64(i << 32 | w_i) over the range's 32-bit words (hash_words below)."""
        v = C.c_ulonglong(0)
        self.check(self.L.dc_hash_device(ptr, nbytes, C.byref(v)), "dc_hash_device")
        return int(v.value)

    def copy_rate(self, src_ptr, dst_ptr, nbytes, reps=10):
        """dc_copy_rate_device: (GB/s read + written, variant) of the best hand-written streaming copy."""
        g, v = C.c_double(0), C.c_int(0)
        self.check(self.L.dc_copy_rate_device(src_ptr, dst_ptr, nbytes, reps, C.byref(g), C.byref(v)), "dc_copy_rate_device")
        return float(g.value), int(v.value)

    def crc32_device(self, s_ptr, nbytes):
        v = C.c_uint32(0)
        self.check(self.L.dc_crc32_device(s_ptr, nbytes, C.byref(v)), "dc_crc32_device")
        return v.value

    def crc32_device_async(self, s_ptr, nbytes, d_crc_ptr):
        self.check(self.L.dc_crc32_device_async(C.c_void_p(s_ptr), C.c_longlong(nbytes), C.c_void_p(d_crc_ptr)),
                   "dc_crc32_device_async")

    def crc_resend_device(self, d_crc2_ptr, src_ptr, dst_ptr, nbytes, copy, d_count_ptr):
        self.check(self.L.dc_crc_resend_device(C.c_void_p(d_crc2_ptr), C.c_void_p(src_ptr), C.c_void_p(dst_ptr),
                                               C.c_longlong(nbytes), C.c_int(copy), C.c_void_p(d_count_ptr)),
                   "dc_crc_resend_device")

    def flip_bits_device(self, s_ptr, nbits, count, seed):
        self.check(self.L.dc_flip_bits_device(C.c_void_p(s_ptr), C.c_ulonglong(nbits), C.c_longlong(count),
                                              C.c_ulonglong(seed)), "dc_flip_bits_device")


def flip_positions(nbits, count, seed):
    """Host restatement of dc_flip_bits_device's positions (splitmix64(seed + i) mod nbits)."""
    M = (1 << 64) - 1
    out = []
    for i in range(count):
        z = (seed + i + 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
        out.append(z % nbits)
    return out


# ---- multi-GPU: one process per GPU, contiguous shards -------------------------
def shard_offsets(bits_per_rank):
    """Exclusive scan of the per-rank stream bit counts -> global start bit of every shard."""
    out, acc = [], 0
    for b in bits_per_rank:
        out.append(acc)
        acc += int(b)
    return out, acc


def gather_stream(local, start_bit, local_bits, group=None):
    """All-gather per-rank shard streams into the single global stream (every rank gets it).

    local: uint8 torch tensor holding this rank's shard, encoded with start_bit = (global start bit
    mod 8) so its first byte's high bits are zero; local_bits = start_bit + the shard's bits.  The
    shards are placed at their global byte offsets and the byte two shards share is OR-ed: the
    result is byte-identical to encoding the whole array in one stream.  Works with
    gloo (CPU tensors) and RCCL (device tensors)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = local.device
    if dev.type == "cuda" and dist.get_backend(group) == "gloo":    # gloo collectives on host copies
        out, total = gather_stream(local.cpu(), start_bit, local_bits, group)
        return out.to(dev), total
    meta = torch.tensor([int(local_bits) - int(start_bit), int(start_bit)], dtype=torch.int64, device=dev)
    metas = [torch.zeros_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    bits = [int(m[0]) for m in metas]
    starts, total = shard_offsets(bits)
    nbytes = [(int(m[1]) + b + 7) // 8 for m, b in zip(metas, bits)]
    pad = max(nbytes) if nbytes else 0
    buf = torch.zeros(pad, dtype=torch.uint8, device=dev)
    buf[: local.numel()] = local[:pad]
    parts = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = torch.zeros((total + 7) // 8, dtype=torch.uint8, device=dev)
    for g in range(world):
        b0, nb = starts[g] // 8, nbytes[g]
        if nb:
            out[b0:b0 + nb] |= parts[g][:nb]
    return out, total


def halo_exchange(streams, nbits, mins, down, up, group=None):
    """Himeno z-halo exchange of compressed planes (impl/himenoBMTxps.c:644-690), one process per GPU.

    streams[0] (plane k = 1) goes to rank `down`, streams[1] (plane k = kmax - 2) to rank `up`; None
    stands for MPI_PROC_NULL (no neighbour: nothing is sent or received on that side).  nbits / mins:
    per-plane stream bit counts and toSmallDataset minima (ints / floats, or 1-element tensors).  As
    the reference, the sizes travel first (one int64 pair per direction: bits and the min's bit pattern),
    then exactly the stream bytes.  Returns [(stream, nbits, min) received from up (for k = kmax - 1),
    the same from down (for k = 0)], None where there is no neighbour.  P2P over RCCL with device
    tensors, or over gloo with host copies.

    The received buffers are complete on torch's current stream; before returning, the library's own
    HIP stream (where halo_decode_device runs) is made to wait for them, so the caller can decode at
    once.  (The sends read streams[] on torch's stream: the caller must have finished the encodes --
    L.synchronize() -- before calling, as the sizes are read on the host anyway.)"""
    import numpy as np
    import torch
    import torch.distributed as dist
    dev = streams[0].device
    host = dev.type == "cuda" and dist.get_backend(group) == "gloo"
    cdev = torch.device("cpu") if host else dev

    def meta(h):
        b = int(nbits[h])
        m = int(np.array([float(mins[h])], np.float32).view(np.int32)[0])
        return torch.tensor([b, m], dtype=torch.int64, device=cdev)

    peers = [(0, down, 0), (1, up, 1)]          # (plane sent, to rank, tag): the receiver gets it from its up / down
    sides = [(up, 0), (down, 1)]                 # (from rank, tag): the planes for k = kmax - 1 and k = 0
    rmeta = [torch.zeros(2, dtype=torch.int64, device=cdev) for _ in sides]
    ops = [dist.P2POp(dist.isend, meta(h), peer, group=group, tag=tag) for h, peer, tag in peers if peer is not None]
    ops += [dist.P2POp(dist.irecv, rmeta[i], peer, group=group, tag=tag)
            for i, (peer, tag) in enumerate(sides) if peer is not None]
    if ops:
        for r in dist.batch_isend_irecv(ops):
            r.wait()
    ops, rbuf = [], [None, None]
    for h, peer, tag in peers:
        nb = (int(nbits[h]) + 7) // 8
        if peer is not None and nb > 0:
            src = streams[h][:nb]
            ops.append(dist.P2POp(dist.isend, src.cpu() if host else src.contiguous(), peer, group=group, tag=2 + tag))
    for i, (peer, tag) in enumerate(sides):
        if peer is None:
            continue
        nb = (int(rmeta[i][0]) + 7) // 8
        rbuf[i] = torch.zeros(nb, dtype=torch.uint8, device=cdev)
        if nb > 0:
            ops.append(dist.P2POp(dist.irecv, rbuf[i], peer, group=group, tag=2 + tag))
    if ops:
        for r in dist.batch_isend_irecv(ops):
            r.wait()
    out = []
    for i, (peer, _) in enumerate(sides):
        if peer is None:
            out.append(None)
            continue
        b, m = int(rmeta[i][0]), int(rmeta[i][1])
        mn = float(np.array([m], np.int32).view(np.float32)[0])
        out.append((rbuf[i].to(dev) if host else rbuf[i], b, mn))
    if dev.type == "cuda":                      # the library stream waits for the received bytes
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        torch.cuda.ExternalStream(lib().L.dc_get_stream(), device=dev).wait_event(ev)
    return out


# ---- CT9 between ranks (BASELINE config 5 across GPUs) ---------------------------
def ct9_partner(rank, world):
    """Rank pairs (0,1), (2,3), ...: each rank sends its stream to its partner and receives the partner's
    (the ping and the pong of impl/pingpong.c at once).  An odd world's last rank is its own partner: its
    channel is a local copy."""
    p = rank ^ 1
    return p if p < world else rank


class LibCT9:
    """The device operations of a CT9 round (ct9_exchange) on the library's HIP stream: the CRC-32 of a
    stream (dc_crc32_device_async: zlib's CRC = the reference's do_crc32, impl/dataCompression.c:5524) into
    the low 4 bytes of an int64 device slot, and floor(bits * BER) bit flips (dc_flip_bits_device, the
    channel's damage).  to_torch / to_lib order torch's current stream (where the collectives run) and the
    library's."""

    def __init__(self, L):
        self.L = L

    def crc(self, buf, nbytes, dst):
        self.L.crc32_device_async(buf.data_ptr(), nbytes, dst.data_ptr())

    def flip(self, buf, nbits, count, seed):
        if count > 0:
            self.L.flip_bits_device(buf.data_ptr(), nbits, count, seed)

    def to_torch(self, dev):
        import torch
        _after(_lib_stream(self.L, dev), torch.cuda.current_stream(dev))

    def to_lib(self, dev):
        import torch
        _after(torch.cuda.current_stream(dev), _lib_stream(self.L, dev))


def _p2p(ops_spec, group, host):
    """Run [(isend|irecv, tensor, peer, tag)] as one batch; gloo moves host copies of device tensors."""
    import torch.distributed as dist
    if not ops_spec:
        return
    ops, back = [], []
    for kind, t, peer, tag in ops_spec:
        if host and t.device.type == "cuda":
            h = t.cpu() if kind == "send" else t.new_empty(t.shape, device="cpu")
            if kind == "recv":
                back.append((t, h))
            t = h
        ops.append(dist.P2POp(dist.isend if kind == "send" else dist.irecv, t, peer, group=group, tag=tag))
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    for t, h in back:
        t.copy_(h)


def ct9_exchange(ops, stream, nbytes_tx, meta_tx, rcv, nbytes_rx, nbits_rx, meta_rx, crc_rx, ack, partner, nflip,
                 seed, group=None, max_rounds=4):
    """One CT9 round with the partner rank (impl/pingpong.c: sender :280-289, receiver :408-447), both directions
    at once, over torch.distributed point-to-point (RCCL on device tensors; gloo on host copies):
      sender    meta_tx = [CRC-32 of its stream, its bit count]; sends the stream bytes and meta_tx;
      receiver  receives them into rcv / meta_rx, the channel flips nflip bits of rcv (seeded), CRCs what
                arrived and answers ack = 1 when the CRC (or the bit count) differs -- 'n' in the reference;
      both      read the two acks on the host (the reference's blocking MPI_Recv of crc_ok); a rejected
                stream is sent again (the reference repeats the round: ping_pong_count--), the receiver
                CRCs the new copy and answers again, until both acks are 0 or max_rounds.
    The stream sizes are known on both sides beforehand (the reference's receiver passes the same byte
    count: both ranks compressed the same data; here ct9_sizes exchanges them once).  meta_tx / meta_rx /
    crc_rx: int64 tensors of 2 / 2 / 1 (CRC in the low 4 bytes; crc_rx's upper bytes zero), ack int64[2]
    (device).  The decode of rcv is the caller's.  Returns (rounds, resent_tx, resent_rx, ok)."""
    import torch.distributed as dist
    dev = stream.device
    cuda = dev.type == "cuda"
    host = cuda and dist.get_backend(group) == "gloo"
    me = dist.get_rank(group)
    ops.crc(stream, nbytes_tx, meta_tx)                     # the sender's CRC of what it sends
    if cuda:
        ops.to_torch(dev)
    if partner == me:                                       # the local channel
        rcv[:nbytes_rx].copy_(stream[:nbytes_tx])
        meta_rx.copy_(meta_tx)
    else:
        _p2p([("send", stream[:nbytes_tx], partner, 0), ("send", meta_tx, partner, 1),
              ("recv", rcv[:nbytes_rx], partner, 0), ("recv", meta_rx, partner, 1)], group, host)
    if cuda:
        ops.to_lib(dev)
    ops.flip(rcv, nbits_rx, nflip, seed)                    # the channel's damage
    resent_tx = resent_rx = 0
    for rnd in range(max_rounds):
        ops.crc(rcv, nbytes_rx, crc_rx)                     # the receiver's check of what arrived
        if cuda:
            ops.to_torch(dev)
        ack[0] = ((crc_rx[0] & 0xFFFFFFFF) != (meta_rx[0] & 0xFFFFFFFF)) | (meta_rx[1] != nbits_rx)
        if partner == me:
            ack[1] = ack[0]
        else:
            _p2p([("send", ack[0:1], partner, 2), ("recv", ack[1:2], partner, 2)], group, host)
        a = ack.cpu()                                       # [my verdict on its stream, its verdict on mine]
        rej_rx, rej_tx = int(a[0]), int(a[1])
        if not rej_rx and not rej_tx:
            return rnd + 1, resent_tx, resent_rx, True
        if partner == me:
            rcv[:nbytes_rx].copy_(stream[:nbytes_tx])
        else:
            spec = []
            if rej_tx:
                spec.append(("send", stream[:nbytes_tx], partner, 3))
            if rej_rx:
                spec.append(("recv", rcv[:nbytes_rx], partner, 3))
            _p2p(spec, group, host)
        resent_tx += rej_tx
        resent_rx += rej_rx
        if cuda:
            ops.to_lib(dev)
    return max_rounds, resent_tx, resent_rx, False


def ct9_sizes(nbits_tx, partner, dev, group=None):
    """The partner's stream bit count (exchanged once, before the rounds)."""
    import torch
    import torch.distributed as dist
    if partner == dist.get_rank(group):
        return int(nbits_tx)
    host = dev.type == "cuda" and dist.get_backend(group) == "gloo"
    t = torch.tensor([int(nbits_tx)], dtype=torch.int64, device=dev)
    r = torch.zeros(1, dtype=torch.int64, device=dev)
    _p2p([("send", t, partner, 9), ("recv", r, partner, 9)], group, host)
    return int(r.item())


def _bcast_scalar(v, src, dev, group=None, dtype=None):
    import torch
    import torch.distributed as dist
    t = torch.tensor([v], dtype=dtype or torch.float32, device=dev)
    dist.broadcast(t, src, group=group)
    return t.cpu().numpy()[0]


def med_apply_shard(e_lo, units, flags, s):
    """The running float sum s after a shard whose whole-shard transducer (dc_med_shard_trans) is
    (e_lo, units, flags), or None when the transducer does not cover s: s outside [2^-100, 3e38), s's
    binade outside the window or marked bad, or the sum leaving its binade (k + units >= 2^24).  Exact:
    s = k * 2^(E-150) with k in [2^23, 2^24) and the result is (k + units) * 2^(E-150)."""
    s = np.float32(s)
    if not (s >= np.float32(2.0 ** -100) and s < np.float32(3.0e38)):
        return None
    b = int(np.array([s], np.float32).view(np.uint32)[0])
    E = (b >> 23) & 0xFF
    w = E - int(e_lo)
    if w < 0 or w >= len(flags) or int(flags[w]) & 4:
        return None
    k = (b & 0x7FFFFF) | 0x800000
    k2 = k + int(units[w][k & 1])
    if k2 >= 1 << 24:
        return None
    return np.float32(k2 * 2.0 ** (E - 150))


def global_med(L, xs_ptr, n, dev, group=None):
    """med_dataset_float of the global array whose contiguous shard of n floats this rank holds (all
    shards the same size), as an exscan over the ranks (impl/dataCompression.c:3593-3620 sums left to
    right, so rank r's shard continues the sum rank r-1 ended with):
      1. every rank: its shard's double sum, max and first value (one pass); one all_gather;
      2. rank 0: its exact float sum from 0 (dc_med_sum_device); every other rank, in parallel: its
         whole-shard binade transducer (dc_med_shard_trans) for the window around the double sum of the
         shards before it; one all_gather;
      3. every rank composes the same walk over the gathered records: a shard whose transducer covers the
         incoming sum is applied exactly on the host; one that does not (the running sum crosses a binade
         inside it -- at most about log2(world) of the ranks after 0) continues the exact sum itself
         and broadcasts it.
    The mean and type every rank returns are those of the single-GPU med_dataset_float of the whole array;
    the max folds rank 0's x[0] with every shard's max (strict >, NaNs never win)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sm, mx, x0 = L.med_shard_stats(xs_ptr, n)
    st = torch.tensor([sm, float(mx), float(x0)], dtype=torch.float64, device=dev)
    parts = [torch.zeros_like(st) for _ in range(world)]
    dist.all_gather(parts, st, group=group)
    stats = [p.cpu().numpy() for p in parts]
    gmax = np.float32(stats[0][2])
    for r in range(world):
        m = np.float32(stats[r][1])
        if m > gmax:
            gmax = m
    mw = int(L.L.dc_med_shard_binades())
    rec = np.zeros(2 + 3 * mw, np.int64)          # [s (rank 0, float bits) | e_lo] units[2 mw] flags[mw]
    if rank == 0:
        s0, _ = L.med_sum_device(xs_ptr, n, 0.0)
        rec[0] = int(np.array([s0], np.float32).view(np.uint32)[0])
    else:
        s_est = 0.0
        for r in range(rank):
            s_est += float(stats[r][0])
        e_lo, units, flags = L.med_shard_trans(xs_ptr, n, s_est)
        rec[1] = e_lo
        rec[2:2 + 2 * mw] = units.reshape(-1)
        rec[2 + 2 * mw:] = flags
    t = torch.from_numpy(rec).to(dev)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    recs = [p.cpu().numpy() for p in parts]
    s = np.array([recs[0][0]], np.uint32).view(np.float32)[0]
    for q in range(1, world):
        r = recs[q]
        s2 = med_apply_shard(r[1], r[2:2 + 2 * mw].reshape(mw, 2), r[2 + 2 * mw:], s)
        if s2 is None:                            # rank q continues the exact sum itself
            if rank == q:
                s2, _ = L.med_sum_device(xs_ptr, n, s)
            s2 = np.float32(_bcast_scalar(float(s2) if rank == q else 0.0, q, dev, group))
        s = s2
    mean = np.float32(s / np.float32(world * n))
    return mean, L.type_from_max(gmax)


def exchange_history(last3, group=None):
    """The 12-byte exchange of the sharded decode: every rank contributes the last three
    values of its shard (x[-1], x[-2], x[-3], a float32 tensor of 3) and receives the previous rank's,
    i.e. its own shard's incoming history b1, b2, b3 (rank 0 gets None)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    parts = [torch_like_zeros(last3) for _ in range(world)]
    dist.all_gather(parts, last3.contiguous(), group=group)
    return parts[rank - 1] if rank > 0 else None


def torch_like_zeros(t):
    import torch
    return torch.zeros_like(t)


def settle_history(tail3, fix, group=None):
    """Run the exchange until no shard's last values change: fix(hin) re-decodes this rank's prefix that
    depends on its incoming values and returns its (possibly updated) last three values.  One round
    unless a prediction chain spans a whole shard, at most world_size rounds."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    last3 = tail3()
    for _ in range(world):
        hin = exchange_history(last3, group)
        changed = torch.zeros(1, dtype=torch.int32, device=last3.device)
        if hin is not None:
            new3 = fix(hin)
            changed[0] = int(not torch.equal(new3, last3))
            last3 = new3
        dist.all_reduce(changed, op=dist.ReduceOp.MAX, group=group)
        if int(changed[0]) == 0:
            break
    return last3


def decode_sharded(L, ct, stream, stream_bytes, start_bit, nbits, num, out, type_=0, mask17=0, group=None):
    """Decode this rank's shard of one global stream on its GPU: rank 0 decodes
    the stream start; the others decode from their start bit with deferred incoming values; then the
    12-byte exchange and the prefix fix-up.  stream / out are device tensors, start_bit / nbits come
    from the encode's shard offsets (shard_offsets), num >= 3."""
    import torch.distributed as dist
    if dist.get_rank(group) == 0:
        L.decode_device(ct, stream.data_ptr(), (int(nbits) + 7) // 8, num, out.data_ptr(), type_, mask17)
    else:
        L.decode_shard_device(ct, stream.data_ptr(), stream_bytes, start_bit, nbits, num, out.data_ptr(), type_, mask17)
    L.decode_finish()

    def tail3():
        return out[num - 3:num].flip(0).contiguous()

    def fix(hin):
        L.decode_shard_fix(hin.data_ptr())
        return tail3()

    settle_history(tail3, fix, group)
    return out


# ---- the device-side multi-GPU step (no host reads inside the step) ---------------
def _lib_stream(L, dev):
    import torch
    return torch.cuda.ExternalStream(L.L.dc_get_stream(), device=dev)


def _after(src, dst):
    """dst waits for the work queued on src so far."""
    import torch
    ev = torch.cuda.Event()
    ev.record(src)
    dst.wait_event(ev)


def _all_gather_flat(t, world, group):
    """all_gather of one tensor per rank into a flat tensor: RCCL on device tensors; gloo on host copies."""
    import torch
    import torch.distributed as dist
    if t.device.type == "cuda" and dist.get_backend(group) == "gloo":
        parts = [torch.empty_like(t, device="cpu") for _ in range(world)]
        dist.all_gather(parts, t.cpu(), group=group)
        return torch.cat(parts).to(t.device)
    out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    return out


def gather_stream_device(L, local, d_count, slot_bytes, out, d_total, group=None):
    """All-gather this rank's shard (encoded at start bit 0 with its global idx0, bit count d_count: a
    1-element int64 device tensor) into the single global stream in `out` (a uint8 device tensor, bit count
    -> d_total), with no host read: the bit counts and the shards (slot_bytes each: >= the largest shard's
    bytes + 8, a multiple of 4 -- e.g. the previous step's largest) are all-gathered, and one merge kernel
    scans the counts and places every shard at its global bit offset (dc_merge_shards_device).  A shard
    longer than its slot sets L.merge_status().  The library stream is ordered after the collectives."""
    import torch.distributed as dist
    import torch
    world = dist.get_world_size(group)
    dev = local.device
    cur, ls = torch.cuda.current_stream(dev), _lib_stream(L, dev)
    _after(ls, cur)                                   # the encode before the collectives
    counts = _all_gather_flat(d_count.view(1), world, group)
    shards = _all_gather_flat(local[:slot_bytes], world, group)
    _after(cur, ls)
    L.merge_shards_device(shards.data_ptr(), slot_bytes, world, counts.data_ptr(), out.data_ptr(), out.numel(),
                          d_total.data_ptr())
    counts.record_stream(ls)
    shards.record_stream(ls)
    return counts


def decode_sharded_device(L, ct, local, d_count, max_bytes, num, out, type_=0, mask17=0, group=None, received=None):
    """Decode this rank's shard (start bit 0, bit count on the device) with the segment decoder; its first
    predictions wait for the previous rank's last three values, which arrive by one all-gather of 12 bytes
    per rank, and a one-wave fix decodes them (dc_decode_shard3_fix).  No host read: L.decode_status() after
    the steps tells whether every shard stayed on this path.

    received = (glob, counts, buf, d_nbits): the shard is cut out of the merged global stream `glob` (the bytes
    that arrived: gather_stream_device's output, `counts` the all-gathered bit counts it returned) into `buf`
    (bit 0, count to d_nbits; dc_extract_shard_device) and decoded from there, as a receiver decodes what it
    received (impl/himenoBMTxps.c:696-697); otherwise from the rank's own encode `local` / d_count."""
    import torch.distributed as dist
    import torch
    rank = dist.get_rank(group)
    dev = out.device
    if received is not None:
        glob, counts, buf, d_nbits = received
        L.extract_shard_device(glob.data_ptr(), glob.numel(), counts.data_ptr(), rank, buf.data_ptr(), buf.numel(),
                               d_nbits.data_ptr())
        local, d_count = buf, d_nbits
    L.decode_shard3_device(ct, local.data_ptr(), d_count.data_ptr(), max_bytes, num, out.data_ptr(), type_, mask17,
                           has_history=rank > 0)
    cur, ls = torch.cuda.current_stream(dev), _lib_stream(L, dev)
    _after(ls, cur)
    hin = exchange_history(out[num - 3:num].flip(0).contiguous(), group)
    _after(cur, ls)
    if hin is not None:
        hin = hin.to(dev)
        L.decode_shard3_fix(hin.data_ptr())
        hin.record_stream(ls)
    return out


def hash_words(buf, nbytes=None):
    """Host twin of dc_hash_device: sum over the 32-bit little-endian words w_i of the first nbytes bytes
    (zero-padded) of splitmix64(i << 32 | w_i) mod 2^64."""
    b = np.frombuffer(memoryview(buf).cast("B"), np.uint8) if not isinstance(buf, np.ndarray) else buf.view(np.uint8).reshape(-1)
    nbytes = b.size if nbytes is None else int(nbytes)
    b = b[:nbytes]
    nw = (nbytes + 3) // 4
    h = np.uint64(0)
    blk = 1 << 24
    with np.errstate(over="ignore"):
        for w0 in range(0, nw, blk):
            w1 = min(nw, w0 + blk)
            chunk = b[4 * w0:4 * w1]
            if chunk.size < 4 * (w1 - w0):
                chunk = np.concatenate([chunk, np.zeros(4 * (w1 - w0) - chunk.size, np.uint8)])
            w = chunk.view("<u4").astype(np.uint64)
            z = (np.arange(w0, w1, dtype=np.uint64) << np.uint64(32)) | w
            z = z + np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            h = h + np.sum(z, dtype=np.uint64)
    return int(h)


def gen_u10(n, seed=42, offset=0):
    """Synthetic U10 input: counter-based splitmix64 -> uniform [0,10) float32.  Generated in
    blocks of 2^22 so that the uint64 temporaries stay small (~100 MB) at any n (2^28: 1 GB of output)."""
    out = np.empty(n, dtype=np.float32)
    blk = 1 << 22
    for b0 in range(0, n, blk):
        m = min(blk, n - b0)
        i = np.arange(offset + b0, offset + b0 + m, dtype=np.uint64) + np.uint64(1)
        with np.errstate(over="ignore"):
            z = np.uint64(0x9E3779B97F4A7C15) * i + np.uint64(seed)
            z ^= z >> np.uint64(30)
            z *= np.uint64(0xBF58476D1CE4E5B9)
            z ^= z >> np.uint64(27)
            z *= np.uint64(0x94D049BB133111EB)
            z ^= z >> np.uint64(31)
        out[b0:b0 + m] = ((z >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)) * np.float32(10.0)
    return out


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = Lib()
    return _lib
