"""The token walk alone out of LDS: padded rows vs per-wave transposed layout, LUT vs ALU length
(diagnostic; tools/walk_bench2.hip).  Cycles per wave-step per SIMD from the kernel wall time."""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "data-compression_amd"))
import dcamd  # noqa: E402

W = ctypes.CDLL(os.path.join(HERE, "libwalkbench2.so"))
W.walk2_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                        ctypes.c_uint, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
L = dcamd.Lib()
L.init(0)
L.set_bound(1e-3)
n = 1 << 24
dev = torch.device("cuda", 0)
x = torch.from_numpy(dcamd.gen_u10(n, 42, 0)).to(dev)
xs = torch.empty_like(x)
mn = ctypes.c_float(0)
L.check(L.L.dc_to_small_device(ctypes.c_void_p(x.data_ptr()), n, ctypes.c_void_p(xs.data_ptr()), ctypes.byref(mn)), "ts")
mean, typ = L.med_device(xs.data_ptr(), n)
mask17 = int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)
stream = torch.zeros(L.stream_capacity(n), dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
L.encode_device(7, xs.data_ptr(), n, stream.data_ptr(), type_=typ, mask17=mask17)
nbytes = (L.encode_result() + 7) // 8
out = torch.zeros(4, dtype=torch.int64, device=dev)
ms = ctypes.c_float(0)
ncu = torch.cuda.get_device_properties(0).multi_processor_count
for v, name in enumerate(["pad lut", "trn lut", "pad alu", "trn alu"]):
    for per_cu in (1, 2, 3, 4):
        grid = ncu * per_cu
        W.walk2_run(v, grid, stream.data_ptr(), nbytes & ~15, 10, typ, mask17, out.data_ptr(), ctypes.byref(ms))
        tok, cyc, waves = int(out[0]), int(out[1]), int(out[2])
        steps_per_wave = tok / waves / 64                        # tokens per lane (the wave runs ~its max)
        cyc_wave = cyc / waves                                   # s_memtime cycles per wave over the walk
        simd_cyc_per_step = cyc_wave / steps_per_wave / per_cu  # per_cu waves share a SIMD
        print(f"{name:8s} {per_cu} WG/CU: {ms.value * 1e3:8.1f} us  {tok / (ms.value * 1e3):9.0f} tok/us  "
              f"wave {cyc_wave:9.0f} cyc, {cyc_wave / steps_per_wave:6.1f} cyc/step/wave, {simd_cyc_per_step:5.1f} per SIMD")
