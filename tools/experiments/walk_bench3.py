"""Latency hiding of the token walk: waves per SIMD x chains per lane (diagnostic; tools/walk_bench3.hip).
Reports SIMD cycles per wave-step (one step of one chain of a whole wave) from the kernel wall time
and the in-kernel clock estimate (2.1 GHz assumed)."""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "data-compression_amd"))
import dcamd  # noqa: E402

W = ctypes.CDLL(os.path.join(HERE, "libwalkbench3.so"))
W.walk3_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                        ctypes.c_uint, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
L = dcamd.Lib()
L.init(0)
L.set_bound(1e-3)
n = 1 << 22
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
for ilp in (1, 2, 4):
    for wpc in (4, 8, 12, 16, 24, 32):
        grid = ncu * wpc
        W.walk3_run(ilp, grid, stream.data_ptr(), nbytes & ~15, 10, typ, mask17, out.data_ptr(), ctypes.byref(ms))
        tok, cyc, waves = int(out[0]), int(out[1]), int(out[2])
        wave_steps = tok / 64.0
        simd_cyc = ms.value * 1e-3 * 2.1e9 * ncu * 4
        print(f"ILP {ilp} waves/CU {wpc:2d}: {ms.value * 1e3:8.1f} us  {tok / (ms.value * 1e3):9.0f} tok/us  "
              f"{simd_cyc / wave_steps:6.1f} SIMD-cyc per wave-step  (wave {cyc / waves / (wave_steps / waves):6.1f} cyc/step)")
        sys.stdout.flush()
