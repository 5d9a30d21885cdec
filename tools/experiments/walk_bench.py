"""Token-walk throughput on the real CT7 U10 2^26 stream (diagnostic; tools/walk_bench.hip)."""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
import dcamd  # noqa: E402

W = ctypes.CDLL(os.path.join(HERE, "libwalkbench.so"))
W.walk_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                       ctypes.c_uint, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
NAMES = ["512 lut", "1024 lut", "2048 lut", "1024 alu", "2048 alu", "1024 lut x2", "1024 alu x2", "1024 lut+pat",
         "1024 alu+pat", "512 lut x2", "512 alu x2", "512 alu"]

L = dcamd.Lib()
L.init(0)
L.set_bound(1e-3)
n = 1 << 26
dev = torch.device("cuda", 0)
x = torch.from_numpy(dcamd.gen_u10(n, 42, 0)).to(dev)
xs = torch.empty_like(x)
mn = ctypes.c_float(0)
L.check(L.L.dc_to_small_device(ctypes.c_void_p(x.data_ptr()), n, ctypes.c_void_p(xs.data_ptr()), ctypes.byref(mn)), "tosmall")
mean, typ = L.med_device(xs.data_ptr(), n)
mask17 = int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)
cap = L.stream_capacity(n)
stream = torch.zeros(cap, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
L.encode_device(7, xs.data_ptr(), n, stream.data_ptr(), type_=typ, mask17=mask17)
nbits = L.encode_result()
nbytes = (nbits + 7) // 8
print(f"stream {nbytes} bytes, type {typ}, mask17 {mask17:#x}")
out = torch.zeros(4, dtype=torch.int64, device=dev)
ms = ctypes.c_float(0)
for v, name in enumerate(NAMES):
    for grid in (0, 1024, 2048):
        rc = W.walk_run(v, grid, stream.data_ptr(), nbytes & ~15, 10, typ, mask17, out.data_ptr(), ctypes.byref(ms))
        tok = int(out[0].item())
        print(f"{name:14s} grid {grid:5d}: {ms.value * 1e3:8.1f} us  tokens {tok}  {tok / (ms.value * 1e3):8.0f} tok/us  rc {rc}")
    sys.stdout.flush()
