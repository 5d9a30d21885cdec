"""Calibrate HBM read/copy bandwidth and shader clock on the box (diagnostic)."""
import ctypes, os, subprocess, sys
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(HERE, "libmicrobench.so")
L = ctypes.CDLL(so)
L.mb_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                     ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_ulonglong)]
nb = 268435456
x = torch.ones(nb // 4, dtype=torch.float32, device="cuda")
y = torch.empty(nb // 4, dtype=torch.float32, device="cuda")
ms = ctypes.c_float(0); clk = (ctypes.c_ulonglong * 2)()
for which, name in [(0, "read"), (1, "read16"), (2, "copy")]:
    for grid in [1024, 2048, 4096, 16384, 65536]:
        L.mb_run(which, x.data_ptr(), y.data_ptr(), nb, grid, 256, 5, ctypes.byref(ms), clk)
        gb = nb * (2 if which == 2 else 1) / (ms.value * 1e-3) / 1e9
        print(f"{name:7s} grid {grid:6d}: {ms.value*1e3:8.1f} us  {gb:7.0f} GB/s")
for grid in [256, 2048]:
    L.mb_run(3, x.data_ptr(), y.data_ptr(), 200000, grid, 256, 1, ctypes.byref(ms), clk)
    print(f"clock grid {grid}: {clk[0] / (clk[1] * 10e-9) / 1e9:.3f} GHz (memtime/memrealtime)")
