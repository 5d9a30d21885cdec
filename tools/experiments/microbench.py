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

# VALU issue rate: W waves per SIMD (blocks of 256 = one wave per SIMD), 8 chains x 6 ops x iters
if len(sys.argv) > 1 and sys.argv[1] == "valu":
    iters = 20000
    for W in (1, 2, 3, 4, 6, 8):
        L.mb_run(4, x.data_ptr(), y.data_ptr(), iters, 256 * W, 256, 3, ctypes.byref(ms), clk)
        waves = 256 * W * 4
        instr = waves * iters * 72.0          # 72 VALU per iteration (checked in the .s)
        print(f"valu W={W}: {ms.value*1e3:9.1f} us  {instr / 1024 / (ms.value * 1e-3) / 1e9:6.3f} G wave-instr/s per SIMD")
