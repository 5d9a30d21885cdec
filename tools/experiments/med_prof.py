"""med_dataset_float compose-kernel sections (DC_MED_PROF build: DCAMD_LIB=data-compression_amd/lib_mp/libdcamd.so)
at 2^26 U10 after toSmallDataset: iterations, ring refills, serial chunks and rounds, and the s_memrealtime
(100 MHz) spent per section by the workgroup's thread 0."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch, dcamd
from pyoracle import Oracle
L = dcamd.Lib(); L.init(0); O = Oracle()
lg = int(sys.argv[1]) if len(sys.argv) > 1 else 26
n = 1 << lg
_, xs = O.to_small(dcamd.gen_u10(n))
x = torch.from_numpy(xs).cuda()
L.med_device(x.data_ptr(), n)
buf = (ctypes.c_longlong * 16)()
L.check(L.L.dc_med_prof_read(ctypes.c_longlong(n), buf), "prof")
v = list(buf)
t = lambda k: v[k] * 10 / 1e3
print(f"2^{lg}: zero-skip rounds {v[0]}, block iterations {v[1]}, ring refills {v[2]}, serial chunks {v[5]}, "
      f"element rounds {v[7]}, single-lane finishes {v[8]}, two-binade finishes {v[6]}")
print(f"  us: iteration head+refill {t(3):.1f}, block rounds {t(4):.1f}, serial chunks {t(9):.1f}")
print(f"  med_round sections (us, all rounds): syncthreads_or {t(10):.1f}, scan..barrier1 {t(11):.1f}, barrier1 {t(12):.1f}, "
      f"prefix {t(13):.1f}, walk+ballot {t(14):.1f}, barrier2+pick {t(15):.1f}")
