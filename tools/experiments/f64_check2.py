"""Debug helper: every chunk record of the double decoder's speculative path vs the true boundaries."""
import os, sys, numpy as np, ctypes as C
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import dcamd
from pyoracle import Oracle
L = dcamd.Lib(); L.init(0); O = Oracle()
n = 1 << int(sys.argv[1]); ct = 7; bound = 1e-3
L.set_bound(bound)
mn, xs = O.to_small64(O.gen_u10_64(n)); mean, t = O.med64(xs); m20 = O.mask20(mean)
so, nbo, _ = O.compress64(ct, xs, bound, t, m20)
cap = (so.size * 8 + 2047) // 2048
TE = np.zeros(cap, np.uint8); TX = np.zeros(cap, np.uint8); TN = np.zeros(cap, np.uint16)
O.L.orc64_chunk_records.argtypes = [C.c_int, C.c_void_p, C.c_long, C.c_long, C.c_double, C.c_int, C.c_uint32, C.c_long] + [C.c_void_p] * 3
O.L.orc64_chunk_records(ct, so.ctypes.data, so.size, n, bound, t, m20, 2048, TE.ctypes.data, TX.ctypes.data, TN.ctypes.data)
L.L.dc64_debug_chunks.argtypes = [C.c_void_p] * 4 + [C.c_longlong]
for it in range(3):
    d = L.decompress64(ct, so, n, t, m20)
    E = np.zeros(cap, np.uint8); X = np.zeros(cap, np.uint8); N = np.zeros(cap, np.uint16); B = np.zeros(cap, np.uint64)
    nc = L.L.dc64_debug_chunks(E.ctypes.data, X.ctypes.data, N.ctypes.data, B.ctypes.data, cap)
    ctr = (C.c_uint * 5)(); L.L.dc64_debug_ctr(ctr)
    we = np.nonzero(E[:nc] != TE[:nc])[0]; wx = np.nonzero(X[:nc - 1] != TX[:nc - 1])[0]; wn = np.nonzero(N[:nc] != TN[:nc])[0]
    print("run", it, "ctr", list(ctr), "wrong entries", we.size, we[:5], "exits", wx.size, wx[:5], "counts", wn.size, wn[:5], flush=True)
    for c in wn[:4]:
        print("   chunk", c, "gpu", (int(E[c]), int(X[c]), int(N[c])), "true", (int(TE[c]), int(TX[c]), int(TN[c])),
              "prev gpu", (int(E[c-1]), int(X[c-1]), int(N[c-1])), "prev true", (int(TE[c-1]), int(TX[c-1]), int(TN[c-1])))
