"""Debug helper: GPU double codec vs the oracle at a given size (first mismatch, decode flags)."""
import os, sys, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch, dcamd
from pyoracle import Oracle
L = dcamd.Lib(); L.init(0); O = Oracle()
log2n = int(sys.argv[1]); ct = int(sys.argv[2]); bound = 1e-3
L.set_bound(bound)
n = 1 << log2n
mn, xs = O.to_small64(O.gen_u10_64(n))
mean, t = O.med64(xs); m20 = O.mask20(mean)
so, nbo, _ = O.compress64(ct, xs, bound, t, m20)
ref, got = O.decompress64(ct, so, n, bound, t, m20)
for force in ("0", "1"):
    os.environ["DC64_FORCE_MAP"] = force
    s, nb, pos = L.compress64(ct, xs, t, m20)
    print("force", force, "enc equal", nb == nbo and np.array_equal(s, so), flush=True)
    d = L.decompress64(ct, so, n, t, m20)
    fl = int(L.L.dc64_last_decode_flags())
    bad = np.nonzero(d.view(np.uint64) != ref.view(np.uint64))[0]
    print("force", force, "flags", fl, "mismatches", bad.size, "first", bad[:5], flush=True)

# chunk records of the speculative path vs a sequential walk around the first mismatch
import ctypes as C
os.environ["DC64_FORCE_MAP"] = "0"
d = L.decompress64(ct, so, n, t, m20)
cap = (so.size * 8 + 2047) // 2048
E = np.zeros(cap, np.uint8); X = np.zeros(cap, np.uint8); N = np.zeros(cap, np.uint16); B = np.zeros(cap, np.uint64)
L.L.dc64_debug_chunks.argtypes = [C.c_void_p] * 4 + [C.c_longlong]
nc = L.L.dc64_debug_chunks(E.ctypes.data, X.ctypes.data, N.ctypes.data, B.ctypes.data, cap)
print("nchunks", nc)
links = np.nonzero(X[:nc - 1] != E[1:nc])[0]
print("broken links", links[:10])
cnt_ok = np.nonzero(np.cumsum(N[:nc].astype(np.uint64)) - N[:nc] != B[:nc])[0]
print("base != exclusive scan of counts at", cnt_ok[:10], B[cnt_ok[:3]] if cnt_ok.size else "")
bad = np.nonzero(d.view(np.uint64) != ref.view(np.uint64))[0]
if bad.size:
    k = bad[0]
    c = int(np.searchsorted(B[:nc], k, side="right")) - 1
    print("first mismatch token", k, "chunk", c, "records", [(int(i), int(E[i]), int(X[i]), int(N[i]), int(B[i])) for i in range(c - 2, c + 3)])
    bits = np.unpackbits(so)
    lens = {}
    def tl(p):
        # CT7 token length (type t, mm from m20)
        if bits[p]: return 3
        if all(bits[p + 1: p + 1 + t]):
            B_ = 10; E_ = (m20 >> 8) & 0x7FF; mm = min(max(B_ + E_ - 1023, 0), 52)
            return t + 2 + (mm if bits[p + 1 + t] else max(mm - 8, 0))
        Ex = int("".join(map(str, bits[p + 1:p + 12])), 2)
        return 12 + min(max(10 + Ex - 1023, 0), 52)
    for cc in (c - 1, c):
        p = cc * 2048 + int(E[cc]); cnt = 0
        while p < (cc + 1) * 2048:
            p += tl(p); cnt += 1
        print("chunk", cc, "walk from entry", int(E[cc]), "-> exit", p - (cc + 1) * 2048, "count", cnt)
