"""Diagnostic (not a test): decoder phase timings from s_memrealtime stamps. DC_DEBUG_STAMPS=1."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
import torch, dcamd
L = dcamd.Lib(); L.init(0); L.set_bound(1e-3)
n = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
kind = sys.argv[2] if len(sys.argv) > 2 else "u10"
ct = int(sys.argv[3]) if len(sys.argv) > 3 else 7
if kind == "eq":
    x = torch.full((n,), 0.123456789, dtype=torch.float32)
elif kind == "plane":            # a Himeno z-halo plane: p = i^2/(imax-1)^2, rows of 256 equal values
    i = np.arange(n) // 256
    x = torch.from_numpy((i * i).astype(np.float32) / np.float32(255 * 255))
else:
    x = torch.from_numpy(dcamd.gen_u10(n))
x = x.cuda()
cap = L.stream_capacity(n)
st = torch.empty(cap, dtype=torch.uint8, device="cuda"); out = torch.empty(n, dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
mean, t = L.med_device(x.data_ptr(), n)
m17 = int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)
L.encode_device(ct, x.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17)
nb = (L.encode_result() + 7) // 8
for rep in range(3):
    L.decode_device(ct, st.data_ptr(), nb, n, out.data_ptr(), type_=t, mask17=m17)
    L.decode_finish()
buf = (ctypes.c_ulonglong * (4096 * 16))()
L.L.dc_debug_stamps(buf, 4096 * 16)
a = np.frombuffer(buf, np.uint64).reshape(4096, 16).astype(np.int64)
ntile = (nb * 8 + 262143) // 262144
a = a[:min(ntile, 4096)]
names = ["stage", "P parse", "round2", "closure", "std+map+write"]
cols = [0, 1, 2, 3, 4, 7]
d = np.diff(a[:, cols], axis=1) * 10.0 / 1000.0   # us
print("tiles", len(a), "rounds(mean)", a[:, 12].mean())
for i, nm in enumerate(names):
    print(f"parse {nm:14s} mean {d[:, i].mean():8.2f} us  p50 {np.median(d[:, i]):8.2f}  max {d[:, i].max():8.2f}")
dd = np.diff(a[:, 8:12], axis=1) * 10.0 / 1000.0
for i, nm in enumerate(["stage+resolve", "decode pass1", "carry+fixup"]):
    print(f"decode {nm:13s} mean {dd[:, i].mean():8.2f} us  p50 {np.median(dd[:, i]):8.2f}  max {dd[:, i].max():8.2f}")
w = a[:, 12:16]
cyc, stp = (w >> 16).astype(np.float64), (w & 0xFFFF).astype(np.float64)
ok = stp > 0
print("pre-loop cycles/wave-step mean %.1f  (steps/wave mean %.1f, cycles/wave mean %.0f)" %
      ((cyc[ok] / stp[ok]).mean(), stp[ok].mean(), cyc[ok].mean()))
t0 = a[:, 0].min()
print("parse span us", (a[:, 7].max() - t0) / 100.0, " decode start->end us", (a[:, 11].max() - a[:, 8].min()) / 100.0)
