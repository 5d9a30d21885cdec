"""Diagnostic (not a test): encoder phase timings from s_memrealtime stamps. DC_DEBUG_STAMPS=1."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
import torch, dcamd
L = dcamd.Lib(); L.init(0); L.set_bound(1e-3)
n = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
x = torch.from_numpy(dcamd.gen_u10(n)).cuda()
st = torch.empty(L.stream_capacity(n), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
mean, t = L.med_device(x.data_ptr(), n)
m17 = int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)
for rep in range(3):
    L.encode_device(7, x.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17)
    L.encode_result()
buf = (ctypes.c_ulonglong * (8192 * 8))()
L.L.dc_debug_enc_stamps(buf, 8192 * 8)
a = np.frombuffer(buf, np.uint64).reshape(8192, 8).astype(np.int64)
a = a[a[:, 0] > 0]
d = np.diff(a[:, :6], axis=1) * 10.0 / 1000.0
for i, nm in enumerate(["load+tokens", "scan+head", "look-back", "assemble", "write"]):
    print(f"encode {nm:12s} mean {d[:, i].mean():8.2f} us  p50 {np.median(d[:, i]):8.2f}  max {d[:, i].max():8.2f}")
t0 = a[:, 0].min()
print("tiles", len(a), "span us", (a[:, 5].max() - t0) / 100.0)
order = np.argsort(a[:, 0])
print("start times of tiles 0,1000,2000,..:", [round((a[i, 0] - t0) / 100.0, 1) for i in range(0, len(a), 1000)])
dur = (a[:, 5] - a[:, 0]) / 100.0
span = (a[:, 5].max() - a[:, 0].min()) / 100.0
print("tile duration mean %.2f us; implied concurrent tiles %.0f" % (dur.mean(), len(a) * dur.mean() / span))
