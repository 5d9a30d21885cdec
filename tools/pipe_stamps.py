"""Diagnostic (not a test): phase stamps of the pipelined encoder (DC_ENC_PIPE=1 DC_DEBUG_STAMPS=1), 2^26 U10 CT7."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
import torch, dcamd
L = dcamd.Lib(); L.init(0); L.set_bound(1e-3)
n = 1 << 26
x = torch.from_numpy(dcamd.gen_u10(n)).cuda()
st = torch.empty(L.stream_capacity(n), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
mean, t = L.med_device(x.data_ptr(), n)
m17 = int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)
for rep in range(4):
    L.encode_device(7, x.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17)
    L.encode_result()
NT = 16384
buf = (ctypes.c_ulonglong * (NT * 8))()
L.L.dc_debug_enc_stamps(buf, NT * 8)
a = np.frombuffer(buf, np.uint64).reshape(NT, 8).astype(np.int64)
t0 = a[:, 0].min()
d = np.diff(a[:, :7], axis=1) / 100.0
for i, nm in enumerate(["transpose+issue", "tokens", "publish", "pack", "lookback", "stores"]):
    print(f"{nm:16s} mean {d[:, i].mean():7.2f} us  p50 {np.median(d[:, i]):7.2f}  p90 {np.percentile(d[:, i], 90):7.2f}  max {d[:, i].max():7.2f}")
blk = a[:, 7]
gaps = []
for bk in np.unique(blk):
    m = np.nonzero(blk == bk)[0]
    o = m[np.argsort(a[m, 0])]
    gaps += list((a[o[1:], 0] - a[o[:-1], 6]) / 100.0)
gaps = np.array(gaps)
print(f"stores -> next top (x wait) mean {gaps.mean():.2f} p50 {np.median(gaps):.2f} p90 {np.percentile(gaps, 90):.2f}")
print("span us", (a[:, 6].max() - t0) / 100.0, "blocks", len(np.unique(blk)))
