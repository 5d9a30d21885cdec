"""Diagnostic (not a test): phase stamps of the single-pass encoder (DC_DEBUG_STAMPS=1), 2^26 U10 CT7.
Per tile: start, tokens made, aggregate published, look-back start/end, stores done (s_memrealtime, 100 MHz),
look-back windows / spins, XCD id."""
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
for rep in range(4):
    L.encode_device(7, x.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17)
    L.encode_result()
NT = 16384
buf = (ctypes.c_ulonglong * (NT * 8))()
L.L.dc_debug_enc_stamps(buf, NT * 8)
a = np.frombuffer(buf, np.uint64).reshape(NT, 8).astype(np.int64)
ok = a[:, 0] > 0
a = a[ok]
idx = np.nonzero(ok)[0]
t0 = a[:, 0].min()
d = np.diff(a[:, :6], axis=1) / 100.0
xa = (a[:, 7] - a[:, 0]) / 100.0                 # wave 0's first x granules arrived (slot 7)
print(f"x arrival    mean {xa.mean():8.2f} us  p50 {np.median(xa):8.2f}  p90 {np.percentile(xa, 90):8.2f}  max {xa.max():8.2f}")
for i, nm in enumerate(["load+tokens", "scan", "tv+pack", "look-back", "tail+store"]):
    print(f"{nm:12s} mean {d[:, i].mean():8.2f} us  p50 {np.median(d[:, i]):8.2f}  p90 {np.percentile(d[:, i], 90):8.2f}  max {d[:, i].max():8.2f}")
print("tiles", len(a), "span us", (a[:, 5].max() - t0) / 100.0)
life = (a[:, 5] - a[:, 0]) / 100.0
st_ = (a[:, 0] - t0) / 100.0
print(f"lifetime mean {life.mean():.2f} us p50 {np.median(life):.2f}; starts: last {st_.max():.1f} us; "
      f"tiles started in the first 5 us {(st_ < 5).sum()}")
win = a[:, 6] & 0xFFFF; spins = a[:, 6] >> 16
print("look-back windows mean %.2f max %d; spins mean %.2f p90 %.0f max %d" % (win.mean(), win.max(), spins.mean(), np.percentile(spins, 90), spins.max()))
xcc = a[:, 7]
for k in range(8):
    m = xcc == k
    if m.any():
        print(f"xcc {k}: tiles {m.sum():5d} start first {((a[m,0].min()-t0)/100):7.1f} last {((a[m,0].max()-t0)/100):7.1f} us; lb mean {d[m,3].mean():6.2f}")
for q in range(0, len(a), 1024):
    s = slice(q, q + 1024)
    print(f"tiles {idx[q]:5d}+: start {((a[s,0].min()-t0)/100):7.1f}..{((a[s,0].max()-t0)/100):7.1f}  agg {((a[s,2].mean()-t0)/100):7.1f}  lb {d[s,3].mean():6.2f} (p90 {np.percentile(d[s,3],90):6.2f})  end {((a[s,5].max()-t0)/100):7.1f}")
