"""Diagnostic (not a test): decode time (parse3 + decode3) of a 2^k U10 CT7 stream per forced segment length."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
import torch, dcamd
L = dcamd.Lib(); L.init(0)
L.set_bound(float(sys.argv[4]) if len(sys.argv) > 4 else 1e-3)
lg = int(sys.argv[1]) if len(sys.argv) > 1 else 26
ct = int(sys.argv[2]) if len(sys.argv) > 2 else 7
n = 1 << lg
kind = sys.argv[5] if len(sys.argv) > 5 else "u10"
if kind == "u10":
    xh = dcamd.gen_u10(n)
elif kind == "sine":
    i = np.arange(n, dtype=np.float64)
    xh = (np.sin(i * 1e-3) * 50.0 + np.sin(i * 0.37) * 0.5).astype(np.float32)
elif kind == "normal":
    xh = np.random.default_rng(1).standard_normal(n).astype(np.float32)
else:                                                  # ramp with noise
    xh = (np.arange(n, dtype=np.float64) * 1e-4 + np.random.default_rng(2).random(n) * 1e-2).astype(np.float32)
xh = xh - xh.min()                                     # (toSmallDataset)
x = torch.from_numpy(np.ascontiguousarray(xh, np.float32)).cuda()
cap = L.stream_capacity(n)
st = torch.zeros(cap, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
mean, t = L.med_device(x.data_ptr(), n)
m17 = int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)
L.encode_device(ct, x.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17)
nbits = L.encode_result()
nb = (nbits + 7) // 8
ls = torch.cuda.ExternalStream(L.L.dc_get_stream())
ref = None
segs = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [16, 8, 16, 8]
for seg in segs:
    L.set_decode3_seg(seg)
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    for _ in range(3):
        L.decode_device(ct, st.data_ptr(), nb, n, out.data_ptr(), type_=t, mask17=m17, max_bytes=cap)
        L.decode_finish()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(ls)
    for _ in range(20):
        L.decode_device(ct, st.data_ptr(), nb, n, out.data_ptr(), type_=t, mask17=m17, max_bytes=cap)
    e1.record(ls)
    stv = L.decode_status()
    L.decode_status_clear()
    L.decode_device(ct, st.data_ptr(), nb, n, out.data_ptr(), type_=t, mask17=m17, max_bytes=cap)
    L.decode_finish()
    torch.cuda.synchronize()
    v3 = L.L.dc_last_decode_was_v3()
    maps = L.L.dc_last_decode_used_maps()
    if ref is None:
        ref = out.clone()
    import time
    t0 = time.perf_counter()
    for _ in range(5):
        L.decode_device(ct, st.data_ptr(), nb, n, out.data_ptr(), type_=t, mask17=m17, max_bytes=cap)
        L.decode_finish()
    full = (time.perf_counter() - t0) / 5 * 1e3
    print(f"   complete decode incl. any slow path (host-synchronised): {full:.3f} ms", flush=True)
    print(f"{kind} 2^{lg} ct{ct} bound {L.get_bound() if hasattr(L, 'get_bound') else ''} seg {seg}: decode {e0.elapsed_time(e1) * 1000 / 20:.1f} us per step, fast-path status 0x{stv:x}, v3 {v3}, maps {maps}, same {bool(torch.equal(out, ref))}", flush=True)
