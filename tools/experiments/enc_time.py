"""Encoder time per launch on the bench's workload (CT7 U10 2^26 after toSmallDataset, med mask, bound 1e-3):
20 back-to-back dc_encode_device calls, HIP events on the library stream.  DCAMD_LIB selects a variant build
(diagnostic builds DC_ENC_DIAG_NOSTORE / DC_ENC_DIAG_NOLB write wrong streams: time only).

usage: python3 tools/experiments/enc_time.py [lg=26] [ct=7] [label]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
import torch, dcamd

L = dcamd.Lib(); L.init(0)
L.set_bound(1e-3)
lg = int(sys.argv[1]) if len(sys.argv) > 1 else 26
ct = int(sys.argv[2]) if len(sys.argv) > 2 else 7
label = sys.argv[3] if len(sys.argv) > 3 else os.environ.get("DCAMD_LIB", "lib")
n = 1 << lg
xh = dcamd.gen_u10(n)
xh = xh - xh.min()
x = torch.from_numpy(np.ascontiguousarray(xh, np.float32)).cuda()
st = torch.zeros(L.stream_capacity(n), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
mean, t = L.med_device(x.data_ptr(), n)
m17 = int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)
ls = torch.cuda.ExternalStream(L.L.dc_get_stream())
for _ in range(5):
    L.encode_device(ct, x.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17)
torch.cuda.synchronize()
K = 20
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
for k in range(K):
    ev[k][0].record(ls)
    L.encode_device(ct, x.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17)
    ev[k][1].record(ls)
torch.cuda.synchronize()
us = [a.elapsed_time(b) * 1000 for a, b in ev]
print(f"{label}: encode 2^{lg} ct{ct} {np.mean(us):.1f} us (min {np.min(us):.1f}, max {np.max(us):.1f}), "
      f"status {L.encode_status()}", flush=True)
